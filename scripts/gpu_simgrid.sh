# One rank's kernel time for G-rank splits x forced lanes-per-pixel x tile order (tuning the auto rules).
set -o pipefail
for g in 1 2 4 8; do
  for e in "RT_LANES_PER_PIXEL=4 RT_TILE_ORDER=1" "RT_LANES_PER_PIXEL=8 RT_TILE_ORDER=1" "RT_LANES_PER_PIXEL=8 RT_TILE_ORDER=0" "RT_LANES_PER_PIXEL=16 RT_TILE_ORDER=0"; do
    if [ $g = 1 ]; then
      env $e timeout -k 10 120 python bench.py --steps 5 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('G=1 $e', d['roofline']['kernel_ms'])" || exit 1
    else
      env $e timeout -k 10 120 python bench.py --steps 5 --no-cpu-baseline --sim-ranks $g 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('G=$g $e', d['rank0_kernel_ms'])" || exit 1
    fi
  done
done
