# Same-box multi-GPU forecast: the 1-GPU C2 frame, then every rank's share of a
# 2-, 4- and 8-GPU frame traced alone (bench.py --sim-ranks), then lanes-per-pixel
# alternatives for residue 0 of each split.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python bench.py --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/fc_c2.json 2> gpurun_out/fc.err || { tail -5 gpurun_out/fc.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/fc_c2.json')); print('C2 1 GPU', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
for g in 2 4 8; do
  echo "== $g ranks"
  bash scripts/gpu_simranks_all.sh $g || exit 1
done
for spec in "2 4" "2 8" "4 8" "4 16" "8 16" "8 32"; do
  set -- $spec
  RT_LANES_PER_PIXEL=$2 timeout -k 10 120 python bench.py --steps 5 --warmup 3 --no-cpu-baseline --sim-ranks $1 --sim-index 0 2> gpurun_out/fc.err | tail -1 | sed "s/^/P=$2 /" || { tail -5 gpurun_out/fc.err; exit 1; }
done
