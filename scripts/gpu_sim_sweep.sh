# One rank's share of a G-GPU C2 frame under several env settings (alternating
# with the default): bash scripts/gpu_sim_sweep.sh <G> "ENV=.." ...
set -o pipefail
mkdir -p gpurun_out
g=$1; shift
for cfg in "$@"; do
  for c in "X=0" "$cfg"; do
    env $c timeout -k 10 120 python bench.py --steps 5 --warmup 3 --no-cpu-baseline --sim-ranks $g > gpurun_out/sw.json 2> gpurun_out/sw.err || { tail -5 gpurun_out/sw.err; exit 1; }
    echo "[$c] $(python -c "import json; d=json.load(open('gpurun_out/sw.json')); print(d['rank0_kernel_ms'])")"
  done
done
