# A/B of env settings on the 1-GPU C2 frame and on one rank's share of a G-GPU frame:
# bash scripts/gpu_ab_sim.sh <G> "ENV=.." ...
set -o pipefail
mkdir -p gpurun_out
g=$1; shift
for cfg in "$@"; do
  env $cfg timeout -k 10 120 python bench.py --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/ab1.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  one=$(python -c "import json; d=json.load(open('gpurun_out/ab1.json')); print(d['value'], d['roofline']['kernel_ms'])")
  env $cfg timeout -k 10 120 python bench.py --steps 5 --warmup 3 --no-cpu-baseline --sim-ranks $g > gpurun_out/abg.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  sim=$(python -c "import json; d=json.load(open('gpurun_out/abg.json')); print(d['rank0_kernel_ms'])")
  echo "[$cfg] 1gpu: $one  sim$g: $sim"
done
