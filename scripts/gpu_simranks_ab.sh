# sim-ranks A/B: bash scripts/gpu_simranks_ab.sh <G> "ENV=.." ...   (one rank's share of a G-GPU C2 frame)
set -o pipefail
mkdir -p gpurun_out
g=$1; shift
for cfg in "$@"; do
  r=$(env $cfg timeout -k 10 120 python bench.py --steps 8 --warmup 3 --no-cpu-baseline --sim-ranks $g 2> gpurun_out/sim.err | tail -1) || { tail -5 gpurun_out/sim.err; exit 1; }
  echo "G=$g $cfg $r"
done
