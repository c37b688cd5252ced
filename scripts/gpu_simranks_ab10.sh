# sim-ranks A/B with 10 timed launches: bash scripts/gpu_simranks_ab10.sh <G> "ENV=.." ...
set -o pipefail
g=$1; shift
for cfg in "$@"; do
  r=$(env $cfg timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --sim-ranks $g 2> gpurun_out/sim.err | tail -1) || { tail -5 gpurun_out/sim.err; exit 1; }
  echo "G=$g $cfg $r"
done
