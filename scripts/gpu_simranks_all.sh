# Every rank's share of a G-GPU C2 frame traced alone on this GPU: bash scripts/gpu_simranks_all.sh <G> [bench args]
# (STEPS / WARMUP: default 10 timed launches after 7 warm-ups, past the 6 launches that learn the wave order)
set -o pipefail
mkdir -p gpurun_out
g=$1; shift
for r in $(seq 0 $((g - 1))); do
  timeout -k 10 120 python bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-7} --no-cpu-baseline "$@" --sim-ranks $g --sim-index $r 2> gpurun_out/sim.err | tail -1 || { tail -5 gpurun_out/sim.err; exit 1; }
done
