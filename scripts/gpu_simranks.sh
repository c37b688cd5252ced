# One rank's share of a G-GPU C2 frame, traced alone on this GPU (strong-scaling forecast).
set -o pipefail
mkdir -p gpurun_out
for g in 2 4 8; do
  env $EXTRA timeout -k 10 120 python bench.py --steps 5 --warmup 3 --no-cpu-baseline --sim-ranks $g 2> gpurun_out/sim.err | tail -1 || { tail -5 gpurun_out/sim.err; exit 1; }
done
