# Lane loss to finished pixels: scheduling counters of the RT_STATS build at 1 GPU
# and at the 8-rank share (needs librt_trace_stats.so: make variant NAME=stats KFLAGS=-DRTK_STATS).
set -o pipefail
mkdir -p gpurun_out
for args in "" "--sim-ranks 8 --sim-index 3"; do
  env RT_STATS=1 RT_TRACE_LIB=librt_trace_stats.so timeout -k 10 120 python bench.py --steps 1 --warmup 2 --no-cpu-baseline $args > gpurun_out/s.json 2> gpurun_out/s.err || { tail -20 gpurun_out/s.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/s.json')); print('$args', d.get('value'), d.get('sched_stats') or d)"
done
