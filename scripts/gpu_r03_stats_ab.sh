# RTK_STATS scheduling counters of two stats builds on C2 (LIBS, default: deferred shading on / off).
set -o pipefail
mkdir -p gpurun_out
for lib in ${LIBS:-librt_trace_stats.so librt_trace_stats0.so}; do
  env RT_STATS=1 RT_TRACE_LIB=$lib timeout -k 10 200 python bench.py --steps 1 --warmup 2 --no-cpu-baseline $ARGS > gpurun_out/s.json 2> gpurun_out/s.err || { tail -20 gpurun_out/s.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/s.json')); print('$lib', d['value'], json.dumps(d.get('sched_stats')))"
done
