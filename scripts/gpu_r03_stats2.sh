# RTK_STATS scheduling counters of RTWeekend (slab walk, K = 40) and C5 at 512 spp.
set -o pipefail
mkdir -p gpurun_out
for args in "--config rtw" "--config c5 --spp 512"; do
  env RT_STATS=1 RT_TRACE_LIB=librt_trace_stats.so timeout -k 10 200 python bench.py --steps 1 --warmup 2 --no-cpu-baseline $args > gpurun_out/s.json 2> gpurun_out/s.err || { tail -20 gpurun_out/s.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/s.json')); print('[$args]', d['value'], json.dumps(d.get('sched_stats')))"
done
