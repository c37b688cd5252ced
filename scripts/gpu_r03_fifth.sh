# Raw wave timelines (C2 and the 8-rank share) for offline schedule simulation,
# and the RTK_STATS scheduling counters of C2, the share, RTWeekend and C5 (1/8 spp).
set -o pipefail
mkdir -p gpurun_out
SAVE=gpurun_out/wt_s8.npz SIM_RANKS=8 timeout -k 10 120 python scripts/wave_tail.py > gpurun_out/wt_s8.txt 2>&1 || { tail -5 gpurun_out/wt_s8.txt; exit 1; }
SAVE=gpurun_out/wt_c2.npz SIM_RANKS=1 timeout -k 10 120 python scripts/wave_tail.py > gpurun_out/wt_c2.txt 2>&1 || { tail -5 gpurun_out/wt_c2.txt; exit 1; }
for args in "" "--sim-ranks 8 --sim-index 0" "--config rtw" "--config c5 --spp 512"; do
  env RT_STATS=1 RT_TRACE_LIB=librt_trace_stats.so timeout -k 10 200 python bench.py --steps 1 --warmup 2 --no-cpu-baseline $args > gpurun_out/s.json 2> gpurun_out/s.err || { tail -20 gpurun_out/s.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/s.json')); print('[$args]', d.get('value'), json.dumps(d.get('sched_stats')))"
done
