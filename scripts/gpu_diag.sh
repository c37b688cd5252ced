# Diagnostics: prefilter flag counters (stats build) and the per-wave
# occupancy timeline of one launch at 1 and 8 simulated ranks.
set -o pipefail
mkdir -p gpurun_out
env RT_STATS=1 RT_TRACE_LIB=librt_trace_stats.so timeout -k 10 120 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
python -c "import json,sys; d=json.load(open('gpurun_out/b.json')); print('stats', d.get('sched_stats'))" || exit 1
for g in 1 8; do
  SIM_RANKS=$g timeout -k 10 120 python scripts/wave_tail.py > gpurun_out/wt_$g.txt 2>&1 || { tail -20 gpurun_out/wt_$g.txt; exit 1; }
  echo "== sim ranks $g"; cat gpurun_out/wt_$g.txt
done
