# 8-rank share diagnosis: every residue's kernel time, then the scheduling
# counters (RTK_STATS build) of residue 0 at 8 ranks and of the 1-GPU frame.
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_simranks_all.sh 8 || exit 1
for g in 8 1; do
  extra=""; [ $g -gt 1 ] && extra="--sim-ranks $g"
  env RT_STATS=1 RT_TRACE_LIB=librt_trace_stats.so timeout -k 10 120 python bench.py --steps 1 --warmup 3 --no-cpu-baseline $extra > gpurun_out/st_$g.json 2> gpurun_out/st.err || { tail -5 gpurun_out/st.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/st_$g.json')); print('$g', d.get('sched_stats'))"
done
