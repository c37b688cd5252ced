# bench A/B over env configs given as args (no parity run), then stats for the default.
set -o pipefail
mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/b.json')); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
env RT_STATS=1 RT_TRACE_LIB=librt_trace_stats.so timeout -k 10 120 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
python -c "import json,sys; d=json.load(open('gpurun_out/b.json')); print('stats', d.get('sched_stats'))"
