# Marginal cost of bounce segments: C2 at several max-bounce settings (timed
# with the production build), then the scheduling counters (RT_STATS build).
set -o pipefail
BOUNCES=${BOUNCES:-1 2 3 4 8}
mkdir -p gpurun_out
for b in $BOUNCES; do
  env $EXTRA timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --bounces $b > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/b.json')); print('B=$b', d['value'], d['roofline']['kernel_ms'], d['config']['rays_per_step'])"
done
for b in 1 8; do
  env RT_STATS=1 RT_TRACE_LIB=librt_trace_stats.so $EXTRA timeout -k 10 120 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --bounces $b > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/b.json')); print('stats B=$b', d.get('sched_stats'))"
done
