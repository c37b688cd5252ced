# Marginal cost of bounce segments: C2 at several max-bounce settings (RT_STATS on).
set -o pipefail
mkdir -p gpurun_out
for b in 1 2 4 8; do
  env RT_STATS=1 $EXTRA timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --bounces $b > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/b.json')); s=d.get('sched_stats',{}); print('B=$b', d['value'], d['roofline']['kernel_ms'], d['config']['rays_per_step'], {k:s[k]//4 for k in ('pri_iters','pri_lanes','sec_iters','sec_lanes','pri_groups')})"
done
