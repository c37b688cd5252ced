set -o pipefail
mkdir -p gpurun_out
for cfg in "RT_STATS=1 RT_CULL=1 RT_SEC_THRESHOLD=16" "RT_STATS=1 RT_CULL=1 RT_SEC_THRESHOLD=1" "RT_STATS=1 RT_CULL=0 RT_SEC_THRESHOLD=1"; do
  env $cfg timeout -k 10 120 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/b.json')); print('$cfg', d['value'], d['roofline']['kernel_ms'], d.get('sched_stats'))"
done
