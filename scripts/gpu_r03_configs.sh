# Current bench lines for C3, RTWeekend, C2-inside and C5 (steps 3, warm-up 3).
set -o pipefail
mkdir -p gpurun_out
for c in rtw c2in c3 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 3 --no-cpu-baseline > gpurun_out/cfg_$c.json 2> gpurun_out/cfg_$c.err || { tail -20 gpurun_out/cfg_$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/cfg_$c.json')); print('$c', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline'].get('frac'), d['cold_ms'])"
done
