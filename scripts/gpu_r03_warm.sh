# The 8-rank share and C2 at the driver's step counts (--steps 20 --warmup 5) against --steps 5 --warmup 3.
set -o pipefail
mkdir -p gpurun_out
for sw in "5 3" "20 5" "20 12"; do
  set -- $sw
  timeout -k 10 120 python bench.py --steps $1 --warmup $2 --no-cpu-baseline --sim-ranks 8 --sim-index 3 2> gpurun_out/w.err | tail -1 | sed "s/^/steps $1 warmup $2 /" || exit 1
done
for sw in "5 3" "20 5"; do
  set -- $sw
  timeout -k 10 120 python bench.py --steps $1 --warmup $2 --no-cpu-baseline > gpurun_out/w.json 2> gpurun_out/w.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/w.json')); print('C2 steps $1 warmup $2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
