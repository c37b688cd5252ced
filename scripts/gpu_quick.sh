# Quick A/B: GPU parity for each lanes-per-pixel shape, then bench for each env config given as args.
set -o pipefail
mkdir -p gpurun_out
for lp in 4 2 1; do
  RT_LANES_PER_PIXEL=$lp timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu_lp$lp.log 2>&1
  rc=$?; echo "pytest P=$lp rc=$rc $(tail -1 gpurun_out/pytest_gpu_lp$lp.log)"; [ $rc -gt 1 ] && exit $rc
done
for cfg in "$@"; do
  env $cfg timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/b.json')); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
