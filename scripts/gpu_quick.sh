# Quick A/B: GPU parity (default variant) + bench for each env config given as args.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
for cfg in "$@"; do
  env $cfg timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/b.json')); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
