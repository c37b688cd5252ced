# Parity under every kernel variant, then a bench sweep of the variants.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest default rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
RT_CULL=0 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu_nocull.log 2>&1
rc=$?; echo "pytest nocull rc=$rc"; tail -2 gpurun_out/pytest_gpu_nocull.log; [ $rc -gt 1 ] && exit $rc
RT_SPHERE_SRC=lds timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu_lds.log 2>&1
rc=$?; echo "pytest lds rc=$rc"; tail -2 gpurun_out/pytest_gpu_lds.log; [ $rc -gt 1 ] && exit $rc
for cfg in "RT_CULL=0 RT_SEC_THRESHOLD=1" "RT_CULL=0 RT_SEC_THRESHOLD=32" "RT_CULL=1 RT_SEC_THRESHOLD=16" "RT_CULL=1 RT_SEC_THRESHOLD=32" "RT_CULL=1 RT_SEC_THRESHOLD=48" "RT_CULL=1 RT_SEC_THRESHOLD=32 RT_SPHERE_SRC=lds"; do
  env $cfg timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/b.json')); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
