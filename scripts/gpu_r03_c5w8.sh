# 8 waves/SIMD for the cl2 walk (C5): GPU suite, full C5 (4096 spp) base vs new, C2 check, VALU op costs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
LIBS="librt_trace_base.so librt_trace.so" ROUNDS=1 CONFIGS="c2;--config c5" timeout -k 10 600 bash scripts/gpu_lib_ab.sh || exit $?
timeout -k 10 120 ./scripts/mb_ops
