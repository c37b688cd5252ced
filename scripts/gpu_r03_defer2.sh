# Deferred shading with the one-wave kernels' cull mask in dynamic LDS: GPU suite, then a
# same-box A/B of HEAD (base), no deferral (nodefer) and deferral (default) on C2 and the 8-rank share.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
LIBS="librt_trace_base.so librt_trace_nodefer.so librt_trace.so" ROUNDS=2 timeout -k 10 600 bash scripts/gpu_lib_ab.sh || exit $?
LIBS="librt_trace_base.so librt_trace_nodefer.so librt_trace.so" ROUNDS=1 CONFIGS="--config rtw" timeout -k 10 600 bash scripts/gpu_lib_ab.sh
