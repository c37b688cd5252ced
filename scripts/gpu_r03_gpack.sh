# Per-class group indices packed in 16-bit halves (two VGPRs fewer: C2's and C5's kernels
# at 63 VGPRs, 8 waves/SIMD without spills): GPU suite, then a same-box A/B against HEAD.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
LIBS="librt_trace_base.so librt_trace.so" ROUNDS=3 timeout -k 10 600 bash scripts/gpu_lib_ab.sh || exit $?
LIBS="librt_trace_base.so librt_trace.so" ROUNDS=2 CONFIGS="--config rtw;--config c5 --spp 512" timeout -k 10 600 bash scripts/gpu_lib_ab.sh
