# Member-level behind-origin test off (RTK_MEMBER_BEHIND=0) against the default: parity of the
# variant on the GPU suite's parity files, then a same-box A/B on C2, the 8-rank share, RTW and C5.
set -o pipefail
mkdir -p gpurun_out
RT_TRACE_LIB=librt_trace_nobehind.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden_regression.py tests/test_gpu_random_scenes.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_nb.log 2>&1
rc=$?; echo "pytest (nobehind) rc=$rc"; tail -2 gpurun_out/pytest_nb.log
[ $rc -ne 0 ] && exit $rc
LIBS="librt_trace.so librt_trace_nobehind.so" ROUNDS=3 timeout -k 10 600 bash scripts/gpu_lib_ab.sh || exit $?
LIBS="librt_trace.so librt_trace_nobehind.so" ROUNDS=1 CONFIGS="--config rtw;--config c5 --spp 512" timeout -k 10 600 bash scripts/gpu_lib_ab.sh
