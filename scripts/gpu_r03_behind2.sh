# Member behind test off for per-lane (REL) tables only: GPU suite, then same-box A/B against HEAD
# on RTWeekend (cl4rel), C2 (cl1, unchanged code) and C5 (cl2, unchanged code).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
LIBS="librt_trace_base.so librt_trace.so" ROUNDS=3 CONFIGS="--config rtw;c2" timeout -k 10 600 bash scripts/gpu_lib_ab.sh
