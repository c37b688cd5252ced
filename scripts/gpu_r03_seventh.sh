# Frontier fold (ring readiness from the lanes' cursors) with three channel lanes, and
# per-wave order: GPU suite, then same-box A/B against the last commit's library.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r03_pytest7.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r03_pytest7.log | head; tail -30 gpurun_out/r03_pytest7.log; exit 1; }
tail -1 gpurun_out/r03_pytest7.log
LIBS="librt_trace_base.so librt_trace.so" ROUNDS=3 bash scripts/gpu_lib_ab.sh || exit 1
CFGS="RT_WAVE_ORDER=0;RT_WAVE_ORDER=1" ROUNDS=2 bash scripts/gpu_env_ab.sh || exit 1
