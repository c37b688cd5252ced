# Height-slab test in the per-lane cluster walk: GPU suite (random scenes include
# per-lane-threshold ones), then RTWeekend / C2 against the previous commit's library.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r03_pytest8.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r03_pytest8.log | head; tail -30 gpurun_out/r03_pytest8.log; exit 1; }
tail -1 gpurun_out/r03_pytest8.log
CONFIGS="--config rtw;c2" LIBS="librt_trace_base.so librt_trace.so" ROUNDS=2 bash scripts/gpu_lib_ab.sh || exit 1
