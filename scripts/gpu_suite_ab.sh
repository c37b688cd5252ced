# GPU suite, then a same-box A/B of this tree against librt_trace_base.so (scripts/build_base_lib.sh):
#   bash scripts/gpu_suite_ab.sh TAG   (CONFIGS / ROUNDS as scripts/gpu_ab.sh; default C2, RTWeekend, the 8-rank share)
set -o pipefail
tag=${1:-ab}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
  > gpurun_out/${tag}_pytest.log 2>&1; rc=$?; tail -1 gpurun_out/${tag}_pytest.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/${tag}_pytest.log | head; exit $rc; }
VARIANTS="RT_TRACE_LIB=librt_trace_base.so;default" CONFIGS="${CONFIGS:-c2;--config rtw;--sim-ranks 8 --sim-index 0}" \
  ROUNDS=${ROUNDS:-3} bash scripts/gpu_ab.sh
