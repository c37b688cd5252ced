# round 5: wave costs recorded only on re-sorting launches (this tree) against HEAD~ (librt_trace_base.so):
# GPU suite, A/B on C2 / RTWeekend / the 8-rank share, trace-kernel HBM bytes
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
  > gpurun_out/r05g_pytest.log 2>&1; rc=$?; tail -1 gpurun_out/r05g_pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r05g_pytest.log | head; exit $rc; }
VARIANTS="RT_TRACE_LIB=librt_trace_base.so;RT_X=0" CONFIGS="c2;--config rtw;--sim-ranks 8 --sim-index 3" ROUNDS=3 bash scripts/gpu_ab.sh && \
VARIANTS="RT_TRACE_LIB=librt_trace_base.so;RT_X=0;RT_PIXEL_SEG=2" CONFIGS="c2;--config rtw" bash scripts/gpu_writes.sh
