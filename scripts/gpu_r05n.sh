# round 5: the primary rounds read C = centre - CameraPosition from the cull pass's table
# (TraceArgs.prim, 16 packed ops per sphere pair instead of 19) -- this tree against HEAD~
# (librt_trace_base.so): GPU suite, then same-box A/B on C2 / RTWeekend / the 8-rank share / C3
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
  > gpurun_out/r05n_pytest.log 2>&1; rc=$?; tail -1 gpurun_out/r05n_pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r05n_pytest.log | head; exit $rc; }
VARIANTS="RT_TRACE_LIB=librt_trace_base.so;RT_X=0" CONFIGS="c2;--config rtw;--sim-ranks 8 --sim-index 0;--config c3" ROUNDS=${ROUNDS:-3} \
  bash scripts/gpu_ab.sh
