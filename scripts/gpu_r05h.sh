# round 5: each block tile's waves grouped onto one XCD (RT_XCD_GROUP, default on): GPU suite, A/B, HBM bytes
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
  > gpurun_out/r05h_pytest.log 2>&1; rc=$?; tail -1 gpurun_out/r05h_pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r05h_pytest.log | head; exit $rc; }
VARIANTS="RT_XCD_GROUP=0;RT_XCD_GROUP=1" CONFIGS="c2;--config rtw;--sim-ranks 8 --sim-index 3" ROUNDS=3 bash scripts/gpu_ab.sh && \
VARIANTS="RT_XCD_GROUP=0;RT_XCD_GROUP=1;RT_XCD_GROUP=1 RT_PIXEL_SEG=2" CONFIGS="c2;--config rtw" bash scripts/gpu_writes.sh
