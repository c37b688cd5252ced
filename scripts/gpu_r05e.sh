# round 5: RGBA8 by a coalesced encode pass after the launch (RT_CUR_PASS=1): parity suite under it, A/B, HBM bytes
set -o pipefail
RT_CUR_PASS=1 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
  > gpurun_out/r05e_pytest_curpass.log 2>&1; rc=$?; tail -2 gpurun_out/r05e_pytest_curpass.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r05e_pytest_curpass.log | head; exit $rc; }
VARIANTS="RT_CUR_PASS=0;RT_CUR_PASS=1" CONFIGS="c2;--config rtw;--sim-ranks 8 --sim-index 3" ROUNDS=2 bash scripts/gpu_ab.sh && \
VARIANTS="RT_CUR_PASS=0;RT_CUR_PASS=1" CONFIGS="c2;--config rtw" bash scripts/gpu_writes.sh
