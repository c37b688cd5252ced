# Whole-batch fold: GPU suite, then same-box A/B against the previous commit (C2, 8-rank share, RTWeekend).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/whole_pytest.log 2>&1 || { tail -30 gpurun_out/whole_pytest.log; exit 1; }
tail -1 gpurun_out/whole_pytest.log
LIBS="librt_trace_base.so librt_trace.so" ROUNDS=2 CONFIGS="c2;--sim-ranks 8 --sim-index 3;--config rtw" bash scripts/gpu_lib_ab.sh
