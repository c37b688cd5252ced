# New OnRender tests (busy poll, moving camera), then the cluster count sweep.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k on_render --timeout 120 --timeout-method thread > gpurun_out/onr_pytest.log 2>&1 || { tail -30 gpurun_out/onr_pytest.log; exit 1; }
tail -1 gpurun_out/onr_pytest.log
bash scripts/gpu_r03_ksweep2.sh
