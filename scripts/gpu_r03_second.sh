# OnRender rework check (C host + multi tests, onrender bench new vs r02) and the
# same-box C2 / 8-rank-share A/B of this tree against the round-2 library.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_c_host.py tests/test_gpu_multi.py -m gpu -x -q --timeout 240 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r03_pytest2.log 2>&1 || { tail -30 gpurun_out/r03_pytest2.log; exit 1; }
tail -2 gpurun_out/r03_pytest2.log
timeout -k 10 300 python bench.py --config onrender --frames 256 > gpurun_out/r03_onrender.log 2>&1 || { tail -5 gpurun_out/r03_onrender.log; exit 1; }
grep '"mode"' gpurun_out/r03_onrender.log | cut -c1-420
LIBS="librt_trace_r02.so librt_trace.so" ROUNDS=3 bash scripts/gpu_lib_ab.sh
