# Round 3 first GPU pass: the GPU suite, the default bench line, the launcher-free
# 8-share bench (all shares on this one GPU), and the OnRender loop against the
# round-2 library (RT_TRACE_LIB=librt_trace_r02.so, built by scripts/build_base_lib.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r03_pytest.log 2>&1
rc=$?
tail -4 gpurun_out/r03_pytest.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" gpurun_out/r03_pytest.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r03_bench.log 2>&1 || { tail -5 gpurun_out/r03_bench.log; exit 1; }
tail -1 gpurun_out/r03_bench.log | cut -c1-600
BENCH_SHARE_GPU=1 timeout -k 10 200 python bench.py --gpus 8 --steps 10 --warmup 3 > gpurun_out/r03_multi8.log 2>&1 || { tail -5 gpurun_out/r03_multi8.log; exit 1; }
tail -1 gpurun_out/r03_multi8.log | cut -c1-900
timeout -k 10 300 python bench.py --config onrender --frames 256 > gpurun_out/r03_onrender.log 2>&1 || { tail -5 gpurun_out/r03_onrender.log; exit 1; }
RT_TRACE_LIB=librt_trace_r02.so timeout -k 10 300 python bench.py --config onrender --frames 256 > gpurun_out/r03_onrender_r02.log 2>&1 || { tail -5 gpurun_out/r03_onrender_r02.log; exit 1; }
grep '"mode"' gpurun_out/r03_onrender.log gpurun_out/r03_onrender_r02.log | cut -c1-400
