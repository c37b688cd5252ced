# fold weights by rcp_rn/div_rn, no per-launch event marker: GPU suite (parity),
# same-box A/B against the round-2 library (C2 + 8-rank share), the share's
# kernel-to-kernel gaps, and its wave timeline.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r03_pytest4.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r03_pytest4.log | head; tail -30 gpurun_out/r03_pytest4.log; exit 1; }
tail -1 gpurun_out/r03_pytest4.log
LIBS="librt_trace_r02.so librt_trace.so" ROUNDS=3 bash scripts/gpu_lib_ab.sh || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/kt4_s8 -o kt --output-format csv -- \
  python bench.py --steps 10 --warmup 6 --no-cpu-baseline --sim-ranks 8 --sim-index 3 > gpurun_out/kt4_s8.log 2>&1 || { tail -5 gpurun_out/kt4_s8.log; exit 1; }
SIM_RANKS=8 timeout -k 10 120 python scripts/wave_tail.py > gpurun_out/r03_wave_tail_s8.txt 2>&1 || { tail -5 gpurun_out/r03_wave_tail_s8.txt; exit 1; }
SIM_RANKS=1 timeout -k 10 120 python scripts/wave_tail.py > gpurun_out/r03_wave_tail_c2.txt 2>&1 || { tail -5 gpurun_out/r03_wave_tail_c2.txt; exit 1; }
head -30 gpurun_out/r03_wave_tail_s8.txt
