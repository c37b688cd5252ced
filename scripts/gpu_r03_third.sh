# Kernel traces: the 8-rank share (this tree against the round-2 library) and the
# OnRender loop; then the round-3 PMC passes (scripts/gpu_r03_pmc.sh).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for lib in librt_trace_r02.so librt_trace.so; do
  RT_TRACE_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_s8_$lib -o kt --output-format csv -- \
    python bench.py --steps 10 --warmup 6 --no-cpu-baseline --sim-ranks 8 --sim-index 3 > gpurun_out/kt_s8_$lib.log 2>&1 || { tail -5 gpurun_out/kt_s8_$lib.log; exit 1; }
  tail -1 gpurun_out/kt_s8_$lib.log
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_onr -o kt --output-format csv -- \
  python bench.py --config onrender --frames 64 --width 1920 --height 1080 > gpurun_out/kt_onr.log 2>&1 || { tail -5 gpurun_out/kt_onr.log; exit 1; }
grep '"mode"' gpurun_out/kt_onr.log | cut -c1-300
bash scripts/gpu_r03_pmc.sh
