# rt_multi new-camera calls under a kernel trace (do the devices' cull passes and
# traces overlap?), then the experiments of scripts/gpu_r03_exp.sh.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ov_kt -o run --output-format csv -- python3 scripts/multi_cold_overlap.py 4 > gpurun_out/ov.log 2>&1 || { tail -5 gpurun_out/ov.log; exit 1; }
grep "calls done" gpurun_out/ov.log
python scripts/multi_trace_report.py gpurun_out/ov_kt | tail -6
bash scripts/gpu_r03_exp.sh
