# PC sampling of one bench launch (stochastic, per-instruction hot spots).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 -L > gpurun_out/pcs_list.txt 2>&1 || true
grep -i -A12 "pc sampling\|pc_sampling" gpurun_out/pcs_list.txt | head -60
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
  --pc-sampling-interval ${PCS_INTERVAL:-65536} -d gpurun_out/pcs -o pcs --output-format csv -- \
  python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pcs.log 2>&1
rc=$?; echo "rc=$rc"; tail -5 gpurun_out/pcs.log; ls -la gpurun_out/pcs | head
