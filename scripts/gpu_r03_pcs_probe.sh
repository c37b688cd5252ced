# PC sampling probe: what rocprofv3 offers on gfx950 and the shape of its output (C2, 2 timed steps).
set -o pipefail
mkdir -p gpurun_out/pcs
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/pcs/list.txt 2>&1 || true
grep -i -B2 -A12 "pc_sampl\|pc sampl" $GRAFT_REPO_ROOT/gpurun_out/pcs/list.txt | head -60 || true
cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1000 -d /tmp/pcs -o pcs --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pcs/run.log 2>&1 || { tail -20 gpurun_out/pcs/run.log; exit 1; }
find /tmp/pcs -type f | xargs ls -la | tee gpurun_out/pcs/files.txt
for f in $(find /tmp/pcs -name "*.csv"); do echo "== $f"; head -3 $f; wc -l $f; done
