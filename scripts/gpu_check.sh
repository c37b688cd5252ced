set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -2 gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r1 --output-format csv -- python bench.py --steps 3 --warmup 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit $?
ls -R gpurun_out/prof | head -20
