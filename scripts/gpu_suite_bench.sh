# GPU parity suite, the default bench line, and the counter list (for the PMC plan).
# usage: bash scripts/gpu_suite_bench.sh <tag>
set -o pipefail
mkdir -p gpurun_out
tag=${1:-run}
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/pytest_gpu_$tag.log)"; [ $rc -ne 0 ] && { grep -E "FAILED|Error|error" gpurun_out/pytest_gpu_$tag.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { tail -20 gpurun_out/bench_$tag.err; exit 1; }
cat gpurun_out/bench_$tag.json
