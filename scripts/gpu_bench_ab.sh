# Same-box A/B of two bench.py versions (bench_prev.py = e.g. git show HEAD~1:bench.py, copied in
# for the call) on C2 and the 8-rank share, after the GPU suite.
# usage: git show <rev>:bench.py > bench_prev.py; bash scripts/gpu_bench_ab.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ctr_pytest.log 2>&1 || { tail -20 gpurun_out/ctr_pytest.log; exit 1; }
tail -1 gpurun_out/ctr_pytest.log
for r in 1 2 3; do
  for b in bench_prev.py bench.py; do
    for a in "" "--sim-ranks 8 --sim-index 3"; do
      timeout -k 10 120 python $b --steps 10 --warmup 6 --no-cpu-baseline $a > gpurun_out/cab.json 2> gpurun_out/cab.err || { tail -20 gpurun_out/cab.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/cab.json')); print('$r', '$b', '[$a]', d.get('value'), d.get('ms_per_step'), d.get('roofline',{}).get('kernel_ms', d.get('rank0_kernel_ms')), d.get('segments',{}).get('counted_equal_every_timed_step'))"
    done
  done
done
