# GPU parity suite (default build), then bench A/B over env configs given as args.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/pytest_gpu.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/pytest_gpu.log; exit $rc; }
for cfg in "$@"; do
  env $cfg timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/b.json')); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
