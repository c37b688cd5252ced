# A/B on one box: GPU parity under each env in $PARITY (';'-separated), then
# bench C2 for each env config given as args (prints value, ms/step, kernel ms).
set -o pipefail
mkdir -p gpurun_out
IFS=';' read -ra PCFG <<< "${PARITY:-RT_LANES_PER_PIXEL=4}"
i=0
for cfg in "${PCFG[@]}"; do
  i=$((i+1))
  env $cfg timeout -k 10 600 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/ab_pytest_$i.log 2>&1
  rc=$?; echo "pytest [$cfg] rc=$rc $(tail -1 gpurun_out/ab_pytest_$i.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/ab_pytest_$i.log; exit $rc; }
done
for cfg in "$@"; do
  env $cfg timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/b.json')); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['config']['rays_per_step'], d.get('sched_stats',''))"
done
