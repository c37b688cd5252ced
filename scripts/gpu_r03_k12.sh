# Parity suite + RTWeekend / C2 bench after the relative-table cluster count change.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/k12_pytest.log 2>&1 || { tail -30 gpurun_out/k12_pytest.log; exit 1; }
tail -2 gpurun_out/k12_pytest.log
for c in rtw c2; do
  timeout -k 10 120 python bench.py --config $c --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/k12_$c.json 2> gpurun_out/k12_$c.err || { tail -5 gpurun_out/k12_$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/k12_$c.json')); print('$c', d['value'], d['ms_per_step'])"
done
