# Two-level defaults: GPU suite, RTWeekend / C5 / C2, the scheduling counters of
# RTWeekend and C5 (512 spp), and the secondary-threshold re-sweep.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tld_pytest.log 2>&1 || { tail -30 gpurun_out/tld_pytest.log; exit 1; }
tail -1 gpurun_out/tld_pytest.log
for c in rtw c5 c2; do
  timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/tld_$c.json 2> gpurun_out/tld_$c.err || { tail -5 gpurun_out/tld_$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/tld_$c.json')); print('$c', d['value'], d['ms_per_step'])"
done
bash scripts/gpu_r03_stats2.sh || exit 1
SS="32 40 56" bash scripts/gpu_r03_ssweep.sh 2>&1 | grep -v "config c2"
