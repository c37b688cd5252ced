# Closing check at HEAD: GPU suite, smoke(), the default bench line, the RTWeekend PMC record
# and bench line (its member rule changed), C5 line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/fin_pytest.log 2>&1 || { tail -20 gpurun_out/fin_pytest.log; exit 1; }
tail -1 gpurun_out/fin_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 || { tail -5 gpurun_out/fin_smoke.log; exit 1; }
tail -2 gpurun_out/fin_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/fin_bench.json 2> gpurun_out/fin_bench.err || { tail -5 gpurun_out/fin_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/fin_bench.json')); print('C2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['source'])"
bash scripts/gpu_pmc.sh fin_rtw --config rtw > gpurun_out/fin_pmc_stdout.txt 2>&1 || { tail -5 gpurun_out/fin_pmc_stdout.txt; exit 1; }
python scripts/pmc_to_json.py gpurun_out pmc_fin_rtw_ gpurun_out/r03b_rtw_pmc.json "RTW: 1920x1080, 64 spp, 482 spheres, 8 bounces, SIMD rules, RTWeekend" > /dev/null || exit 1
python scripts/pmc_brief.py gpurun_out/r03b_rtw_pmc.json
for cfg in rtw c3 c2in; do
  timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 3 --no-cpu-baseline >> gpurun_out/fin_configs.jsonl 2>> gpurun_out/fin_configs.err || exit 1
done
timeout -k 10 300 python bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline >> gpurun_out/fin_configs.jsonl 2>> gpurun_out/fin_configs.err || exit 1
python -c "
import json
for l in open('gpurun_out/fin_configs.jsonl'):
    d=json.loads(l); print(d['config']['workload'][:40], d['value'], d['ms_per_step'], d['roofline'].get('frac'))"
