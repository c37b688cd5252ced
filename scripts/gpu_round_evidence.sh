# Round evidence in one call: GPU suite, the default bench line, rocprofv3 kernel
# trace + stats, the PMC passes, every 8-rank share, the other bench configurations.
# usage: bash scripts/gpu_round_evidence.sh <tag>   (writes gpurun_out/ev_<tag>_*)
set -o pipefail
mkdir -p gpurun_out
tag=${1:-ev}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ev_${tag}_pytest.log 2>&1 || { tail -20 gpurun_out/ev_${tag}_pytest.log; exit 1; }
tail -1 gpurun_out/ev_${tag}_pytest.log
timeout -k 10 300 python bench.py > gpurun_out/ev_${tag}_bench.json 2> gpurun_out/ev_${tag}_bench.err || { tail -5 gpurun_out/ev_${tag}_bench.err; exit 1; }
tail -c 400 gpurun_out/ev_${tag}_bench.json; echo
TAG=ev_${tag}_trace bash scripts/gpu_trace_launches.sh > gpurun_out/ev_${tag}_launches.txt 2>&1 || { tail -5 gpurun_out/ev_${tag}_launches.txt; exit 1; }
bash scripts/gpu_pmc.sh ev_${tag} > gpurun_out/ev_${tag}_pmc_stdout.txt 2>&1 || { tail -5 gpurun_out/ev_${tag}_pmc_stdout.txt; exit 1; }
python scripts/pmc_to_json.py gpurun_out pmc_ev_${tag}_ gpurun_out/ev_${tag}_c2_pmc.json "C2: 1920x1080, 256 spp, 64 spheres, 8 bounces, SIMD rules" || exit 1
bash scripts/gpu_pmc.sh ev_${tag}rtw --config rtw > gpurun_out/ev_${tag}_rtw_pmc_stdout.txt 2>&1 || { tail -5 gpurun_out/ev_${tag}_rtw_pmc_stdout.txt; exit 1; }
python scripts/pmc_to_json.py gpurun_out pmc_ev_${tag}rtw_ gpurun_out/ev_${tag}_rtw_pmc.json "RTW: 1920x1080, 64 spp, 482 spheres, 8 bounces, SIMD rules, RTWeekend" || exit 1
bash scripts/gpu_simranks_all.sh 8 > gpurun_out/ev_${tag}_simranks8.txt 2>&1 || exit 1
for cfg in c3 rtw c2in; do
  timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 3 --no-cpu-baseline >> gpurun_out/ev_${tag}_configs.jsonl 2>> gpurun_out/ev_${tag}_configs.err || exit 1
done
timeout -k 10 300 python bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline >> gpurun_out/ev_${tag}_configs.jsonl 2>> gpurun_out/ev_${tag}_configs.err || exit 1
echo done
