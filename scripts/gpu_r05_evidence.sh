# Round-5 evidence at the final kernel (writes gpurun_out/ev_<tag>_*):
#   part 1: smoke, the default bench line, kernel trace + stats, C2 and RTWeekend PMC records
#   part 2: every 8-rank share, the 2- and 4-rank shares, the share PMC records, the other configs, OnRender
# usage: bash scripts/gpu_r05_evidence.sh <tag> [1|2|all]
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r05}; part=${2:-all}
if [ "$part" = 1 ] || [ "$part" = all ]; then
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ev_${tag}_smoke.log 2>&1 || { tail -5 gpurun_out/ev_${tag}_smoke.log; exit 1; }
  tail -1 gpurun_out/ev_${tag}_smoke.log
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ev_${tag}_bench.json 2> gpurun_out/ev_${tag}_bench.err || { tail -5 gpurun_out/ev_${tag}_bench.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ev_${tag}_bench.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], 'verified', d.get('verified'), 'cpu', d['cpu_baseline']['value'])"
  TAG=ev_${tag}_trace bash scripts/gpu_trace_launches.sh > gpurun_out/ev_${tag}_launches.txt 2>&1 || { tail -5 gpurun_out/ev_${tag}_launches.txt; exit 1; }
  bash scripts/gpu_pmc.sh ev_${tag} > gpurun_out/ev_${tag}_pmc_stdout.txt 2>&1 || { tail -5 gpurun_out/ev_${tag}_pmc_stdout.txt; exit 1; }
  python scripts/pmc_to_json.py gpurun_out pmc_ev_${tag}_ gpurun_out/ev_${tag}_c2_pmc.json "C2: 1920x1080, 256 spp, 64 spheres, 8 bounces, SIMD rules" || exit 1
  bash scripts/gpu_pmc.sh ev_${tag}rtw --config rtw > gpurun_out/ev_${tag}_rtw_pmc_stdout.txt 2>&1 || { tail -5 gpurun_out/ev_${tag}_rtw_pmc_stdout.txt; exit 1; }
  python scripts/pmc_to_json.py gpurun_out pmc_ev_${tag}rtw_ gpurun_out/ev_${tag}_rtw_pmc.json "RTW: 1920x1080, 64 spp, 482 spheres, 8 bounces, SIMD rules, RTWeekend" || exit 1
  echo part1 done
fi
if [ "$part" = 2 ] || [ "$part" = all ]; then
  bash scripts/gpu_simranks_all.sh 8 > gpurun_out/ev_${tag}_simranks8.txt 2>&1 || exit 1
  { bash scripts/gpu_simranks_all.sh 2 && bash scripts/gpu_simranks_all.sh 4; } > gpurun_out/ev_${tag}_simranks24.txt 2>&1 || exit 1
  for g in 8 4 2; do
    bash scripts/gpu_pmc.sh ev_${tag}r$g --sim-ranks $g --sim-index 0 > gpurun_out/ev_${tag}_r${g}_pmc_stdout.txt 2>&1 || { tail -5 gpurun_out/ev_${tag}_r${g}_pmc_stdout.txt; exit 1; }
    python scripts/pmc_to_json.py gpurun_out pmc_ev_${tag}r${g}_ gpurun_out/ev_${tag}_c2_rank${g}_pmc.json "C2: 1920x1080, 256 spp, 64 spheres, 8 bounces, SIMD rules" $g || exit 1
  done
  for cfg in c3 rtw c2in; do
    timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 3 --no-cpu-baseline >> gpurun_out/ev_${tag}_configs.jsonl 2>> gpurun_out/ev_${tag}_configs.err || exit 1
  done
  timeout -k 10 300 python bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline >> gpurun_out/ev_${tag}_configs.jsonl 2>> gpurun_out/ev_${tag}_configs.err || exit 1
  timeout -k 10 300 python bench.py --config onrender > gpurun_out/ev_${tag}_onrender.json 2> gpurun_out/ev_${tag}_onrender.err || exit 1
  echo part2 done
fi
