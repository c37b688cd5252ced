# Round-5 PMC records at steady state (gpu_pmc.sh: the timed launch after 7 warm-ups) for C2, RTWeekend and the
# 8/4/2-rank shares, plus the same-box whole frame and every 8-rank residue (the multi-GPU forecast)
set -o pipefail
tag=${1:-r05p}
bash scripts/gpu_pmc.sh ev_${tag} > gpurun_out/ev_${tag}_pmc_stdout.txt 2>&1 || { tail -5 gpurun_out/ev_${tag}_pmc_stdout.txt; exit 1; }
python scripts/pmc_to_json.py gpurun_out pmc_ev_${tag}_ gpurun_out/ev_${tag}_c2_pmc.json "C2: 1920x1080, 256 spp, 64 spheres, 8 bounces, SIMD rules" || exit 1
bash scripts/gpu_pmc.sh ev_${tag}rtw --config rtw > gpurun_out/ev_${tag}_rtw_pmc_stdout.txt 2>&1 || { tail -5 gpurun_out/ev_${tag}_rtw_pmc_stdout.txt; exit 1; }
python scripts/pmc_to_json.py gpurun_out pmc_ev_${tag}rtw_ gpurun_out/ev_${tag}_rtw_pmc.json "RTW: 1920x1080, 64 spp, 482 spheres, 8 bounces, SIMD rules, RTWeekend" || exit 1
for g in 8 4 2; do
  bash scripts/gpu_pmc.sh ev_${tag}r$g --sim-ranks $g --sim-index 0 > gpurun_out/ev_${tag}_r${g}_pmc_stdout.txt 2>&1 || { tail -5 gpurun_out/ev_${tag}_r${g}_pmc_stdout.txt; exit 1; }
  python scripts/pmc_to_json.py gpurun_out pmc_ev_${tag}r${g}_ gpurun_out/ev_${tag}_c2_rank${g}_pmc.json "C2: 1920x1080, 256 spp, 64 spheres, 8 bounces, SIMD rules" $g || exit 1
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ev_${tag}_c2_sameboxes.json 2>/dev/null || exit 1
bash scripts/gpu_simranks_all.sh 8 > gpurun_out/ev_${tag}_simranks8.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/ev_${tag}_c2_sameboxes.json 2>/dev/null || exit 1
python -c "import json; [print('c2', json.loads(l)['value'], json.loads(l)['ms_per_step']) for l in open('gpurun_out/ev_${tag}_c2_sameboxes.json')]"
cat gpurun_out/ev_${tag}_simranks8.txt
