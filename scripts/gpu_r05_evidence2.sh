# Round-5 evidence part 2 at the final kernel: the same-box forecast (whole frame, every residue of the 8/4/2-rank
# splits at steady state, whole frame), the share PMC records, the other configs, OnRender.  usage: bash ... <tag>
set -o pipefail
tag=${1:-r05y}
bash scripts/gpu_forecast.sh ev_${tag} > gpurun_out/ev_${tag}_fc_stdout.txt 2>&1 || { tail -5 gpurun_out/ev_${tag}_fc_stdout.txt; exit 1; }
tail -4 gpurun_out/ev_${tag}_fc_stdout.txt
for g in 8 4 2; do
  bash scripts/gpu_pmc.sh ev_${tag}r$g --sim-ranks $g --sim-index 0 > gpurun_out/ev_${tag}_r${g}_pmc_stdout.txt 2>&1 || { tail -5 gpurun_out/ev_${tag}_r${g}_pmc_stdout.txt; exit 1; }
  python scripts/pmc_to_json.py gpurun_out pmc_ev_${tag}r${g}_ gpurun_out/ev_${tag}_c2_rank${g}_pmc.json "C2: 1920x1080, 256 spp, 64 spheres, 8 bounces, SIMD rules" $g > /dev/null || exit 1
done
for cfg in c3 rtw c2in; do
  timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 5 --no-cpu-baseline >> gpurun_out/ev_${tag}_configs.jsonl 2>> gpurun_out/ev_${tag}_configs.err || exit 1
done
timeout -k 10 300 python bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline >> gpurun_out/ev_${tag}_configs.jsonl 2>> gpurun_out/ev_${tag}_configs.err || exit 1
timeout -k 10 300 python bench.py --config onrender > gpurun_out/ev_${tag}_onrender.json 2> gpurun_out/ev_${tag}_onrender.err || exit 1
echo part2 done
