# Round-3 counter evidence: the six PMC passes (scripts/gpu_pmc.sh) over the
# trace kernel of C2, one 8-GPU band share (residue 0), RTWeekend and C5, folded
# into profiles-ready JSON records (scripts/pmc_to_json.py).
set -o pipefail
mkdir -p gpurun_out
W2="C2: 1920x1080, 256 spp, 64 spheres, 8 bounces, SIMD rules"
bash scripts/gpu_pmc.sh r03c2 && python scripts/pmc_to_json.py gpurun_out pmc_r03c2_ gpurun_out/r03_c2_pmc.json "$W2" > /dev/null || exit 1
bash scripts/gpu_pmc.sh r03s8 --sim-ranks 8 --sim-index 0 && python scripts/pmc_to_json.py gpurun_out pmc_r03s8_ gpurun_out/r03_c2_rank8_pmc.json "$W2" 8 > /dev/null || exit 1
bash scripts/gpu_pmc.sh r03rtw --config rtw && python scripts/pmc_to_json.py gpurun_out pmc_r03rtw_ gpurun_out/r03_rtw_pmc.json "RTW: 1920x1080, 64 spp, 482 spheres, 8 bounces, SIMD rules, RTWeekend" > /dev/null || exit 1
bash scripts/gpu_pmc.sh r03c5 --config c5 --warmup 2 && python scripts/pmc_to_json.py gpurun_out pmc_r03c5_ gpurun_out/r03_c5_pmc.json "C5: 7680x4320, 4096 spp, 256 spheres, 16 bounces, SIMD rules" > /dev/null || exit 1
for f in c2 c2_rank8 rtw c5; do python scripts/pmc_brief.py gpurun_out/r03_${f}_pmc.json; done
ls gpurun_out/r03_*_pmc.json
