# PMC records of the 2- and 4-rank shares (residue 0) with the round-3 end kernel.
set -o pipefail
mkdir -p gpurun_out
W2="C2: 1920x1080, 256 spp, 64 spheres, 8 bounces, SIMD rules"
bash scripts/gpu_pmc.sh r03s2 --sim-ranks 2 --sim-index 0 && python scripts/pmc_to_json.py gpurun_out pmc_r03s2_ gpurun_out/r03_c2_rank2_pmc.json "$W2" 2 > /dev/null || exit 1
bash scripts/gpu_pmc.sh r03s4 --sim-ranks 4 --sim-index 0 && python scripts/pmc_to_json.py gpurun_out pmc_r03s4_ gpurun_out/r03_c2_rank4_pmc.json "$W2" 4 > /dev/null || exit 1
for f in c2_rank2 c2_rank4; do python scripts/pmc_brief.py gpurun_out/r03_${f}_pmc.json; done
