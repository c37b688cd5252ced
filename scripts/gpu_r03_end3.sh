# Round-3 closing evidence at HEAD (cull mask in dynamic LDS): C2 PMC record, every 8-rank
# share, the 2- and 4-rank shares, the 1-GPU C2 line on the same box.
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_pmc.sh e3c2 > gpurun_out/e3_pmc_stdout.txt 2>&1 || { tail -5 gpurun_out/e3_pmc_stdout.txt; exit 1; }
python scripts/pmc_to_json.py gpurun_out pmc_e3c2_ gpurun_out/r03b_c2_pmc.json "C2: 1920x1080, 256 spp, 64 spheres, 8 bounces, SIMD rules" > /dev/null || exit 1
python scripts/pmc_brief.py gpurun_out/r03b_c2_pmc.json
timeout -k 10 120 python bench.py --steps 10 --warmup 6 --no-cpu-baseline > gpurun_out/e3_c2.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/e3_c2.json')); print('C2 1 GPU', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
for g in 8 4 2; do
  echo "== $g ranks"; bash scripts/gpu_simranks_all.sh $g || exit 1
done
