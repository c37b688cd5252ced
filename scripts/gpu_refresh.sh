# Round-end evidence refresh: GPU parity, the default bench line, rocprofv3
# kernel stats, PMC passes, sim-ranks forecast and the C3/C5 configurations.
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_check.sh || exit $?
bash scripts/gpu_pmc.sh c2 > gpurun_out/pmc_c2_stdout.txt 2>&1 || exit $?
python scripts/pmc_to_json.py gpurun_out pmc_c2_ gpurun_out/c2_pmc.json "C2: 1920x1080, 256 spp, 64 spheres, 8 bounces, SIMD rules" || exit $?
bash scripts/gpu_simranks.sh > gpurun_out/simranks.txt 2>&1 || exit $?
cat gpurun_out/simranks.txt
for c in c3 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit $?
  tail -1 gpurun_out/bench_$c.json
done
