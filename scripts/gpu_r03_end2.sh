# Second round-3 evidence pass (after the cl2 occupancy change): GPU suite, the default
# bench line, kernel trace + stats of C2, the C5 PMC record, the other configurations.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/e2_pytest.log 2>&1 || { tail -20 gpurun_out/e2_pytest.log; exit 1; }
tail -1 gpurun_out/e2_pytest.log
timeout -k 10 300 python bench.py > gpurun_out/e2_bench.json 2> gpurun_out/e2_bench.err || { tail -5 gpurun_out/e2_bench.err; exit 1; }
tail -c 300 gpurun_out/e2_bench.json; echo
TAG=e2_trace bash scripts/gpu_trace_launches.sh > gpurun_out/e2_launches.txt 2>&1 || { tail -5 gpurun_out/e2_launches.txt; exit 1; }
bash scripts/gpu_pmc.sh e2c5 --config c5 --warmup 2 > gpurun_out/e2_pmc_stdout.txt 2>&1 || { tail -5 gpurun_out/e2_pmc_stdout.txt; exit 1; }
python scripts/pmc_to_json.py gpurun_out pmc_e2c5_ gpurun_out/r03b_c5_pmc.json "C5: 7680x4320, 4096 spp, 256 spheres, 16 bounces, SIMD rules" > /dev/null || exit 1
python scripts/pmc_brief.py gpurun_out/r03b_c5_pmc.json
for cfg in c3 rtw c2in; do
  timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 3 --no-cpu-baseline >> gpurun_out/e2_configs.jsonl 2>> gpurun_out/e2_configs.err || exit 1
done
timeout -k 10 300 python bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline >> gpurun_out/e2_configs.jsonl 2>> gpurun_out/e2_configs.err || exit 1
echo done
