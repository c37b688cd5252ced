# Per-wave heaviest-first order: GPU suite, raw wave timelines of both orders
# (offline schedule simulation: scripts/sched_sim.py), same-box env A/B
# (RT_WAVE_ORDER=0 = round-2 tile order) on C2 and the 8-rank share, and the
# RTK_STATS scheduling counters of C2, the share, RTWeekend and C5 (1/8 spp).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r03_pytest6.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r03_pytest6.log | head; tail -30 gpurun_out/r03_pytest6.log; exit 1; }
tail -1 gpurun_out/r03_pytest6.log
for wo in 0 1; do
  RT_WAVE_ORDER=$wo SAVE=gpurun_out/wt_s8_wo$wo.npz SIM_RANKS=8 timeout -k 10 120 python scripts/wave_tail.py > gpurun_out/wt_s8_wo$wo.txt 2>&1 || { tail -5 gpurun_out/wt_s8_wo$wo.txt; exit 1; }
  RT_WAVE_ORDER=$wo SAVE=gpurun_out/wt_c2_wo$wo.npz SIM_RANKS=1 timeout -k 10 120 python scripts/wave_tail.py > gpurun_out/wt_c2_wo$wo.txt 2>&1 || { tail -5 gpurun_out/wt_c2_wo$wo.txt; exit 1; }
  head -3 gpurun_out/wt_s8_wo$wo.txt gpurun_out/wt_c2_wo$wo.txt
done
CFGS="RT_WAVE_ORDER=0;RT_WAVE_ORDER=1" ROUNDS=3 bash scripts/gpu_env_ab.sh || exit 1
for args in "" "--sim-ranks 8 --sim-index 0" "--config rtw" "--config c5 --spp 512"; do
  env RT_STATS=1 RT_TRACE_LIB=librt_trace_stats.so timeout -k 10 200 python bench.py --steps 1 --warmup 2 --no-cpu-baseline $args > gpurun_out/s.json 2> gpurun_out/s.err || { tail -20 gpurun_out/s.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/s.json')); print('[$args]', d.get('value'), json.dumps(d.get('sched_stats')))"
done
