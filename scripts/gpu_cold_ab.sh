# Cold-launch A/B: for each "LIB ENV..." config (';'-separated in $CFGS), ROUNDS x bench with
# 6 warm-ups (cold_ms, warm value) and with 1 warm-up (how fast the learned order settles).
set -o pipefail
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
IFS=';' read -ra CFG <<< "${CFGS:-librt_trace_base.so;librt_trace.so}"
for r in $(seq $ROUNDS); do
  for c in "${CFG[@]}"; do
    set -- $c; lib=$1; shift
    for w in 6 1; do
      env RT_TRACE_LIB=$lib "$@" timeout -k 10 120 python bench.py --steps 5 --warmup $w --no-cpu-baseline $BENCH_ARGS > gpurun_out/cab.json 2> gpurun_out/cab.err || { tail -20 gpurun_out/cab.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/cab.json')); print('$r [$c] w=$w', d.get('value'), d.get('ms_per_step'), 'cold', d.get('cold_ms'))"
    done
  done
done
