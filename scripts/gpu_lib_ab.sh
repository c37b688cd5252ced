# Same-box A/B of kernel libraries: ROUNDS x (each lib in $LIBS) bench runs, C2 and
# the 8-rank share (sim-ranks 8, residue 3), printing value / ms per step / kernel ms.
# usage: LIBS="librt_trace_base.so librt_trace.so" ROUNDS=3 bash scripts/gpu_lib_ab.sh [extra bench args]
set -o pipefail
mkdir -p gpurun_out
LIBS=${LIBS:-librt_trace_base.so librt_trace.so}
ROUNDS=${ROUNDS:-3}
CONFIGS=${CONFIGS:-"c2;--sim-ranks 8 --sim-index 3"}
IFS=';' read -ra CFG <<< "$CONFIGS"
for r in $(seq $ROUNDS); do
  for lib in $LIBS; do
    for c in "${CFG[@]}"; do
      args=$c; [ "$c" = "c2" ] && args=""
      RT_TRACE_LIB=$lib timeout -k 10 120 python bench.py --steps 10 --warmup 6 --no-cpu-baseline $args "$@" > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$r', '$lib', '[$c]', d.get('value'), d.get('ms_per_step'), d.get('roofline',{}).get('kernel_ms', d.get('rank0_kernel_ms')))"
    done
  done
done
