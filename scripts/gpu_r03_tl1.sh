# A/B: C2's one-word cluster table with two levels (librt_trace_tl1.so + RT_TWO_LEVEL_W1=1)
# against the one-level default, C2 and the 8-rank share, then top count / sub size.
set -o pipefail
mkdir -p gpurun_out
run() {  # label, bench args, env...
  local label=$1 args=$2; shift 2
  env "$@" timeout -k 10 150 python bench.py --steps 10 --warmup 6 --no-cpu-baseline $args > gpurun_out/p.json 2> gpurun_out/p.err || { tail -5 gpurun_out/p.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/p.json')); print('$label', '[$args]', d.get('value'), d['ms_per_step'])"
}
for r in 1 2; do
  for a in "" "--sim-ranks 8 --sim-index 3"; do
    run base "$a" RT_X=0
    run tl1 "$a" RT_TRACE_LIB=librt_trace_tl1.so RT_TWO_LEVEL_W1=1
  done
done
for k in 6 8; do for s in 2 3 4; do run tl1K${k}S$s "" RT_TRACE_LIB=librt_trace_tl1.so RT_TWO_LEVEL_W1=1 RT_CLUSTER_K=$k RT_SUB_SPHERES=$s; done; done
