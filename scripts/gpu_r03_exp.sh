# Experiments: slab test at the sub level (librt_trace_noss.so), lanes per pixel for
# RTWeekend / C5 with the cheap fold, P = 32 for the 8-rank share.
set -o pipefail
mkdir -p gpurun_out
run() {  # label, bench args, env...
  local label=$1 args=$2; shift 2
  env "$@" timeout -k 10 150 python bench.py --steps 5 --warmup 3 --no-cpu-baseline $args > gpurun_out/p.json 2> gpurun_out/p.err || { tail -5 gpurun_out/p.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/p.json')); print('$label', '[$args]', d.get('value'), d['ms_per_step'])"
}
for r in 1 2; do
  run base "--config rtw" RT_X=0
  run noss "--config rtw" RT_TRACE_LIB=librt_trace_noss.so
done
run P8 "--config rtw" RT_LANES_PER_PIXEL=8
run P8 "--config c5 --spp 512" RT_LANES_PER_PIXEL=8
run base "--config c5 --spp 512" RT_X=0
run P32 "--sim-ranks 8 --sim-index 3" RT_LANES_PER_PIXEL=32
run P16 "--sim-ranks 8 --sim-index 3" RT_X=0
