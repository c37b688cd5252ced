# Lanes per pixel and secondary-round threshold on RTWeekend and C5 (512 spp).
set -o pipefail
mkdir -p gpurun_out
run() {  # label, env..., -- bench args
  local label=$1; shift
  env "$@" timeout -k 10 150 python bench.py --steps 3 --warmup 3 --no-cpu-baseline $BARGS > gpurun_out/p.json 2> gpurun_out/p.err || { tail -5 gpurun_out/p.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/p.json')); print('$BARGS $label', d['value'], d['ms_per_step'])"
}
for BARGS in "--config rtw" "--config c5 --spp 512"; do
  run base RT_X=0
  for p in 2 8 16; do run P$p RT_LANES_PER_PIXEL=$p; done
  for s in 8 24 32; do run S$s RT_SEC_THRESHOLD=$s; done
done
