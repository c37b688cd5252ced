# Secondary-round threshold sweep (RT_SEC_THRESHOLD) on RTWeekend, C5 (512 spp) and C2.
set -o pipefail
mkdir -p gpurun_out
run() {
  local label=$1; shift
  env "$@" timeout -k 10 150 python bench.py --steps 3 --warmup 3 --no-cpu-baseline $BARGS > gpurun_out/p.json 2> gpurun_out/p.err || { tail -5 gpurun_out/p.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/p.json')); print('$BARGS $label', d['value'], d['ms_per_step'])"
}
for BARGS in "--config rtw" "--config c5 --spp 512" "--config c2"; do
  for s in ${SS:-16 32 40 48 56}; do run S$s RT_SEC_THRESHOLD=$s; done
done
