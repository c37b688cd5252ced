# Cluster count (RT_CLUSTER_K) with the per-scene secondary threshold: RTWeekend and C5 (512 spp).
set -o pipefail
mkdir -p gpurun_out
run() {
  local label=$1; shift
  env "$@" timeout -k 10 150 python bench.py --steps 3 --warmup 3 --no-cpu-baseline $BARGS > gpurun_out/p.json 2> gpurun_out/p.err || { tail -5 gpurun_out/p.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/p.json')); print('$BARGS $label', d['value'], d['ms_per_step'])"
}
BARGS="--config rtw"; for k in 32 40 48; do run K$k RT_CLUSTER_K=$k; done
BARGS="--config c5 --spp 512"; for k in 24 32 40 48; do run K$k RT_CLUSTER_K=$k; done
