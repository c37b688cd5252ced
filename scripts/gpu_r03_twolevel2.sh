# Two-level tables: finer top-count / sub-size sweep on RTWeekend and C5 (512 spp).
set -o pipefail
mkdir -p gpurun_out
run() {
  local label=$1; shift
  env "$@" timeout -k 10 150 python bench.py --steps 3 --warmup 3 --no-cpu-baseline $BARGS > gpurun_out/p.json 2> gpurun_out/p.err || { tail -5 gpurun_out/p.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/p.json')); print('$BARGS $label', d['value'], d['ms_per_step'])"
}
BARGS="--config rtw"; for k in 24 28 32; do for s in 2 3 4; do run K${k}S$s RT_CLUSTER_K=$k RT_SUB_SPHERES=$s; done; done
BARGS="--config c5 --spp 512"; for k in 20 24 28; do for s in 2 3 4; do run K${k}S$s RT_CLUSTER_K=$k RT_SUB_SPHERES=$s; done; done
