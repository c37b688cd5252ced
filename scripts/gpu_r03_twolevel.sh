# Two-level cluster tables (W >= 2): GPU suite, same-box A/B against the one-level
# build (C5 at 512 spp, RTWeekend, C2), then a top-count / sub-size sweep.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tl_pytest.log 2>&1 || { tail -30 gpurun_out/tl_pytest.log; exit 1; }
tail -1 gpurun_out/tl_pytest.log
LIBS="librt_trace_base.so librt_trace.so" ROUNDS=2 CONFIGS="--config c5 --spp 512;--config rtw;c2" bash scripts/gpu_lib_ab.sh
run() {
  local label=$1; shift
  env "$@" timeout -k 10 150 python bench.py --steps 3 --warmup 3 --no-cpu-baseline $BARGS > gpurun_out/p.json 2> gpurun_out/p.err || { tail -5 gpurun_out/p.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/p.json')); print('$BARGS $label', d['value'], d['ms_per_step'])"
}
BARGS="--config rtw"; for k in 20 28 40; do for s in 4 6; do run K${k}S$s RT_CLUSTER_K=$k RT_SUB_SPHERES=$s; done; done
BARGS="--config c5 --spp 512"; for k in 16 24 32; do for s in 4 6; do run K${k}S$s RT_CLUSTER_K=$k RT_SUB_SPHERES=$s; done; done
