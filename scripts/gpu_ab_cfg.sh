# A/B of env settings on one bench config: bash scripts/gpu_ab_cfg.sh <config> <steps> "ENV=.. ENV2=.." ...
set -o pipefail
mkdir -p gpurun_out
cfgname=$1; steps=$2; shift 2
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python bench.py --config $cfgname --steps $steps --warmup 1 --no-cpu-baseline > gpurun_out/b_$cfgname.json 2> gpurun_out/b_$cfgname.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/b_$cfgname.json')); print('$cfgname', '$cfg', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
