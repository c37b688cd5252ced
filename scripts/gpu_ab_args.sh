# A/B of env settings with explicit bench args: bash scripts/gpu_ab_args.sh "<bench args>" "ENV=.." ...
set -o pipefail
mkdir -p gpurun_out
args=$1; shift
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python bench.py $args --warmup 1 --no-cpu-baseline > gpurun_out/b_args.json 2> gpurun_out/b_args.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/b_args.json')); print('$args', '$cfg', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
