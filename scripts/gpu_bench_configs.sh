# Bench lines for several configs (first one with the CPU baseline), then the
# rocprofv3 kernel-trace summary of the default bench command.
# usage: bash scripts/gpu_bench_configs.sh <tag> c2 rtw c2in ...
set -o pipefail
mkdir -p gpurun_out
tag=$1; shift
first=1
for c in "$@"; do
  extra="--no-cpu-baseline"; [ $first = 1 ] && extra=""; first=0
  timeout -k 10 300 python bench.py --config $c $extra > gpurun_out/bench_${tag}_$c.json 2> gpurun_out/bench_${tag}_$c.err || { tail -20 gpurun_out/bench_${tag}_$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_${tag}_$c.json')); print('$c', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['cold_ms'], d['segments'])"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o k --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/prof_$tag.log 2>&1 || { tail -5 gpurun_out/prof_$tag.log; exit 1; }
echo profiled
