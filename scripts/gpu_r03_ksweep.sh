# Cluster count sweep on RTWeekend with the height-slab walk (RT_CLUSTER_K).
set -o pipefail
mkdir -p gpurun_out
for k in ${KS:-40 60 90 120 160}; do
  RT_CLUSTER_K=$k timeout -k 10 120 python bench.py --config rtw --steps 3 --warmup 3 --no-cpu-baseline > gpurun_out/k.json 2> gpurun_out/k.err || { tail -5 gpurun_out/k.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/k.json')); print('K=$k', d['value'], d['ms_per_step'])"
done
