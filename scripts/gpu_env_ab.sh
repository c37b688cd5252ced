# Same-box A/B of env configs (';'-separated in $CFGS) over ROUNDS rounds: C2 and the
# 8-rank share (sim-ranks 8, residue 3), printing value / ms per step / kernel ms.
set -o pipefail
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-3}
IFS=';' read -ra CFG <<< "${CFGS:-RT_X=0}"
CONFIGS=${CONFIGS:-"c2;--sim-ranks 8 --sim-index 3"}
IFS=';' read -ra BC <<< "$CONFIGS"
for r in $(seq $ROUNDS); do
  for c in "${CFG[@]}"; do
    for b in "${BC[@]}"; do
      args=$b; [ "$b" = "c2" ] && args=""
      env $c timeout -k 10 120 python bench.py --steps 10 --warmup 6 --no-cpu-baseline $args > gpurun_out/eab.json 2> gpurun_out/eab.err || { tail -20 gpurun_out/eab.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/eab.json')); print('$r', '[$c]', '[$b]', d.get('value'), d.get('ms_per_step'), d.get('roofline',{}).get('kernel_ms', d.get('rank0_kernel_ms')), 'cold', d.get('cold_ms'))"
    done
  done
done
