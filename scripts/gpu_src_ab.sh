# SMEM vs LDS sphere staging at C2 (north star: "the sphere array staged in LDS"):
# bench + two PMC passes for the one-wave default (groups through the scalar cache,
# no LDS image), four-wave workgroups with the LDS image (groups still through the
# scalar cache, per-lane gathers from LDS), and four-wave with the groups read from LDS.
set -o pipefail
mkdir -p gpurun_out
for c in "RT_X=0" "RT_SOLO=0" "RT_SOLO=0 RT_SPHERE_SRC=lds"; do
  for r in 1 2; do
    env $c timeout -k 10 100 python bench.py --steps 10 --warmup 6 --no-cpu-baseline > gpurun_out/src.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/src.json')); print('[$c] bench', d['value'], 'Mrays/s', d['roofline']['kernel_ms'], 'ms', d['roofline']['kernel'])"
  done
done
for c in "RT_X=0" "RT_SOLO=0" "RT_SOLO=0 RT_SPHERE_SRC=lds"; do
  env $c bash scripts/gpu_pmc_quick.sh src "" 2>&1 | grep "|" | sed "s/^/[$c] /" || exit 1
done
