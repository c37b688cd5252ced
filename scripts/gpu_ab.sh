# Same-box A/B of variants (the one A/B launcher; gpurun -- 'bash scripts/gpu_ab.sh').
#   VARIANTS  ';'-separated; each a list of tokens (scripts/variant.sh): rt_device_options as bench
#             arguments and library builds as env, e.g. "default;--opt SecondaryThreshold=16;
#             RT_TRACE_LIB=librt_trace_base.so" (library builds: scripts/build_base_lib.sh, or
#             make -C simd-ray-tracer_amd variant NAME=.. KFLAGS=..)
#   CONFIGS   ';'-separated bench.py argument sets, "c2" = the defaults
#             (default: "c2;--sim-ranks 8 --sim-index 3", the 8-rank share)
#   ROUNDS    interleaved repetitions (default 3)
#   PARITY=1  run the GPU suite under each library build first (stops at the first failure; options
#             are parity-tested by tests/test_gpu_parity.py's VARIANT_OPTIONS)
#   STEPS / WARMUP  bench steps (default 10 / 6)
#   LEGS      bench.py --legs (default none; "distinct" also times the steps on unseen samples)
# Prints one line per run: round, variant, config, Mrays/s, ms per step, kernel ms, cold ms.
set -o pipefail
mkdir -p gpurun_out
. "$(dirname "$0")/variant.sh"
IFS=';' read -ra VAR <<< "${VARIANTS:-default}"
IFS=';' read -ra CFG <<< "${CONFIGS:-c2;--sim-ranks 8 --sim-index 3}"
ROUNDS=${ROUNDS:-3}
if [ "${PARITY:-0}" = 1 ]; then
  i=0
  for v in "${VAR[@]}"; do
    i=$((i+1))
    split_variant "$v"
    env "${VENV[@]}" RT_X=0 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 200 \
      --timeout-method thread > gpurun_out/ab_pytest_$i.log 2>&1
    rc=$?; echo "parity [$v] rc=$rc $(tail -1 gpurun_out/ab_pytest_$i.log)"
    [ $rc -ne 0 ] && { tail -30 gpurun_out/ab_pytest_$i.log; exit $rc; }
  done
fi
for r in $(seq $ROUNDS); do
  for v in "${VAR[@]}"; do
    for c in "${CFG[@]}"; do
      args=$c; [ "$c" = "c2" ] && args=""
      split_variant "$v"
      env "${VENV[@]}" RT_X=0 timeout -k 10 180 python bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-6} --no-cpu-baseline \
        --legs ${LEGS:-none} "${VARGS[@]}" $args \
        > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
      python - "$r" "$v" "$c" <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/ab.json") if l.startswith("{")][-1])
kern = d.get("roofline", {}).get("kernel_ms", d.get("rank0_kernel_ms"))
print(sys.argv[1], f"[{sys.argv[2]}]", f"[{sys.argv[3]}]", d.get("value"), d.get("ms_per_step"), kern, "cold", d.get("cold_ms"),
      *(["distinct", d["value_distinct_samples"], d["distinct_samples"]["kernel_ms"]] if "distinct_samples" in d else []),
      flush=True)
for r in d.get("runs", [])[1:]:  # (onrender: the other sizes / modes)
    print("   ", r["width"], r["mode"], r["mrays_per_s"], r["ms_per_frame"], "gpu", r.get("gpu_ms_per_frame"), flush=True)
PY
    done
  done
done
