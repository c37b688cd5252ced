# Scheduling counters of the -DRTK_STATS build (make -C simd-ray-tracer_amd variant NAME=stats KFLAGS=-DRTK_STATS)
# for each ';'-separated variant in $VARIANTS (scripts/variant.sh) and each bench config in $CONFIGS (';'-separated, "c2" = defaults).
# Prints the lane-trip shares: done (finished lanes), primary/secondary lanes per round.
set -o pipefail
mkdir -p gpurun_out
. "$(dirname "$0")/variant.sh"
IFS=';' read -ra VAR <<< "${VARIANTS:-default}"
IFS=';' read -ra CFG <<< "${CONFIGS:-c2}"
for v in "${VAR[@]}"; do
  for c in "${CFG[@]}"; do
    args=$c; [ "$c" = "c2" ] && args=""
    split_variant "$v"
    env RT_STATS=1 RT_TRACE_LIB=librt_trace_stats.so "${VENV[@]}" timeout -k 10 180 python bench.py --steps 1 \
      --warmup ${WARMUP:-6} --no-cpu-baseline --headline-only "${VARGS[@]}" $args > gpurun_out/st.json 2> gpurun_out/st.err || { tail -5 gpurun_out/st.err; exit 1; }
    python - "$v" "$c" <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/st.json") if l.startswith("{")][-1])
s = d.get("sched_stats") or {}
trips = s.get("pri_iters", 0) + s.get("sec_iters", 0)
print(f"[{sys.argv[1]}] [{sys.argv[2]}] {d.get('value')} Mrays/s; trips {trips}; done lane-trips share "
      f"{s.get('done_lane_trips', 0) / max(64 * trips, 1):.3f}; primary lanes/round {s.get('pri_lanes', 0) / max(s.get('pri_iters', 1), 1):.1f}; "
      f"secondary lanes/round {s.get('sec_lanes', 0) / max(s.get('sec_iters', 1), 1):.1f}", flush=True)
print("  ", json.dumps(s), flush=True)
PY
  done
done
