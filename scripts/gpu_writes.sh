# HBM write/fetch bytes of the trace kernel's last (warm) dispatch per env variant and config:
# one FETCH_SIZE and one WRITE_SIZE pass each (kernel-trace counters only).
#   VARIANTS ';'-separated variants (scripts/variant.sh); CONFIGS ';'-separated bench args ("c2" = defaults); WARMUP (default 8)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
. scripts/variant.sh
IFS=';' read -ra VAR <<< "${VARIANTS:-default}"
IFS=';' read -ra CFG <<< "${CONFIGS:-c2}"
n=0
for v in "${VAR[@]}"; do
  for c in "${CFG[@]}"; do
    args=$c; [ "$c" = "c2" ] && args=""
    for ctr in FETCH_SIZE WRITE_SIZE; do
      n=$((n+1))
      split_variant "$v"
      env "${VENV[@]}" RT_X=0 timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/wr_$n -o p --output-format csv -- \
        python bench.py --steps 1 --warmup ${WARMUP:-8} --no-cpu-baseline --headline-only "${VARGS[@]}" $args > gpurun_out/wr_$n.log 2>&1 || { tail -5 gpurun_out/wr_$n.log; exit 1; }
      python - "$v" "$c" "$ctr" gpurun_out/wr_$n <<'PY'
import csv, glob, sys
rows = [r for f in glob.glob(sys.argv[4] + "/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))
        if "trace_kernel" in r["Kernel_Name"]]
last = max(int(r["Dispatch_Id"]) for r in rows)
kb = sum(float(r["Counter_Value"]) for r in rows if int(r["Dispatch_Id"]) == last)
print(f"[{sys.argv[1]}] [{sys.argv[2]}] {sys.argv[3]} {kb * 1024 / 1e6:.2f} MB (last trace_kernel dispatch)", flush=True)
PY
    done
  done
done
