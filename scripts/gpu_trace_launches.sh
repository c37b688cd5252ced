# rocprofv3 kernel trace of a short C2 bench (cold launch, warm-ups, timed steps):
# every kernel in launch order with its duration, plus the --stats summary.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tag=${TAG:-tl}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag -o run --output-format csv -- python bench.py --steps 5 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/$tag.log 2>&1 || exit $?
tail -1 gpurun_out/$tag.log
f=$(find gpurun_out/$tag -name "*kernel_trace.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    n = r["Kernel_Name"]
    if "rtk::" not in n: continue
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e6:10.3f} ms  {(e - s) / 1e6:8.3f} ms  {n[:70]}")
PY
