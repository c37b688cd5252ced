# Same-box multi-GPU forecast: the whole C2 frame, every residue of the 8-, 4- and 2-rank splits
# (bench.py --sim-ranks), the whole frame again.  usage: bash scripts/gpu_forecast.sh <tag>
set -o pipefail
tag=${1:-fc}
out=gpurun_out/${tag}_forecast.txt
: > $out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --headline-only 2>/dev/null \
  | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'c2_before': d['value'], 'ms_per_step': d['ms_per_step']}))" >> $out || exit 1
for g in 8 4 2; do bash scripts/gpu_simranks_all.sh $g >> $out 2>&1 || exit 1; done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --headline-only 2>/dev/null \
  | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'c2_after': d['value'], 'ms_per_step': d['ms_per_step']}))" >> $out || exit 1
python - $out <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
c2 = [r["ms_per_step"] for r in rows if "c2_before" in r or "c2_after" in r]
one = sum(c2) / len(c2)
print(f"1 GPU: {c2} ms (mean {one:.3f})")
for g in (8, 4, 2):
    sh = [r["ms_per_step"] for r in rows if r.get("sim_ranks") == g]
    print(f"{g} ranks: residues {min(sh):.3f}-{max(sh):.3f} ms, forecast {one / max(sh):.2f}x (slowest residue)")
PY
