# Two PMC passes (instruction counts, VALU occupancy) over the trace kernel for
# several bench argument sets: bash scripts/gpu_pmc_quick.sh <tag> "<bench args>" ...
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tag=$1; shift
j=0
for args in "$@"; do
  j=$((j+1))
  i=0
  for set in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/pq_${tag}_${j}_$i -o p --output-format csv -- python bench.py --steps 1 --warmup 3 --no-cpu-baseline $args > gpurun_out/pq_${tag}_${j}_$i.log 2>&1 || { tail -5 gpurun_out/pq_${tag}_${j}_$i.log; exit 1; }
  done
  python scripts/pmc_to_json.py gpurun_out pq_${tag}_${j}_ gpurun_out/pq_${tag}_$j.json "$args" > /dev/null || exit 1
  python - "$args" gpurun_out/pq_${tag}_$j.json <<'PY'
import json, sys
r = json.load(open(sys.argv[2])); c = r["counters_per_dispatch"]; cyc = r["gpu_cycles_per_dispatch"]
qc = 1024 * cyc / 4
print(sys.argv[1], "| cycles %.3e" % cyc, "insts_valu %.4e" % c["SQ_INSTS_VALU"], "busy %.3f" % ((c["SQ_ACTIVE_INST_VALU"] - c["SQ_ACTIVE_INST_VALU2"]) / qc),
      "dual %.3f" % (2 * c["SQ_ACTIVE_INST_VALU2"] / c["SQ_ACTIVE_INST_VALU"]), "lanes %.3f" % (c["SQ_THREAD_CYCLES_VALU"] / 64 / c["SQ_ACTIVE_INST_VALU"]),
      "waves %d" % c["SQ_WAVES"], "wavecyc %.3e" % c["SQ_WAVE_CYCLES"], "occ %.2f" % (c["SQ_WAVE_CYCLES"] * 4 / (1024 * cyc)),
      "salu %.3e" % c["SQ_INSTS_SALU"], "waitinst %.3f" % (c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]), "waitany %.3f" % (c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]),
      "lds %.3e conf %.3e" % (c["SQ_INSTS_LDS"], c["SQ_LDS_BANK_CONFLICT"]), "smem %.3e" % c["SQ_INSTS_SMEM"], "ms %.3f" % (cyc / 2.4e6))
PY
done
