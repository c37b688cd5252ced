"""Fold the per-pass rocprofv3 --pmc CSVs of scripts/gpu_pmc.sh into one JSON
record for the trace kernel (per-dispatch averages + derived figures) that
bench.py reports as roofline.traffic / roofline.issue.

usage: python scripts/pmc_to_json.py gpurun_out pmc_r01_ profiles/r01_c2_pmc.json "<workload>"

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md § HBM: FETCH_SIZE and
WRITE_SIZE are KiB; gfx950 FETCH_SIZE counts half the bytes of wide streaming
reads, so it is doubled; WRITE_SIZE is taken as is.
"""
import collections
import csv
import glob
import json
import sys

root, prefix, out, workload = sys.argv[1:5]
agg = collections.defaultdict(float)
disp = collections.defaultdict(set)
dur = []
for f in sorted(glob.glob(f"{root}/{prefix}*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if "trace_kernel" not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
        kernel = r["Kernel_Name"]
per = {k: agg[k] / max(1, len(disp[k])) for k in agg}
rec = {"workload": workload, "kernel": kernel, "counters_per_dispatch": per}
if "FETCH_SIZE" in per and "WRITE_SIZE" in per:
    rec["hbm_bytes_per_dispatch"] = 2.0 * per["FETCH_SIZE"] * 1024 + per["WRITE_SIZE"] * 1024
if "SQ_INSTS_VALU" in per and "GRBM_GUI_ACTIVE" in per:
    cycles = per["GRBM_GUI_ACTIVE"] / 8.0  # summed over the 8 XCDs
    # wave64 VALU instructions issued per SIMD per cycle (1024 SIMDs).  The
    # ceiling is 0.5 for full-rate ops (f32 add/mul/fma, 32-bit logic: 2 cyc)
    # and 0.25 for half-rate ones (v_pk_*_f32, integer mul/cvt/64-bit shifts,
    # f64: 4 cyc); transcendentals 8 cyc (scripts/mb_ops.hip on gfx950)
    rec["gpu_cycles_per_dispatch"] = cycles
    rec["valu_inst_per_simd_cycle"] = per["SQ_INSTS_VALU"] / (1024.0 * cycles)
if "SQ_THREAD_CYCLES_VALU" in per and "SQ_ACTIVE_INST_VALU" in per:
    rec["valu_lane_utilisation"] = per["SQ_THREAD_CYCLES_VALU"] / (64.0 * per["SQ_ACTIVE_INST_VALU"])
json.dump(rec, open(out, "w"), indent=1, sort_keys=True)
print(json.dumps({k: v for k, v in rec.items() if k != "counters_per_dispatch"}, indent=1))
