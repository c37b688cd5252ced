"""Fold the per-pass rocprofv3 --pmc CSVs of scripts/gpu_pmc.sh into one JSON
record for the trace kernel that bench.py reports as roofline.traffic and as
the executed-work roofline fraction.

usage: python scripts/pmc_to_json.py gpurun_out pmc_r02_c2_ profiles/r02_c2_pmc.json "<workload>" [bands]
(bands: the band split of a --sim-ranks share, e.g. 8; bench.py matches records on workload + bands +
binary_hash).  Run it on the GPU box right after the passes: the record is stamped with the code-object
hash of the library the passes ran (simd_ray_tracer_amd.code_object_hash, or RT_TRACE_LIB's build) and the
time it was folded (taken_unix); bench.py uses a record only for a library with the same hash.

Per pass only the LAST trace_kernel dispatch is kept (the bench's timed, warm
launch; the earlier ones are the cold launch and warm-up launches that learn
the tile order).  HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md
§ HBM: FETCH_SIZE and WRITE_SIZE are KiB; gfx950 FETCH_SIZE counts half the
bytes of wide streaming reads, so it is doubled; WRITE_SIZE is taken as is.

VALU issue model (gfx950, measured by scripts/mb_ops.hip and the counter
calibration scripts/gpu_pmc_calib.sh -> profiles/r02_pmc_calib.txt): a SIMD
retires one wave64 full-rate VALU instruction every 2 cycles; half-rate ones
(v_pk_*_f32, 64-bit integer, conversions, f64) take 4 and transcendentals 8.
valu_pipe_frac = sum(instructions x cycles) / (1024 SIMDs x kernel cycles):
the executed-work roofline fraction (<= 1).  See bench.py valu_issue().
"""
import collections
import csv
import glob
import json
import os
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import __graft_entry__ as graft  # noqa: E402  (the package's code_object_hash: reads the .so, no GPU)

root, prefix, out, workload = sys.argv[1:5]
bands = int(sys.argv[5]) if len(sys.argv) > 5 else 1
per = {}
kernel = None
for f in sorted(glob.glob(f"{root}/{prefix}*/**/*counter_collection.csv", recursive=True)):
    rows = [r for r in csv.DictReader(open(f)) if "trace_kernel" in r["Kernel_Name"]]
    if not rows:
        continue
    last = max(int(r["Dispatch_Id"]) for r in rows)
    vals = collections.defaultdict(float)
    for r in rows:
        if int(r["Dispatch_Id"]) == last:
            vals[r["Counter_Name"]] += float(r["Counter_Value"])
            kernel = r["Kernel_Name"]
    for k, v in vals.items():
        if k == "GRBM_GUI_ACTIVE":
            per.setdefault("GRBM_GUI_ACTIVE_passes", []).append(v)
        else:
            per[k] = v
g = per.pop("GRBM_GUI_ACTIVE_passes", [])
if g:
    per["GRBM_GUI_ACTIVE"] = sum(g) / len(g)
rt = graft.load_package()
lib = rt.LIB_PATH
rec = {"workload": workload, "bands": bands, "kernel": kernel, "dispatch": "last trace_kernel dispatch of each pass (warm)",
       "counters_per_dispatch": per, "binary_hash": rt.code_object_hash(lib), "library": lib.name,
       "taken_unix": int(time.time()), "passes": len(glob.glob(f"{root}/{prefix}*/"))}
if "FETCH_SIZE" in per and "WRITE_SIZE" in per:
    rec["hbm_bytes_per_dispatch"] = 2.0 * per["FETCH_SIZE"] * 1024 + per["WRITE_SIZE"] * 1024
if "GRBM_GUI_ACTIVE" in per:
    rec["gpu_cycles_per_dispatch"] = per["GRBM_GUI_ACTIVE"] / 8.0  # summed over the 8 XCDs
json.dump(rec, open(out, "w"), indent=1, sort_keys=True)
print(json.dumps({k: v for k, v in rec.items() if k != "counters_per_dispatch"}, indent=1))
