"""One-line summary of a profiles-style PMC record (scripts/pmc_to_json.py):
VALU issue occupancy, lane utilisation, dual issue, SALU / SMEM per CU cycle.
usage: python scripts/pmc_brief.py <record.json> [kernel_ms]"""
import json
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import bench  # noqa: E402

rec = json.load(open(sys.argv[1]))
ms = float(sys.argv[2]) if len(sys.argv) > 2 else rec["gpu_cycles_per_dispatch"] / 2.4e6
out = bench.valu_roofline(rec, ms)
out["kernel_ms_assumed"] = round(ms, 4)
print(sys.argv[1], json.dumps(out))
