"""Sums rocprofv3 --pmc CSVs per counter for the trace kernel (per dispatch)."""
import collections
import csv
import glob
import sys

root, prefix = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in sorted(glob.glob(f"{root}/{prefix}*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if "trace_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r["Dispatch_Id"])
for k in sorted(agg):
    n = max(1, len(disp[k]))
    print(f"{k:28s} {agg[k] / n:18.4e}  (per dispatch, {n} dispatch)")
