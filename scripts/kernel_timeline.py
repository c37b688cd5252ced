"""Summarise a rocprofv3 --kernel-trace CSV: per-kernel mean durations over
the last `--tail` dispatches of the trace kernel's frames, the gaps between
consecutive kernels there, and the last few frames' timeline.

usage: python scripts/kernel_timeline.py <kernel_trace.csv> [--tail 64] [--show 24]
"""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--tail", type=int, default=64, help="steady-state frames (trace-kernel dispatches) summarised")
ap.add_argument("--show", type=int, default=24, help="kernels listed at the end")
ap.add_argument("--kernel", default="trace_kernel",
                help="name substring of the trace kernel whose dispatches mark the frames (e.g. 'trace_kernel<true, 0, "
                     "true' for the culled headline kernel of a run that also has a brute-force leg)")
a = ap.parse_args()

rows = list(csv.DictReader(open(a.csv)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
trace_idx = [i for i, r in enumerate(rows) if a.kernel in r["Kernel_Name"]]
rows = rows[:trace_idx[-1] + 1]  # up to the last dispatch of that kernel
first = trace_idx[-a.tail] if len(trace_idx) >= a.tail else trace_idx[0]
steady = rows[first:]
t0, t1 = int(steady[0]["Start_Timestamp"]), int(steady[-1]["End_Timestamp"])
frames = sum(1 for r in steady if a.kernel in r["Kernel_Name"])
dur = collections.defaultdict(list)
busy = 0
prev_end = None
gaps = []
for r in steady:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0][-60:]
    dur[name].append((e - s) / 1e3)
    busy += e - s
    if prev_end is not None:
        gaps.append((s - prev_end) / 1e3)
    prev_end = max(prev_end or 0, e)
span = (t1 - t0) / 1e3
print(f"steady state: {frames} trace dispatches, {len(steady)} kernels, span {span:.1f} us, "
      f"{span / frames:.2f} us per frame, kernels busy {busy / 1e3 / frames:.2f} us per frame")
for name, d in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {len(d) / frames:5.2f}/frame  mean {sum(d) / len(d):8.2f} us  min {min(d):8.2f}  max {max(d):8.2f}  {name}")
if gaps:
    gaps.sort()
    print(f"  gaps between kernels: mean {sum(gaps) / len(gaps):.2f} us, median {gaps[len(gaps) // 2]:.2f}, "
          f"max {gaps[-1]:.2f}, total {sum(gaps) / frames:.2f} us per frame")
print("last kernels (start offset, duration):")
tail = rows[-a.show:]
b = int(tail[0]["Start_Timestamp"])
for r in tail:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"  {(s - b) / 1e3:10.2f} us  {(e - s) / 1e3:8.2f} us  {r['Kernel_Name'].split('(')[0][-70:]}")
