"""rt_multi kernel trace report (rocprofv3 --kernel-trace of
`BENCH_SHARE_GPU=1 bench.py --gpus G` or scripts/multi_cold_overlap.py).

Prints the cull passes, trace kernels and assembly kernels in time order with
their HIP queue and stream, then for every group of cull passes (one call's new
camera on every device) how much of the time from its first cull pass to the
end of its last trace had kernels of two or more devices (streams) in flight.

usage: python scripts/multi_trace_report.py gpurun_out/me_kt
"""
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    files = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    kt = list(csv.DictReader(open(files[0])))
    ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Queue_Id"], r["Kernel_Name"])
                 for r in kt), key=lambda e: e[0])
    t0 = ev[0][0]
    shown = [e for e in ev if any(k in e[4] for k in ("cull_kernel", "trace_kernel", "assemble_kernel"))]
    for s, e, st, q, n in shown:
        print(f"  {(s - t0) / 1e6:9.3f} -> {(e - t0) / 1e6:9.3f} ms  stream {st:>3} queue {q:>2}  {n[:58]}")
    culls = [x for x in ev if "cull_kernel" in x[4]]
    groups, cur = [], []
    for c in culls:
        if cur and c[0] - cur[-1][1] > 2_000_000 and len({x[2] for x in cur}) > 1:  # > 2 ms after the last cull
            groups.append(cur)
            cur = []
        cur.append(c)
    if cur:
        groups.append(cur)
    for gi, grp in enumerate(groups):
        streams = {x[2] for x in grp}
        lo = grp[0][0]
        traces = [x for x in ev if "trace_kernel" in x[4] and x[0] >= lo and x[2] in streams]
        first = {}
        for x in traces:
            first.setdefault(x[2], x)
        hi = max([x[1] for x in first.values()] + [grp[-1][1]])
        win = [x for x in ev if x[0] < hi and x[1] > lo and x[2] in streams]
        pts = sorted({max(x[0], lo) for x in win} | {min(x[1], hi) for x in win})
        busy = multi = 0
        for a, b in zip(pts, pts[1:]):
            act = {x[2] for x in win if x[0] <= a and x[1] >= b}
            if act:
                busy += b - a
                if len(act) >= 2:
                    multi += b - a
        print(f"cull group {gi}: {len(grp)} cull passes on {len(streams)} streams, first at {(lo - t0) / 1e6:.3f} ms; "
              f"to the end of every stream's first trace {(hi - lo) / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, "
              f"two or more devices in flight {multi / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
