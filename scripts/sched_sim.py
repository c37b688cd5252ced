"""Offline list-scheduling simulation of one trace launch from its measured
per-wave durations (scripts/wave_tail.py SAVE=...npz): how long would the
launch take if its waves were dispatched in another order?

Model: SLOTS wave slots (256 CUs x 4 SIMDs x 7 waves); waves are dispatched in
the given order, each to the earliest free slot, and keep their measured
duration (contention is ignored, so absolute numbers are approximate; the
comparison between orders is the point).

Orders compared:
  measured     the launch's actual start order (sanity check against its span)
  tile         heaviest-first by block tile (max of its four waves), the
               kernel's current order (tile costs bucketed per quarter octave)
  wave         heaviest-first by wave (every wave its own entry)
  wave_exact   heaviest-first by exact wave duration (no buckets)

usage: python scripts/sched_sim.py gpurun_out/wt_s8.npz [slots]
"""
import heapq
import sys

import numpy as np


def makespan(durations, slots):
    free = [0.0] * min(slots, len(durations))
    heapq.heapify(free)
    end = 0.0
    for d in durations:
        t = heapq.heappop(free)
        heapq.heappush(free, t + d)
        end = max(end, t + d)
    return end


def bucket(c):
    """Quarter-octave bucket of a cost (rt_kernel.hip tile_bucket, without the clamp)."""
    c = np.maximum(c, 1.0)
    l = np.floor(np.log2(c))
    frac = np.floor((c / 2.0 ** l - 1.0) * 4.0)
    return 4 * l + frac


def main():
    z = np.load(sys.argv[1])
    slots = int(sys.argv[2]) if len(sys.argv) > 2 else 256 * 4 * 7
    wt = z["wave_times"].astype(np.int64)
    n = (len(wt) // 4) * 4
    wt = wt[:n]
    live = wt[:, 1] > 0
    st = np.where(live, (wt[:, 0] - wt[live, 0].min()) / 100.0, 0.0)
    du = np.where(live, (wt[:, 1] - wt[:, 0]) / 100.0, 0.0)
    span = (wt[live, 1].max() - wt[live, 0].min()) / 100.0
    ids = np.flatnonzero(live)
    print(f"waves {len(ids)}, measured span {span:.0f} us, total wave time {du.sum() / 1e3:.1f} ms, "
          f"bound max(longest {du.max():.0f}, total/slots {du.sum() / slots:.0f}) us")
    orders = {}
    orders["measured"] = ids[np.argsort(st[ids], kind="stable")]
    tile_cost = du.reshape(-1, 4).max(1)
    tb = bucket(tile_cost * 2400.0)  # us -> cycles at 2.4 GHz, as the kernel measures
    tiles = np.argsort(-tb, kind="stable")
    orders["tile"] = np.array([4 * t + w for t in tiles for w in range(4) if live[4 * t + w]])
    wb = bucket(du * 2400.0)
    orders["wave"] = ids[np.argsort(-wb[ids], kind="stable")]
    orders["wave_exact"] = ids[np.argsort(-du[ids], kind="stable")]
    for name, o in orders.items():
        print(f"  {name:11s} makespan {makespan(du[o], slots):7.0f} us")


if __name__ == "__main__":
    main()


def split_tail(durations, slots, x):
    """The last x jobs (in order) split into two halves of half the duration;
    the second halves go after everything else and may start only when their
    first half has finished (a dispatched second half occupies its slot
    while it waits)."""
    d = list(durations)
    n = len(d)
    x = min(x, n)
    jobs = [(di, None) for di in d[: n - x]] + [(di / 2.0, ("a", k)) for k, di in enumerate(d[n - x:])] + \
           [(di / 2.0, ("b", k)) for k, di in enumerate(d[n - x:])]
    free = [0.0] * min(slots, len(jobs))
    heapq.heapify(free)
    done_a = {}
    end = 0.0
    for dur, tag in jobs:
        t = heapq.heappop(free)
        start = t
        if tag and tag[0] == "b":
            start = max(t, done_a[tag[1]])
        fin = start + dur
        if tag and tag[0] == "a":
            done_a[tag[1]] = fin
        heapq.heappush(free, fin)
        end = max(end, fin)
    return end


if __name__ == "__main__" and len(sys.argv) > 1:
    z = np.load(sys.argv[1])
    wt = z["wave_times"].astype(np.int64)
    live = wt[:, 1] > 0
    du = (wt[live, 1] - wt[live, 0]) / 100.0
    slots = 256 * 4 * 7
    order = np.sort(du)[::-1]
    for x in (0, 3584, 7168, 14336):
        print(f"  wave_exact + split of the last {x:5d} waves: makespan {split_tail(order, slots, x):7.0f} us")
