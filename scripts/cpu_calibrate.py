"""Same-host calibration of the CPU baseline (bench.py's cpu_baseline leg)
against the reference's own compiled code.

Times, alternately and on the same cores of THIS host:
  - the reference: main.cpp:7-640 compiled from /root/reference with its own
    codegen flags (oracle/Makefile, oracle/_ref/librefpix.so: SURVEY 8c's
    pixel-seed / bounce-count patches), its RenderTile over every 32x32 tile;
  - the port bench.py times: oracle/liboracle.so (the C restatement).
Workload: SURVEY 8d's calibration frame, 480x270, 8 spp, the first 64
Floating Spheres, 8 bounces, pixel seeds -- one thread (ref_render /
or_render threads=1), then `--threads` workers on both sides (the reference's
tiles pulled from one counter as its work queue deals them,
ref_render_threads; the port's pthread tile queue).  Both frames must be
identical.  Writes profiles/<tag>_cpu_calibration.json; bench.py reports its
ratio as cpu_baseline.same_host_ratio_to_reference.  Needs /root/reference
(this container), so the GPU box only reads the committed record.

    python scripts/cpu_calibrate.py r06 [--rounds 9] [--threads 8] [--warmup 3]

Round 6: each thread count starts with --warmup discarded alternating rounds (the round-5 record's first 8-worker
rounds ran at the single-thread rate on both sides: the pool's threads had not spread over the cores yet).
"""
import argparse
import ctypes
import json
import os
import pathlib
import statistics
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from oracle import oracle as orc  # noqa: E402  (the port under calibration)

W, H, FRAMES, N, B = 480, 270, 8, 64, 8


def cpu_model() -> str:
    for line in pathlib.Path("/proc/cpuinfo").read_text().splitlines():
        if line.startswith("model name"):
            return line.split(":", 1)[1].strip()
    return "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--warmup", type=int, default=3, help="discarded alternating rounds before each thread count")
    a = ap.parse_args()
    P = ctypes.CDLL(str(ROOT / "oracle" / "_ref" / "librefpix.so"))
    v, u32 = ctypes.c_void_p, ctypes.c_uint32
    P.ref_set_patch.argtypes = [u32, ctypes.c_int]
    P.ref_render.argtypes = [v, u32, v, u32, v, u32, u32, v, u32, u32, u32, u32, ctypes.c_int, v, v, v, v]
    P.ref_render_threads.argtypes = [v, u32, v, u32, v, u32, u32, v, u32, u32, u32, u32, ctypes.c_int, u32, v, v, v]
    o = orc.scene_builtin(1).prefix(N)
    cam = orc.camera(o, W, H)
    P.ref_set_patch(B, 1)
    scene_args = (o.spheres.ctypes.data, len(o.spheres), o.groups.ctypes.data, len(o.groups), o.materials.ctypes.data,
                  len(o.materials), int(o.use_sky), cam.ctypes.data, W, H, 0, FRAMES, 1)

    def ref(threads):
        prev = np.zeros((W * H, 4), np.float32)
        cur = np.zeros(W * H, np.uint32)
        rays = np.zeros(1, np.uint64)
        st = np.zeros(1, np.uint64)
        t = time.perf_counter()
        if threads == 1:
            P.ref_render(*scene_args, st.ctypes.data, prev.ctypes.data, cur.ctypes.data, rays.ctypes.data)
        else:
            P.ref_render_threads(*scene_args, threads, prev.ctypes.data, cur.ctypes.data, rays.ctypes.data)
        dt = time.perf_counter() - t
        return int(rays[0]) / dt / 1e6, cur, int(rays[0])

    def port(threads):
        t = time.perf_counter()
        _, cur, rays = orc.render(o, cam, W, H, frames=FRAMES, max_bounce=B, threads=threads)
        dt = time.perf_counter() - t
        return rays / dt / 1e6, cur, rays

    out = {"tag": a.tag, "script": "scripts/cpu_calibrate.py", "host_cpu": cpu_model(), "nproc": os.cpu_count(),
           "workload": f"{W}x{H}, {FRAMES} spp, first {N} Floating Spheres, {B} bounces, pixel seeds "
                       "(SURVEY 8d calibration frame)",
           "reference": "oracle/_ref/librefpix.so: /root/reference/main.cpp:7-640 (+ SURVEY 8c patches), clang++ "
                        "-O3 -mavx2 -mfma -DSIMD_WIDTH=4 (win32/compile.ps1:15 codegen flags)",
           "port": "oracle/liboracle.so (oracle/rt_oracle.c), the code bench.py's cpu_baseline times",
           "runs": {}}
    for threads in (1, a.threads):
        rr, pr = [], []
        for i in range(a.warmup):
            ref(threads)
            port(threads)
        for i in range(a.rounds):  # alternate, so drifting host load hits both sides alike
            r, rc, rrays = ref(threads)
            p, pc, prays = port(threads)
            assert rrays == prays and np.array_equal(rc, pc), "the port's frame differs from the reference's"
            rr.append(r)
            pr.append(p)
        run = {"threads": threads, "rounds": a.rounds, "warmup_rounds_discarded": a.warmup, "rays": rrays,
               "reference_mrays_per_s": {"median": round(statistics.median(rr), 3), "best": round(max(rr), 3),
                                         "all": [round(x, 3) for x in rr]},
               "port_mrays_per_s": {"median": round(statistics.median(pr), 3), "best": round(max(pr), 3),
                                    "all": [round(x, 3) for x in pr]},
               "ratio_median": round(statistics.median(pr) / statistics.median(rr), 4),
               "ratio_best": round(max(pr) / max(rr), 4),
               "frames_identical": True}
        run["within_10pct"] = bool(abs(run["ratio_median"] - 1) <= 0.10)
        out["runs"][str(threads)] = run
        print(json.dumps(run), flush=True)
    one = out["runs"]["1"]
    out["same_host_ratio_to_reference"] = one["ratio_median"]
    out["within_10pct"] = one["within_10pct"]
    path = ROOT / "profiles" / f"{a.tag}_cpu_calibration.json"
    path.write_text(json.dumps(out, indent=1) + "\n")
    print(f"wrote {path}: single-thread ratio {one['ratio_median']} (median), {one['ratio_best']} (best)")


if __name__ == "__main__":
    main()
