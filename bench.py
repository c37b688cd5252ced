"""bench.py — Mrays/s of the MI355X sphere trace path (BASELINE.json metric).

Workload (BASELINE.json configs[1], "C2"): 1920x1080, 256 spp, 64 spheres
(first 64 of the reference's Floating Spheres scene, main.cpp:96-167, with
that scene's default camera), 8 bounces, per-(pixel, frame) PCG seeds.
One step = one complete 256-spp render of the frame: every pixel's 256
progressive frames folded into the running mean and the sRGB RGBA8 stored;
for N > 1 GPUs the frame is dealt out in interleaved 8-row bands (one rank
per GPU) and gathered to rank 0 over RCCL, then assembled (strong scaling:
the total work per step is fixed).  Rays = bounce segments counted as the
reference counts them (main.cpp:390).

Run:  python bench.py [--gpus N --steps K --warmup W]
      python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

# MI355X constants (/opt/skills/guides/MI355X_MICROARCH.md, chip table):
# a SIMD retires 16 f32 lanes/clk (a wave64 VALU op every 4 clk), 32 with
# packed v_pk_{add,mul}_f32: 256 CUs x 4 SIMDs x 32 x 2.4 GHz = 78.6 T f32
# add/mul ops/s (the 157 TFLOP/s spec figure counts an FMA as 2; the path
# cannot fuse: every op must round separately to match the reference).
# HBM3E 8 TB/s.
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
HBM_PEAK_GBS = 8000.0
SIMDS = 256 * 4


def ops_per_segment(n_spheres: int) -> int:
    """~21 f32 ops per sphere test + ~70 per segment of shading."""
    return 21 * n_spheres + 70


# BASELINE.json configs: C2 is the headline (1 GPU) and the
# default; C4 is C2 on several GPUs; C3 / C5 are the large single- and
# multi-GPU cases.  C1 is the CPU-only plumbing case (tests, not a bench line).
# "rtw" and "c2in" are frames the primary-ray cull cannot empty:
# RTWeekend (main.cpp:193-268, 482 spheres, sky term: every pixel is traced)
# and C2's 64 spheres seen from inside the sphere cloud (camera 1.0 from the
# look-at point instead of 3.0).
CONFIGS = {
    "c2": dict(width=1920, height=1080, spp=256, spheres=64, bounces=8, scene=1, distance=None),
    "c3": dict(width=3840, height=2160, spp=1024, spheres=64, bounces=8, scene=1, distance=None),
    "c5": dict(width=7680, height=4320, spp=4096, spheres=256, bounces=16, scene=1, distance=None),
    "rtw": dict(width=1920, height=1080, spp=64, spheres=482, bounces=8, scene=2, distance=None),
    "c2in": dict(width=1920, height=1080, spp=256, spheres=64, bounces=8, scene=1, distance=1.0),
}
SCENE_NAMES = {0: "RGB Glass", 1: "Floating Spheres", 2: "RTWeekend"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", choices=sorted(CONFIGS) + ["onrender"], default="c2",
                   help="BASELINE.json workload preset; 'onrender': the reference's per-frame OnRender loop")
    p.add_argument("--width", type=int)
    p.add_argument("--height", type=int)
    p.add_argument("--spp", type=int)
    p.add_argument("--spheres", type=int)
    p.add_argument("--bounces", type=int)
    p.add_argument("--scene", type=int, choices=(0, 1, 2), help="built-in scene (default: the config's)")
    p.add_argument("--distance", type=float, help="camera distance from the look-at point (default: the scene's)")
    p.add_argument("--scalar", action="store_true", help="RenderTileScalar rules instead of RenderTile")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target wall time of the CPU baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--band-rows", type=int, default=8, help="rows per interleaved band (multiple of 8)")
    p.add_argument("--verify", action="store_true",
                   help="after timing, rank 0 re-renders the whole frame alone and checks the gathered frame is "
                        "bit-identical (adds 'verified' to the line)")
    p.add_argument("--sim-ranks", type=int, default=0,
                   help="diagnostic (1 GPU): trace only band residue --sim-index of this many ranks, i.e. one rank's "
                        "share of a multi-GPU frame; prints that rank's kernel time, not a bench line")
    p.add_argument("--sim-index", type=int, default=0, help="band residue (rank) traced by --sim-ranks")
    p.add_argument("--devices", help="HIP devices of a single-process multi-GPU run (default 0..N-1)")
    p.add_argument("--transport", choices=("auto", "rccl", "peer"), default="auto",
                   help="single-process multi-GPU gather: RCCL, peer copies, or RCCL where it can be used")
    p.add_argument("--no-verify", action="store_true", help="multi-GPU: skip the whole-frame check (on by default)")
    p.add_argument("--frames", type=int, default=256, help="onrender: completed frames per measured run")
    p.add_argument("--modes", default="static,moving", help="onrender: camera modes to run (static, moving)")
    p.add_argument("--no-register", action="store_true",
                   help="onrender: hand frames out through the library's staging buffer (no registered image)")
    p.add_argument("--opt", action="append", default=[], metavar="FIELD=VALUE",
                   help="rt_device_options field for every device (include/rt_trace.h), e.g. --opt XcdGroup=off "
                        "--opt LanesPerPixel=16; switches take on/off/default.  A/B experiments only: every "
                        "option gives the same bits")
    p.add_argument("--brute", action="store_true",
                   help="time the brute-force kernel (Cull=off, Prefilter=off: every counted segment tests every "
                        "sphere, main.cpp:399-430) as the main line; its roofline is SURVEY 8d's algorithmic one")
    p.add_argument("--headline-only", action="store_true",
                   help="skip the extra legs after the timed steps (the brute-force roofline leg and the "
                        "distinct-samples leg): the PMC passes and kernel traces record the headline launches only")
    p.add_argument("--distinct-base", type=int, default=-1,
                   help="distinct leg: first frame of its first step (default spp x (warmup + 1))")
    p.add_argument("--distinct-stride", type=int, default=-1,
                   help="distinct leg: frames between its steps' first frames (default spp; 0 replays one range, "
                        "the leg's control)")
    p.add_argument("--legs", default="distinct,brute",
                   help="extra legs after the timed steps (1 GPU, whole frame): 'distinct' (the same steps on "
                        "samples no launch has seen), 'brute' (the brute-force kernel's roofline), both, or 'none'")
    a = p.parse_args()
    if a.config == "onrender":
        return a
    for k, v in CONFIGS[a.config].items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    return a


def device_options(rt, args) -> dict:
    """The rt_device_options of this run (--opt, --brute); {} = the library's defaults."""
    opts = rt.parse_options(args.opt)
    if args.brute:
        opts.update(Cull=rt.RT_OPT_OFF, Prefilter=rt.RT_OPT_OFF)
    return {k: v for k, v in opts.items() if v}


BRUTE = {"Cull": -1, "Prefilter": -1}  # rt_device_options of the brute-force kernel (RT_OPT_OFF)


def make_scene(rt, args):
    """The workload's scene: the first `spheres` spheres of a built-in scene."""
    scene = rt.scene_builtin(args.scene)
    if args.spheres < scene.ScalarSpheres.Count:
        scene = rt.scene_prefix(scene, args.spheres)
    args.spheres = scene.ScalarSpheres.Count
    return scene


GOLDEN = ROOT / "tests" / "golden" / "oracle_regression.json"


def golden_for(args, W, H, S, N, B):
    """The committed fixture of this exact workload (tests/golden/oracle_regression.json;
    every pixel-mode entry there was also rendered by the reference itself,
    tests/golden/reference_frames.json "pixel_cases"), or None."""
    try:
        gold = json.loads(GOLDEN.read_text())
    except (OSError, ValueError):
        return None, None
    for name, g in gold.items():
        if (g.get("seed_mode") == "pixel" and g["scene"] == args.scene and g["width"] == W and g["height"] == H
                and g["frames"] == S and g["bounces"] == B and g["simd"] == (not args.scalar)
                and (g["spheres"] is None or g["spheres"] == N) and g.get("distance") == args.distance):
            return name, g
    return None, None


ROWS_GOLDEN = ROOT / "tests" / "golden" / "c5_rows.json"


def rows_golden_for(args, W, H, S, N, B):
    """The committed tile-row fixture of this workload (tests/golden/c5_rows.json:
    whole 32-row tile rows of C5 rendered by the reference's own RenderTile and
    by the oracle, tests/golden/make_c5_rows.py), or None."""
    try:
        g = json.loads(ROWS_GOLDEN.read_text())
    except (OSError, ValueError):
        return None
    if (g["scene"] == args.scene and g["width"] == W and g["height"] == H and g["frames"] == S
            and g["bounces"] == B and g["spheres"] == N and g["simd"] == (not args.scalar) and args.distance is None):
        return g
    return None


def check_rows(rt, g, W, cur_host, prev_host):
    """A whole frame too large for a CPU render (C5): its fixture's tile rows, hashed."""
    got, ok = {}, True
    for ty, e in g["tile_rows"].items():
        y0, y1 = e["rows"]
        h = {"rgba8": f"{rt.frame_hash(cur_host[y0 * W:y1 * W]):016x}"}
        ok = ok and h["rgba8"] == e["fnv1a64_rgba8"]
        if prev_host is not None:
            h["v4"] = f"{rt.frame_hash(prev_host[y0 * W:y1 * W]):016x}"
            ok = ok and h["v4"] == e["fnv1a64_v4"]
        got[ty] = h
    return {"verified": bool(ok), "golden": "tests/golden/c5_rows.json",
            "rows": {ty: e["rows"] for ty, e in g["tile_rows"].items()}, "hashes": got,
            "expected": {ty: {"rgba8": e["fnv1a64_rgba8"], "v4": e["fnv1a64_v4"]} for ty, e in g["tile_rows"].items()},
            "note": "FNV-1a 64 (rt_frame_hash) of the fixture's 32-row tile rows of the last timed frame (the rows "
                    "0-1, 2160-2161, 4318-4319 among them); the fixture was rendered by the reference's own "
                    "RenderTile over those tiles and by the oracle (tests/golden/make_c5_rows.py).  The whole "
                    "frame's ray count has no CPU reference (about 2e11 segments); it is checked equal on every "
                    "timed step"}


def check_frame(rt, args, W, H, S, N, B, cur_host, prev_host, rays):
    """Hashes the last timed frame (RGBA8 and, when given, the v4 running mean)
    with the library's rt_frame_hash and compares it with the committed
    fixture: {"verified": bool or None, "golden": name, ...}."""
    name, g = golden_for(args, W, H, S, N, B)
    if g is None:
        rg = rows_golden_for(args, W, H, S, N, B)
        if rg is not None:
            return check_rows(rt, rg, W, cur_host, prev_host)
        return {"verified": None, "golden": None, "note": "no committed fixture for this workload"}
    got = {"rgba8": f"{rt.frame_hash(cur_host):016x}", "rays": rays}
    ok = got["rgba8"] == g["fnv1a64_rgba8"] and rays == g["rays"]
    if prev_host is not None:
        got["v4"] = f"{rt.frame_hash(prev_host):016x}"
        ok = ok and got["v4"] == g["fnv1a64_v4"]
    return {"verified": bool(ok), "golden": f"tests/golden/oracle_regression.json:{name}",
            "hashes": got, "expected": {"rgba8": g["fnv1a64_rgba8"], "v4": g["fnv1a64_v4"], "rays": g["rays"]},
            "note": "FNV-1a 64 (rt_frame_hash) of the last timed frame copied to the host after timing; the fixture "
                    "was rendered by the oracle and by the reference's own RenderTile (SURVEY 8c pixel mode)"}


def combine_verified(vs_one_gpu, vs_golden):
    """False if either check failed, True if one passed and none failed, None if neither ran."""
    checks = [v for v in (vs_one_gpu, vs_golden) if v is not None]
    return None if not checks else all(checks)


def reference_lib():
    """oracle/_ref/librefpix.so: the reference's own main.cpp:7-640 (RenderTile, with SURVEY 8c's pixel-seed and
    bounce-count patches) compiled from /root/reference in the build container by `make -C oracle ref` with its own
    codegen flags; the built .so travels with the tree (git-ignored, not gpurun-ignored), so the GPU box can time
    the reference itself.  None when it was not built."""
    import ctypes
    path = ROOT / "oracle" / "_ref" / "librefpix.so"
    if not path.exists():
        return None
    L = ctypes.CDLL(str(path))
    v, u32 = ctypes.c_void_p, ctypes.c_uint32
    L.ref_set_patch.restype = None
    L.ref_set_patch.argtypes = [u32, ctypes.c_int]
    L.ref_render_threads.restype = None
    L.ref_render_threads.argtypes = [v, u32, v, u32, v, u32, u32, v, u32, u32, u32, u32, ctypes.c_int, u32, v, v, v]
    return L


def cpu_baseline(args, n_rays_gpu_step: int):
    """The CPU baseline on this host's cores, on a bounded sample of the same workload: the full frame at k spp, k
    chosen from a 1-spp probe so the alternating rounds take ~--cpu-seconds in all.

    kind "reference": the reference's own compiled RenderTile (oracle/_ref/librefpix.so, its tiles pulled by
    `threads` workers from one counter as its work queue deals them, wasm/wasm.cpp:624-694), pixel seeds, the
    workload's bounce count.  The port (oracle/rt_oracle.c, the C restatement) is timed on the same sample beside it,
    so the line carries their live same-host ratio, also on the single-thread SURVEY 8d probe.  (The reference's
    NormalizeFast is the host's rsqrtss: on a non-Intel host its frames differ from the Intel-table port's in a few
    bits, `frames_identical`; the speed comparison does not depend on that.)  Without the reference build, kind
    "port" with the committed same-host calibration record."""
    import numpy as np
    from oracle import oracle as orc
    threads = orc.cpu_threads()
    env_cap = os.environ.get("OMP_NUM_THREADS")
    if env_cap and env_cap.isdigit():
        threads = min(threads, int(env_cap))
    o = orc.scene_builtin(args.scene)
    if args.spheres < len(o.spheres):
        o = o.prefix(args.spheres)
    W, H, B = args.width, args.height, args.bounces
    cam = orc.camera(o, W, H, distance=args.distance)
    ref = reference_lib()

    def port(scene, c, w, h, frames, thr, bounces):
        t = time.perf_counter()
        _, cur, rays = orc.render(scene, c, w, h, frames=frames, max_bounce=bounces, threads=thr,
                                  simd=not args.scalar)
        return rays, time.perf_counter() - t, cur

    def reference(scene, c, w, h, frames, thr, bounces):
        prev = np.zeros((w * h, 4), np.float32)
        cur = np.zeros(w * h, np.uint32)
        rays = np.zeros(1, np.uint64)
        ref.ref_set_patch(bounces, 1)
        t = time.perf_counter()
        ref.ref_render_threads(scene.spheres.ctypes.data, len(scene.spheres), scene.groups.ctypes.data,
                               len(scene.groups), scene.materials.ctypes.data, len(scene.materials), int(scene.use_sky),
                               c.ctypes.data, w, h, 0, frames, int(not args.scalar), thr, prev.ctypes.data,
                               cur.ctypes.data, rays.ctypes.data)
        dt = time.perf_counter() - t
        ref.ref_set_patch(5, 0)
        return int(rays[0]), dt, cur

    timed = reference if ref is not None else port
    # warm-up (the host's scheduler spreads a fresh pool over the cores only after a while: short first runs
    # measured single-core rates, profiles/r05_cpu_calibration.json) and the 1-spp probe that sizes k
    timed(o, cam, W, H, 1, threads, B)
    if ref is not None:
        port(o, cam, W, H, 1, threads, B)
    _, dt1, _ = timed(o, cam, W, H, 1, threads, B)
    rounds = 3 if ref is not None else 1
    k = max(1, min(args.spp, int(args.cpu_seconds / (2 * rounds if ref is not None else 1) / max(dt1, 1e-3))))
    # SURVEY §8d's single-thread probe (480x270, 8 spp, N = 64, 8 bounces, one thread)
    pr = orc.scene_builtin(1).prefix(64)
    pcam = orc.camera(pr, 480, 270)
    runs, pruns, probes, pprobes = [], [], [], []
    for _ in range(rounds):  # alternating rounds (reference, port), medians reported
        runs.append(timed(o, cam, W, H, k, threads, B))
        probes.append(timed(pr, pcam, 480, 270, 8, 1, 8))
        if ref is not None:
            pruns.append(port(o, cam, W, H, k, threads, B))
            pprobes.append(port(pr, pcam, 480, 270, 8, 1, 8))

    def median(rs):  # (rays, seconds, frame) of the median-rate run
        return sorted(rs, key=lambda r: r[0] / r[1])[len(rs) // 2]
    rays, dt, cur = median(runs)
    prays, pdt, _ = median(probes)
    out = {"value": round(rays / dt / 1e6, 2), "unit": "Mrays/s", "cores": threads,
           "kind": "reference" if ref is not None else "port",
           "sample": f"{W}x{H}, {k} spp (of {args.spp}), {args.spheres} spheres, {B} bounces, {rays} rays in "
                     f"{dt:.2f} s on {threads} threads (" +
                     ("the reference's own RenderTile, main.cpp:7-640 compiled with its codegen flags "
                      "(oracle/_ref/librefpix.so), pixel seeds, its tiles pulled from one counter"
                      if ref is not None else "oracle/rt_oracle.c, lane-4 SSE RenderTile restatement, pixel seeds") +
                     ")",
           "cpu": cpu_model(), "nproc": os.cpu_count(),
           "single_thread": {"value": round(prays / pdt / 1e6, 2), "unit": "Mrays/s",
                             "sample": f"480x270, 8 spp, 64 spheres, 8 bounces, 1 thread, {prays} rays in "
                                       f"{pdt:.2f} s (SURVEY 8d calibration workload)"}}
    if ref is not None:
        # the port on the same sample and cores, alternating with the reference: the live same-host ratio
        p_rays, p_dt, p_cur = median(pruns)
        pp_rays, pp_dt, _ = median(pprobes)
        out["rounds"] = {"reference": [round(r[0] / r[1] / 1e6, 2) for r in runs],
                         "port": [round(r[0] / r[1] / 1e6, 2) for r in pruns],
                         "note": "alternating rounds after a warm-up; value and port.value are the medians"}
        out["port"] = {"value": round(p_rays / p_dt / 1e6, 2), "unit": "Mrays/s", "cores": threads,
                       "single_thread": round(pp_rays / pp_dt / 1e6, 2),
                       "note": "oracle/rt_oracle.c (the C restatement, lane-4 SSE, pthread tile queue, clang -O3 "
                               "-mavx2 -mfma) on the same sample and cores"}
        out["same_host_ratio_to_reference"] = round((p_rays / p_dt) / (rays / dt), 4)
        out["within_10pct"] = bool(abs(out["same_host_ratio_to_reference"] - 1.0) <= 0.10)
        out["same_host_ratio_single_thread"] = round((pp_rays / pp_dt) / (prays / pdt), 4)
        out["frames_identical"] = bool(np.array_equal(cur, p_cur) and p_rays == rays)
    calib = cpu_calibration()
    if calib:
        # the build container's alternating-rounds record (scripts/cpu_calibrate.py)
        if ref is None:
            out["same_host_ratio_to_reference"] = calib["same_host_ratio_to_reference"]
            out["within_10pct"] = calib["within_10pct"]
        out["calibration"] = {"source": calib["file"], "host_cpu": calib["host_cpu"],
                              "ratio_median_1_thread": calib["runs"]["1"]["ratio_median"],
                              "ratio_median_n_threads": {k: r["ratio_median"] for k, r in calib["runs"].items()
                                                         if k != "1"},
                              "note": "port / compiled reference (main.cpp:7-640, its own codegen flags) on the "
                                      "build container's host and the SURVEY 8d probe, frames identical; median of "
                                      "alternating rounds"}
    return out


def cpu_calibration():
    """The newest committed same-host calibration record (scripts/cpu_calibrate.py)."""
    for f in sorted((ROOT / "profiles").glob("r*_cpu_calibration.json"), reverse=True):
        try:
            rec = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        rec["file"] = f"profiles/{f.name}"
        return rec
    return None


def cpu_model() -> str:
    try:
        for line in pathlib.Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def pmc_record(workload: str, bands: int = 1, binary_hash: str | None = None):
    """The committed rocprofv3 --pmc record (profiles/*_pmc.json, written by
    scripts/pmc_to_json.py) of this workload and band split taken on THIS
    library's code objects: its `binary_hash` must equal the loaded library's
    (simd_ray_tracer_amd.code_object_hash, the .hip_fatbin section).  Among
    several, the one taken last (`taken_unix`).  Returns (record, reason):
    record None with the reason when no record fits."""
    best, others = None, 0
    for f in (ROOT / "profiles").glob("*_pmc.json"):
        try:
            rec = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        if rec.get("workload") != workload or int(rec.get("bands", 1)) != bands:
            continue
        if rec.get("binary_hash") != binary_hash:
            others += 1
            continue
        if best is None or (rec.get("taken_unix", 0), f.name) > (best.get("taken_unix", 0), best["file"]):
            rec["file"] = f"profiles/{f.name}"
            best = rec
    if best is not None:
        return best, None
    return None, (f"no committed PMC record of this workload for the loaded code objects (binary_hash "
                  f"{binary_hash}); {others} record(s) of it belong to other builds")


def valu_roofline(pmc, kern_ms: float):
    """Executed-work roofline of the trace kernel from its committed PMC record
    (scripts/gpu_pmc.sh -> scripts/pmc_to_json.py, the warm dispatch).

    gfx950 VALU issue, calibrated on scripts/mb_ops (profiles/r02_pmc_calib.txt):
    SQ_ACTIVE_INST_VALU counts one quad-cycle per wave64 VALU instruction (two
    for transcendentals); full-rate ops (f32 add/mul/fma, 32-bit logic) can
    pair, and SQ_ACTIVE_INST_VALU2 counts the quad-cycles in which two issued.
    So a SIMD's VALU is occupied for ACTIVE_INST_VALU - ACTIVE_INST_VALU2
    quad-cycles, out of cycles/4:
        frac      = (ACTIVE_INST_VALU - ACTIVE_INST_VALU2) / (1024 SIMDs x cycles / 4)
                    (VALU issue occupancy, <= 1)
        lane_util = THREAD_CYCLES_VALU / (64 x ACTIVE_INST_VALU)
        frac_lane = frac x lane_util   (the share of issue capacity doing useful lanes)
        achieved  = INSTS_VALU_FLOPS_FP32 x 64 x lane_util / kernel time   (f32 lane flops/s;
                    the counter counts per wave instruction, 2 per FMA, packed ops per element)
        issue_capacity_tops = (ACTIVE_INST_VALU - ACTIVE_INST_VALU2) x 128 / kernel time
                    (one quad-cycle slot = 128 f32 add/mul lane-op capacity)"""
    c = pmc["counters_per_dispatch"]
    cycles = pmc["gpu_cycles_per_dispatch"]
    slots = c["SQ_ACTIVE_INST_VALU"] - c["SQ_ACTIVE_INST_VALU2"]
    frac = slots / (SIMDS * cycles / 4.0)
    lane = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"])
    flops = c["SQ_INSTS_VALU_FLOPS_FP32"] * 64.0 * lane
    sec = kern_ms / 1e3
    out = {"frac": round(frac, 4), "frac_lane": round(frac * lane, 4),
           "achieved": round(flops / sec / 1e12, 2), "issue_capacity_tops": round(slots * 128 / sec / 1e12, 2),
           "valu_slots_per_launch": slots,
           "valu_instructions_per_launch": c["SQ_INSTS_VALU"],
           "f32_lane_flops_per_launch": round(flops),
           "dual_issue_share": round(2 * c["SQ_ACTIVE_INST_VALU2"] / c["SQ_ACTIVE_INST_VALU"], 4),
           "lane_utilisation": round(lane, 4),
           "wave_cycles_issue_stalled": round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 4),
           "salu_per_valu": round(c["SQ_INSTS_SALU"] / c["SQ_INSTS_VALU"], 4),
           "gpu_cycles_per_launch": cycles}
    # the scalar unit: one per CU (256), at most one SALU instruction per CU cycle (the
    # sequencer serves the CU's four SIMDs in turn, one scalar issue each); SQ_ACTIVE_INST_SCA
    # counts wave quad-cycles like the VALU counter (so per SIMD)
    out["salu_per_cu_cycle"] = round(c["SQ_INSTS_SALU"] / (256.0 * cycles), 4)
    if "SQ_ACTIVE_INST_SCA" in c:
        out["sca_active_per_simd_quad_cycle"] = round(c["SQ_ACTIVE_INST_SCA"] / (SIMDS * cycles / 4.0), 4)
    if "SQ_INSTS_SMEM" in c:
        out["smem_per_cu_cycle"] = round(c["SQ_INSTS_SMEM"] / (256.0 * cycles), 4)
    return out


def workload_name(args, W, H, S, N, B, opts=None) -> str:
    """The workload a PMC record is matched on: the config and, when a run sets
    rt_device_options, those options (a record of the brute-force kernel is
    'C2: ... [Cull=-1, Prefilter=-1]')."""
    preset = all(getattr(args, k) == v for k, v in CONFIGS[args.config].items())
    tag = args.config.upper() if preset else "custom"
    view = "" if args.distance is None else f", camera {args.distance:g} from look-at"
    o = "" if not opts else " [" + ", ".join(f"{k}={v}" for k, v in sorted(opts.items())) + "]"
    return (f"{tag}: {W}x{H}, {S} spp, {N} spheres, {B} bounces, {'scalar' if args.scalar else 'SIMD'} rules"
            + ("" if args.scene == 1 else f", {SCENE_NAMES[args.scene]}") + view + o)


def roofline(args, info, kern_ms: float, rays_local: int, rows0: int, W: int, N: int, workload: str, bands: int,
             binary_hash: str | None = None, culled: bool = True):
    """The dominant kernel's roofline object (one device's trace kernel)."""
    ops = rays_local * ops_per_segment(N)
    achieved_alg = ops / (kern_ms / 1e3) / 1e12
    fb_bytes = rows0 * W * (16 + 4)  # accumulation + RGBA8 written once per launch
    hbm_achieved = fb_bytes / (kern_ms / 1e3) / 1e9
    pmc, why = pmc_record(workload, bands, binary_hash)
    walks = {0: "any", 1: "groups", 2: "cl1", 3: "cl2", 4: "cl4", 5: "cl1rel", 6: "cl2rel", 7: "cl4rel"}
    kernel = (f"trace_kernel<{'SIMD' if not args.scalar else 'scalar'},SMEM,{'CULL' if culled else 'NOCULL'},"
              f"{info['LanesPerPixel']},{'one-wave' if info['OneWaveGroups'] else 'four-wave'},"
              f"walk={walks.get(info['Walk'], '?')}>")
    roof = {"bound": "valu", "achieved": None, "peak": round(VALU_PEAK_TOPS, 1), "unit": "TFLOP/s",
            "frac": None, "traffic": None, "kernel": kernel, "kernel_ms": round(kern_ms, 3),
            "binary_hash": binary_hash}
    if pmc is None:
        roof["frac_null_reason"] = why
    if pmc:
        ex = valu_roofline(pmc, kern_ms)
        roof["achieved"], roof["frac"] = ex.pop("achieved"), ex.pop("frac")
        roof["frac_lane"] = ex.pop("frac_lane")
        roof["frac_flops"] = round(roof["achieved"] / VALU_PEAK_TOPS, 4)
        roof["issue_capacity_tops"] = ex.pop("issue_capacity_tops")
        roof["traffic"] = round(pmc["hbm_bytes_per_dispatch"]) if "hbm_bytes_per_dispatch" in pmc else None
        roof["executed"] = ex
        roof["source"] = pmc["file"]
        roof["source_binary_hash"] = pmc["binary_hash"]
        roof["note"] = ("frac = VALU issue occupancy of the trace kernel from the committed PMC record: "
                        "(SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) / (1024 SIMDs x GRBM_GUI_ACTIVE/8 / 4); "
                        "frac_lane = frac x lane utilisation (SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU)); "
                        "achieved = f32 lane flops = SQ_INSTS_VALU_FLOPS_FP32 x 64 x lane utilisation / live kernel "
                        "ms, against the 78.6 T f32 add/mul peak (frac_flops; the FMA-counted spec is 157.3 T); "
                        "issue_capacity_tops = issued quad-cycle slots x 128 / kernel ms (bench.py valu_roofline). "
                        "traffic = FETCH_SIZE x2 + WRITE_SIZE (KiB), per launch.")
    roof["frac_algorithmic"] = round(achieved_alg / VALU_PEAK_TOPS, 4)
    roof["achieved_algorithmic"] = round(achieved_alg, 2)
    roof["work_per_launch"] = (f"{rays_local} segments x (21*{N}+70) f32 ops (SURVEY 8d brute force" +
                               ("; the kernel skips most sphere tests exactly, so this rate can exceed the peak)"
                                if culled else "; this kernel tests every sphere for every segment, as "
                                               "main.cpp:399-430 does)"))
    roof["hbm"] = {"achieved": round(hbm_achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": round(hbm_achieved / HBM_PEAK_GBS, 6), "bytes_per_launch": fb_bytes}
    return roof


def base_line(args, *, world, elapsed, seg_counted, seg_folded, W, H, S, N, B, workload, parallelism, gather=None):
    value = seg_counted * args.steps / elapsed / 1e6
    seg_traced = seg_counted - seg_folded
    return {
        "metric": f"Mrays/sec at {W}x{H}, {S}spp, {B} bounces, {N} spheres",
        "value": round(value, 1),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic ({'first ' + str(N) + ' spheres of ' if args.scene == 1 else ''}the reference's "
                f"{SCENE_NAMES[args.scene]} scene, {'default camera' if args.distance is None else 'camera moved'}"
                ", per-(pixel,frame) PCG seeds)",
        "config": {"workload": workload,
                   "width": W, "height": H, "spp": S, "spheres": N, "bounces": B, "scene": args.scene,
                   "parallelism": parallelism,
                   **({"gather": gather} if gather else {}),
                   "rays_per_step": seg_counted},
        "segments": {"counted_per_step": seg_counted, "traced_per_step": seg_traced,
                     "counted_equal_every_timed_step": True,  # one counter per step, checked by the caller
                     "folded_per_step": seg_folded,
                     "traced_mrays_per_s": round(seg_traced * args.steps / elapsed / 1e6, 1),
                     "note": "every segment is counted as the reference counts it (main.cpp:390); 'folded' "
                             "ones belong to pixels whose every sample provably misses (dead tiles), folded "
                             "by the empty-tile kernel instead of traced"},
    }


def brute_leg(rt, torch, args, scene, cam, W, H, S, N, B, gpu, stream, binary_hash, workload_of):
    """SURVEY 8d's roofline on the work it defines: the same frame on a device
    created with the brute-force kernel (Cull off: no cone cull, no dead-tile
    fold; Prefilter off: no prefilter, no cluster walk), so every counted
    segment tests every sphere as main.cpp:399-430 does.  2 warm-up + 3 timed
    launches (HIP events around each), the last frame checked against the same
    fixture; frac_algorithmic = segments x (21 N + 70) / kernel time / 78.6 T."""
    dev = rt.Device(gpu, options=BRUTE)
    try:
        dev.upload_scene(scene)
        dev.reserve(W, H)
        prev = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
        cur = torch.zeros(H * W, dtype=torch.int32, device="cuda")
        ctr = torch.zeros(5, dtype=torch.int64, device="cuda")
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
        for i in range(5):
            if i >= 2:
                ev[i - 2][0].record(stream)
            dev.trace(cam, width=W, height=H, prev_ptr=prev.data_ptr(), cur_ptr=cur.data_ptr(),
                      rays_ptr=ctr[i].data_ptr(), prev_count=0, frames=S, max_bounce=B, simd=not args.scalar,
                      band_rows=args.band_rows, accum_zero=True, stream=stream.cuda_stream)
            if i >= 2:
                ev[i - 2][1].record(stream)
        torch.cuda.synchronize()
        counts = ctr.tolist()
        ms = sum(a.elapsed_time(b) for a, b in ev) / 3
        info = dev.last_info()
        fc = check_frame(rt, args, W, H, S, N, B, cur.cpu().numpy().view("uint32"), prev.cpu().numpy(), counts[-1])
    finally:
        dev.close()
    wl = workload_of(BRUTE)
    roof = roofline(args, info, ms, counts[-1], H, W, N, wl, 1, binary_hash, culled=False)
    out = {"ms": round(ms, 3), "frac_algorithmic": roof["frac_algorithmic"],
           "achieved_algorithmic": roof["achieved_algorithmic"], "frac": roof["frac"],
           "frac_lane": roof.get("frac_lane"), "achieved": roof["achieved"], "traffic": roof["traffic"],
           "source": roof.get("source"), "kernel": roof["kernel"], "workload": wl,
           "segments": counts[-1], "segments_folded": info["SegmentsFolded"],
           "counted_equal": len(set(counts)) == 1, "verified": fc["verified"], "frame_check": fc,
           "note": "brute-force kernel of the same frame (rt_device_options Cull=off, Prefilter=off): every "
                   "counted segment tests every sphere (main.cpp:399-430), so frac_algorithmic = segments x "
                   "(21N+70) f32 ops / kernel ms / 78.6 T is SURVEY 8d's roofline on work the kernel really "
                   "executes; frac / frac_lane come from that kernel's committed PMC record (bench.py --brute)"}
    if "frac_null_reason" in roof:
        out["frac_null_reason"] = roof["frac_null_reason"]
    return out


def distinct_leg(rt, torch, args, dev, scene, cam, W, H, S, N, B, gpu, stream, opts):
    """The headline on samples no launch has seen: timed step i renders frames
    [S (w+1+i), S (w+2+i)) (PreviousRayCount with RT_FLAG_ACCUM_ZERO: new pixel
    seeds, main.cpp:797-806's progressive count), so no timed launch repeats
    the samples its learned wave order and pixel permutation were measured on.
    The last step is checked bit for bit against a FRESH device's cold render
    of the same frame range (its first launch: cull pass, split head, no
    learned order)."""
    pc0 = S * (args.warmup + 1) if args.distinct_base < 0 else args.distinct_base
    stride = S if args.distinct_stride < 0 else args.distinct_stride
    prev = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
    cur = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    warm = max(args.warmup, 6)
    n = warm + args.steps
    ctr = torch.zeros(n, dtype=torch.int64, device="cuda")
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    def launch(i):
        dev.trace(cam, width=W, height=H, prev_ptr=prev.data_ptr(), cur_ptr=cur.data_ptr(),
                  rays_ptr=ctr[i].data_ptr(), prev_count=pc0 + stride * i, frames=S, max_bounce=B,
                  simd=not args.scalar, band_rows=args.band_rows, accum_zero=True, stream=stream.cuda_stream)

    # untimed warm-up launches (at least 6) on unseen frames too: the host work between the headline's timed
    # steps and this leg idles the GPU, and its clock takes ~6 launches of C2 to ramp back
    # (measured: 5.0, 4.7, 4.6, 4.4, 4.3, 4.2 ms, then steady, profiles/r06b_distinct_warmup.txt)
    for i in range(warm):
        launch(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        launch(warm + i)
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    counts = ctr[warm:].tolist()
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    last_pc = pc0 + stride * (n - 1)
    fresh = rt.Device(gpu, options=opts)
    try:
        fresh.upload_scene(scene)
        cprev = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
        ccur = torch.zeros(H * W, dtype=torch.int32, device="cuda")
        crays = torch.zeros(1, dtype=torch.int64, device="cuda")
        fresh.trace(cam, width=W, height=H, prev_ptr=cprev.data_ptr(), cur_ptr=ccur.data_ptr(),
                    rays_ptr=crays.data_ptr(), prev_count=last_pc, frames=S, max_bounce=B, simd=not args.scalar,
                    band_rows=args.band_rows, accum_zero=True, stream=stream.cuda_stream)
        torch.cuda.synchronize()
        cold_split = fresh.last_info()["SplitHeadFrames"]
    finally:
        fresh.close()
    same = (torch.equal(prev.view(torch.int32), cprev.view(torch.int32)) and torch.equal(cur, ccur)
            and counts[-1] == int(crays.item()))
    return {"value": round(sum(counts) / elapsed / 1e6, 1), "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "kernel_ms": round(kern_ms, 3), "kernel_ms_per_step": [round(a.elapsed_time(b), 3) for a, b in ev],
            "segments_per_step": counts,
            "frames_timed": [pc0 + stride * warm, last_pc + S], "warmup_frames": [pc0, pc0 + stride * warm],
            "verified_vs_fresh_device": bool(same),
            "fresh_device_split_head_frames": cold_split,
            "note": f"after {warm} untimed launches (also on unseen frames), each timed step folds the next "
                    f"{S} frames with RT_FLAG_ACCUM_ZERO: every launch traces samples (pixel "
                    "seeds) no earlier launch traced, with the wave order and pixel permutation learned on other "
                    "samples; the last step equals a fresh device's cold render of the same frames (v4, RGBA8, "
                    "ray count)"}


def one_gpu_reference(rt, torch, dev, cam, args, W, H, S, B, stream, steps: int):
    """The whole frame on one device alone (multi-GPU lines): its RGBA8 frame
    (the --verify reference) and its ms per frame over `steps` warm launches."""
    cur = torch.zeros(H * W, dtype=torch.int32, device=torch.cuda.current_device())
    prev = torch.zeros((H * W, 4), dtype=torch.float32, device=torch.cuda.current_device())
    ctr = torch.zeros(steps + 3, dtype=torch.int64, device=torch.cuda.current_device())
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for i in range(steps + 3):
        if i == 3:
            torch.cuda.synchronize()
            ev[0].record(stream)
        dev.trace(cam, width=W, height=H, prev_ptr=prev.data_ptr(), cur_ptr=cur.data_ptr(),
                  rays_ptr=ctr[i].data_ptr(), prev_count=0, frames=S, max_bounce=B, simd=not args.scalar,
                  band_rows=args.band_rows, band_count=1, band_index=0, accum_zero=True, stream=stream.cuda_stream)
    ev[1].record(stream)
    torch.cuda.synchronize()
    return cur, ev[0].elapsed_time(ev[1]) / steps, int(ctr[steps + 2].item())


def main_multi_device(args):
    """--gpus N (N > 1) without a launcher: ONE process drives N devices through
    the C-ABI's rt_multi (include/rt_trace.h): interleaved 8-row bands dealt
    over the devices, each traced on its own stream, RCCL grouped send/recv to
    devices[0] (ncclCommInitAll; peer copies where RCCL cannot be used, e.g. a
    device listed twice) and the assembly -- all inside the timed region.  The
    reference drives its worker pool from one process the same way
    (main.cpp:851-856, wasm/wasm.cpp:651-678)."""
    import torch
    import __graft_entry__ as graft

    rt = graft.load_package()
    opts = device_options(rt, args)
    binary_hash = rt.code_object_hash()
    if os.environ.get("BENCH_SHARE_GPU") == "1":
        devices = [0] * args.gpus
    elif args.devices:
        devices = [int(d) for d in args.devices.split(",")]
    else:
        devices = list(range(args.gpus))
    if len(devices) != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but --devices lists {len(devices)}")
    visible = torch.cuda.device_count()  # does not initialise the GPU
    if visible < max(devices) + 1:
        print(f"bench.py: --gpus {args.gpus} needs HIP devices {sorted(set(devices))}, but {visible} "
              f"{'is' if visible == 1 else 'are'} visible (set BENCH_SHARE_GPU=1 to deal the bands over one "
              "device, or launch one process per GPU with torch.distributed.run)", file=sys.stderr)
        raise SystemExit(2)
    d0 = devices[0]
    torch.cuda.set_device(d0)
    scene = make_scene(rt, args)
    W, H, S, B, N = args.width, args.height, args.spp, args.bounces, args.spheres
    cam = rt.camera_setup(scene, W, H, distance=args.distance)
    transport = rt.RT_MULTI_PEER if args.transport == "peer" else rt.RT_MULTI_RCCL if args.transport == "rccl" \
        else rt.RT_MULTI_AUTO
    multi = rt.Multi(devices, transport=transport, options=opts)
    multi.upload_scene(scene)
    # every buffer a call of this geometry needs, allocated now: no call of the
    # timed region allocates or waits for a device (rt_multi_reserve)
    multi.reserve(W, H, args.band_rows)
    full = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    ctr = torch.zeros(args.warmup + args.steps + 2, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream()
    tiny = torch.zeros(64 * 8, dtype=torch.int32, device="cuda")
    tiny_rays = torch.zeros(1, dtype=torch.int64, device="cuda")
    band_rows = args.band_rows

    def call(c):
        multi.trace(cam, width=W, height=H, cur_ptr=full.data_ptr(), rays_ptr=ctr[c].data_ptr(), frames=S,
                    max_bounce=B, simd=not args.scalar, band_rows=band_rows, accum_zero=True,
                    stream=stream.cuda_stream)

    # code objects on every device (a tiny frame), then the cold call of this geometry
    multi.trace(cam, width=64, height=8 * len(devices), cur_ptr=torch.zeros(64 * 8 * len(devices), dtype=torch.int32,
                device="cuda").data_ptr(), rays_ptr=tiny_rays.data_ptr(), frames=1, max_bounce=1,
                simd=not args.scalar, band_rows=8, accum_zero=True, stream=stream.cuda_stream)
    multi.synchronize()
    del tiny
    t = time.perf_counter()
    call(0)
    multi.synchronize()
    cold_ms = (time.perf_counter() - t) * 1e3
    for c in range(1, args.warmup):
        call(c)
    multi.synchronize()
    c_last = max(args.warmup - 1, 0)
    rays_per_step = int(ctr[c_last].item())
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    growths0 = [multi.shard_info(i)["BufferGrowths"] for i in range(len(devices))]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        call(args.warmup + i)
        ev[i][1].record(stream)
    multi.synchronize()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    timed = ctr[args.warmup:args.warmup + args.steps].tolist()
    if any(n != rays_per_step for n in timed):
        raise SystemExit(f"bench.py: timed steps counted {timed} segments, expected {rays_per_step} each")
    per_dev_ms = multi.last_trace_ms(len(devices))
    gather_ms = multi.last_gather_ms()
    growths = sum(multi.shard_info(i)["BufferGrowths"] - g for i, g in enumerate(growths0))
    minfo = multi.info()
    call_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    frame = full.clone()
    # the whole frame on devices[0] alone: the 1-GPU time on this box and the --verify reference
    dev = rt.Device(d0, options=opts)
    dev.upload_scene(scene)
    ref, one_ms, one_rays = one_gpu_reference(rt, torch, dev, cam, args, W, H, S, B, stream, min(args.steps, 5))
    verified = bool(torch.equal(frame, ref)) and one_rays == rays_per_step
    frame_check = check_frame(rt, args, W, H, S, N, B, frame.cpu().numpy().view("uint32"), None, rays_per_step)
    workload = workload_name(args, W, H, S, N, B, opts)
    gather = ("RCCL grouped send/recv to devices[0] (ncclCommInitAll) + rt_assemble scatter, overlapping the next "
              "call's traces" if minfo["Transport"] == rt.RT_MULTI_RCCL else
              "hipMemcpyPeerAsync to devices[0] + rt_assemble scatter, overlapping the next call's traces")
    elapsed_share = elapsed
    line = base_line(args, world=args.gpus, elapsed=elapsed_share, seg_counted=rays_per_step,
                     seg_folded=minfo["SegmentsFolded"], W=W, H=H, S=S, N=N, B=B, workload=workload,
                     parallelism=f"{args.gpus} GPU x interleaved {band_rows}-row bands, one process (rt_multi)",
                     gather=gather)
    line["config"]["launcher"] = "single process: rt_multi over devices " + ",".join(map(str, devices))
    line["config"]["devices"] = devices
    line["cold_ms"] = round(cold_ms, 3)
    line["cold"] = {"ms": round(cold_ms, 3), "note": "first call for this camera/geometry on every device (cull "
                    "passes + untrained tile orders + RCCL/peer setup), wall clock incl. its synchronisation"}
    line["per_device_trace_ms"] = [round(v, 3) for v in per_dev_ms]
    line["gather_ms"] = round(gather_ms, 4)
    line["gather"] = {"ms": round(gather_ms, 4), "bytes": W * H * 4,
                      "note": "last timed call: from every device's trace done to the frame assembled on devices[0] "
                              "(HIP events on its gather stream: band transfer + scatter, rt_multi_last_gather_ms)"}
    line["call_ms_events"] = round(call_ms, 3)
    # launch-buffer (re)allocations during the timed calls, over every device (rt_multi_reserve sized them: 0)
    line["buffer_growths_timed"] = growths
    line["one_gpu"] = {"ms_per_frame": round(one_ms, 3), "device": d0,
                       "speedup_vs_one_gpu": round(one_ms / (elapsed / args.steps * 1e3), 3),
                       "note": "the same frame traced whole on devices[0] alone, in this run"}
    line["verified_vs_one_gpu"] = verified
    line["frame_check"] = frame_check
    line["verified"] = combine_verified(verified, frame_check["verified"])
    # the roofline of the slowest device's share (its trace kernel; counters: the committed share record)
    slowest = max(range(len(devices)), key=lambda i: per_dev_ms[i])
    rows0 = rt.band_local_rows(H, band_rows, args.gpus, slowest)
    share_info = multi.shard_info(slowest)  # what the slowest device's last launch really ran
    line["roofline"] = roofline(args, share_info, per_dev_ms[slowest], rays_per_step // args.gpus, rows0, W, N,
                                workload, args.gpus, binary_hash, culled=opts.get("Cull", 0) != -1)
    if opts:
        line["config"]["device_options"] = opts
    line["roofline"]["device"] = slowest
    print(json.dumps(line), flush=True)
    dev.close()
    multi.close()
    if line["verified"] is False:
        print(f"bench.py: the gathered frame does NOT match: {frame_check}", file=sys.stderr)
        raise SystemExit(3)


def main_onrender(args):
    """The reference's own per-frame unit: OnRender (main.cpp:705-859), called
    by the platform once per animation frame (wasm/wasm.cpp:176-218) with one
    progressive sample per pixel per call, MaxBounce 5 (main.cpp:387), the
    completed frame handed back one call late.  Driven here through the C-ABI
    (rt_on_init / rt_on_init_devices + rt_on_render, busy-polling like a
    platform loop with a GPU behind it) at 1920x1080 and at 960x540 (the
    default 1280x720 window x the 0.75 render scale, main.cpp:649-650,
    wasm/wasm.cpp:78), scene 0 (RGB Glass, wasm/wasm.cpp:20) unless --scene:
      static: the camera stays, so every call folds one more frame;
      moving: RT_KEY_LEFT on every call (main.cpp:743-746), so every frame
              restarts the mean, re-runs the cull pass, and waits for the
              previous frame (WorkQueueWaitUntilCompletion, main.cpp:792).
    The line reports Mrays/s and ms per completed frame for each, and where
    the host time went (rt_on_render_get_profile)."""
    import numpy as np
    import torch
    import __graft_entry__ as graft

    rt = graft.load_package()
    if os.environ.get("BENCH_SHARE_GPU") == "1":
        devices = [0] * args.gpus
    elif args.devices:
        devices = [int(d) for d in args.devices.split(",")]
    else:
        devices = list(range(args.gpus))
    visible = torch.cuda.device_count()
    if visible < max(devices) + 1:
        print(f"bench.py: onrender over devices {sorted(set(devices))} but {visible} visible", file=sys.stderr)
        raise SystemExit(2)
    scene = 0 if args.scene is None else args.scene
    sizes = [(args.width, args.height)] if args.width and args.height else [(1920, 1080), (960, 540)]
    device_sets = [devices[:1]] + ([devices] if len(devices) > 1 else [])
    has_profile = hasattr(rt.lib(), "rt_on_render_get_profile")
    runs = []
    for devs in device_sets:
        for (W, H) in sizes:
            for mode, keys in (("static", 0), ("moving", rt.KEY_LEFT)):
                if mode not in args.modes.split(","):
                    continue
                rt.on_init(devs if len(devs) > 1 else None)
                img = np.zeros((H, W), np.uint32)
                if not args.no_register:  # the platform's persistent image (wasm/wasm.cpp:179)
                    rt.on_render_register_image(img)
                warm = 0
                while warm < 8:  # code objects, allocations, the first cull pass
                    ok, _, _ = rt.on_render(img, scene, True, keys)
                    warm += int(ok)
                if has_profile:
                    rt.on_render_profile(reset=True)
                done = rays = calls = 0
                t0 = time.perf_counter()
                while done < args.frames:
                    ok, r, _ = rt.on_render(img, scene, True, keys)
                    calls += 1
                    if ok:
                        done += 1
                        rays += r
                wall = time.perf_counter() - t0
                run = {"devices": devs, "width": W, "height": H, "mode": mode,
                       "image": "staged" if args.no_register else "registered", "frames": done, "calls": calls,
                       "rays": rays, "mrays_per_s": round(rays / wall / 1e6, 1),
                       "ms_per_frame": round(wall / done * 1e3, 4)}
                if has_profile:
                    prof = rt.on_render_profile()
                    wall_ms = wall * 1e3
                    run["host_ms_per_frame"] = {k: round(prof[k] / done, 4) for k in
                                                ("CallMs", "HostCopyMs", "HostWaitMs")}
                    run["gpu_ms_per_frame"] = round(prof["GpuFrameMs"] / max(prof["FramesCopied"], 1), 4)
                    run["share_of_wall"] = {"host_copy": round(prof["HostCopyMs"] / wall_ms, 4),
                                            "host_wait": round(prof["HostWaitMs"] / wall_ms, 4),
                                            "gpu_frame": round(prof["GpuFrameMs"] / wall_ms, 4)}
                rt.on_shutdown()
                runs.append(run)
                print(json.dumps(run), file=sys.stderr, flush=True)
    line = {"metric": "OnRender Mrays/sec (1 spp per call, 5 bounces)", "value": runs[0]["mrays_per_s"],
            "unit": "Mrays/s", "n_gpus": len(set(devices)) if len(devices) > 1 else 1, "steps": args.frames,
            "warmup": 8, "ms_per_step": runs[0]["ms_per_frame"], "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f32",
            "data": f"the reference's built-in scene {scene} ({SCENE_NAMES[scene]}), its default camera",
            "config": {"workload": "onrender", "scene": scene, "lib": os.environ.get("RT_TRACE_LIB", "librt_trace.so"),
                       "note": "value/ms_per_step: the first run (1 device, static camera, "
                               f"{sizes[0][0]}x{sizes[0][1]}); every run is in 'runs'"},
            "runs": runs}
    print(json.dumps(line), flush=True)


def main():
    args = parse()
    if args.config == "onrender":
        return main_onrender(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 and args.gpus > 1 and args.sim_ranks == 0:
        return main_multi_device(args)
    import torch
    import torch.distributed as dist
    import __graft_entry__ as graft

    rt = graft.load_package()
    opts = device_options(rt, args)
    binary_hash = rt.code_object_hash()
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # BENCH_BACKEND=gloo + BENCH_SHARE_GPU=1: rehearsal of the multi-rank
    # path with every rank on cuda:0 (a 1-GPU box); the real runs use RCCL
    backend = os.environ.get("BENCH_BACKEND", "nccl")
    gpu = 0 if os.environ.get("BENCH_SHARE_GPU") == "1" else local
    torch.cuda.set_device(gpu)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)

    scene = make_scene(rt, args)
    W, H, S, B, N = args.width, args.height, args.spp, args.bounces, args.spheres
    cam = rt.camera_setup(scene, W, H, distance=args.distance)
    dev = rt.Device(gpu, options=opts)
    dev.upload_scene(scene)
    band_rows = args.band_rows
    bands = args.sim_ranks if (world == 1 and args.sim_ranks > 1) else world
    rows = [rt.band_local_rows(H, band_rows, bands, r) for r in range(bands)]
    maxr = max(rows)
    band_index = args.sim_index if bands != world else rank
    dev.reserve(W, maxr)  # launch buffers for this band geometry: no timed launch allocates (rt_device_reserve)
    # Two frame slots: frame i's band image is gathered to rank 0 while frame
    # i+1 is traced; rank 0 assembles frame i before frame i+2 reuses its slot.
    # The gather is the C-ABI's RCCL band gather (rt_comm_gather_bands: grouped
    # send/recv to rank 0 over xGMI, then the scatter into the full frame) on a
    # side stream; a rehearsal with every rank on one GPU (BENCH_SHARE_GPU=1,
    # which RCCL refuses) uses a torch.distributed gather.  The timed region
    # ends only after the last frame is assembled on rank 0.
    cur = [torch.zeros(maxr * W, dtype=torch.int32, device="cuda") for _ in range(2)]
    prev = torch.zeros((maxr * W, 4), dtype=torch.float32, device="cuda")
    rays = torch.zeros(1, dtype=torch.int64, device="cuda")  # the tiny code-object launch's counter
    # one pre-zeroed ray counter per step (cold, warm-ups, timed): no counter
    # reset between launches, and every timed step's count is checked after
    ctr = torch.zeros(args.warmup + args.steps + 2, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream()
    comm, gather_kind = None, None
    if world > 1:
        gather_kind = f"torch.distributed {backend} gather + rt_assemble_bands"
        if backend == "nccl" and os.environ.get("BENCH_SHARE_GPU") != "1":
            uid = [rt.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            err = ""
            try:
                comm = rt.Comm(gpu, uid[0], world, rank)
            except rt.RtError as e:
                err = str(e)
            ok = torch.tensor([1 if comm else 0], dtype=torch.int32, device="cuda")
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok.item()) == 1:
                gather_kind = "RCCL grouped send/recv to rank 0 + scatter (rt_comm_gather_bands)"
            else:
                if comm:
                    comm.close()
                comm = None
                gather_kind += f" (rt_comm unavailable: {err or 'on another rank'})"
                print(f"bench.py: {gather_kind}", file=sys.stderr)
    gbuf = full = None
    if world > 1 and rank == 0:
        full = torch.empty(H * W, dtype=torch.int32, device="cuda")
        if comm is None:
            gdev = "cuda" if backend == "nccl" else "cpu"
            gbuf = [torch.empty((world, maxr * W), dtype=torch.int32, device=gdev) for _ in range(2)]
    side = torch.cuda.Stream() if comm else None
    gathered = [None, None]  # per slot: event after its gather on the side stream
    # HIP events around every timed launch give the kernel's own average time on
    # one whole-frame GPU (the roofline's denominator).  A band share (world > 1 or
    # --sim-ranks) takes one pair around the whole timed loop instead: every event
    # marker between launches widens the dispatch gap (measured ~4.6 us each), a
    # measurable share of a 0.8 ms launch; its kernel time is then GPU ms per step.
    per_launch_events = world == 1 and bands == 1
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps if per_launch_events else 1)]
    state = {"n": 0, "pending": None, "c": 0}

    def finish():  # frame whose gather is in flight -> assembled on rank 0
        if state["pending"] is None:
            return
        work, slot = state["pending"]
        state["pending"] = None
        work.wait()
        if rank == 0:
            src = gbuf[slot] if backend == "nccl" else gbuf[slot].to("cuda")
            rt.assemble_bands(src.data_ptr(), maxr * W * 4, full.data_ptr(), W, H, 4, band_rows, world,
                              stream=stream.cuda_stream)

    def step(i=None):
        slot = state["n"] % 2
        state["n"] += 1
        if gathered[slot] is not None:  # the gather two frames back has read this slot
            stream.wait_event(gathered[slot])
        c = state["c"]
        state["c"] += 1
        if i is not None and (per_launch_events or i == 0):
            ev[i][0].record(stream)
        dev.trace(cam, width=W, height=H, prev_ptr=prev.data_ptr(), cur_ptr=cur[slot].data_ptr(),
                  rays_ptr=ctr[c].data_ptr(), prev_count=0, frames=S, max_bounce=B, simd=not args.scalar,
                  band_rows=band_rows, band_count=bands, band_index=band_index, accum_zero=True,
                  stream=stream.cuda_stream)
        if i is not None and (per_launch_events or i == args.steps - 1):
            ev[i if per_launch_events else 0][1].record(stream)
        if world > 1 and comm is not None:
            traced = torch.cuda.Event()
            traced.record(stream)
            side.wait_event(traced)
            comm.gather_bands(cur[slot].data_ptr(), full.data_ptr() if rank == 0 else 0, W, H, 4, band_rows,
                              stream=side.cuda_stream)
            gathered[slot] = torch.cuda.Event()
            gathered[slot].record(side)
        elif world > 1:
            send = cur[slot] if backend == "nccl" else cur[slot].cpu()
            work = dist.gather(send, list(gbuf[slot].unbind(0)) if rank == 0 else None, dst=0, async_op=True)
            finish()
            state["pending"] = (work, slot)

    # Cold launch: the first launch for this camera / scene / geometry runs the
    # primary-ray cull pass and traces in the cull pass's live-first tile order
    # (the heaviest-first order is learned over the next launches).  A tiny
    # launch first loads the code objects, so cold_ms is the render's own cost.
    tiny_prev = torch.zeros((64 * 8, 4), dtype=torch.float32, device="cuda")
    tiny_cur = torch.zeros(64 * 8, dtype=torch.int32, device="cuda")
    dev.trace(cam, width=64, height=8, prev_ptr=tiny_prev.data_ptr(), cur_ptr=tiny_cur.data_ptr(),
              rays_ptr=rays.data_ptr(), frames=1, max_bounce=1, simd=not args.scalar, band_rows=8,
              accum_zero=True, stream=stream.cuda_stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t = time.perf_counter()
    step()
    finish()
    torch.cuda.synchronize()
    cold_ms = (time.perf_counter() - t) * 1e3
    cold_info = dev.last_info()
    for _ in range(max(args.warmup - 1, 0)):
        step()
    finish()
    torch.cuda.synchronize()
    rays_local = int(ctr[state["c"] - 1].item())  # this rank's segments per launch (last warm-up)
    first_timed = state["c"]
    rays_per_step = torch.tensor([rays_local, dev.last_info()["SegmentsFolded"]], dtype=torch.int64,
                                 device="cuda")
    if world > 1:
        dist.all_reduce(rays_per_step)
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    finish()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    info = dev.last_info()
    timed_counts = ctr[first_timed:first_timed + args.steps].tolist()
    if any(n != rays_local for n in timed_counts):
        raise SystemExit(f"bench.py: timed steps counted {timed_counts} segments, expected {rays_local} each")
    verified, one_ms = None, None
    if (args.verify or world > 1) and not args.no_verify and bands == world:
        # rank 0 renders the whole frame alone: the 1-GPU time and the reference the gathered frame must equal
        if rank == 0:
            ref_cur, one_ms, one_rays = one_gpu_reference(rt, torch, dev, cam, args, W, H, S, B, stream,
                                                          min(args.steps, 5))
            got = full if world > 1 else cur[(state["n"] - 1) % 2]
            verified = bool(torch.equal(got, ref_cur))
        if world > 1:
            dist.barrier()
    frame_check = None
    if rank == 0 and bands == world:
        # the last timed frame against the committed fixture of this workload
        last = full if world > 1 else cur[(state["n"] - 1) % 2]
        torch.cuda.synchronize()
        frame_check = check_frame(rt, args, W, H, S, args.spheres, B, last.cpu().numpy().view("uint32"),
                                  prev.cpu().numpy() if world == 1 else None, int(rays_per_step[0].item()))
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    t = torch.tensor([elapsed, kern_ms, cold_ms], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms_max, cold_ms = float(t[0]), float(t[1]), float(t[2])
    seg_counted, seg_folded = int(rays_per_step[0].item()), int(rays_per_step[1].item())
    total_rays = seg_counted * args.steps

    if bands != world:
        if rank == 0:
            out = {"sim_ranks": bands, "sim_index": band_index, "rank0_rows": rows[band_index],
                   "rank0_kernel_ms": round(kern_ms, 3), "lanes_per_pixel": info["LanesPerPixel"],
                   "rank0_rays": rays_local, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
                   "cold_ms": round(cold_ms, 3)}
            stats = dev.debug_stats()
            if stats:
                out["sched_stats"] = stats
            print(json.dumps(out))
        if comm:
            comm.close()
        dev.close()
        return
    legs = {}
    want = set() if args.headline_only else set(args.legs.split(","))
    if world == 1 and bands == 1:
        if "distinct" in want:
            legs["distinct"] = distinct_leg(rt, torch, args, dev, scene, cam, W, H, S, N, B, gpu, stream, opts)
        if "brute" in want and not args.brute and not opts and W * H * S * N <= 2.2 * 1920 * 1080 * 256 * 64:
            legs["brute"] = brute_leg(rt, torch, args, scene, cam, W, H, S, N, B, gpu, stream, binary_hash,
                                      lambda o: workload_name(args, W, H, S, N, B, o))
    if rank == 0:
        workload = workload_name(args, W, H, S, N, B, opts)
        line = base_line(args, world=world, elapsed=elapsed, seg_counted=seg_counted, seg_folded=seg_folded,
                         W=W, H=H, S=S, N=N, B=B, workload=workload,
                         parallelism=f"{world} GPU x interleaved {band_rows}-row bands"
                                     + (", one process per GPU (torch.distributed.run)" if world > 1 else ""),
                         gather=gather_kind)
        line["cold_ms"] = round(cold_ms, 3)
        line["cold"] = {"ms": round(cold_ms, 3), "cull_pass": bool(cold_info["CullPassRan"]),
                        "note": "first launch for this camera/scene/geometry (cull pass + untrained tile order), "
                                "wall clock incl. its host synchronisation; the timed steps reuse the cull masks "
                                "and the learned heaviest-first order"}
        line["roofline"] = roofline(args, info, kern_ms, rays_local, rows[0], W, N, workload, world, binary_hash,
                                    culled=opts.get("Cull", 0) != -1)
        if per_launch_events:
            line["kernel_ms_per_step"] = [round(a.elapsed_time(b), 3) for a, b in ev]
        if opts:
            line["config"]["device_options"] = opts
        if "brute" in legs:
            line["roofline"]["brute"] = legs["brute"]
        if "distinct" in legs:
            line["value_distinct_samples"] = legs["distinct"]["value"]
            line["distinct_samples"] = legs["distinct"]
        if world > 1:
            line["kernel_ms_max_over_ranks"] = round(kern_ms_max, 3)
        if one_ms is not None and world > 1:
            line["one_gpu"] = {"ms_per_frame": round(one_ms, 3),
                               "speedup_vs_one_gpu": round(one_ms / (elapsed / args.steps * 1e3), 3),
                               "note": "the same frame traced whole on rank 0's GPU alone, in this run"}
        stats = dev.debug_stats()
        if stats:
            line["sched_stats"] = stats
        if verified is not None:
            line["verified_vs_one_gpu"] = verified
        if frame_check is not None:
            line["frame_check"] = frame_check
            line["verified"] = combine_verified(verified, frame_check["verified"])
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args, total_rays)
        print(json.dumps(line), flush=True)
        if line.get("verified") is False:
            print(f"bench.py: the timed frame does NOT match {frame_check.get('golden')}: {frame_check}",
                  file=sys.stderr)
            raise SystemExit(3)
        bad = [k for k, leg in (("distinct samples", legs.get("distinct", {}).get("verified_vs_fresh_device")),
                                ("brute force", legs.get("brute", {}).get("verified"))) if leg is False]
        if bad:
            print(f"bench.py: the {' and '.join(bad)} leg's frame does NOT match", file=sys.stderr)
            raise SystemExit(3)
    if comm:
        comm.close()
    dev.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
