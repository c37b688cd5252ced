"""Generates tests/golden/reference_frames.json from the REFERENCE'S OWN CODE.

Runs main.cpp's RenderTile / RenderTileScalar (compiled from /root/reference
by `make -C oracle ref` into oracle/_ref/librefmath.so, see
oracle/ref_harness.cpp) over whole frames on one worker thread -- the thread-0
PCG stream in tile order, MaxRayBounce 5 (main.cpp:387) -- and records, per
case, the bounce-segment count, the final PCG state and FNV-1a-64 hashes of
the RGBA8 image and of the v4 f32 accumulation.  The fixture is data: it lets
tests/test_oracle_vs_reference_render.py check the oracle against the
reference where /root/reference is absent.  Needs an Intel host (the
reference's NormalizeFast is the host's rsqrtss).

Round 5 adds "pixel_cases": every pixel-seed case of
tests/golden/oracle_regression.json (the fixtures the GPU path is checked
against, tests/test_golden_regression.py), rendered by the reference itself in
SURVEY §8c's `pixel` mode at the case's bounce count -- main.cpp:7-640 with the
two textual patches on a temporary copy (oracle/Makefile, librefpix.so) --
including the full BASELINE frames (C2, C3, RTWeekend, C2 from inside).  The
patched build runs the reference's tiles on a pthread pool (the output is
schedule-independent in pixel mode).

    python tests/golden/make_reference_golden.py [--pixel-only] [--skip-c3]
"""
import ctypes
import json
import os
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import oracle as orc  # noqa: E402  (scene/camera inputs and the FNV hash only)

OUT = pathlib.Path(__file__).with_name("reference_frames.json")
PIXEL_SOURCE = ("/root/reference/main.cpp:7-640 with SURVEY 8c's patches (MaxRayBounce :387,536; per-pixel seed "
                "after :373,522 with the mixer of :668-675) via oracle/ref_harness.cpp -DRT_REF_PATCHED")

# (name, builtin scene, sphere prefix or None, W, H, frames, simd, prev_count)
CASES = [
    ("rgb_glass_96x64x3", 0, None, 96, 64, 3, True, 0),
    ("rgb_glass_96x64x3_scalar", 0, None, 96, 64, 3, False, 0),
    ("floating_256x256x4", 1, None, 256, 256, 4, True, 0),        # SURVEY §8c probe: 440,334 segments
    ("floating_256x256x4_scalar", 1, None, 256, 256, 4, False, 0),
    ("rtweekend_96x64x3", 2, None, 96, 64, 3, True, 0),
    ("rtweekend_96x64x3_scalar", 2, None, 96, 64, 3, False, 0),
    ("n64_128x72x2", 1, 64, 128, 72, 2, True, 0),
    ("n64_128x72x2_scalar", 1, 64, 128, 72, 2, False, 0),
    ("n4_37x29x2_pc5", 1, 4, 37, 29, 2, True, 5),
    ("rtweekend_160x90x2_pc3", 2, None, 160, 90, 2, True, 3),
]


def scene_of(index, prefix):
    o = orc.scene_builtin(index)
    return o.prefix(prefix) if prefix else o


def pixel_cases(skip_c3: bool) -> dict:
    """Every pixel-mode case of oracle_regression.json, rendered by librefpix.so."""
    sys.path.insert(0, str(ROOT / "tests" / "golden"))
    import make_golden
    P = ctypes.CDLL(str(ROOT / "oracle" / "_ref" / "librefpix.so"))
    v, u32 = ctypes.c_void_p, ctypes.c_uint32
    P.ref_set_patch.argtypes = [u32, ctypes.c_int]
    P.ref_render_threads.argtypes = [v, u32, v, u32, v, u32, u32, v, u32, u32, u32, u32, ctypes.c_int, u32, v, v, v]
    threads = min(8, os.cpu_count() or 1)
    out = {}
    for name, idx, n, w, h, frames, bounces, simd, seed in make_golden.CASES:
        if seed != "pixel" or (skip_c3 and name in make_golden.SLOW):
            continue
        o = scene_of(idx, n)
        cam = orc.camera(o, w, h, distance=make_golden.DISTANCE.get(name))
        prev = np.zeros((w * h, 4), np.float32)
        cur = np.zeros(w * h, np.uint32)
        rays = np.zeros(1, np.uint64)
        P.ref_set_patch(bounces, 1)
        t = time.time()
        P.ref_render_threads(o.spheres.ctypes.data, len(o.spheres), o.groups.ctypes.data, len(o.groups),
                             o.materials.ctypes.data, len(o.materials), int(o.use_sky), cam.ctypes.data, w, h, 0,
                             frames, int(simd), threads, prev.ctypes.data, cur.ctypes.data, rays.ctypes.data)
        out[name] = {"scene": idx, "spheres": n, "width": w, "height": h, "frames": frames, "bounces": bounces,
                     "simd": simd, **({"distance": make_golden.DISTANCE[name]} if name in make_golden.DISTANCE else {}),
                     "rays": int(rays[0]), "fnv1a64_rgba8": f"{orc.fnv1a64(cur):016x}",
                     "fnv1a64_v4": f"{orc.fnv1a64(prev):016x}", "ref_seconds": round(time.time() - t, 2),
                     "ref_threads": threads}
        print(name, out[name]["rays"], out[name]["fnv1a64_rgba8"], out[name]["ref_seconds"], "s", flush=True)
    return out


def main():
    keep = json.loads(OUT.read_text()) if OUT.exists() else {}
    pixel_only = "--pixel-only" in sys.argv
    px = pixel_cases("--skip-c3" in sys.argv)
    if "--skip-c3" in sys.argv:  # keep a previously rendered C3 entry
        for k, e in keep.get("pixel_cases", {}).items():
            px.setdefault(k, e)
    if pixel_only:
        keep["pixel_cases"] = px
        keep["pixel_source"] = PIXEL_SOURCE
        OUT.write_text(json.dumps(keep, indent=1) + "\n")
        return
    L = ctypes.CDLL(str(ROOT / "oracle" / "_ref" / "librefmath.so"))
    v, u32 = ctypes.c_void_p, ctypes.c_uint32
    L.ref_render.argtypes = [v, u32, v, u32, v, u32, u32, v, u32, u32, u32, u32, ctypes.c_int, v, v, v, v]
    out = {}
    for name, idx, prefix, w, h, frames, simd, pc in CASES:
        o = scene_of(idx, prefix)
        cam = orc.camera(o, w, h)
        seed = orc.seed_mix(0)
        prev = np.zeros((w * h, 4), np.float32)
        cur = np.zeros(w * h, np.uint32)
        st = np.array([seed], np.uint64)
        rays = np.zeros(1, np.uint64)
        L.ref_render(o.spheres.ctypes.data, len(o.spheres), o.groups.ctypes.data, len(o.groups),
                     o.materials.ctypes.data, len(o.materials), int(o.use_sky), cam.ctypes.data, w, h, pc, frames,
                     int(simd), st.ctypes.data, prev.ctypes.data, cur.ctypes.data, rays.ctypes.data)
        out[name] = {"scene": idx, "prefix": prefix, "width": w, "height": h, "frames": frames, "simd": simd,
                     "prev_count": pc, "seed": f"{seed:016x}", "rays": int(rays[0]), "final_state": f"{int(st[0]):016x}",
                     "rgba8_fnv1a64": f"{orc.fnv1a64(cur):016x}", "v4_fnv1a64": f"{orc.fnv1a64(prev):016x}",
                     "non_black_pixels": int(np.count_nonzero(cur != 0xFF000000))}
        print(name, out[name]["rays"], out[name]["rgba8_fnv1a64"])
    OUT.write_text(json.dumps({"generator": "tests/golden/make_reference_golden.py",
                               "source": "/root/reference/main.cpp:7-640 via oracle/ref_harness.cpp",
                               "max_bounce": 5, "cases": out, "pixel_source": PIXEL_SOURCE, "pixel_cases": px},
                              indent=1) + "\n")


if __name__ == "__main__":
    main()
