"""Generates tests/golden/c5_rows.json: BASELINE config C5 (7680x4320, 4096 spp,
scene 1's first 256 spheres, 16 bounces, pixel seeds) on whole 32-row tile rows,
rendered twice on the CPU --

* by the REFERENCE'S OWN CODE: main.cpp:7-640 with SURVEY §8c's two textual
  patches (oracle/_ref/librefpix.so, oracle/Makefile), the reference's
  RenderTile over just those tiles (ref_render_tile_list, the work entries
  main.cpp:362-368 decodes), pulled by 8 worker threads;
* by the oracle's row mode (oracle/rt_oracle.c, rows=(y0, y1)).

The two must agree field for field (the script exits 1 otherwise), and the
fixture records, per tile row, the bounce-segment count and FNV-1a-64 hashes of
its rows of the v4 f32 running mean and of the RGBA8 image.  A whole C5 frame is
about 2.2e11 segments (~5e4 core-seconds), out of a CPU render's
reach; five tile rows are ~1e10 segments, about 12 minutes per renderer on the
container's 8 threads.  The tile rows hold the verdict's rows 0-1, 2160-2161
and 4318-4319 (tile rows 0, 67, 134) and the two geometry-heavy bands of the
frame (tile rows 50 and 95: the most hit pixels at 1 spp).

The GPU checks its full-frame C5 render against these hashes
(tests/test_golden_regression.py::test_gpu_c5_tile_rows) and bench.py --config
c5 checks its last timed frame the same way (`frame_check`).  Needs an Intel
host (NormalizeFast is the host's rsqrtss; the oracle uses the captured table).

    python tests/golden/make_c5_rows.py [--frames F] [--tile-rows 0,67,...] [--out PATH]
"""
import argparse
import ctypes
import json
import os
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import oracle as orc  # noqa: E402

OUT = pathlib.Path(__file__).with_name("c5_rows.json")
W, H, N, B, FRAMES = 7680, 4320, 256, 16, 4096
TILE_ROWS = (0, 50, 67, 95, 134)
TILE = 32


def band_hashes(prev, cur, y0, y1):
    p = prev.reshape(H, W, 4)[y0:y1]
    c = cur.reshape(H, W)[y0:y1]
    return f"{orc.fnv1a64(p):016x}", f"{orc.fnv1a64(c):016x}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=FRAMES)
    ap.add_argument("--tile-rows", default=",".join(map(str, TILE_ROWS)))
    ap.add_argument("--out", default=str(OUT))
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    a = ap.parse_args()
    tile_rows = [int(t) for t in a.tile_rows.split(",")]
    o = orc.scene_builtin(1).prefix(N)
    cam = orc.camera(o, W, H)
    tiles_x = (W + TILE - 1) // TILE

    P = ctypes.CDLL(str(ROOT / "oracle" / "_ref" / "librefpix.so"))
    v, u32 = ctypes.c_void_p, ctypes.c_uint32
    P.ref_set_patch.argtypes = [u32, ctypes.c_int]
    P.ref_render_tile_list.argtypes = [v, u32, v, u32, v, u32, u32, v, u32, u32, u32, u32, ctypes.c_int, u32, v, u32,
                                       v, v, v]
    out = {"generator": "tests/golden/make_c5_rows.py", "scene": 1, "spheres": N, "width": W, "height": H,
           "frames": a.frames, "bounces": B, "simd": True, "seed": "pixel", "tile_rows": {},
           "source": "oracle/_ref/librefpix.so (main.cpp:7-640, SURVEY 8c patches) and oracle/liboracle.so rows mode"}
    ok = True
    for ty in tile_rows:
        y0, y1 = ty * TILE, min(H, (ty + 1) * TILE)
        # the reference: its RenderTile over this tile row's tiles only
        rprev = np.zeros((W * H, 4), np.float32)
        rcur = np.zeros(W * H, np.uint32)
        rays = np.zeros(1, np.uint64)
        tiles = np.arange(ty * tiles_x, (ty + 1) * tiles_x, dtype=np.uint32)
        P.ref_set_patch(B, 1)
        t = time.time()
        P.ref_render_tile_list(o.spheres.ctypes.data, len(o.spheres), o.groups.ctypes.data, len(o.groups),
                               o.materials.ctypes.data, len(o.materials), int(o.use_sky), cam.ctypes.data, W, H, 0,
                               a.frames, 1, a.threads, tiles.ctypes.data, len(tiles), rprev.ctypes.data,
                               rcur.ctypes.data, rays.ctypes.data)
        ref_s = time.time() - t
        ref_rays = int(rays[0])
        ref_v4, ref_rgba = band_hashes(rprev, rcur, y0, y1)
        del rprev, rcur
        # the oracle's row mode on the same rows
        t = time.time()
        oprev, ocur, orays = orc.render(o, cam, W, H, frames=a.frames, max_bounce=B, rows=(y0, y1),
                                        threads=a.threads)
        or_s = time.time() - t
        or_v4, or_rgba = band_hashes(oprev, ocur, y0, y1)
        hit = int(np.count_nonzero(ocur.reshape(H, W)[y0:y1] != 0xFF000000))
        del oprev, ocur
        same = (ref_rays, ref_v4, ref_rgba) == (orays, or_v4, or_rgba)
        ok &= same
        out["tile_rows"][str(ty)] = {"rows": [y0, y1], "rays": ref_rays, "fnv1a64_v4": ref_v4,
                                     "fnv1a64_rgba8": ref_rgba, "non_black_pixels": hit,
                                     "oracle_equal": same, "ref_seconds": round(ref_s, 1),
                                     "oracle_seconds": round(or_s, 1), "threads": a.threads}
        print(ty, (y0, y1), ref_rays, ref_v4, ref_rgba, "oracle", orays, or_v4, or_rgba, "equal" if same else "DIFFER",
              f"ref {ref_s:.0f} s, oracle {or_s:.0f} s", flush=True)
    pathlib.Path(a.out).write_text(json.dumps(out, indent=1) + "\n")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
