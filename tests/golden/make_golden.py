"""Generates tests/golden/oracle_regression.json: FNV-1a-64 hashes, ray counts
and a few raw pixels of oracle renders (pixel and stream seed modes) for the
configurations the parity tests use.  These are REGRESSION vectors of the
oracle (which is itself pinned to the reference by test_oracle_reference.py),
committed so the GPU path can be checked against fixed data too.

    python tests/golden/make_golden.py [case ...]   (only the named cases are re-rendered)
"""
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import oracle as orc  # noqa: E402

OUT = ROOT / "tests" / "golden" / "oracle_regression.json"

CASES = [
    # name, scene, N, W, H, frames, bounces, simd, seed mode
    ("c1_simd", 1, 4, 256, 256, 1, 1, True, "pixel"),
    ("c1_scalar", 1, 4, 256, 256, 1, 1, False, "pixel"),
    ("n64_b8_128x96x8", 1, 64, 128, 96, 8, 8, True, "pixel"),
    ("n256_b16_64x64x2", 1, 256, 64, 64, 2, 16, True, "pixel"),
    ("rgb_glass_96x64x4", 0, None, 96, 64, 4, 5, True, "pixel"),
    ("rtweekend_80x48x2", 2, None, 80, 48, 2, 5, True, "pixel"),
    ("rtweekend_80x48x2_scalar", 2, None, 80, 48, 2, 5, False, "pixel"),
    ("ragged_n13_37x23x3", 1, 13, 37, 23, 3, 6, True, "pixel"),
    ("survey_scene1_stream_256x4", 1, None, 256, 256, 4, 5, True, "stream"),
    # round 5: the parity mode at B = 8 on the colour scenes and the scalar rules at
    # B = 8 / 16 -- these, like every pixel case, are also rendered by the reference
    # itself (tests/golden/make_reference_golden.py, SURVEY 8c patches)
    ("rgb_glass_b8_96x64x4", 0, None, 96, 64, 4, 8, True, "pixel"),
    ("rgb_glass_b8_96x64x4_scalar", 0, None, 96, 64, 4, 8, False, "pixel"),
    ("rtweekend_b8_80x48x2", 2, None, 80, 48, 2, 8, True, "pixel"),
    ("rtweekend_b8_80x48x2_scalar", 2, None, 80, 48, 2, 8, False, "pixel"),
    ("n64_b8_128x96x8_scalar", 1, 64, 128, 96, 8, 8, False, "pixel"),
    ("n256_b16_64x64x2_scalar", 1, 256, 64, 64, 2, 16, False, "pixel"),
    ("survey_n64_pixel_256x4", 1, 64, 256, 256, 4, 8, True, "pixel"),
    # BASELINE.json configs[1] (C2) at full size: the whole 1920x1080 frame, 256 spp
    ("c2_full_1920x1080x256", 1, 64, 1920, 1080, 256, 8, True, "pixel"),
    # configs[2] (C3) at full size: ~16x C2 on the CPU (minutes), so its CPU
    # re-render runs only with RT_SLOW_ORACLE=1 (tests/test_golden_regression.py)
    ("c3_full_3840x2160x1024", 1, 64, 3840, 2160, 1024, 8, True, "pixel"),
    # bench.py's frames the primary-ray cull cannot empty: RTWeekend (sky term,
    # 482 spheres) and C2's scene seen from inside the sphere cloud
    ("rtw_full_1920x1080x64", 2, None, 1920, 1080, 64, 8, True, "pixel"),
    ("c2in_full_1920x1080x256", 1, 64, 1920, 1080, 256, 8, True, "pixel"),
]
SLOW = {"c3_full_3840x2160x1024"}
# camera distance from the look-at point where a case does not use the scene's default
DISTANCE = {"c2in_full_1920x1080x256": 1.0}


def render_case(scene, n, W, H, frames, bounces, simd, seed, distance=None):
    o = orc.scene_builtin(scene)
    if n is not None:
        o = o.prefix(n)
    mode = orc.SEED_PIXEL if seed == "pixel" else orc.SEED_STREAM
    return orc.render(o, orc.camera(o, W, H, distance=distance), W, H, frames=frames, max_bounce=bounces, simd=simd,
                      seed_mode=mode, threads=1 if seed == "stream" else orc.cpu_threads())


def main():
    out = {}
    keep = json.loads(OUT.read_text()) if OUT.exists() else {}
    only = set(sys.argv[1:])  # optional: regenerate just these cases
    for name, scene, n, W, H, frames, bounces, simd, seed in CASES:
        if only and name not in only and name in keep:
            out[name] = keep[name]
            continue
        prev, cur, rays = render_case(scene, n, W, H, frames, bounces, simd, seed, DISTANCE.get(name))
        mid = (H // 2) * W + W // 2
        out[name] = {"scene": scene, "spheres": n, "width": W, "height": H, "frames": frames, "bounces": bounces,
                     "simd": simd, "seed_mode": seed, "rays": rays,
                     **({"distance": DISTANCE[name]} if name in DISTANCE else {}),
                     "fnv1a64_rgba8": f"{orc.fnv1a64(cur):016x}", "fnv1a64_v4": f"{orc.fnv1a64(prev):016x}",
                     "center_rgba8": f"{int(cur[mid]):08x}",
                     "center_v4_bits": [f"{int(v):08x}" for v in prev[mid].view(np.uint32)]}
    OUT.write_text(json.dumps(out, indent=1) + "\n")
    print(f"wrote {OUT} ({len(out)} cases)")


if __name__ == "__main__":
    main()
