"""Diagnostic (CPU): which spheres can a pixel's jittered primary rays hit (f64
line test over a jitter grid), and are their groups in the cull mask of the
pixel's wave tile (numpy restatement in tests/cull_ref.py)?
Usage: python scripts/diag/pixel_hits.py N W H P x y"""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as g  # noqa: E402

sys.path.insert(0, str(ROOT / "tests"))
from cull_ref import SHAPE, np_masks  # noqa: E402

rt = g.load_package()

n, W, H, P, x, y = (int(v) for v in sys.argv[1:7])
s = rt.scene_prefix(rt.scene_builtin(1), n)
cam = rt.camera_setup(s, W, H)
m = np_masks(rt, s, cam, W, H, P)
_, groups, _ = rt.scene_arrays(s)
c = np.stack([groups[:, 0:4].ravel(), groups[:, 4:8].ravel(), groups[:, 8:12].ravel()], 1).astype(np.float64)
r = groups[:, 12:16].ravel().astype(np.float64)
v3 = lambda q: np.array([q.x, q.y, q.z], np.float64)  # noqa: E731
cp, cx, cy, fc = v3(cam.CameraPosition), v3(cam.CameraX), v3(cam.CameraY), v3(cam.FilmCenter)
hits = set()
for jx in np.linspace(-0.5, 0.5, 21):
    for jy in np.linspace(-0.5, 0.5, 21):
        fx = -1 + (x + jx) * 2 / W
        fy = -1 + (y + jy) * 2 / H
        p = fc + fx * cam.FilmW * 0.5 * cx + fy * cam.FilmH * 0.5 * cy
        d = p - cp
        d /= np.linalg.norm(d)
        C = c - cp
        T = C @ d
        dist = (C * C).sum(1) - T * T
        for i in np.flatnonzero(dist < r * r):
            hits.add((int(i), round(float(T[i]), 3)))
TW, TH = SHAPE[P]
tx = (W + 2 * TW - 1) // (2 * TW)
t = (y // (2 * TH)) * tx + x // (2 * TW)
w = (1 if (x % (2 * TW)) >= TW else 0) + (2 if (y % (2 * TH)) >= TH else 0)
nw = (groups.shape[0] + 63) // 64
mask = [int(m[(t * 4 + w) * nw + k]) for k in range(nw)]
print("pixel", (x, y), "tile", t, "wave", w, "mask", [hex(v) for v in mask])
for i, T in sorted(hits):
    gi = i // 4
    print(f"  sphere {i} group {gi} T={T} in_mask={(mask[gi // 64] >> (gi % 64)) & 1}")
