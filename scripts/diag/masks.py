"""Diagnostic: are the cull pass's masks deterministic and do they match a numpy f64 restatement?"""
import os, sys, pathlib
import numpy as np
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import torch
import __graft_entry__ as g
rt = g.load_package()
SHAPE = {1: (8, 8), 2: (8, 4), 4: (4, 4), 8: (4, 2), 16: (2, 2)}

def np_masks(scene, cam, W, H, P, simd=True):
    _, groups, _ = rt.scene_arrays(scene)  # (ng, 16): x[4] y[4] z[4] r[4] (SIMD groups)
    ng = groups.shape[0]
    cx, cy, cz = groups[:, 0:4].ravel().astype(np.float64), groups[:, 4:8].ravel().astype(np.float64), groups[:, 8:12].ravel().astype(np.float64)
    r = groups[:, 12:16].ravel().astype(np.float32)
    r2 = (r * r).astype(np.float32).astype(np.float64)
    cp = np.array([cam.CameraPosition.x, cam.CameraPosition.y, cam.CameraPosition.z], np.float32).astype(np.float64)
    camx = np.array([cam.CameraX.x, cam.CameraX.y, cam.CameraX.z], np.float32).astype(np.float64)
    camy = np.array([cam.CameraY.x, cam.CameraY.y, cam.CameraY.z], np.float32).astype(np.float64)
    fc = np.array([cam.FilmCenter.x, cam.FilmCenter.y, cam.FilmCenter.z], np.float32).astype(np.float64)
    fw, fh = float(np.float32(cam.FilmW)), float(np.float32(cam.FilmH))
    TW, TH = SHAPE[P]
    tx, ty = (W + 2 * TW - 1) // (2 * TW), (H + 2 * TH - 1) // (2 * TH)
    nw = (ng + 63) // 64
    out = np.zeros(tx * ty * 4 * nw, np.uint64)
    for t in range(tx * ty):
        for w in range(4):
            x0 = (t % tx) * 2 * TW + (w & 1) * TW
            y0 = (t // tx) * 2 * TH + (w >> 1) * TH
            u = [x0 - 0.501, x0 + TW - 1 + 0.501]
            v = [y0 - 0.501, y0 + TH - 1 + 0.501]
            dirs = []
            for i in range(4):
                ka = (-1.0 + (u[i & 1] * 2.0) / W) * fw * 0.5
                kb = (-1.0 + (v[i >> 1] * 2.0) / H) * fh * 0.5
                d = (fc - cp) + ka * camx + kb * camy
                dirs.append(d / np.sqrt((d * d).sum()))
            dirs = np.array(dirs)
            s = dirs.sum(0); ax = s / np.sqrt((s * s).sum())
            ct = min(1.0, (dirs @ ax).min()); st = np.sqrt(max(0.0, 1 - ct * ct))
            cd, sd = 0.99999999995, 1e-5
            cos_t, sin_t = ct * cd - st * sd, st * cd + ct * sd
            q = np.stack([cx - cp[0], cy - cp[1], cz - cp[2]], 1)
            c2 = (q * q).sum(1)
            rr = r2 * (1 + 1e-5) + 1e-5 * c2
            with np.errstate(invalid="ignore", divide="ignore"):
                sb, cb = np.sqrt(rr / c2), np.sqrt(1 - rr / c2)
                cos_lim = cos_t * cb - sin_t * sb
                cos_phi = np.abs(q @ ax) / np.sqrt(c2)
                cand = (r2 >= 0) & ((rr >= c2) | (cos_t <= 0) | (cos_phi >= cos_lim - 1e-12))
            gm = cand.reshape(-1, 4).any(1)
            for wd in range(nw):
                bits = 0
                for gi in range(64 * wd, min(ng, 64 * wd + 64)):
                    if gm[gi]:
                        bits |= 1 << (gi - 64 * wd)
                out[(t * 4 + w) * nw + wd] = np.uint64(bits)
    return out

for n, W, H, P in [(128, 16, 8, 2), (128, 40, 32, 1), (128, 40, 32, 2), (200, 40, 32, 2), (64, 40, 32, 2)]:
    os.environ["RT_LANES_PER_PIXEL"] = str(P)
    dev = rt.Device(0)
    s = rt.scene_prefix(rt.scene_builtin(1), n)
    cam = rt.camera_setup(s, W, H)
    ref = np_masks(s, cam, W, H, P)
    seen = []
    for rep in range(8):
        dev.upload_scene(s)
        prev = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
        cur = torch.zeros(H * W, dtype=torch.int32, device="cuda")
        rays = torch.zeros(1, dtype=torch.int64, device="cuda")
        dev.trace(cam, width=W, height=H, prev_ptr=prev.data_ptr(), cur_ptr=cur.data_ptr(), rays_ptr=rays.data_ptr(),
                  frames=1, max_bounce=1, stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        m = dev.debug_masks()
        seen.append(m)
    dev.close()
    same = all(np.array_equal(seen[0], x) for x in seen)
    diff = np.flatnonzero(seen[0] != ref)
    print(f"n={n} {W}x{H} P={P}: words={len(seen[0])} deterministic={same} vs_numpy_diff={len(diff)}",
          [(int(i), hex(int(seen[0][i])), hex(int(ref[i]))) for i in diff[:4]],
          [int(np.count_nonzero(x != seen[0])) for x in seen], flush=True)
