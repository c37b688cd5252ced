"""CPU restatement (numpy, f64) of the cull pass's primary masks
(rt_kernel.hip tile_cone / cone_may_hit / wave_tile_mask), SIMD rule set,
one band: one bit per sphere pair (bit p: sphere slots 2p, 2p + 1), one u64
word per 64 pairs per wave tile, word ((tile * 4 + wave) * n_words + w),
n_words = ceil(2 groups / 64) (rt_kernel.h rtk_mask_words).  Test helper
(test_gpu_parity.py, test_cull_bound.py, test_random_scene_bounds.py)."""
import numpy as np

SHAPE = {1: (8, 8), 2: (8, 4), 4: (4, 4), 8: (4, 2), 16: (2, 2)}  # wave tile TW x TH per lanes-per-pixel


def _v3(v):
    return np.array([v.x, v.y, v.z], np.float32).astype(np.float64)


def scene_spheres(rt, scene):
    """Centres (f64), r^2 (the kernel's f32 r*r, as f64) per SIMD sphere slot."""
    _, groups, _ = rt.scene_arrays(scene)  # (ng, 16): x[4] y[4] z[4] r[4]
    c = np.stack([groups[:, 0:4].ravel(), groups[:, 4:8].ravel(), groups[:, 8:12].ravel()], 1).astype(np.float64)
    r = groups[:, 12:16].ravel().astype(np.float32)
    return c, (r * r).astype(np.float32).astype(np.float64), groups.shape[0]


def wave_tiles(W, H, P):
    TW, TH = SHAPE[P]
    tx, ty = (W + 2 * TW - 1) // (2 * TW), (H + 2 * TH - 1) // (2 * TH)
    for t in range(tx * ty):
        for w in range(4):
            yield t, w, (t % tx) * 2 * TW + (w & 1) * TW, (t // tx) * 2 * TH + (w >> 1) * TH


def np_masks(rt, scene, cam, W, H, P):
    c, r2, ng = scene_spheres(rt, scene)
    cp, camx, camy, fc = _v3(cam.CameraPosition), _v3(cam.CameraX), _v3(cam.CameraY), _v3(cam.FilmCenter)
    fw, fh = float(np.float32(cam.FilmW)), float(np.float32(cam.FilmH))
    TW, TH = SHAPE[P]
    nw = (2 * ng + 63) // 64
    tiles = list(wave_tiles(W, H, P))
    out = np.zeros(len(tiles) * nw, np.uint64)
    q = c - cp
    c2 = (q * q).sum(1)
    rr = r2 * (1 + 1e-5) + 1e-5 * c2
    for t, w, x0, y0 in tiles:
        u = [x0 - 0.501, x0 + TW - 1 + 0.501]
        v = [y0 - 0.501, y0 + TH - 1 + 0.501]
        dirs = []
        for i in range(4):
            ka = (-1.0 + (u[i & 1] * 2.0) / W) * fw * 0.5
            kb = (-1.0 + (v[i >> 1] * 2.0) / H) * fh * 0.5
            d = (fc - cp) + ka * camx + kb * camy
            dirs.append(d / np.sqrt((d * d).sum()))
        dirs = np.array(dirs)
        s = dirs.sum(0)
        ax = s / np.sqrt((s * s).sum())
        ct = min(1.0, (dirs @ ax).min())
        st = np.sqrt(max(0.0, 1 - ct * ct))
        cd, sd = 0.99999999995, 1e-5  # cos / sin of the 1e-5 rad margin
        cos_t, sin_t = ct * cd - st * sd, st * cd + ct * sd
        with np.errstate(invalid="ignore", divide="ignore"):
            sb, cb = np.sqrt(rr / c2), np.sqrt(1 - rr / c2)
            cos_lim = cos_t * cb - sin_t * sb
            cos_phi = np.abs(q @ ax) / np.sqrt(c2)
            cand = (r2 >= 0) & ((rr >= c2) | (cos_t <= 0) | (cos_phi >= cos_lim - 1e-12))
        gm = cand.reshape(-1, 2).any(1)  # per sphere pair
        for wd in range(nw):
            bits = 0
            for gi in np.flatnonzero(gm[64 * wd:64 * wd + 64]):
                bits |= 1 << int(gi)
            out[(t * 4 + w) * nw + wd] = np.uint64(bits)
    return out


def sampled_hit_pairs(rt, scene, cam, W, H, x, y, n_jitter=9):
    """Sphere pairs (slots 2p, 2p + 1) some f64 primary ray of pixel (x, y)
    passes within r of (a jitter grid over the pixel's +-0.5 px)."""
    c, r2, _ = scene_spheres(rt, scene)
    cp, camx, camy, fc = _v3(cam.CameraPosition), _v3(cam.CameraX), _v3(cam.CameraY), _v3(cam.FilmCenter)
    hits = set()
    C = c - cp
    for jx in np.linspace(-0.5, 0.5, n_jitter):
        for jy in np.linspace(-0.5, 0.5, n_jitter):
            fx = -1 + (x + jx) * 2 / W
            fy = -1 + (y + jy) * 2 / H
            d = (fc - cp) + fx * cam.FilmW * 0.5 * camx + fy * cam.FilmH * 0.5 * camy
            d /= np.linalg.norm(d)
            T = C @ d
            dist = (C * C).sum(1) - T * T
            hits.update(int(i) // 2 for i in np.flatnonzero((dist < r2) & (r2 > 0)))
    return hits
