"""CPU property test of the secondary-ray prefilter.

The kernel skips a sphere for a secondary ray when the FMA estimate
e = |C|^2 - (C.D)^2 satisfies e >= r2p, where r2p comes from the host
(rt_scene_prefilter, the same code rt_scene_upload runs).  Skipping is only
allowed if the reference-rounded exact test (main.cpp:401-409, restated op
for op in numpy f32) rejects the sphere.  This checks that on rays the bound
is meant for -- origins on scene spheres, |D|^2 within 2^-16 of 1 -- with
random and near-tangent directions, under both rule sets.
"""
import numpy as np
import pytest

F = np.float32


def fma(a, b, c):
    # exact f32 product in f64, one rounding of the sum to f64, one to f32:
    # within 1 ulp of a true fma -- far inside the bound's slack
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(F)


def exact_dist(cx, cy, cz, dx, dy, dz):
    """main.cpp:401-407 with every f32 op rounded separately."""
    T = (cx * dx + cy * dy) + cz * dz
    qx, qy, qz = cx - dx * T, cy - dy * T, cz - dz * T
    return (qx * qx + qy * qy) + qz * qz


def prefilter(cx, cy, cz, dx, dy, dz, with_t=False, with_cc=False):
    """rt_kernel.hip pair_prefilter, lane by lane: e (and its FMA T, and cc = |C|^2)."""
    cc = fma(cx, cx, fma(cy, cy, cz * cz))
    T = fma(cz, dz, fma(cy, dy, cx * dx))
    e = fma(-T, T, cc)
    if with_cc:
        return e, T, cc
    return (e, T) if with_t else e


PF_REL = F(2.0 ** -15)  # rt_kernel.hip kPfRel


CL_REL = F(9.2e-4)            # rt_kernel.hip kClRel
BEHIND_REL = F(4.5 * 2.0 ** -24)  # rt_kernel.hip kBehindRel
SLAB_REL = F(2.0 ** -9)       # rt_kernel.h kSlabRel


def slab_skip(tc, cc, oy, dy, srho, ymid, yhalf):
    """rt_kernel.hip clustered_groups, per-lane tables: the height-slab test skips a
    cluster when |RN(fma(D.y, T, O.y)) - ymid| > RN(fma(|D.y|, srho, yhalf + E)),
    E = RN(fma(cc, kSlabRel, RN(fma(|O.y|, 2^-21, kSlabRel))))."""
    with np.errstate(invalid="ignore", over="ignore"):
        e0 = fma(np.abs(oy), np.broadcast_to(F(2.0 ** -21), oy.shape), np.broadcast_to(SLAB_REL, oy.shape))
        E = fma(cc, np.broadcast_to(SLAB_REL, cc.shape), e0)
        c = fma(dy, tc, oy)
        d = (c - F(ymid)).astype(F)
        thr = fma(np.abs(dy), np.broadcast_to(F(srho), dy.shape), (F(yhalf) + E).astype(F))
        return np.abs(d) > thr


def cluster_threshold(t, cc, relative):
    """Cluster skip threshold: the stored rc2p, or RN(cc kClRel + R_c) per lane."""
    if not relative:
        return t
    with np.errstate(invalid="ignore"):
        return fma(cc, np.broadcast_to(CL_REL, cc.shape), np.broadcast_to(F(t), cc.shape))


def behind_threshold(b, cc, relative):
    """Behind threshold: the stored b, or RN(b - cc kBehindRel) per lane."""
    if not relative:
        return b
    with np.errstate(invalid="ignore"):
        return fma(cc, np.broadcast_to(-BEHIND_REL, cc.shape), np.broadcast_to(b, cc.shape))


def threshold(r2p, cc, relative):
    """The kernel's skip threshold: r2p (scene-wide), or RN(cc 2^-15 + r^2) per lane."""
    if not relative:
        return r2p
    with np.errstate(invalid="ignore"):
        return fma(cc, np.broadcast_to(PF_REL, cc.shape), np.broadcast_to(r2p, cc.shape))


def could_accept(cx, cy, cz, dx, dy, dz, r2, simd):
    """main.cpp:401-429 per sphere with every f32 op rounded separately: the
    exact test passes AND the candidate's it clears eps (the current minimum
    is ignored, so this over-approximates what a lane can accept)."""
    T = (cx * dx + cy * dy) + cz * dz
    dist = exact_dist(cx, cy, cz, dx, dy, dz)
    hit = (dist < r2) if simd else ~(dist > r2)
    with np.errstate(invalid="ignore"):
        X = np.sqrt((r2 - dist).astype(F))
    it = T - X
    it = np.where(it < F(1e-4), T + X, it)
    ok = (it > F(1e-4)) if simd else ~(it < F(1e-4))
    return hit & ok


def unit(v):
    v = v.astype(F)
    n = np.sqrt((v.astype(np.float64) ** 2).sum(-1, keepdims=True))
    return (v / n).astype(F)


def rays(rng, centres, radii, n):
    """Origins on random scene spheres; half random directions, half aimed
    at a random sphere's silhouette (d ~ r^2: the bound's tight case);
    |D|^2 pushed up to 2^-17 away from 1."""
    i = rng.integers(0, len(centres), n)
    u = unit(rng.normal(size=(n, 3)))
    o = (centres[i] + radii[i, None] * u).astype(F)
    d = unit(rng.normal(size=(n, 3)))
    half = n // 2
    j = rng.integers(0, len(centres), half)
    to = (centres[j] - o[:half]).astype(np.float64)
    w = np.cross(to, rng.normal(size=(half, 3)))
    w /= np.linalg.norm(w, axis=1, keepdims=True)
    tangent = to + w * radii[j, None] * (1.0 + rng.uniform(-2e-6, 2e-6, (half, 1)))
    d[:half] = unit(tangent)
    d = (d * F(1.0) + d * F(rng.uniform(-2**-18, 2**-18, (n, 1)))).astype(F)
    u2 = (d.astype(np.float64) ** 2).sum(1)
    assert np.all(np.abs(1.0 - u2) <= 2**-16)
    return o, d


def slot_spheres(rt, scene, simd):
    """Centres and radii per sphere slot 4*group+lane of one rule set."""
    sp, groups, _ = rt.scene_arrays(scene)
    if simd:
        cx_, cy_, cz_ = groups[:, 0:4].ravel(), groups[:, 4:8].ravel(), groups[:, 8:12].ravel()
        radius = groups[:, 12:16].ravel()
    else:
        pad = (-len(sp)) % 4
        cx_, cy_, cz_ = (np.concatenate([sp[:, k], np.zeros(pad, F)]) for k in range(3))
        radius = np.concatenate([sp[:, 4], np.zeros(pad, F)])
    return np.stack([cx_, cy_, cz_], 1).astype(F), radius


@pytest.mark.parametrize("idx,n_spheres", [(1, 64), (1, 256), (0, None), (2, None)])
@pytest.mark.parametrize("simd", [True, False])
def test_prefilter_never_skips_an_exact_hit(rt, idx, n_spheres, simd):
    scene = rt.scene_builtin(idx)
    if n_spheres:
        scene = rt.scene_prefix(scene, n_spheres)
    check_prefilter(rt, scene, simd, 7 + idx)


def check_prefilter(rt, scene, simd, seed, n_rays=4000, require_hits=True):
    """No ray the bound is meant for has e >= r2p on a sphere its exact test
    accepts; where the prefilter is on by default it must actually cull."""
    r2, r2p, flags = rt.scene_prefilter(scene, simd)
    centres, radius = slot_spheres(rt, scene, simd)
    assert np.array_equal(r2[: len(radius)][r2 >= 0], (radius * radius)[r2 >= 0])
    live = r2 > 0 if simd else r2 >= 0
    rng = np.random.default_rng(seed)
    o, d = rays(rng, centres[live], np.abs(radius[live]).astype(F), n_rays)
    cx = centres[None, :, 0] - o[:, None, 0]
    cy = centres[None, :, 1] - o[:, None, 1]
    cz = centres[None, :, 2] - o[:, None, 2]
    dx, dy, dz = d[:, None, 0], d[:, None, 1], d[:, None, 2]
    dist = exact_dist(cx, cy, cz, dx, dy, dz)
    e, _, cc = prefilter(cx, cy, cz, dx, dy, dz, with_cc=True)
    hit = (dist < r2) if simd else ~(dist > r2)
    hit &= live[None, :]
    relative = bool(flags & 4)
    skipped = ~(e < threshold(r2p[None, :], cc, relative))
    assert not np.any(hit & skipped), "prefilter skipped a sphere the exact test accepts"
    if require_hits:
        assert hit.sum() > 0
    if relative and require_hits:  # the per-lane threshold must cull too
        assert (~skipped & live[None, :]).sum() < 1.5 * hit.sum() + 0.2 * live.sum() * len(o)
    return bool(flags & 5), int((skipped & live[None, :]).sum())

    if flags & 1 and require_hits:  # where it is enabled, the prefilter must actually cull
        assert (~skipped).sum() < 1.5 * hit.sum() + 0.05 * hit.size


def test_prefilter_rows_of_padding_are_never_flagged(rt):
    s = rt.scene_prefix(rt.scene_builtin(1), 13)  # scalar packing pads 3 lanes
    r2, r2p, _ = rt.scene_prefilter(s, simd=False)
    assert len(r2) == 16 and np.all(np.isneginf(r2p[13:])) and np.all(np.isfinite(r2p[:13]))
    assert np.all(r2p[:13] > r2[:13])


def test_short_sqrt_flag_follows_the_radius_range(rt):
    base = rt.scene_prefix(rt.scene_builtin(1), 16)
    assert rt.scene_prefilter(base, True)[2] & 2 and rt.scene_prefilter(base, False)[2] & 2
    sp, _, _ = rt.scene_arrays(base)
    sp = sp.copy()
    sp[3, 4] = np.float32(2e-6)  # r^2 = 4e-12 < 2^-36: outside the verified range
    tiny = rt.scene_from_spheres(sp)
    assert not rt.scene_prefilter(tiny, True)[2] & 2 and not rt.scene_prefilter(tiny, False)[2] & 2


@pytest.mark.parametrize("idx,n_spheres", [(1, 64), (1, 37), (1, 16), (1, 100), (1, 256), (0, None), (2, None)])
@pytest.mark.parametrize("simd", [True, False])
def test_cluster_prefilter_never_skips_an_exact_hit(rt, idx, n_spheres, simd):
    """The clustered loop (rt_kernel.hip clustered_groups) skips every member
    of a cluster when e_c >= rc2p_c on all lanes; the members of a tested
    cluster are flagged by their own r2p.  Every exact hit must survive both
    levels, and every hittable sphere must be a member of exactly one cluster."""
    scene = rt.scene_builtin(idx)
    if n_spheres:
        scene = rt.scene_prefix(scene, n_spheres)
    if rt.scene_clusters(scene, simd)[1] == 0:
        pytest.skip("scene uses the per-group prefilter loop")
    check_clusters(rt, scene, simd, 11 + idx, require_culls=True)


def check_clusters(rt, scene, simd, seed, require_culls=False, n_rays=4000):
    """Decodes the cluster table; no skipped cluster (near-line or behind
    rule) and no skipped member holds a sphere a lane can accept.  Returns
    (rays x clusters skipped, of them by the behind rule)."""
    tab, ncp = rt.scene_clusters(scene, simd)
    r2, r2p, flags = rt.scene_prefilter(scene, simd)
    if ncp == 0:
        return 0, 0
    relative = bool(flags & 4)  # per-lane thresholds (rt_kernel.hip kClRel / kPfRel / kBehindRel)
    centres, radius = slot_spheres(rt, scene, simd)
    live = np.isfinite(r2p)
    # decode the table: clusters -> member spheres (by centre and r2p) and pair indices;
    # two-level tables: top entries -> sub-cluster entries -> member entries
    levels, n_sub = rt.scene_cluster_layout(scene, simd)
    groups = scene.SIMDSpheres.Count if simd else (scene.ScalarSpheres.Count + 3) // 4
    assert levels == (1 if groups <= 32 else 2), "two levels exactly for tables of two or more mask words"
    members = []  # (qx, qy, qz, t, spheres under the cluster, b, slab), both levels
    used = set()
    beta_of = {}  # per-sphere behind threshold (member rows)

    def decode_members(first, count):
        ms = []
        for m in range(first, first + count):
            e = tab[m]
            # member k's pair q: bit q & 63 in the row of mask word q >> 6 (row 2, then rows 4 ..)
            rows = [e[2]] + [e[3 + w] for w in range(1, max(1, len(e) - 3))]
            bits = [[int(r.view(np.uint32)[2 * k]) | (int(r.view(np.uint32)[2 * k + 1]) << 32) for r in rows]
                    for k in range(2)]
            pair = [0, 0]
            for w in range(2):
                set_words = [i for i, b in enumerate(bits[w]) if b]
                if np.isneginf(e[1][2 + w]):
                    assert not set_words
                    continue
                assert len(set_words) == 1, "one mask word per member"
                b = bits[w][set_words[0]]
                assert b & (b - 1) == 0, "one pair bit per member"
                pair[w] = b.bit_length() - 1 + 64 * set_words[0]
                x, y, z, t = e[0][w], e[0][2 + w], e[1][w], e[1][2 + w]
                s = np.flatnonzero((centres[:, 0] == x) & (centres[:, 1] == y) & (centres[:, 2] == z) &
                                   (r2p == t) & live)
                assert len(s) >= 1
                s = [k for k in s if pair[w] == int(k) >> 1]
                assert len(s) >= 1, "member pair index is not its sphere's pair in group order"
                s = [k for k in s if k not in used] or s  # two spheres of one pair with equal rows
                used.add(s[0])
                ms.append(s[0])
                beta_of[s[0]] = np.float32(e[3][w])
        return ms

    def cluster(q, h, ms):
        slab = (np.float32(q[3][2 + h]), np.float32(q[4][h]), np.float32(q[4][2 + h])) if relative else None
        return (np.float32(q[0][h]), np.float32(q[0][2 + h]), np.float32(q[1][h]), np.float32(q[1][2 + h]), ms,
                np.float32(q[3][h]), slab)

    leaves = []
    sub_seen = set()
    for c in range(ncp):
        q = tab[c]
        u = q[2].view(np.uint32)
        for h in range(2):
            first, count = int(u[2 * h]), int(u[2 * h + 1])
            if levels == 2:
                under = []
                for e in range(first, first + count):
                    assert ncp <= e < ncp + n_sub and e not in sub_seen, "sub-cluster entry outside its range"
                    sub_seen.add(e)
                    qs, us = tab[e], tab[e][2].view(np.uint32)
                    for h2 in range(2):
                        ms = decode_members(int(us[2 * h2]), int(us[2 * h2 + 1]))
                        members.append(cluster(qs, h2, ms))
                        leaves += ms
                        under += ms
                members.append(cluster(q, h, under))
            else:
                ms = decode_members(first, count)
                members.append(cluster(q, h, ms))
                leaves += ms
    if levels == 2:
        assert len(sub_seen) == n_sub
    covered = sorted(leaves)
    assert covered == sorted(np.flatnonzero(live)), "every hittable sphere is in exactly one cluster"
    rng = np.random.default_rng(seed)
    o, d = rays(rng, centres[live], np.abs(radius[live]).astype(F), n_rays)
    dx, dy, dz = d[:, None, 0], d[:, None, 1], d[:, None, 2]
    cx = centres[None, :, 0] - o[:, None, 0]
    cy = centres[None, :, 1] - o[:, None, 1]
    cz = centres[None, :, 2] - o[:, None, 2]
    accept = could_accept(cx, cy, cz, dx, dy, dz, r2[None, :], simd) & live[None, :]
    if require_culls:
        assert accept.sum() > 0
    # sphere level: near-line estimate or wholly behind the origin (member rows)
    e_s, t_s, cc_s = prefilter(cx, cy, cz, dx, dy, dz, with_cc=True)
    beta = np.array([beta_of.get(k, -np.inf) for k in range(len(r2))], F)
    thr_s = threshold(r2p[None, :], cc_s, relative)
    beta_s = behind_threshold(beta[None, :], cc_s, relative)
    skip_s = ~(e_s < thr_s) | (t_s < beta_s)
    assert not np.any(accept & skip_s), "the member test skipped a sphere a lane can accept"
    if require_culls:
        assert np.any((t_s < beta_s) & (e_s < thr_s) & live[None, :]), "the behind rule culls nothing"
    skipped_any = behind_any = slab_any = 0
    for qx, qy, qz, t, ms, bc, slab in members:
        if np.isneginf(t):
            continue
        ex, tx, cq = prefilter((qx - o[:, 0])[:, None], (qy - o[:, 1])[:, None], (qz - o[:, 2])[:, None],
                               d[:, 0:1], d[:, 1:2], d[:, 2:3], with_cc=True)
        tc = cluster_threshold(t, cq[:, 0], relative)
        behind = tx[:, 0] < behind_threshold(bc, cq[:, 0], relative)
        skip = ~(ex[:, 0] < tc) | behind
        if slab is not None:
            sl = slab_skip(tx[:, 0], cq[:, 0], o[:, 1], d[:, 1], *slab)
            slab_any += int((sl & ~skip).sum())
            skip = skip | sl
        skipped_any += int(skip.sum())
        behind_any += int((behind & (ex[:, 0] < tc)).sum())
        assert not np.any(accept[skip][:, ms]), "a skipped cluster holds a sphere a lane can accept"
    if require_culls:
        assert skipped_any > 0 and behind_any > 0  # both cluster rules cull
        if relative:
            assert slab_any > 0, "the height-slab rule culls nothing"
    return skipped_any, behind_any
