"""Pins the CPU oracle to the reference.

1. Known-answer values recorded from the verbatim reference build (SURVEY.md
   §7 step 1 and §8(c)/(d)): PCG outputs, RandomFloat bits, the thread-0
   seed, NormalizeFast/Normalize bits, the default camera position, and the
   bounce-segment counts of two end-to-end renders.
2. Differential tests against the reference's own math layer — base.h and
   x64_math.h compiled from /root/reference by oracle/Makefile into
   oracle/_ref/librefmath.so (skipped where that build is absent).
"""
import ctypes
import struct

import numpy as np
import pytest

from conftest import host_is_intel


def bits(f: float) -> int:
    return struct.unpack("<I", struct.pack("<f", f))[0]


def test_pcg_known_answers(orc):
    s = ctypes.c_uint64(0x29D7A0A514F22432)
    got = [orc.lib().or_pcg(ctypes.byref(s)) for _ in range(4)]
    assert got == [0xb9e92c24, 0xa9cb1a46, 0xd6756c1b, 0xaa61a1f5]


def test_random_float_known_answers(orc):
    s = ctypes.c_uint64(0x29D7A0A514F22432)
    a = orc.lib().or_random_float(ctypes.byref(s), -1.0, 1.0)
    b = orc.lib().or_random_float(ctypes.byref(s), -1.0, 1.0)
    assert (bits(a), bits(b)) == (0x3ee7a4b0, 0x3ea72c68)


def test_thread0_seed(orc):
    assert orc.seed_mix(0) == 0x59daf6ff03286ede  # main.cpp:668-675 with i = 0


def test_normalize_known_answers(orc):
    v = np.array([0.3, -0.7, 0.2], np.float32)
    fast = np.zeros(3, np.float32)
    exact = np.zeros(3, np.float32)
    orc.lib().or_normalize_fast(v.ctypes.data, fast.ctypes.data)
    orc.lib().or_normalize(v.ctypes.data, exact.ctypes.data)
    assert [bits(x) for x in fast] == [0x3ec31334, 0xbf639666, 0x3e820ccd]
    assert [bits(x) for x in exact] == [0x3ec3127c, 0xbf639590, 0x3e820c52]


def test_default_camera_position(orc):
    o = orc.scene_builtin(1)
    cam = orc.camera(o, 256, 256)
    np.testing.assert_allclose(cam[:3], [-1.44249487, 0.0, -2.43292093], rtol=0, atol=5e-8)


def test_reference_ray_counts_scene1_stream_mode(orc):
    """Scene 1 verbatim (256 spheres), 256x256, 4 frames, 5 bounces, ONE thread
    drawing from the thread-0 PCG stream in tile order (the reference as
    shipped): 440334 bounce segments."""
    o = orc.scene_builtin(1)
    _, _, rays = orc.render(o, orc.camera(o, 256, 256), 256, 256, frames=4, max_bounce=5,
                            seed_mode=orc.SEED_STREAM, threads=1)
    assert rays == 440334


def test_reference_ray_counts_n64_pixel_mode(orc):
    """First 64 spheres, 256x256, 4 frames, 8 bounces, pixel seeds: 341802
    segments."""
    o = orc.scene_builtin(1).prefix(64)
    _, _, rays = orc.render(o, orc.camera(o, 256, 256), 256, 256, frames=4, max_bounce=8)
    assert rays == 341802


def test_simd_and_scalar_rules_agree_on_builtin_scenes(orc):
    """RenderTile and RenderTileScalar agree on all three scenes."""
    for idx in range(3):
        o = orc.scene_builtin(idx)
        cam = orc.camera(o, 64, 48)
        a = orc.render(o, cam, 64, 48, frames=2, max_bounce=5, simd=True)
        b = orc.render(o, cam, 64, 48, frames=2, max_bounce=5, simd=False)
        assert np.array_equal(a[1], b[1]) and a[2] == b[2], idx


def test_pixel_mode_independent_of_thread_count(orc):
    o = orc.scene_builtin(1).prefix(32)
    cam = orc.camera(o, 96, 64)
    a = orc.render(o, cam, 96, 64, frames=3, max_bounce=6, threads=1)
    b = orc.render(o, cam, 96, 64, frames=3, max_bounce=6, threads=4)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2]


def test_row_subset_matches_full_render(orc):
    o = orc.scene_builtin(1).prefix(16)
    cam = orc.camera(o, 70, 90)
    full = orc.render(o, cam, 70, 90, frames=2, max_bounce=4)
    part = orc.render(o, cam, 70, 90, frames=2, max_bounce=4, rows=(33, 61))
    assert np.array_equal(full[1].reshape(90, 70)[33:61], part[1].reshape(90, 70)[33:61])


# ------------------------------------------------- vs the reference math layer
RNG = np.random.default_rng(1234)


def test_pcg_and_random_float_vs_reference(orc, refmath):
    for seed in [0, 1, 0x29D7A0A514F22432, 0xCD46749A57ACB371, 0xFFFFFFFFFFFFFFFF]:
        for lo, hi in [(-1.0, 1.0), (-0.5, 0.5), (0.0, 1.0), (0.15, 1.0), (2.0, 8.0), (1.0, 4.0)]:
            a, b = ctypes.c_uint64(seed), ctypes.c_uint64(seed)
            for _ in range(64):
                x = orc.lib().or_random_float(ctypes.byref(a), lo, hi)
                y = refmath.ref_random_float(ctypes.byref(b), lo, hi)
                assert bits(x) == bits(y)
            assert a.value == b.value


def _vecs(n):
    v = RNG.uniform(-1, 1, size=(n, 3)).astype(np.float32)
    v[: n // 8] *= np.float32(0.004)  # around the 1e-4 masking threshold
    return np.ascontiguousarray(v)


def test_normalize_vs_reference(orc, refmath):
    for v in _vecs(20000):
        a = np.zeros(3, np.float32)
        b = np.zeros(3, np.float32)
        orc.lib().or_normalize(v.ctypes.data, a.ctypes.data)
        refmath.ref_normalize(v.ctypes.data, b.ctypes.data)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), v


@pytest.mark.skipif(not host_is_intel(), reason="the captured rsqrtss table is Intel's; this host's rsqrtss differs")
def test_normalize_fast_vs_reference_rsqrtss(orc, refmath):
    for v in _vecs(20000):
        a = np.zeros(3, np.float32)
        b = np.zeros(3, np.float32)
        orc.lib().or_normalize_fast(v.ctypes.data, a.ctypes.data)
        refmath.ref_normalize_fast(v.ctypes.data, b.ctypes.data)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), v


@pytest.mark.skipif(not host_is_intel(), reason="the captured rsqrtss table is Intel's")
def test_rsqrt_table_vs_reference_rsqrtss(orc, refmath):
    xs = np.concatenate([RNG.uniform(1e-4, 3.0, 50000), np.geomspace(1e-6, 1e6, 5000)]).astype(np.float32)
    for x in xs:
        assert bits(orc.lib().or_rsqrt(float(x))) == bits(refmath.ref_rsqrt(float(x)))


def test_cross_with_fma_contraction_vs_reference(orc, refmath):
    a, b = _vecs(5000), _vecs(5000)
    for u, w in zip(a, b):
        x = np.zeros(3, np.float32)
        y = np.zeros(3, np.float32)
        orc.lib().or_cross(u.ctypes.data, w.ctypes.data, x.ctypes.data)
        refmath.ref_cross(u.ctypes.data, w.ctypes.data, y.ctypes.data)
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32))


def test_x87_trig_and_camera_vs_reference(orc, refmath):
    """The oracle camera (main.cpp:776-838) rebuilt from the reference's own
    Cosine/Sin/Normalize/Cross: bit-identical for all three scenes' defaults
    and a sweep of orbit angles."""
    for idx in range(3):
        o = orc.scene_builtin(idx)
        for ang in [o.x_angle, 0.3, -2.0, 5.9]:
            cam = orc.camera(o, 200, 120, x_angle=ang)
            la = o.look_at[:3]
            c, s = np.float32(refmath.ref_cos(ang)), np.float32(refmath.ref_sin(ang))
            d = np.float32(o.distance)
            pos = np.array([c * d + la[0], np.float32(o.y_height) + la[1], s * d + la[2]], np.float32)

            def norm(v):
                v = np.ascontiguousarray(v, np.float32)
                r = np.zeros(3, np.float32)
                refmath.ref_normalize(v.ctypes.data, r.ctypes.data)
                return r

            def cross(p, q):
                p, q = np.ascontiguousarray(p, np.float32), np.ascontiguousarray(q, np.float32)
                r = np.zeros(3, np.float32)
                refmath.ref_cross(p.ctypes.data, q.ctypes.data, r.ctypes.data)
                return r

            z = norm(pos - la)
            x = norm(cross(np.array([0, 1, 0], np.float32), z))
            y = norm(cross(z, x))
            for got, want in [(cam[0:3], pos), (cam[4:7], z), (cam[8:11], x), (cam[12:15], y),
                              (cam[16:19], pos - z)]:
                assert np.array_equal(got.view(np.uint32), want.astype(np.float32).view(np.uint32)), (idx, ang)


def test_group_intersection_arithmetic_vs_reference(orc, refmath):
    """The lane-4 sphere-group arithmetic of main.cpp:400-417 evaluated with the
    reference's f32x4/v3x4 operators vs the oracle's SSE restatement."""
    o = orc.scene_builtin(1)
    for _ in range(4000):
        org = RNG.uniform(-4, 4, 3).astype(np.float32)
        d = RNG.uniform(-1, 1, 3).astype(np.float32)
        d /= np.float32(np.linalg.norm(d))
        g = o.groups[RNG.integers(0, o.groups.shape[0])].copy()
        a_d, a_t, b_d, b_t = (np.zeros(4, np.float32) for _ in range(4))
        orc.lib().or_group_test(org.ctypes.data, d.ctypes.data, g.ctypes.data, a_d.ctypes.data, a_t.ctypes.data)
        refmath.ref_group_test(org.ctypes.data, d.ctypes.data, g[0:4].ctypes.data, g[4:8].ctypes.data,
                               g[8:12].ctypes.data, g[12:16].ctypes.data, b_d.ctypes.data, b_t.ctypes.data)
        assert np.array_equal(a_d.view(np.uint32), b_d.view(np.uint32))
        assert np.array_equal(a_t.view(np.uint32), b_t.view(np.uint32))


def test_horizontal_min_vs_reference(orc, refmath):
    for _ in range(2000):
        v = RNG.choice(np.array([1e30, 0.5, 0.25, 2.0, 1e-3], np.float32), 4).astype(np.float32)
        lane = ctypes.c_uint32()
        m = orc.lib().or_horizontal_min(v.ctypes.data, ctypes.byref(lane))
        assert bits(m) == bits(refmath.ref_horizontal_min(v.ctypes.data))
        assert lane.value == int(np.flatnonzero(v == np.float32(m))[0])
