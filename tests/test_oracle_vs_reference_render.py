"""Pins the oracle's colour path and whole framebuffers to the reference's own
compiled code.

`make -C oracle ref` compiles /root/reference/main.cpp lines 7-640 (scene
generators, Reflectance, LinearToSRGB, ColorFromV4, RenderTile,
RenderTileScalar), extracted by line range at build time, against the
reference's base.h + x64_math.h into oracle/_ref/librefmath.so
(oracle/ref_harness.cpp).  These tests compare the oracle (oracle/rt_oracle.c,
the checker the GPU parity suite uses) with it bit for bit:

- Reflectance (main.cpp:292-300) over random (cos, eta) with eta < 1 and > 1
  and cos near 0 and 1;
- LinearToSRGB + ColorFromV4 (main.cpp:312-346) exhaustively over every f32
  in [-1, 2] plus NaN and +-inf;
- the running-mean blend and store (main.cpp:484-492, compiled verbatim)
  at PreviousRayCount 0, 1, 3, 2^24-1, 2^24+1 and 4294967000;
- the emission / attenuation update (main.cpp:446-447, compiled verbatim);
- the three built-in scenes as the reference's own generators build them
  (main.cpp:96-268);
- whole framebuffers: the reference's RenderTile and RenderTileScalar run
  over every tile on one worker thread (its PCG stream in tile order,
  MaxRayBounce 5 as in main.cpp:387), against the oracle's stream seed mode.
  The accumulation (v4 f32), the RGBA8 image, the ray count and the final
  PCG state must all be identical.

RenderTile calls three lane helpers the reference's x64 layer declares but
never defines (base.h:503-504,546); the harness defines them with the WASM
layer's semantics (wasm_math.h:286-323).  RenderTileScalar needs none.

The diffuse bounce uses rsqrtss (NormalizeFast, x64_math.h:246-257), which the
oracle reproduces with a table captured from an Intel CPU, so the render tests
need an Intel host (this container).  All tests skip where the reference is
absent (the GPU box).
"""
import ctypes

import numpy as np
import pytest

from conftest import host_is_intel

RNG = np.random.default_rng(20261017)
F = np.float32

intel_only = pytest.mark.skipif(not host_is_intel(), reason="the oracle's rsqrtss table is Intel's")


def _u(a):
    return np.ascontiguousarray(a).view(np.uint32)


# ------------------------------------------------------------- Reflectance
def test_reflectance_vs_reference(orc, refmath):
    L = orc.lib()
    cos = np.concatenate([RNG.uniform(0, 1, 40000), RNG.uniform(0, 1e-3, 5000), 1 - RNG.uniform(0, 1e-3, 5000),
                          [0.0, 1.0, 1e-30, 0.5, -0.25, 1.5]]).astype(F)
    eta = np.concatenate([RNG.uniform(0.3, 1.0, 20000), RNG.uniform(1.0, 3.0, 20000), RNG.choice(
        [1 / 1.5, 1.5, 1.0, 0.999999, 1.000001], 10000), [1.5, 1 / 1.5, 1.0, 2.0, 0.5, 1.5]]).astype(F)
    for c, e in zip(cos, eta):
        a = F(L.or_reflectance(float(c), float(e)))
        b = F(refmath.ref_reflectance(float(c), float(e)))
        assert a.view(np.uint32) == b.view(np.uint32), (c, e, a, b)


# --------------------------------------------- LinearToSRGB + ColorFromV4
def _bit_ranges():
    """Every f32 bit pattern in [-1, 2] (both zeros), then NaNs and infinities."""
    yield np.uint32(0x00000000), np.uint32(0x40000000)  # +0 .. 2.0
    yield np.uint32(0x80000000), np.uint32(0xBF800000)  # -0 .. -1.0


def test_srgb_and_rgba8_exhaustive_vs_reference(orc, refmath):
    """Every f32 in [-1, 2] (2,139,095,042 values) plus NaN/inf edge values:
    LinearToSRGB's f32 bits and the RGBA8 of ColorFromV4(LinearToSRGB(v)),
    oracle against the reference's compiled main.cpp:312-346."""
    L = orc.lib()
    chunk = 3 << 22
    total = 0
    for lo, hi in _bit_ranges():
        start = int(lo)
        while start <= int(hi):
            n = min(chunk, int(hi) - start + 1)
            x = np.arange(start, start + n, dtype=np.uint32).view(F)
            _check_srgb(L, refmath, x)
            total += n
            start += n
    assert total == 0x40000001 + 0x3F800001
    edge = np.array([np.nan, -np.nan, np.inf, -np.inf, 3e38, -3e38, 0.0031308, np.nextafter(F(0.0031308), F(0)),
                     1.0, np.nextafter(F(1), F(2)), 254.5 / 255, 255.0 / 255],
                    F)
    edge = np.concatenate([edge, np.array([0x7FC00001, 0xFF800001, 0x7F800001], np.uint32).view(F)])
    _check_srgb(L, refmath, edge)


def _check_srgb(L, refmath, x):
    x = np.ascontiguousarray(x, F)
    n = x.size
    a = np.empty(n, F)
    b = np.empty(n, F)
    L.or_srgb_n(x.ctypes.data, a.ctypes.data, n)
    refmath.ref_linear_to_srgb_n(x.ctypes.data, b.ctypes.data, n)
    bad = np.flatnonzero(a.view(np.uint32) != b.view(np.uint32))
    assert bad.size == 0, ("LinearToSRGB", x[bad[:4]], a[bad[:4]], b[bad[:4]])
    # three values per pixel (x, y, z); w = 1 as the blend writes it
    m = (n + 2) // 3
    v = np.ones((m, 4), F)
    flat = np.zeros(m * 3, F)
    flat[:n] = x
    v[:, :3] = flat.reshape(m, 3)
    ra = np.empty(m, np.uint32)
    rb = np.empty(m, np.uint32)
    L.or_encode_rgba8(v.ctypes.data, ra.ctypes.data, m, 0)
    refmath.ref_encode_rgba8(v.ctypes.data, rb.ctypes.data, m)
    bad = np.flatnonzero(ra != rb)
    assert bad.size == 0, ("RGBA8", v[bad[:4]], ra[bad[:4]], rb[bad[:4]])


def test_color_from_v4_vs_reference(orc, refmath):
    """ColorFromV4 alone (main.cpp:340-346): saturate, x255, truncate to u8."""
    v = np.concatenate([RNG.uniform(-0.5, 1.5, (20000, 4)), np.array([[np.nan, np.inf, -np.inf, 1.0]])]).astype(F)
    for row in v:
        row = np.ascontiguousarray(row)
        want = refmath.ref_color_from_v4(row.ctypes.data)
        got = 0
        for k in range(3):  # the oracle's to_u8 through its encode of a value already in sRGB space is not
            s = F(row[k])    # exposed alone, so restate ColorFromV4's byte the reference's way here
            s = F(0) if s < 0 else (F(1) if s > 1 else s)
            s = F(s * F(255))
            got |= (0 if np.isnan(s) else int(s) & 0xFF) << (8 * k)
        got |= 255 << 24
        assert got == want, row


# ----------------------------------------------------------- blend / store
@pytest.mark.parametrize("prev_count", [0, 1, 3, (1 << 24) - 1, (1 << 24) + 1, 4294967000])
def test_blend_store_vs_reference(orc, refmath, prev_count):
    """main.cpp:484-492 compiled verbatim: FinalColor = Out*(1/n) + Prev*(p/n),
    w = 1, then ColorFromV4(LinearToSRGB(FinalColor))."""
    L = orc.lib()
    out = np.concatenate([RNG.uniform(0, 1, (3000, 3)), RNG.uniform(0, 40, (1000, 3)),
                          RNG.choice([0.0, 1.0, 8.0, 1e-30, 3e38], (200, 3))]).astype(F)
    prev = np.concatenate([RNG.uniform(0, 1, (3000, 4)), RNG.uniform(0, 40, (1000, 4)),
                           RNG.choice([0.0, 1.0, 0.5, 1e-30], (200, 4))]).astype(F)
    for o, p in zip(out, prev):
        o = np.ascontiguousarray(o)
        pa, pb = p.copy(), p.copy()
        xa, xb = np.zeros(1, np.uint32), np.zeros(1, np.uint32)
        L.or_blend_store(prev_count, o.ctypes.data, pa.ctypes.data, xa.ctypes.data)
        refmath.ref_blend_store(prev_count, o.ctypes.data, pb.ctypes.data, xb.ctypes.data)
        assert np.array_equal(_u(pa), _u(pb)) and xa[0] == xb[0], (prev_count, o, p, pa, pb)


def test_emit_attenuate_vs_reference(orc, refmath):
    """main.cpp:446-447 compiled verbatim: Out += Emissive*Att; Att *= Color."""
    L = orc.lib()
    for _ in range(20000):
        e, c, att, out = (RNG.uniform(0, 8, 3).astype(F) for _ in range(4))
        if RNG.random() < 0.3:
            e[:] = 0
        a1, o1, a2, o2 = att.copy(), out.copy(), att.copy(), out.copy()
        L.or_emit_attenuate(e.ctypes.data, c.ctypes.data, a1.ctypes.data, o1.ctypes.data)
        refmath.ref_emit_attenuate(e.ctypes.data, c.ctypes.data, a2.ctypes.data, o2.ctypes.data)
        assert np.array_equal(_u(a1), _u(a2)) and np.array_equal(_u(o1), _u(o2))


# ---------------------------------------------------------- built-in scenes
def _ref_scene(refmath, index):
    sp = np.zeros((512, 20), F)
    gr = np.zeros((128, 16), F)
    ma = np.zeros((512, 12), F)
    info = np.zeros(10, F)
    assert refmath.ref_scene_builtin(index, sp.ctypes.data, 512, gr.ctypes.data, 128, ma.ctypes.data, 512,
                                     info.ctypes.data) == 0
    n, g, m = int(info[7]), int(info[8]), int(info[9])
    return sp[:n], gr[:g], ma[:m], info


SPHERE_FIELDS = [0, 1, 2, 4, 8, 9, 10, 12, 13, 14, 16, 17]  # Position.xyz, Radius, Color, Emissive, Specular, IOR
MATERIAL_FIELDS = [0, 1, 2, 4, 5, 6, 8, 9]


@pytest.mark.parametrize("index", [0, 1, 2])
def test_builtin_scenes_vs_reference_generators(rt, orc, refmath, index):
    """The reference's InitRGBSphereScene / InitRandomizedSphereScene /
    InitRTWeekendSphereScene (main.cpp:96-268) against the oracle's scene and
    the product library's (rt_scene_builtin): every sphere, group lane and
    material field bit for bit, plus look-at, sky flag and default camera."""
    sp, gr, ma, info = _ref_scene(refmath, index)
    o = orc.scene_builtin(index)
    lsp, lgr, lma = rt.scene_arrays(rt.scene_builtin(index))
    for name, s, g, m in (("oracle", o.spheres, o.groups, o.materials), ("library", lsp, lgr, lma)):
        s, g, m = np.asarray(s, F).reshape(-1, 20), np.asarray(g, F).reshape(-1, 16), np.asarray(m, F).reshape(-1, 12)
        assert s.shape == sp.shape and g.shape == gr.shape, (name, s.shape, sp.shape, g.shape, gr.shape)
        assert np.array_equal(_u(s[:, SPHERE_FIELDS]), _u(sp[:, SPHERE_FIELDS])), name
        assert np.array_equal(_u(g), _u(gr)), name
        # the reference's Materials array has Count = N + 1; its last entry is never written
        assert np.array_equal(_u(m[:len(sp), MATERIAL_FIELDS]), _u(ma[:len(sp), MATERIAL_FIELDS])), name
    assert np.array_equal(_u(o.look_at[:3]), _u(info[:3]))
    assert o.use_sky == bool(info[3])
    assert (F(o.distance), F(o.x_angle), F(o.y_height)) == (info[4], info[5], info[6])


# ------------------------------------------------------ whole framebuffers
def _ref_render(refmath, o, cam, w, h, frames, simd, seed, prev_count=0, prev=None):
    prev = np.zeros((w * h, 4), F) if prev is None else prev.copy()
    cur = np.zeros(w * h, np.uint32)
    st = np.array([seed], np.uint64)
    rays = np.zeros(1, np.uint64)
    refmath.ref_render(o.spheres.ctypes.data, len(o.spheres), o.groups.ctypes.data, len(o.groups),
                       o.materials.ctypes.data, len(o.materials), int(o.use_sky), cam.ctypes.data, w, h, prev_count,
                       frames, int(simd), st.ctypes.data, prev.ctypes.data, cur.ctypes.data, rays.ctypes.data)
    return prev, cur, int(rays[0]), int(st[0])


def _compare(orc, refmath, o, w, h, frames, simd, seed=None, prev_count=0, prev=None, cam=None):
    cam = orc.camera(o, w, h) if cam is None else cam
    seed = orc.seed_mix(0) if seed is None else seed
    rp, rc, rr, rs = _ref_render(refmath, o, cam, w, h, frames, simd, seed, prev_count, prev)
    st = np.array([seed], np.uint64)
    op, oc, orr = orc.render(o, cam, w, h, prev_count=prev_count, frames=frames, max_bounce=5, simd=simd,
                             seed_mode=orc.SEED_STREAM, threads=1, stream_states=st,
                             prev=None if prev is None else prev.copy())
    assert rr == orr, (rr, orr)
    assert rs == int(st[0])
    bad = np.flatnonzero(np.any(_u(op) != _u(rp), axis=1))
    assert bad.size == 0, ("v4", bad[:5], op[bad[:3]], rp[bad[:3]])
    assert np.array_equal(oc, rc)
    return rp, rc, rr


@intel_only
@pytest.mark.parametrize("simd", [True, False], ids=["RenderTile", "RenderTileScalar"])
@pytest.mark.parametrize("index", [0, 1, 2], ids=["rgb_glass", "floating", "rtweekend"])
def test_builtin_scene_framebuffers_vs_reference(orc, refmath, index, simd):
    o = orc.scene_builtin(index)
    _, cur, rays = _compare(orc, refmath, o, 96, 64, 3, simd)
    assert rays > 96 * 64 * 3
    assert np.count_nonzero(cur != 0xFF000000) > cur.size // 25  # colour-bearing, not a black frame


@intel_only
@pytest.mark.parametrize("simd", [True, False], ids=["RenderTile", "RenderTileScalar"])
def test_survey_probe_frame_vs_reference(orc, refmath, simd):
    """SURVEY §8c's probe: scene 1 verbatim, 256x256, 4 frames, thread-0 stream:
    440,334 segments, and now the framebuffer itself."""
    o = orc.scene_builtin(1)
    _, cur, rays = _compare(orc, refmath, o, 256, 256, 4, simd)
    assert rays == 440334
    assert np.count_nonzero(cur != 0xFF000000) > 2000


@intel_only
@pytest.mark.parametrize("simd", [True, False], ids=["RenderTile", "RenderTileScalar"])
def test_synthetic_prefix_scenes_and_continuation_vs_reference(orc, refmath, simd):
    """The BASELINE scene family (first N spheres of Floating Spheres, N = 4, 13,
    64) on ragged sizes, and a continued accumulation from a random non-zero
    running mean at PreviousRayCount 7 (the blend's prev term)."""
    base = orc.scene_builtin(1)
    for n, (w, h) in ((4, (37, 29)), (13, (70, 33)), (64, (128, 72))):
        _compare(orc, refmath, base.prefix(n), w, h, 2, simd, seed=orc.seed_mix(n))
    o = base.prefix(64)
    prev = RNG.uniform(0, 1.5, (64 * 48, 4)).astype(F)
    _compare(orc, refmath, o, 64, 48, 2, simd, prev_count=7, prev=prev)


@intel_only
def test_moved_camera_and_inside_sphere_vs_reference(orc, refmath):
    """Cameras the defaults never take: an orbit angle and height off the
    default, and one inside the RGB-glass sphere (sticky inside flag)."""
    o = orc.scene_builtin(0)
    for simd in (True, False):
        cam = orc.camera(o, 64, 40, distance=0.5, x_angle=2.2, y_height=0.3)
        _compare(orc, refmath, o, 64, 40, 2, simd, cam=cam)
        cam = orc.camera(o, 48, 48, distance=0.01, x_angle=0.4, y_height=0.0)
        _compare(orc, refmath, o, 48, 48, 2, simd, cam=cam)


# --------------------------------- committed vectors from the reference itself
GOLDEN = __import__("pathlib").Path(__file__).with_name("golden") / "reference_frames.json"


def _golden_cases():
    import json
    return list(json.loads(GOLDEN.read_text())["cases"].items())


@intel_only
@pytest.mark.parametrize("name,case", _golden_cases(), ids=[n for n, _ in _golden_cases()])
def test_oracle_matches_reference_golden_frames(orc, name, case):
    """tests/golden/reference_frames.json was written by
    tests/golden/make_reference_golden.py from the reference's own compiled
    RenderTile/RenderTileScalar; this needs no /root/reference."""
    o = orc.scene_builtin(case["scene"])
    if case["prefix"]:
        o = o.prefix(case["prefix"])
    w, h = case["width"], case["height"]
    st = np.array([int(case["seed"], 16)], np.uint64)
    prev, cur, rays = orc.render(o, orc.camera(o, w, h), w, h, prev_count=case["prev_count"], frames=case["frames"],
                                 max_bounce=5, simd=case["simd"], seed_mode=orc.SEED_STREAM, threads=1,
                                 stream_states=st)
    assert rays == case["rays"]
    assert f"{int(st[0]):016x}" == case["final_state"]
    assert f"{orc.fnv1a64(cur):016x}" == case["rgba8_fnv1a64"]
    assert f"{orc.fnv1a64(prev):016x}" == case["v4_fnv1a64"]


# -------------------- the parity mode itself: SURVEY 8c's patched reference
# librefpix.so is main.cpp:7-640 with SURVEY 8c's two textual patches applied to
# a temporary copy by oracle/Makefile: (i) MaxRayBounce reads a harness global
# (main.cpp:387,536), (ii) the pixel loops re-seed the thread's PCG with
# OnInit's mixer (main.cpp:668-675) at i = (PreviousRayCount*H + y)*W + x
# (after main.cpp:373,522).  That is the `pixel` seed mode and the bounce
# counts the GPU is held to.
sys_path_golden = str(GOLDEN.parent)


def _make_golden():
    import sys
    if sys_path_golden not in sys.path:
        sys.path.insert(0, sys_path_golden)
    import make_golden
    return make_golden


def _refpix_render(refpix, o, cam, w, h, frames, simd, bounces, threads=0, prev_count=0, prev=None, seed=None):
    prev = np.zeros((w * h, 4), F) if prev is None else prev.copy()
    cur = np.zeros(w * h, np.uint32)
    rays = np.zeros(1, np.uint64)
    args = (o.spheres.ctypes.data, len(o.spheres), o.groups.ctypes.data, len(o.groups), o.materials.ctypes.data,
            len(o.materials), int(o.use_sky), cam.ctypes.data, w, h, prev_count, frames, int(simd))
    st = np.array([seed if seed is not None else 0], np.uint64)
    if threads:
        refpix.ref_render_threads(*args, threads, prev.ctypes.data, cur.ctypes.data, rays.ctypes.data)
    else:
        refpix.ref_render(*args, st.ctypes.data, prev.ctypes.data, cur.ctypes.data, rays.ctypes.data)
    return prev, cur, int(rays[0]), int(st[0])


@pytest.mark.parametrize("simd", [True, False], ids=["RenderTile", "RenderTileScalar"])
def test_patched_reference_is_neutral_at_five_bounces(orc, refmath, refpix, simd):
    """With MaxRayBounce 5 and pixel seeds off, the patched build renders the
    verbatim build's frames: same v4, RGBA8, ray count and final PCG state
    (stream mode, so every draw of the thread's one PCG stream is compared)."""
    refpix.ref_set_patch(5, 0)
    for idx, n, (w, h), frames in ((1, None, (256, 256), 4), (0, None, (96, 64), 3), (2, None, (96, 64), 2),
                                   (1, 13, (70, 33), 2)):
        o = orc.scene_builtin(idx)
        o = o.prefix(n) if n else o
        cam = orc.camera(o, w, h)
        seed = orc.seed_mix(idx)
        a = _ref_render(refmath, o, cam, w, h, frames, simd, seed)
        b = _refpix_render(refpix, o, cam, w, h, frames, simd, 5, seed=seed)
        assert np.array_equal(_u(a[0]), _u(b[0])) and np.array_equal(a[1], b[1]), (idx, n)
        assert (a[2], a[3]) == (b[2], b[3]), (idx, n, a[2:], b[2:])


def _pixel_cases(max_rays=2_000_000):
    mg = _make_golden()
    gold = __import__("json").loads((GOLDEN.parent / "oracle_regression.json").read_text())
    return [c for c in mg.CASES if c[8] == "pixel" and gold[c[0]]["rays"] <= max_rays]


@intel_only
@pytest.mark.parametrize("case", _pixel_cases(), ids=[c[0] for c in _pixel_cases()])
def test_oracle_pixel_mode_vs_patched_reference(orc, refpix, case):
    """The oracle's `pixel` seed mode -- the mode every GPU parity test and
    BASELINE config runs -- against the reference's own RenderTile /
    RenderTileScalar in that mode at the case's bounce count, bit for bit:
    C1 (256^2, N=4, B=1), N=64 at B=8, N=256 at B=16, RGB Glass and RTWeekend
    at B=5 and B=8, both rule sets, and SURVEY 8c's 341,802-segment probe."""
    name, idx, n, w, h, frames, bounces, simd, _ = case
    o = orc.scene_builtin(idx)
    o = o.prefix(n) if n else o
    cam = orc.camera(o, w, h, distance=_make_golden().DISTANCE.get(name))
    refpix.ref_set_patch(bounces, 1)
    rp, rc, rr, _ = _refpix_render(refpix, o, cam, w, h, frames, simd, bounces)
    refpix.ref_set_patch(5, 0)
    op, oc, orr = orc.render(o, cam, w, h, frames=frames, max_bounce=bounces, simd=simd, seed_mode=orc.SEED_PIXEL,
                             threads=4)
    assert rr == orr, (rr, orr)
    bad = np.flatnonzero(np.any(_u(op) != _u(rp), axis=1))
    assert bad.size == 0, ("v4", bad[:5], op[bad[:3]], rp[bad[:3]])
    assert np.array_equal(oc, rc)
    if name == "survey_n64_pixel_256x4":
        assert rr == 341802  # SURVEY 8c's probe value, reproduced by the reference itself


@intel_only
def test_patched_reference_pixel_mode_continuation_and_threads(orc, refpix):
    """A continued accumulation (PreviousRayCount 9, random non-zero mean) in
    pixel mode, and the reference's tiles pulled by 1 or 5 worker threads (its
    work queue, wasm/wasm.cpp:624-694): pixel seeds make the frame independent
    of the schedule, and the oracle matches it."""
    o = orc.scene_builtin(1).prefix(64)
    w, h = 100, 70
    cam = orc.camera(o, w, h)
    prev = RNG.uniform(0, 1.5, (w * h, 4)).astype(F)
    refpix.ref_set_patch(8, 1)
    a = _refpix_render(refpix, o, cam, w, h, 3, True, 8, prev_count=9, prev=prev)
    b = _refpix_render(refpix, o, cam, w, h, 3, True, 8, threads=5, prev_count=9, prev=prev)
    c = _refpix_render(refpix, o, cam, w, h, 3, True, 8, threads=1, prev_count=9, prev=prev)
    refpix.ref_set_patch(5, 0)
    for x in (b, c):
        assert np.array_equal(_u(a[0]), _u(x[0])) and np.array_equal(a[1], x[1]) and a[2] == x[2]
    op, oc, orr = orc.render(o, cam, w, h, prev_count=9, frames=3, max_bounce=8, seed_mode=orc.SEED_PIXEL, threads=3,
                             prev=prev.copy())
    assert orr == a[2] and np.array_equal(_u(op), _u(a[0])) and np.array_equal(oc, a[1])


def test_reference_pixel_frames_equal_the_gpu_fixtures():
    """tests/golden/reference_frames.json "pixel_cases" were rendered by the
    patched reference itself (make_reference_golden.py), including the full
    BASELINE frames: C2 (1920x1080x256, N=64, B=8), C3 (3840x2160x1024), the
    RTWeekend and inside-the-cloud frames.  Every one must equal the fixture of
    the same name in oracle_regression.json, which the GPU path is checked
    against (test_golden_regression.py::test_gpu_matches_golden) and bench.py
    checks its timed frame against.  So reference == fixture == GPU, with no
    live reference needed (this runs on any host)."""
    import json
    ref = json.loads(GOLDEN.read_text())["pixel_cases"]
    gold = json.loads((GOLDEN.parent / "oracle_regression.json").read_text())
    pixel = {k for k, g in gold.items() if g["seed_mode"] == "pixel"}
    assert set(ref) == pixel, sorted(set(ref) ^ pixel)
    for k in sorted(pixel):
        r, g = ref[k], gold[k]
        for f in ("scene", "spheres", "width", "height", "frames", "bounces", "simd", "rays", "fnv1a64_rgba8",
                  "fnv1a64_v4"):
            assert r[f] == g[f], (k, f, r[f], g[f])
        assert r.get("distance") == g.get("distance"), k
    for k in ("c2_full_1920x1080x256", "c3_full_3840x2160x1024", "rtw_full_1920x1080x64"):
        assert k in ref
