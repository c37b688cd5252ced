"""CPU-side checks of the C-ABI library (no GPU needed): it loads, exports
every symbol include/rt_trace.h declares, keeps the reference's struct
layouts, and its host-side inputs (scenes, camera, seeds, band plan) are
bit-identical to the oracle's restatement of the reference."""
import ctypes
import pathlib
import re

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "rt_trace.h"


def declared_functions():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(rt_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_the_expected_surface():
    names = declared_functions()
    for must in ["rt_device_create", "rt_scene_upload", "rt_trace", "rt_on_init", "rt_on_render",
                 "rt_assemble_bands", "rt_camera_setup", "rt_scene_builtin"]:
        assert must in names


def test_library_exports_every_declared_symbol(rt):
    L = rt.lib()
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing
    assert set(declared_functions()) == set(rt.SIGNATURES), "python SIGNATURES out of sync with the header"


def test_struct_layouts_match_reference(rt):
    # SURVEY §8b offsets (verified by offsetof on the reference in the survey probe)
    assert rt.RtScene.UseSkyColor.offset == 16
    assert rt.RtScene.DefaultDistanceFromLookAt.offset == 20
    assert rt.RtScene.ScalarSpheres.offset == 32
    assert rt.RtScene.SIMDSpheres.offset == 48
    assert rt.RtScene.Materials.offset == 64
    assert rt.RtCameraInfo.FilmW.offset == 80 and rt.RtCameraInfo.FilmH.offset == 84
    assert rt.RtCameraInfo.TilesX.offset == 88
    assert rt.RtCameraInfo.CurrentImage.offset == 96 and rt.RtCameraInfo.PreviousImage.offset == 120
    assert rt.RtMaterial.Specular.offset == 32 and rt.RtMaterial.IndexOfRefraction.offset == 36
    assert rt.RtScalarSphere.Material.offset == 32
    assert ctypes.sizeof(rt.RtCameraInfo) == 144 and ctypes.sizeof(rt.RtScene) == 80


@pytest.mark.parametrize("idx,n", [(0, 5), (1, 256), (2, 482)])
def test_builtin_scenes_match_oracle(rt, orc, idx, n):
    s = rt.scene_builtin(idx)
    o = orc.scene_builtin(idx)
    sp, gr, ma = rt.scene_arrays(s)
    assert sp.shape[0] == n and gr.shape[0] == (n + 3) // 4 and ma.shape[0] == n + 1
    for a, b in [(sp, o.spheres), (gr, o.groups), (ma, o.materials)]:
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert bool(s.UseSkyColor) == o.use_sky
    for a, b in [(s.DefaultDistanceFromLookAt, o.distance), (s.DefaultXAngle, o.x_angle),
                 (s.DefaultYHeight, o.y_height), (s.LookAt.x, o.look_at[0]), (s.LookAt.y, o.look_at[1]),
                 (s.LookAt.z, o.look_at[2])]:
        assert np.float32(a) == np.float32(b)


def test_scene_prefix_counts(rt):
    s = rt.scene_prefix(rt.scene_builtin(1), 13)
    assert (s.ScalarSpheres.Count, s.SIMDSpheres.Count, s.Materials.Count) == (13, 4, 14)
    with pytest.raises(rt.RtError):
        rt.scene_prefix(rt.scene_builtin(0), 6)


@pytest.mark.parametrize("idx", [0, 1, 2])
@pytest.mark.parametrize("W,H", [(256, 256), (1920, 1080), (37, 91), (1, 1)])
def test_camera_matches_oracle(rt, orc, idx, W, H):
    s = rt.scene_builtin(idx)
    o = orc.scene_builtin(idx)
    for ang, dist, yh in [(None, None, None), (0.7, 0.4, 0.1), (-5.5, 2.0, -0.3)]:
        c = rt.camera_floats(rt.camera_setup(s, W, H, dist, ang, yh))
        oc = orc.camera(o, W, H, dist, ang, yh)
        assert np.array_equal(c[:23].view(np.uint32), oc[:23].view(np.uint32))


def test_pixel_seed_matches_oracle(rt, orc):
    for x, y, k, W, H in [(0, 0, 0, 1, 1), (3, 5, 2, 100, 50), (1919, 1079, 255, 1920, 1080),
                          (7679, 4319, 4095, 7680, 4320)]:
        assert rt.pixel_seed(x, y, k, W, H) == orc.seed_mix((k * H + y) * W + x)


def test_band_plan_matches_library(rt):
    import __graft_entry__ as graft
    mg = __import__("simd_ray_tracer_amd.multigpu", fromlist=["x"])
    for H in [1, 31, 32, 33, 150, 1080, 4320]:
        for G in [1, 2, 3, 4, 8]:
            rows, maxr = mg.band_plan(H, 32, G)
            assert rows == [rt.band_local_rows(H, 32, G, r) for r in range(G)]
            assert sum(rows) == H
            m = mg.row_owner_map(H, 32, G)
            for r in range(G):
                assert (m[:, 0] == r).sum() == rows[r]
                assert sorted(m[m[:, 0] == r, 1]) == list(range(rows[r]))
    assert graft is not None


def test_rsqrt_builtin_table_is_the_fixture(rt):
    fixture = np.fromfile(ROOT / "tests" / "golden" / "rsqrt_lut_intel.bin", dtype=np.float32)
    assert np.array_equal(rt.rsqrt_table_builtin().view(np.uint32), fixture.view(np.uint32))
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_rsqrt_inc", ROOT / "tests" / "golden" / "make_rsqrt_inc.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    inc = ROOT / "simd-ray-tracer_amd" / "csrc" / "rsqrt_table_intel.inc"
    assert inc.read_text() == mod.render(), "regenerate with tests/golden/make_rsqrt_inc.py"


def test_rsqrt_capture_host(rt):
    from conftest import host_is_intel
    t = np.zeros(2048, np.float32)
    rc = rt.lib().rt_rsqrt_table_capture_host(t.ctypes.data)
    if host_is_intel():
        assert rc == 0 and np.array_equal(t.view(np.uint32), rt.rsqrt_table_builtin().view(np.uint32))
    else:
        assert rc in (0, -22)


def test_device_create_fails_loudly_without_gpu(rt):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(rt.RtError, match="no HIP device"):
        rt.Device(0)


def test_trace_rejects_bad_arguments(rt):
    L = rt.lib()
    cam = rt.RtCameraInfo()
    d = rt.RtTraceDesc()
    assert L.rt_trace(None, ctypes.byref(cam), ctypes.byref(d), None, None) == -22
    assert L.rt_scene_upload(None, None) == -22
    assert L.rt_assemble_bands(None, 0, None, 0, 0, 0, 0, 0, None) == -22
    assert b"bad argument" in L.rt_last_error()
    assert L.rt_encode_rgba8(None, None, 1, 0, None) == -22
    assert L.rt_encode_rgba8(None, None, 0, 4, None) == -22 and b"unknown flags" in L.rt_last_error()
    assert L.rt_encode_rgba8(None, None, 0, rt.RT_FLAG_SRGB_POW, None) == 0  # nothing to encode: no launch


def test_scene_size_limits(rt):
    """rt_scene_upload's packer (shared with rt_scene_prefilter, no GPU needed)
    rejects an empty scene and one past RT_MAX_SPHERES; scenes past the LDS
    image's 656 spheres (164 groups) are accepted (they stay in HBM)."""
    empty = rt.scene_from_spheres(np.zeros((0, 20), np.float32), use_sky=True)
    with pytest.raises(rt.RtError, match="empty scene"):
        rt.scene_prefilter(empty, True)
    sp = np.zeros((rt.RT_MAX_SPHERES + 1, 20), np.float32)
    sp[:, 0] = np.arange(len(sp), dtype=np.float32)
    sp[:, 4] = 0.25
    with pytest.raises(rt.RtError, match="exceed the limit"):
        rt.scene_prefilter(rt.scene_from_spheres(sp[:]), True)
    r2, _, _ = rt.scene_prefilter(rt.scene_from_spheres(sp[:4 * 164 + 1]), True)  # one past the LDS image
    assert len(r2) == 4 * 165


def test_frame_hash_is_the_fixtures_fnv1a(rt, orc):
    """rt_frame_hash (the bench's frame check) is the FNV-1a 64 the committed
    fixtures hold (the oracle's or_fnv1a64), on empty, odd-sized and random
    buffers."""
    rng = np.random.default_rng(5)
    for n in (0, 1, 7, 4096, 100003):
        a = rng.integers(0, 256, n, dtype=np.uint8)
        assert rt.frame_hash(a) == orc.fnv1a64(a), n
    assert rt.frame_hash(np.zeros(0, np.uint8)) == 0xcbf29ce484222325


def test_bench_finds_the_fixture_of_each_preset():
    """bench.py checks its last timed frame against the committed fixture of
    the workload (golden_for): C2, C3, RTWeekend and C2-inside each have one,
    a custom workload has none."""
    import sys
    sys.path.insert(0, str(ROOT))
    import bench

    class A:
        pass
    for cfg, name in (("c2", "c2_full_1920x1080x256"), ("c3", "c3_full_3840x2160x1024"),
                      ("rtw", "rtw_full_1920x1080x64"), ("c2in", "c2in_full_1920x1080x256")):
        a = A()
        for k, v in bench.CONFIGS[cfg].items():
            setattr(a, k, v)
        a.scalar = False
        n = 482 if cfg == "rtw" else a.spheres
        got, g = bench.golden_for(a, a.width, a.height, a.spp, n, a.bounces)
        assert got == name, (cfg, got)
        assert g["seed_mode"] == "pixel"
    a.spp = 3
    assert bench.golden_for(a, a.width, a.height, a.spp, 64, a.bounces) == (None, None)
    assert bench.combine_verified(None, True) is True and bench.combine_verified(True, False) is False
    assert bench.combine_verified(None, None) is None


def test_device_options_are_checked_before_any_device(rt):
    """rt_device_options (rt_device_create_ex) replaces the environment knobs the
    library read before round 6: bad values are refused before the call looks
    for a device (so this runs without one), unknown names never reach C, and a
    zero-filled struct is rt_device_create's behaviour.  The library reads no
    environment variable that selects kernels or schedules."""
    import ctypes
    with pytest.raises(rt.RtError, match="switch is 5"):
        rt.Device(0, options={"Cull": 5})
    with pytest.raises(rt.RtError, match="LanesPerPixel 3"):
        rt.Device(0, options={"LanesPerPixel": 3})
    with pytest.raises(rt.RtError, match="count is out of range"):
        rt.Device(0, options={"SplitParts": 9})
    with pytest.raises(KeyError, match="unknown device option"):
        rt.device_options({"RT_CULL": 0})
    o = rt.RtDeviceOptions()
    o.Size = 7
    h = ctypes.c_void_p()
    assert rt.lib().rt_device_create_ex(0, ctypes.byref(o), ctypes.byref(h)) == -22
    assert b"Size 7" in rt.lib().rt_last_error()
    assert rt.parse_options(["Cull=off", "LanesPerPixel=16", "XcdGroup=on", "Prefilter=default"]) == {
        "Cull": -1, "LanesPerPixel": 16, "XcdGroup": 1, "Prefilter": 0}
    assert rt.device_options({"Cull": False, "TileOrder": True}).Cull == -1
    assert ctypes.sizeof(rt.RtDeviceOptions) == 4 * (1 + len(rt.OPTION_FIELDS))
    import subprocess
    syms = subprocess.run(["nm", "-D", "--undefined-only", str(rt.LIB_PATH)], capture_output=True, text=True).stdout
    assert "getenv" in syms  # the diagnostic hooks (RT_STATS, RT_WAVETIMES) only:
    src = (ROOT / "simd-ray-tracer_amd" / "csrc" / "rt_host.cpp").read_text()
    names = re.findall(r'getenv\("(\w+)"\)', src)
    assert sorted(names) == ["RT_STATS", "RT_WAVETIMES"], names
    for f in (ROOT / "simd-ray-tracer_amd" / "csrc").glob("*"):
        if f.name != "rt_host.cpp" and f.suffix in (".cpp", ".hip", ".h"):
            assert "getenv" not in f.read_text(), f.name


def test_code_object_hash_reads_the_fatbin(rt, tmp_path):
    """The binary hash bench.py ties PMC records to: the .hip_fatbin section
    of the library (stable across a host-only relink, moved by any kernel
    change); a file without the section is refused."""
    h = rt.code_object_hash()
    assert len(h) == 16 and int(h, 16) >= 0
    assert rt.code_object_hash(rt.LIB_PATH) == h
    bad = tmp_path / "x.so"
    bad.write_bytes(b"not an elf")
    with pytest.raises(rt.RtError, match="ELF64"):
        rt.code_object_hash(bad)
