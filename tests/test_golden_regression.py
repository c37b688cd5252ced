"""Regression vectors (tests/golden/oracle_regression.json, made by
tests/golden/make_golden.py): the oracle must keep reproducing them (CPU),
and the GPU path must match them directly (GPU) — i.e. the HIP kernel is
checked against fixed committed data, not only against a live oracle."""
import json
import os
import pathlib
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
GOLD = json.loads((ROOT / "tests" / "golden" / "oracle_regression.json").read_text())
sys.path.insert(0, str(ROOT / "tests" / "golden"))
import make_golden  # noqa: E402

CASES = {c[0]: c for c in make_golden.CASES}
FAST = [k for k in GOLD if not k.startswith("survey_")]


@pytest.mark.parametrize("name", list(GOLD))
def test_oracle_reproduces_golden(orc, name):
    if name in make_golden.SLOW and os.environ.get("RT_SLOW_ORACLE") != "1":
        pytest.skip("full-size C3 oracle render takes minutes: RT_SLOW_ORACLE=1")
    _, scene, n, W, H, frames, bounces, simd, seed = CASES[name]
    prev, cur, rays = make_golden.render_case(scene, n, W, H, frames, bounces, simd, seed,
                                              make_golden.DISTANCE.get(name))
    g = GOLD[name]
    assert rays == g["rays"]
    assert f"{orc.fnv1a64(cur):016x}" == g["fnv1a64_rgba8"]
    assert f"{orc.fnv1a64(prev):016x}" == g["fnv1a64_v4"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", [k for k in GOLD if GOLD[k]["seed_mode"] == "pixel"])
def test_gpu_matches_golden(rt, orc, torch_cuda, name):
    torch = torch_cuda
    _, scene, n, W, H, frames, bounces, simd, seed = CASES[name]
    s = rt.scene_builtin(scene)
    if n is not None:
        s = rt.scene_prefix(s, n)
    dev = rt.Device(0)
    dev.upload_scene(s)
    prev = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
    cur = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    rays = torch.zeros(1, dtype=torch.int64, device="cuda")
    dev.trace(rt.camera_setup(s, W, H, distance=make_golden.DISTANCE.get(name)), width=W, height=H, prev_ptr=prev.data_ptr(), cur_ptr=cur.data_ptr(),
              rays_ptr=rays.data_ptr(), frames=frames, max_bounce=bounces, simd=simd)
    torch.cuda.synchronize()
    g = GOLD[name]
    assert int(rays.item()) == g["rays"]
    assert f"{orc.fnv1a64(cur.cpu().numpy().view(np.uint32)):016x}" == g["fnv1a64_rgba8"]
    assert f"{orc.fnv1a64(prev.cpu().numpy()):016x}" == g["fnv1a64_v4"]
    dev.close()


C5_ROWS = ROOT / "tests" / "golden" / "c5_rows.json"


def _c5_rows():
    return json.loads(C5_ROWS.read_text())


def test_c5_rows_fixture_covers_the_frame_and_agrees():
    """tests/golden/c5_rows.json (tests/golden/make_c5_rows.py): BASELINE C5 at
    its full workload (7680x4320, 4096 spp, 256 spheres, 16 bounces) on whole
    32-row tile rows, rendered by the reference's own RenderTile (librefpix.so,
    main.cpp:7-640 with SURVEY 8c's patches) and by the oracle's row mode: the
    two agreed on every field (oracle_equal), and the rows cover the top, middle
    and bottom of the frame (rows 0-1, 2160-2161, 4318-4319) and its two
    densest bands of geometry."""
    g = _c5_rows()
    assert (g["width"], g["height"], g["frames"], g["spheres"], g["bounces"], g["scene"]) == (7680, 4320, 4096, 256,
                                                                                               16, 1)
    covered = set()
    for e in g["tile_rows"].values():
        assert e["oracle_equal"] is True
        assert e["rays"] > 0 and e["rows"][1] - e["rows"][0] == 32
        covered.update(range(*e["rows"]))
    assert {0, 1, 2160, 2161, 4318, 4319} <= covered
    assert max(e["non_black_pixels"] for e in g["tile_rows"].values()) > 50000


@pytest.mark.gpu
@pytest.mark.timeout(280)
def test_gpu_c5_tile_rows_match_the_reference(rt, torch_cuda):
    """The full C5 frame (7680x4320, 4096 spp, 256 spheres, 16 bounces) in one
    launch on one device, then dealt over eight shards of this GPU (rt_multi, 8-row
    bands, the running mean gathered too): the tile rows of c5_rows.json equal
    the reference-rendered hashes (v4 and RGBA8) in both, and both count the same
    segments."""
    torch = torch_cuda
    g = _c5_rows()
    W, H, S, B = g["width"], g["height"], g["frames"], g["bounces"]
    s = rt.scene_prefix(rt.scene_builtin(1), g["spheres"])
    cam = rt.camera_setup(s, W, H)
    prev = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
    cur = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    rays = torch.zeros(2, dtype=torch.int64, device="cuda")

    def check(tag):
        hp = prev.view(H, W, 4)
        hc = cur.view(H, W)
        for ty, e in g["tile_rows"].items():
            y0, y1 = e["rows"]
            v4 = hp[y0:y1].cpu().numpy()
            rgba = hc[y0:y1].cpu().numpy().view(np.uint32)
            assert f"{rt.frame_hash(rgba):016x}" == e["fnv1a64_rgba8"], (tag, ty)
            assert f"{rt.frame_hash(v4):016x}" == e["fnv1a64_v4"], (tag, ty)

    dev = rt.Device(0)
    try:
        dev.upload_scene(s)
        dev.trace(cam, width=W, height=H, prev_ptr=prev.data_ptr(), cur_ptr=cur.data_ptr(),
                  rays_ptr=rays[0].data_ptr(), frames=S, max_bounce=B)
        torch.cuda.synchronize()
    finally:
        dev.close()
    check("one device")
    prev.fill_(float("nan"))
    cur.zero_()
    m = rt.Multi([0] * 8)
    try:
        m.upload_scene(s)
        m.trace(cam, width=W, height=H, cur_ptr=cur.data_ptr(), prev_ptr=prev.data_ptr(), rays_ptr=rays[1].data_ptr(),
                frames=S, max_bounce=B, band_rows=8, accum_zero=True)
        torch.cuda.synchronize()
    finally:
        m.close()
    check("eight shards")
    assert int(rays[0].item()) == int(rays[1].item()) > 1e11
