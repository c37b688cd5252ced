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
