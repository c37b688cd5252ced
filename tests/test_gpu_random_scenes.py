"""GPU parity on adversarial random scenes (tests/random_scenes.py): 56
seeded scenes x 4 cameras (outside, inside a sphere, on a sphere, grazing
spheres) x both rule sets, bit-exact against the oracle.  The kernel's
proof-based skips -- the cone cull with its dead tiles, the secondary-ray
prefilter (scene-wide or per-lane thresholds), the cluster walk with the
behind-origin rule -- run with their default per-scene choices, and the set
must exercise every one of them."""
import numpy as np
import pytest

import random_scenes

pytestmark = pytest.mark.gpu

SEEDS = list(range(56))
W, H, S, B = 40, 24, 2, 6
_seen = {"culled_groups": 0, "dead_tiles": 0, "prefilter": 0, "relative": 0, "clusters": 0, "inside": 0}


@pytest.fixture(scope="module")
def rdev(rt, torch_cuda):
    dev = rt.Device(0)
    yield dev
    dev.close()


@pytest.mark.parametrize("seed", SEEDS)
def test_random_scene_matches_oracle(rt, orc, torch_cuda, rdev, seed):
    torch = torch_cuda
    spec = random_scenes.make(seed)
    spheres = random_scenes.add_grazing_spheres(rt, spec, W, H, seed=seed)
    first = True
    for look, dist, ang, yh, kind in spec["cameras"]:
        s, o = random_scenes.build(rt, orc, spheres, spec["use_sky"], look, dist, ang, yh)
        if first:
            rdev.upload_scene(s)
            first = False
            for simd in (True, False):
                flags = rt.scene_prefilter(s, simd)[2]
                _seen["prefilter"] += flags & 1
                _seen["relative"] += (flags >> 2) & 1
                _seen["clusters"] += (flags & 1) and rt.scene_clusters(s, simd)[1] > 0
        cam = rt.camera_setup(s, W, H)
        ocam = orc.camera(o, W, H)
        for simd in (True, False):
            prev = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
            cur = torch.zeros(W * H, dtype=torch.int32, device="cuda")
            rays = torch.zeros(1, dtype=torch.int64, device="cuda")
            rdev.trace(cam, width=W, height=H, prev_ptr=prev.data_ptr(), cur_ptr=cur.data_ptr(),
                       rays_ptr=rays.data_ptr(), frames=S, max_bounce=B, simd=simd, band_rows=8,
                       stream=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            op, oc, orays = orc.render(o, ocam, W, H, frames=S, max_bounce=B, simd=simd)
            gp = prev.cpu().numpy().view(np.uint32).reshape(-1, 4)
            bad = np.argwhere(gp != op.view(np.uint32).reshape(-1, 4))
            assert bad.size == 0, f"{kind} simd={simd}: {len(bad)} accumulation words differ, first {bad[:3].tolist()}"
            assert np.array_equal(cur.cpu().numpy().view(np.uint32), oc), f"{kind} simd={simd}: RGBA8 differs"
            assert int(rays.item()) == orays, f"{kind} simd={simd}"
            info = rdev.last_info()
            _seen["dead_tiles"] += info["SegmentsFolded"] > 0
            if simd:
                m = rdev.debug_masks()
                ng = (len(spheres) + 3) // 4
                full = sum(bin(int(v)).count("1") for v in m) if m is not None else 0
                words = (ng + 63) // 64
                _seen["culled_groups"] += m is not None and full < (len(m) // words) * ng
        _seen["inside"] += kind == "inside"


def test_random_scenes_exercise_every_skip():
    if not _seen["inside"]:
        pytest.skip("run with the per-seed tests")
    assert all(v > 0 for v in _seen.values()), _seen
