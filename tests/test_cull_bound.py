"""CPU check of the primary-ray cull proof (rt_kernel.hip
cone_may_hit): every sphere pair a pixel's primary rays can reach (f64 line
test over a jitter grid) is in its wave tile's pair mask, as the numpy
restatement of the cull pass computes it.  test_gpu_parity.py pins the GPU's masks to the
same restatement bit for bit."""
import numpy as np
import pytest

from cull_ref import SHAPE, np_masks, sampled_hit_pairs, scene_spheres, wave_tiles


@pytest.mark.parametrize("idx,n,W,H,P", [(1, 64, 48, 32, 4), (1, 128, 16, 16, 1), (1, 200, 40, 24, 2),
                                         (0, None, 32, 24, 8), (1, 256, 24, 16, 16)])
def test_cull_masks_keep_every_reachable_pair(rt, idx, n, W, H, P):
    scene = rt.scene_builtin(idx)
    if n:
        scene = rt.scene_prefix(scene, n)
    cam = rt.camera_setup(scene, W, H)
    masks = np_masks(rt, scene, cam, W, H, P)
    tiles = list(wave_tiles(W, H, P))
    nw = len(masks) // len(tiles)
    n_pairs = 2 * scene_spheres(rt, scene)[2]
    TW, TH = SHAPE[P]
    culled = reached = 0
    for t, w, x0, y0 in tiles:
        words = [int(masks[(t * 4 + w) * nw + k]) for k in range(nw)]
        for y in range(y0, min(y0 + TH, H)):
            for x in range(x0, min(x0 + TW, W)):
                for pi in sampled_hit_pairs(rt, scene, cam, W, H, x, y, n_jitter=3):
                    reached += 1
                    assert (words[pi // 64] >> (pi % 64)) & 1, f"pixel ({x},{y}) reaches pair {pi}, culled"
        culled += n_pairs - sum(bin(v).count("1") for v in words)
    assert reached > 0 and culled > 0
