"""The skip proofs' host-side bounds on adversarial random scenes (CPU; see
tests/random_scenes.py): the prefilter thresholds and the cluster table never
skip a sphere the reference-rounded exact test can accept, and the cull
pass's primary masks keep every group a pixel's rays can reach -- for scenes
with radii over five decades, tangent / nested / coincident spheres and
cameras inside or on a sphere.  The GPU parity of the same scenes is
tests/test_gpu_random_scenes.py."""
import numpy as np
import pytest

import random_scenes
from cull_ref import SHAPE, np_masks, sampled_hit_pairs, scene_spheres, wave_tiles
from test_prefilter_bound import check_clusters, check_prefilter

SEEDS = list(range(40))
_seen = {"prefilter_on": 0, "prefilter_culls": 0, "cluster_skips": 0, "behind_skips": 0, "cull_culls": 0}


@pytest.mark.parametrize("seed", SEEDS)
def test_random_scene_bounds(rt, orc, seed):
    spec = random_scenes.make(seed)
    look, dist, ang, yh, _ = spec["cameras"][0]
    scene, _ = random_scenes.build(rt, orc, spec["spheres"], spec["use_sky"], look, dist, ang, yh)
    for simd in (True, False):
        on, culled = check_prefilter(rt, scene, simd, seed, n_rays=1500, require_hits=False)
        _seen["prefilter_on"] += on
        _seen["prefilter_culls"] += culled > 0
        sk, bh = check_clusters(rt, scene, simd, seed, n_rays=1500)
        _seen["cluster_skips"] += sk > 0
        _seen["behind_skips"] += bh > 0
    W, H, P = 24, 16, 4
    TW, TH = SHAPE[P]
    for look, dist, ang, yh, kind in spec["cameras"]:
        s, _ = random_scenes.build(rt, orc, spec["spheres"], spec["use_sky"], look, dist, ang, yh)
        cam = rt.camera_setup(s, W, H)
        masks = np_masks(rt, s, cam, W, H, P)
        tiles = list(wave_tiles(W, H, P))
        nw = len(masks) // len(tiles)
        n_pairs = 2 * scene_spheres(rt, s)[2]
        for t, w, x0, y0 in tiles:
            words = [int(masks[(t * 4 + w) * nw + k]) for k in range(nw)]
            _seen["cull_culls"] += n_pairs - sum(bin(v).count("1") for v in words) > 0
            for y in range(y0, min(y0 + TH, H), 2):
                for x in range(x0, min(x0 + TW, W), 2):
                    for pi in sampled_hit_pairs(rt, s, cam, W, H, x, y, n_jitter=3):
                        assert (words[pi // 64] >> (pi % 64)) & 1, f"{kind}: pixel ({x},{y}) reaches pair {pi}"


def test_random_scenes_exercise_every_skip(rt, orc):
    """Over the seed set, every proof-based skip actually fires somewhere (counted
    afresh here, so the test does not depend on the per-seed tests' process)."""
    seen = dict.fromkeys(_seen, 0)
    for seed in SEEDS:
        spec = random_scenes.make(seed)
        look, dist, ang, yh, _ = spec["cameras"][0]
        scene, _ = random_scenes.build(rt, orc, spec["spheres"], spec["use_sky"], look, dist, ang, yh)
        for simd in (True, False):
            on, culled = check_prefilter(rt, scene, simd, seed, n_rays=300, require_hits=False)
            seen["prefilter_on"] += on
            seen["prefilter_culls"] += culled > 0
            sk, bh = check_clusters(rt, scene, simd, seed, n_rays=300)
            seen["cluster_skips"] += sk > 0
            seen["behind_skips"] += bh > 0
        cam = rt.camera_setup(scene, 24, 16)
        masks = np_masks(rt, scene, cam, 24, 16, 4)
        n_pairs = 2 * scene_spheres(rt, scene)[2]
        nw = (n_pairs + 63) // 64
        seen["cull_culls"] += sum(bin(int(v)).count("1") for v in masks) < (len(masks) // nw) * n_pairs
    assert all(v > 0 for v in seen.values()), seen
