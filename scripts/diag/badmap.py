"""Diagnostic: where do culled primary-only launches differ from brute force (RT_CULL=0)?"""
import os
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import __graft_entry__ as g  # noqa: E402

rt = g.load_package()
SHAPE = {1: (8, 8), 2: (8, 4), 4: (4, 4), 8: (4, 2), 16: (2, 2)}


def render(n, W, H, S, B, P, cull):
    os.environ["RT_LANES_PER_PIXEL"] = str(P)
    os.environ["RT_CULL"] = "1" if cull else "0"
    dev = rt.Device(0)
    s = rt.scene_prefix(rt.scene_builtin(1), n)
    cam = rt.camera_setup(s, W, H)
    dev.upload_scene(s)
    prev = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
    cur = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    rays = torch.zeros(1, dtype=torch.int64, device="cuda")
    dev.trace(cam, width=W, height=H, prev_ptr=prev.data_ptr(), cur_ptr=cur.data_ptr(), rays_ptr=rays.data_ptr(),
              frames=S, max_bounce=B, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    masks = dev.debug_masks() if cull else None
    dev.close()
    return prev.cpu().numpy().reshape(H, W, 4), int(rays.item()), masks


for n, W, H, S, B in [(128, 16, 8, 1, 1), (128, 32, 8, 1, 1), (128, 16, 16, 1, 1), (128, 40, 32, 3, 8)]:
    for P in (1, 2, 4):
        a, ra, masks = render(n, W, H, S, B, P, True)
        b, rb, _ = render(n, W, H, S, B, P, False)
        bad = np.argwhere((a.view(np.uint32) != b.view(np.uint32)).any(2))
        TW, TH = SHAPE[P]
        desc = []
        for y, x in bad[:6]:
            w = (1 if x % (2 * TW) >= TW else 0) + (2 if y % (2 * TH) >= TH else 0)
            pl = (y % TH) * TW + (x % TW)
            desc.append(f"({x},{y}) w{w} pix{pl} cull={a[y, x, :3].round(3).tolist()} brute={b[y, x, :3].round(3).tolist()}")
        if len(bad):
            y, x = bad[0]
            TWp, THp = SHAPE[P]
            tx = (W + 2 * TWp - 1) // (2 * TWp)
            t = (y // (2 * THp)) * tx + x // (2 * TWp)
            w = (1 if x % (2 * TWp) >= TWp else 0) + (2 if y % (2 * THp) >= THp else 0)
            nw = len(masks) // (4 * (len(masks) // 4 // max(1, (len(masks) // 4))))
            desc.append(f"tile {t} masks {[hex(int(v)) for v in masks[4 * t:4 * t + 4]]}")
        print(f"n={n} {W}x{H} S={S} B={B} P={P}: bad={len(bad)} drays={ra - rb}", desc, flush=True)
