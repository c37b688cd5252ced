"""Diagnostic: GPU vs oracle ray counts for culled launches (scene 1 prefixes)."""
import os, sys, pathlib
import numpy as np
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import torch
import __graft_entry__ as g
from oracle import oracle as orc
rt = g.load_package()

def run(dev, n, W, H, S, B, simd, band_count=1, band_index=0):
    s = rt.scene_prefix(rt.scene_builtin(1), n)
    cam = rt.camera_setup(s, W, H)
    dev.upload_scene(s)
    local = rt.band_local_rows(H, 32, band_count, band_index)
    prev = torch.zeros((local * W, 4), dtype=torch.float32, device="cuda")
    cur = torch.zeros(local * W, dtype=torch.int32, device="cuda")
    rays = torch.zeros(1, dtype=torch.int64, device="cuda")
    dev.trace(cam, width=W, height=H, prev_ptr=prev.data_ptr(), cur_ptr=cur.data_ptr(), rays_ptr=rays.data_ptr(),
              frames=S, max_bounce=B, simd=simd, band_count=band_count, band_index=band_index,
              stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return prev.cpu().numpy(), int(rays.item())

for lpp in ("2", "4", "1"):
    os.environ["RT_LANES_PER_PIXEL"] = lpp
    for cull in ("1", "0"):
        os.environ["RT_CULL"] = cull
        dev = rt.Device(0)
        out = []
        for n, W, H, S, B in [(128, 40, 32, 3, 8), (128, 40, 32, 1, 1), (128, 40, 32, 1, 8), (128, 16, 8, 1, 1),
                              (128, 64, 64, 1, 1), (64, 40, 32, 1, 1), (100, 40, 32, 1, 1)]:
            o = orc.scene_builtin(1).prefix(n)
            op, _, orays = orc.render(o, orc.camera(o, W, H), W, H, frames=S, max_bounce=B)
            gp, grays = run(dev, n, W, H, S, B, True)
            nbad = int((gp.view(np.uint32) != op.reshape(-1, 4).view(np.uint32)).any(1).sum())
            out.append(f"{n}/{W}x{H}/{S}/{B}: d={grays - orays} bad={nbad}")
        dev.close()
        print(f"P={lpp} cull={cull}", "; ".join(out), flush=True)
