"""Diagnostic: does a culled launch's result depend on the device's launch history?"""
import os, sys, pathlib
import numpy as np
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import torch
import __graft_entry__ as g
from oracle import oracle as orc
rt = g.load_package()
REF = {}

def run(dev, n, W, H, S, B, simd=True):
    s = rt.scene_prefix(rt.scene_builtin(1), n)
    cam = rt.camera_setup(s, W, H)
    dev.upload_scene(s)
    prev = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
    cur = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    rays = torch.zeros(1, dtype=torch.int64, device="cuda")
    dev.trace(cam, width=W, height=H, prev_ptr=prev.data_ptr(), cur_ptr=cur.data_ptr(), rays_ptr=rays.data_ptr(),
              frames=S, max_bounce=B, simd=simd, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    key = (n, W, H, S, B, simd)
    if key not in REF:
        o = orc.scene_builtin(1).prefix(n)
        REF[key] = orc.render(o, orc.camera(o, W, H), W, H, frames=S, max_bounce=B, simd=simd)
    op, _, orays = REF[key]
    gp = prev.cpu().numpy()
    bad = np.flatnonzero((gp.view(np.uint32) != op.reshape(-1, 4).view(np.uint32)).any(1))
    info = f"{n}/{W}x{H}/{S}/{B}{'' if simd else 's'}:bad={len(bad)} d={int(rays.item()) - orays}"
    if len(bad):
        i = bad[0]
        info += f" px{i} gpu={gp[i].tolist()} ref={op.reshape(-1, 4)[i].tolist()}"
    return info

seqs = {
    "A": [(128, 16, 8, 1, 1)],
    "B": [(128, 40, 32, 3, 8), (128, 16, 8, 1, 1)],
    "C": [(200, 40, 32, 3, 8), (128, 16, 8, 1, 1), (128, 40, 32, 3, 8)],
    "C2": [(256, 40, 32, 3, 8), (128, 40, 32, 3, 8), (64, 40, 32, 3, 8)],
}
for envname, env in [("smem", {}), ("lds", {"RT_SPHERE_SRC": "lds"}), ("noorder", {"RT_TILE_ORDER": "0"})]:
    for k in ("RT_SPHERE_SRC", "RT_TILE_ORDER"):
        os.environ.pop(k, None)
    os.environ.update(env)
    os.environ["RT_LANES_PER_PIXEL"] = "2"
    for name, seq in seqs.items():
        dev = rt.Device(0)
        print(envname, name, " | ".join(run(dev, *c) for c in seq), flush=True)
        dev.close()
