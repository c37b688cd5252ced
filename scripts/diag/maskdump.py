"""Diagnostic (RTK_DIAG_MASKDUMP build, RT_WAVETIMES=1): the mask word each wave read vs the cull pass's."""
import os, pathlib, sys
import numpy as np
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
os.environ["RT_WAVETIMES"] = "1"
import torch
import __graft_entry__ as g
rt = g.load_package()
for n, W, H, P in [(128, 16, 16, 1), (128, 16, 8, 2), (128, 40, 32, 1)]:
    os.environ["RT_LANES_PER_PIXEL"] = str(P)
    dev = rt.Device(0)
    s = rt.scene_prefix(rt.scene_builtin(1), n)
    cam = rt.camera_setup(s, W, H)
    dev.upload_scene(s)
    prev = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
    cur = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    rays = torch.zeros(1, dtype=torch.int64, device="cuda")
    dev.trace(cam, width=W, height=H, prev_ptr=prev.data_ptr(), cur_ptr=cur.data_ptr(), rays_ptr=rays.data_ptr(),
              frames=1, max_bounce=1, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    m = dev.debug_masks()
    wt = dev.debug_wave_times(len(m))
    dev.close()
    for wid in range(len(m)):
        if wt[wid, 0] != m[wid] or wt[wid, 1] != m[wid]:
            print(f"n={n} {W}x{H} P={P} wave {wid}: cull {hex(int(m[wid]))} read {hex(int(wt[wid, 0]))} end {hex(int(wt[wid, 1]))}")
    print(f"n={n} {W}x{H} P={P} checked {len(m)} waves", flush=True)
