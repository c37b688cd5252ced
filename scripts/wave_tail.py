"""Diagnostic: per-wave start/end times of one C2 launch -> occupancy over time.
env: SPP (256), SIM_RANKS (1: whole frame; G: rank 0's bands of a G-GPU split),
SCENE (1) / SPHERES (64) / BOUNCES (8), CONTINUE (1: launches continue the running mean,
as OnRender's frames do; default: every launch restarts it),
LPP (lanes per pixel, rt_device_options LanesPerPixel; 0 auto), LAUNCHES (8: the learned order settles), SAVE (a .npz
path: the raw per-wave {start, end} of the last launch, indexed 4 * block tile + wave,
for offline schedule simulation: scripts/sched_sim.py)."""
import os
import sys
import pathlib
import numpy as np
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
os.environ["RT_WAVETIMES"] = "1"
import torch
import __graft_entry__ as graft
rt = graft.load_package()
W, H, S = 1920, 1080, int(os.environ.get("SPP", "256"))
B, N = int(os.environ.get("BOUNCES", "8")), int(os.environ.get("SPHERES", "64"))
scene = rt.scene_builtin(int(os.environ.get("SCENE", "1")))
if N < scene.ScalarSpheres.Count:
    scene = rt.scene_prefix(scene, N)
cont = os.environ.get("CONTINUE") == "1"
cam = rt.camera_setup(scene, W, H)
dev = rt.Device(0, options={"LanesPerPixel": int(os.environ.get("LPP", "0"))})
dev.upload_scene(scene)
G = int(os.environ.get("SIM_RANKS", "1"))
rows = rt.band_local_rows(H, 8, G, 0)
prev = torch.zeros((rows * W, 4), dtype=torch.float32, device="cuda")
cur = torch.zeros(rows * W, dtype=torch.int32, device="cuda")
rays = torch.zeros(1, dtype=torch.int64, device="cuda")
for i in range(int(os.environ.get("LAUNCHES", "8"))):
    dev.trace(cam, width=W, height=H, prev_ptr=prev.data_ptr(), cur_ptr=cur.data_ptr(), rays_ptr=rays.data_ptr(),
              prev_count=i * S if cont else 0, frames=S, max_bounce=B, accum_zero=not cont, band_rows=8,
              band_count=G, band_index=0)
torch.cuda.synchronize()
wt_all = dev.debug_wave_times().astype(np.int64)
if os.environ.get("SAVE"):
    np.savez_compressed(os.environ["SAVE"], wave_times=wt_all, info=np.array(list(dev.last_info().values())))
wt = wt_all[wt_all[:, 1] > 0]
t0 = wt[:, 0].min()
st, en = (wt[:, 0] - t0) / 100.0, (wt[:, 1] - t0) / 100.0  # microseconds
dur = en - st
print(f"waves {len(wt)}  kernel span {en.max():.0f} us  wave dur mean {dur.mean():.0f} p50 {np.median(dur):.0f} "
      f"p90 {np.percentile(dur, 90):.0f} max {dur.max():.0f} us")
T = en.max()
fin = np.sort(en)
print("finished fraction -> time (us):", {q: round(float(fin[int(q * (len(fin) - 1))]), 0) for q in (0.5, 0.9, 0.99, 1.0)})
for f in np.linspace(0, 1, 21)[:-1]:
    t = f * T
    print(f"t={t:8.0f}us active waves {int(((st <= t) & (en > t)).sum()):6d}")
print("slowest wave durations (us):", [int(d) for d in np.sort(dur)[-10:]])
late = np.argsort(en)[-10:]
print("last-ending waves (start, dur) us:", [(int(st[i]), int(dur[i])) for i in late])
# block occupancy: a 4-wave block holds its slots until its last wave ends
blk = wt_all[: (len(wt_all) // 4) * 4].reshape(-1, 4, 2)
blk = blk[(blk[:, :, 1] > 0).all(1)]
span = blk[:, :, 1].max(1) - blk[:, :, 0].min(1)
busy = (blk[:, :, 1] - blk[:, :, 0]).sum(1)
print(f"blocks {len(blk)}: wave-slot time idle inside blocks {1 - busy.sum() / (4 * span.sum()):.3f} "
      f"(waves ending before their block's last wave)")
