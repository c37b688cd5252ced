"""Two C2 frames in flight on one GPU: two rt_device contexts on device 0, each
with its own stream and buffers, trace alternate frames; measured against one
context tracing the same frames one after another.  A launch's ramp and tail
leave SIMDs idle; a second launch in flight on another stream can fill them.

usage: python scripts/frames_in_flight.py [steps] [contexts] [extra bench-style args: --sim-ranks G --sim-index r]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import __graft_entry__ as graft  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    n_ctx = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    bands, band = 1, 0
    if "--sim-ranks" in sys.argv:
        bands = int(sys.argv[sys.argv.index("--sim-ranks") + 1])
        band = int(sys.argv[sys.argv.index("--sim-index") + 1])
    rt = graft.load_package()
    scene = rt.scene_prefix(rt.scene_builtin(1), 64)
    W, H, S, B = 1920, 1080, 256, 8
    rows = rt.band_local_rows(H, 8, bands, band)
    cam = rt.camera_setup(scene, W, H)
    ctx = []
    for i in range(n_ctx):
        dev = rt.Device(0)
        dev.upload_scene(scene)
        st = torch.cuda.Stream()
        prev = torch.zeros((rows * W, 4), dtype=torch.float32, device="cuda")
        cur = torch.zeros(rows * W, dtype=torch.int32, device="cuda")
        ctx.append((dev, st, prev, cur))
    rays = torch.zeros(4 * steps + 64, dtype=torch.int64, device="cuda")
    c = [0]

    def launch(i):
        dev, st, prev, cur = ctx[i]
        dev.trace(cam, width=W, height=H, prev_ptr=prev.data_ptr(), cur_ptr=cur.data_ptr(),
                  rays_ptr=rays[c[0]].data_ptr(), prev_count=0, frames=S, max_bounce=B, simd=True,
                  band_rows=8, band_count=bands, band_index=band, accum_zero=True, stream=st.cuda_stream)
        c[0] += 1

    for i in range(n_ctx):  # warm every context: cull pass, learned order (6 re-sorts), code objects
        for _ in range(8):
            launch(i)
    torch.cuda.synchronize()
    out = {}
    for mode in ("one", "flight"):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k in range(steps):
            launch(0 if mode == "one" else k % n_ctx)
        torch.cuda.synchronize()
        out[mode] = (time.perf_counter() - t) * 1e3 / steps
    n = int(rays[c[0] - 1].item())
    assert all(int(v) == n for v in rays[c[0] - 2 * steps:c[0]].tolist()), "every frame counts the same rays"
    print(f"bands {bands} index {band}: one context {out['one']:.3f} ms/frame, {n_ctx} in flight "
          f"{out['flight']:.3f} ms/frame ({out['one'] / out['flight']:.3f}x), {n} rays per frame")


if __name__ == "__main__":
    main()
