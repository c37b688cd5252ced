"""rt_multi: does a new camera's first call overlap across devices?

Drives rt_multi over `G` device slots (default four times device 0) at C2's
geometry: one warm call (buffers sized, code objects loaded), then calls with
a new camera each, no host synchronisation in between.  Run it under
`rocprofv3 --kernel-trace` and read the trace with
scripts/multi_trace_report.py: every new-camera call must show the devices'
cull passes and traces in flight together (rt_trace never blocks the host on a
new key).

usage: python scripts/multi_cold_overlap.py [G]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import __graft_entry__ as graft  # noqa: E402


def main():
    g = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    rt = graft.load_package()
    scene = rt.scene_prefix(rt.scene_builtin(1), 64)
    W, H = 1920, 1080
    multi = rt.Multi([0] * g)
    multi.upload_scene(scene)
    full = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    rays = torch.zeros(8, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream()
    for c, angle in enumerate((None, 0.3, 0.6, 0.9)):
        cam = rt.camera_setup(scene, W, H, x_angle=angle)
        multi.trace(cam, width=W, height=H, cur_ptr=full.data_ptr(), rays_ptr=rays[c].data_ptr(), frames=256,
                    max_bounce=8, simd=True, band_rows=8, accum_zero=True, stream=stream.cuda_stream)
        if c == 0:
            multi.synchronize()  # the warm call: buffers sized, code objects loaded
    multi.synchronize()
    torch.cuda.synchronize()
    print("calls done, rays per call:", rays[:4].tolist())
    multi.close()


if __name__ == "__main__":
    main()
