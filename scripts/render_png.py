"""Render a built-in scene on the GPU and write the frame (output path).

usage: python scripts/render_png.py out.png [--scene 1] [--spheres N] [--width 1920] [--height 1080]
                                     [--spp 64] [--bounces 8] [--scalar]
One rt_trace launch of all --spp frames (pixel seeds) into a device-resident
accumulation, the RGBA8 frame copied to the host and written by
rt_image_write_png / rt_image_write_ppm (by suffix), on-screen orientation."""
import argparse
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("out")
    p.add_argument("--scene", type=int, default=1)
    p.add_argument("--spheres", type=int)
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--spp", type=int, default=64)
    p.add_argument("--bounces", type=int, default=8)
    p.add_argument("--scalar", action="store_true")
    a = p.parse_args()
    import torch
    import __graft_entry__ as graft
    rt = graft.load_package()
    scene = rt.scene_builtin(a.scene)
    if a.spheres:
        scene = rt.scene_prefix(scene, a.spheres)
    W, H = a.width, a.height
    cam = rt.camera_setup(scene, W, H)
    dev = rt.Device(0)
    dev.upload_scene(scene)
    prev = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
    cur = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    rays = torch.zeros(1, dtype=torch.int64, device="cuda")
    dev.trace(cam, width=W, height=H, prev_ptr=prev.data_ptr(), cur_ptr=cur.data_ptr(), rays_ptr=rays.data_ptr(),
              frames=a.spp, max_bounce=a.bounces, simd=not a.scalar, accum_zero=True,
              stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    img = cur.cpu().numpy().view("uint32").reshape(H, W).copy()
    rt.write_image(img, a.out)
    dev.close()
    print(f"{a.out}: {W}x{H}, {a.spp} spp, {int(rays.item())} rays")


if __name__ == "__main__":
    main()
