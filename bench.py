"""bench.py — Mrays/s of the MI355X sphere trace path (BASELINE.json metric).

Workload (BASELINE.json configs[1], "C2"): 1920x1080, 256 spp, 64 spheres
(first 64 of the reference's Floating Spheres scene, main.cpp:96-167, with
that scene's default camera), 8 bounces, per-(pixel, frame) PCG seeds.
One step = one complete 256-spp render of the frame: every pixel's 256
progressive frames folded into the running mean and the sRGB RGBA8 stored;
for N > 1 GPUs the frame is dealt out in interleaved 8-row bands (one rank
per GPU) and gathered to rank 0 over RCCL, then assembled (strong scaling:
the total work per step is fixed).  Rays = bounce segments counted as the
reference counts them (main.cpp:390).

Run:  python bench.py [--gpus N --steps K --warmup W]
      python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

# MI355X constants (/opt/skills/guides/MI355X_MICROARCH.md, chip table):
# a SIMD retires 16 f32 lanes/clk (a wave64 VALU op every 4 clk), 32 with
# packed v_pk_{add,mul}_f32: 256 CUs x 4 SIMDs x 32 x 2.4 GHz = 78.6 T f32
# add/mul ops/s (the 157 TFLOP/s spec figure counts an FMA as 2; the path
# cannot fuse: every op must round separately to match the reference).
# HBM3E 8 TB/s.
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
HBM_PEAK_GBS = 8000.0


def ops_per_segment(n_spheres: int) -> int:
    """~21 f32 ops per sphere test + ~70 per segment of shading."""
    return 21 * n_spheres + 70


# BASELINE.json configs: C2 is the headline (1 GPU) and the
# default; C4 is C2 on several GPUs; C3 / C5 are the large single- and
# multi-GPU cases.  C1 is the CPU-only plumbing case (tests, not a bench line).
CONFIGS = {
    "c2": dict(width=1920, height=1080, spp=256, spheres=64, bounces=8),
    "c3": dict(width=3840, height=2160, spp=1024, spheres=64, bounces=8),
    "c5": dict(width=7680, height=4320, spp=4096, spheres=256, bounces=16),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", choices=sorted(CONFIGS), default="c2", help="BASELINE.json workload preset")
    p.add_argument("--width", type=int)
    p.add_argument("--height", type=int)
    p.add_argument("--spp", type=int)
    p.add_argument("--spheres", type=int)
    p.add_argument("--bounces", type=int)
    p.add_argument("--scalar", action="store_true", help="RenderTileScalar rules instead of RenderTile")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target wall time of the CPU baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--band-rows", type=int, default=8, help="rows per interleaved band (multiple of 8)")
    p.add_argument("--verify", action="store_true",
                   help="after timing, rank 0 re-renders the whole frame alone and checks the gathered frame is "
                        "bit-identical (adds 'verified' to the line)")
    p.add_argument("--sim-ranks", type=int, default=0,
                   help="diagnostic (1 GPU): trace only band residue --sim-index of this many ranks, i.e. one rank's "
                        "share of a multi-GPU frame; prints that rank's kernel time, not a bench line")
    p.add_argument("--sim-index", type=int, default=0, help="band residue (rank) traced by --sim-ranks")
    a = p.parse_args()
    for k, v in CONFIGS[a.config].items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    return a


def cpu_baseline(args, n_rays_gpu_step: int):
    """The oracle (C restatement of RenderTile, lane-4 SSE, pthread 32x32 tile
    queue) on this host's cores, on a bounded sample of the same workload:
    the full 1920x1080 frame, 64 spheres, 8 bounces, k spp, k chosen from a
    1-spp calibration so the sample takes ~--cpu-seconds."""
    from oracle import oracle as orc
    threads = orc.cpu_threads()
    env_cap = os.environ.get("OMP_NUM_THREADS")
    if env_cap and env_cap.isdigit():
        threads = min(threads, int(env_cap))
    o = orc.scene_builtin(1).prefix(args.spheres)
    W, H = args.width, args.height
    cam = orc.camera(o, W, H)
    t = time.perf_counter()
    _, _, rays1 = orc.render(o, cam, W, H, frames=1, max_bounce=args.bounces, threads=threads, simd=not args.scalar)
    dt1 = time.perf_counter() - t
    k = max(1, min(args.spp, int(args.cpu_seconds / max(dt1, 1e-3))))
    t = time.perf_counter()
    _, _, rays = orc.render(o, cam, W, H, frames=k, max_bounce=args.bounces, threads=threads, simd=not args.scalar)
    dt = time.perf_counter() - t
    return {"value": round(rays / dt / 1e6, 2), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{W}x{H}, {k} spp (of {args.spp}), {args.spheres} spheres, {args.bounces} bounces, "
                      f"{rays} rays in {dt:.2f} s on {threads} threads (oracle/rt_oracle.c, lane-4 SSE "
                      f"RenderTile restatement, pixel seeds)"}


def lanes_per_pixel(band_pixels: int, frames: int) -> int:
    """The P rt_trace picks for a band (rt_host.cpp rt_trace; RT_LANES_PER_PIXEL overrides), for the line's label."""
    import torch
    forced = os.environ.get("RT_LANES_PER_PIXEL")
    if forced in ("1", "2", "4", "8", "16", "32"):
        return int(forced)
    cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    p = 4 if band_pixels >= cus * 6144 else 8 if band_pixels >= cus * 1536 else 16
    while p > 1 and p // 2 >= frames:
        p //= 2
    return p


def pmc_record(workload: str):
    """The newest committed rocprofv3 --pmc record of this workload
    (profiles/rNN_*_pmc.json, written by scripts/pmc_to_json.py)."""
    for f in sorted((ROOT / "profiles").glob("r*_pmc.json"), reverse=True):
        try:
            rec = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        if rec.get("workload") == workload:
            rec["file"] = f"profiles/{f.name}"
            return rec
    return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import __graft_entry__ as graft

    rt = graft.load_package()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # BENCH_BACKEND=gloo + BENCH_SHARE_GPU=1: rehearsal of the multi-rank
    # path with every rank on cuda:0 (a 1-GPU box); the real runs use RCCL
    backend = os.environ.get("BENCH_BACKEND", "nccl")
    gpu = 0 if os.environ.get("BENCH_SHARE_GPU") == "1" else local
    torch.cuda.set_device(gpu)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)

    W, H, S, B, N = args.width, args.height, args.spp, args.bounces, args.spheres
    scene = rt.scene_prefix(rt.scene_builtin(1), N)
    cam = rt.camera_setup(scene, W, H)
    dev = rt.Device(gpu)
    dev.upload_scene(scene)
    band_rows = args.band_rows
    bands = args.sim_ranks if (world == 1 and args.sim_ranks > 1) else world
    rows = [rt.band_local_rows(H, band_rows, bands, r) for r in range(bands)]
    maxr = max(rows)
    band_index = args.sim_index if bands != world else rank
    # Two frame slots: frame i's band image is gathered to rank 0 (RCCL, async)
    # while frame i+1 is traced; rank 0 assembles frame i before frame i+2
    # reuses its slot.  The timed region ends only after the last frame is
    # assembled on rank 0.
    cur = [torch.zeros(maxr * W, dtype=torch.int32, device="cuda") for _ in range(2)]
    prev = torch.zeros((maxr * W, 4), dtype=torch.float32, device="cuda")
    rays = torch.zeros(1, dtype=torch.int64, device="cuda")
    gbuf = full = None
    if world > 1 and rank == 0:
        gdev = "cuda" if backend == "nccl" else "cpu"
        gbuf = [torch.empty((world, maxr * W), dtype=torch.int32, device=gdev) for _ in range(2)]
        full = torch.empty(H * W, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    state = {"n": 0, "pending": None}

    def finish():  # frame whose gather is in flight -> assembled on rank 0
        if state["pending"] is None:
            return
        work, slot = state["pending"]
        state["pending"] = None
        work.wait()
        if rank == 0:
            src = gbuf[slot] if backend == "nccl" else gbuf[slot].to("cuda")
            rt.assemble_bands(src.data_ptr(), maxr * W * 4, full.data_ptr(), W, H, 4, band_rows, world,
                              stream=stream.cuda_stream)

    def step(i=None):
        slot = state["n"] % 2
        state["n"] += 1
        rays.zero_()
        if i is not None:
            ev[i][0].record(stream)
        dev.trace(cam, width=W, height=H, prev_ptr=prev.data_ptr(), cur_ptr=cur[slot].data_ptr(),
                  rays_ptr=rays.data_ptr(), prev_count=0, frames=S, max_bounce=B, simd=not args.scalar,
                  band_rows=band_rows, band_count=bands, band_index=band_index, accum_zero=True,
                  stream=stream.cuda_stream)
        if i is not None:
            ev[i][1].record(stream)
        if world > 1:  # RCCL gather of the band images to rank 0 over xGMI, then assembly
            send = cur[slot] if backend == "nccl" else cur[slot].cpu()
            work = dist.gather(send, list(gbuf[slot].unbind(0)) if rank == 0 else None, dst=0, async_op=True)
            finish()
            state["pending"] = (work, slot)

    for _ in range(max(args.warmup, 1)):
        step()
    finish()
    torch.cuda.synchronize()
    rays_per_step = torch.tensor([int(rays.item())], dtype=torch.int64, device="cuda")
    if world > 1:
        dist.all_reduce(rays_per_step)
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    finish()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    verified = None
    if args.verify and bands == world:  # rank 0 renders the whole frame alone and compares
        if rank == 0:
            ref_cur = torch.zeros(H * W, dtype=torch.int32, device="cuda")
            ref_prev = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
            ref_rays = torch.zeros(1, dtype=torch.int64, device="cuda")
            dev.trace(cam, width=W, height=H, prev_ptr=ref_prev.data_ptr(), cur_ptr=ref_cur.data_ptr(),
                      rays_ptr=ref_rays.data_ptr(), prev_count=0, frames=S, max_bounce=B, simd=not args.scalar,
                      band_rows=band_rows, band_count=1, band_index=0, accum_zero=True, stream=stream.cuda_stream)
            torch.cuda.synchronize()
            got = full if world > 1 else cur[(state["n"] - 1) % 2]
            verified = bool(torch.equal(got, ref_cur))
        if world > 1:
            dist.barrier()
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms_max = float(t[0]), float(t[1])
    total_rays = int(rays_per_step.item()) * args.steps
    value = total_rays / elapsed / 1e6

    if bands != world:
        if rank == 0:
            print(json.dumps({"sim_ranks": bands, "sim_index": band_index, "rank0_rows": rows[band_index],
                              "rank0_kernel_ms": round(kern_ms, 3),
                              "rank0_rays": int(rays.item()), "ms_per_step": round(elapsed / args.steps * 1e3, 3)}))
        dev.close()
        return
    if rank == 0:
        rays_local = int(rays.item())  # rank 0's rays per launch
        ops = rays_local * ops_per_segment(N)
        achieved = ops / (kern_ms / 1e3) / 1e12
        fb_bytes = rows[0] * W * (16 + 4)  # accumulation + RGBA8 written once per launch
        hbm_achieved = fb_bytes / (kern_ms / 1e3) / 1e9
        preset = all(getattr(args, k) == v for k, v in CONFIGS[args.config].items())
        tag = args.config.upper() if preset else "custom"
        workload = f"{tag}: {W}x{H}, {S} spp, {N} spheres, {B} bounces, {'scalar' if args.scalar else 'SIMD'} rules"
        pmc = pmc_record(workload)
        roof = {"bound": "valu", "achieved": round(achieved, 2), "peak": round(VALU_PEAK_TOPS, 1),
                "unit": "TFLOP/s", "frac": round(achieved / VALU_PEAK_TOPS, 4),
                "traffic": round(pmc["hbm_bytes_per_dispatch"]) if pmc and "hbm_bytes_per_dispatch" in pmc else None,
                "kernel": f"trace_kernel<{'SIMD' if not args.scalar else 'scalar'},SMEM,CULL,{lanes_per_pixel(rows[0] * W, S)}>",
                "kernel_ms": round(kern_ms, 3),
                "work_per_launch": f"{rays_local} segments x (21*{N}+70) f32 ops (SURVEY 8d, brute force)",
                "note": "algorithmic ops count every sphere for every segment; the kernel culls sphere groups "
                        "for primary rays exactly, so it executes fewer ops and frac may exceed 1. The "
                        "executed-instruction view is 'issue' (PMC).",
                "hbm": {"achieved": round(hbm_achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(hbm_achieved / HBM_PEAK_GBS, 6), "bytes_per_launch": fb_bytes}}
        if pmc:
            roof["issue"] = {k: round(pmc[k], 4) for k in ("valu_inst_per_simd_cycle", "valu_lane_utilisation") if k in pmc}
            roof["issue"]["ceiling"] = "0.5 full-rate / 0.25 half-rate (v_pk_*, int mul) wave-instr per SIMD-cycle"
            roof["issue"]["source"] = pmc["file"]
            roof["traffic_source"] = pmc["file"] + " (FETCH_SIZE x2 + WRITE_SIZE, per launch)"
        line = {
            "metric": f"Mrays/sec at {W}x{H}, {S}spp, {B} bounces, {N} spheres",
            "value": round(value, 1),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic (first {N} spheres of the reference's Floating Spheres scene, default camera, "
                    "per-(pixel,frame) PCG seeds)",
            "config": {"workload": workload,
                       "width": W, "height": H, "spp": S, "spheres": N, "bounces": B,
                       "parallelism": f"{world} GPU x interleaved {band_rows}-row bands" +
                                      (" + RCCL gather" if world > 1 else ""),
                       "rays_per_step": int(rays_per_step.item())},
            "roofline": roof,
        }
        stats = dev.debug_stats()
        if stats:
            line["sched_stats"] = stats
        if verified is not None:
            line["verified"] = verified
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args, total_rays)
        print(json.dumps(line), flush=True)
    dev.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
