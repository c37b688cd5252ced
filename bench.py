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
SIMDS = 256 * 4
# the verbatim reference, one thread, N=64, 8 bounces, pixel
# seeds, measured on the survey host: about 11-12.5 Mrays/s per core.
REF_SINGLE_THREAD_MRAYS = (11.0, 12.5)


def ops_per_segment(n_spheres: int) -> int:
    """~21 f32 ops per sphere test + ~70 per segment of shading."""
    return 21 * n_spheres + 70


# BASELINE.json configs: C2 is the headline (1 GPU) and the
# default; C4 is C2 on several GPUs; C3 / C5 are the large single- and
# multi-GPU cases.  C1 is the CPU-only plumbing case (tests, not a bench line).
# "rtw" and "c2in" are frames the primary-ray cull cannot empty:
# RTWeekend (main.cpp:193-268, 482 spheres, sky term: every pixel is traced)
# and C2's 64 spheres seen from inside the sphere cloud (camera 1.0 from the
# look-at point instead of 3.0).
CONFIGS = {
    "c2": dict(width=1920, height=1080, spp=256, spheres=64, bounces=8, scene=1, distance=None),
    "c3": dict(width=3840, height=2160, spp=1024, spheres=64, bounces=8, scene=1, distance=None),
    "c5": dict(width=7680, height=4320, spp=4096, spheres=256, bounces=16, scene=1, distance=None),
    "rtw": dict(width=1920, height=1080, spp=64, spheres=482, bounces=8, scene=2, distance=None),
    "c2in": dict(width=1920, height=1080, spp=256, spheres=64, bounces=8, scene=1, distance=1.0),
}
SCENE_NAMES = {0: "RGB Glass", 1: "Floating Spheres", 2: "RTWeekend"}


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
    p.add_argument("--scene", type=int, choices=(0, 1, 2), help="built-in scene (default: the config's)")
    p.add_argument("--distance", type=float, help="camera distance from the look-at point (default: the scene's)")
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


def make_scene(rt, args):
    """The workload's scene: the first `spheres` spheres of a built-in scene."""
    scene = rt.scene_builtin(args.scene)
    if args.spheres < scene.ScalarSpheres.Count:
        scene = rt.scene_prefix(scene, args.spheres)
    args.spheres = scene.ScalarSpheres.Count
    return scene


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
    o = orc.scene_builtin(args.scene)
    if args.spheres < len(o.spheres):
        o = o.prefix(args.spheres)
    W, H = args.width, args.height
    cam = orc.camera(o, W, H, distance=args.distance)
    t = time.perf_counter()
    _, _, rays1 = orc.render(o, cam, W, H, frames=1, max_bounce=args.bounces, threads=threads, simd=not args.scalar)
    dt1 = time.perf_counter() - t
    k = max(1, min(args.spp, int(args.cpu_seconds / max(dt1, 1e-3))))
    t = time.perf_counter()
    _, _, rays = orc.render(o, cam, W, H, frames=k, max_bounce=args.bounces, threads=threads, simd=not args.scalar)
    dt = time.perf_counter() - t
    # the port counts as the reference's speed only if its single-thread
    # rate is within +-10 % of the verbatim reference's on the probe workload
    # (480x270, 8 spp, N = 64, 8 bounces, one thread: ~11-12.5 Mrays/s on the survey host)
    p = orc.scene_builtin(1).prefix(64)
    pc = orc.camera(p, 480, 270)
    t = time.perf_counter()
    _, _, prays = orc.render(p, pc, 480, 270, frames=8, max_bounce=8, threads=1)
    pdt = time.perf_counter() - t
    single = prays / pdt / 1e6
    lo, hi = REF_SINGLE_THREAD_MRAYS
    return {"value": round(rays / dt / 1e6, 2), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{W}x{H}, {k} spp (of {args.spp}), {args.spheres} spheres, {args.bounces} bounces, "
                      f"{rays} rays in {dt:.2f} s on {threads} threads (oracle/rt_oracle.c, lane-4 SSE "
                      f"RenderTile restatement, pixel seeds)",
            "cpu": cpu_model(), "nproc": os.cpu_count(),
            "single_thread": {"value": round(single, 2), "unit": "Mrays/s",
                              "sample": f"480x270, 8 spp, 64 spheres, 8 bounces, 1 thread, {prays} rays in "
                                        f"{pdt:.2f} s (SURVEY 8d calibration workload)",
                              "reference_single_thread": [lo, hi],
                              "ratio_to_reference": round(single / ((lo + hi) / 2), 3),
                              "within_10pct": bool(0.9 * lo <= single <= 1.1 * hi)}}


def cpu_model() -> str:
    try:
        for line in pathlib.Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


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


def valu_roofline(pmc, kern_ms: float):
    """Executed-work roofline of the trace kernel from its committed PMC record
    (scripts/gpu_pmc.sh -> scripts/pmc_to_json.py, the warm dispatch).

    gfx950 VALU issue, calibrated on scripts/mb_ops (profiles/r02_pmc_calib.txt):
    SQ_ACTIVE_INST_VALU counts one quad-cycle per wave64 VALU instruction (two
    for transcendentals); full-rate ops (f32 add/mul/fma, 32-bit logic) can
    pair, and SQ_ACTIVE_INST_VALU2 counts the quad-cycles in which two issued.
    So a SIMD's VALU is occupied for ACTIVE_INST_VALU - ACTIVE_INST_VALU2
    quad-cycles, out of cycles/4:
        frac = (ACTIVE_INST_VALU - ACTIVE_INST_VALU2) / (1024 SIMDs x cycles / 4)
    (<= 1: a VALU-bound kernel reaches 1 when every SIMD issues every
    quad-cycle).  One quad-cycle slot is the capacity of 128 f32 add/mul lane
    ops (a dual-issued wave64 pair, or one v_pk_*_f32), so `achieved` =
    slots x 128 / live kernel time is in f32 add/mul-equivalent TFLOP/s
    against the 78.6 T peak."""
    c = pmc["counters_per_dispatch"]
    cycles = pmc["gpu_cycles_per_dispatch"]
    slots = c["SQ_ACTIVE_INST_VALU"] - c["SQ_ACTIVE_INST_VALU2"]
    frac = slots / (SIMDS * cycles / 4.0)
    return {"frac": round(frac, 4), "achieved": round(slots * 128 / (kern_ms / 1e3) / 1e12, 2),
            "valu_slots_per_launch": slots,
            "valu_instructions_per_launch": c["SQ_INSTS_VALU"],
            "dual_issue_share": round(2 * c["SQ_ACTIVE_INST_VALU2"] / c["SQ_ACTIVE_INST_VALU"], 4),
            "lane_utilisation": round(c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"]), 4),
            "wave_cycles_issue_stalled": round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 4),
            "salu_per_valu": round(c["SQ_INSTS_SALU"] / c["SQ_INSTS_VALU"], 4),
            "gpu_cycles_per_launch": cycles}


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

    scene = make_scene(rt, args)
    W, H, S, B, N = args.width, args.height, args.spp, args.bounces, args.spheres
    cam = rt.camera_setup(scene, W, H, distance=args.distance)
    dev = rt.Device(gpu)
    dev.upload_scene(scene)
    band_rows = args.band_rows
    bands = args.sim_ranks if (world == 1 and args.sim_ranks > 1) else world
    rows = [rt.band_local_rows(H, band_rows, bands, r) for r in range(bands)]
    maxr = max(rows)
    band_index = args.sim_index if bands != world else rank
    # Two frame slots: frame i's band image is gathered to rank 0 while frame
    # i+1 is traced; rank 0 assembles frame i before frame i+2 reuses its slot.
    # The gather is the C-ABI's RCCL band gather (rt_comm_gather_bands: grouped
    # send/recv to rank 0 over xGMI, then the scatter into the full frame) on a
    # side stream; a rehearsal with every rank on one GPU (BENCH_SHARE_GPU=1,
    # which RCCL refuses) uses a torch.distributed gather.  The timed region
    # ends only after the last frame is assembled on rank 0.
    cur = [torch.zeros(maxr * W, dtype=torch.int32, device="cuda") for _ in range(2)]
    prev = torch.zeros((maxr * W, 4), dtype=torch.float32, device="cuda")
    rays = torch.zeros(1, dtype=torch.int64, device="cuda")  # the tiny code-object launch's counter
    # one pre-zeroed ray counter per step (cold, warm-ups, timed): no counter
    # reset between launches, and every timed step's count is checked after
    ctr = torch.zeros(args.warmup + args.steps + 2, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream()
    comm, gather_kind = None, None
    if world > 1:
        gather_kind = f"torch.distributed {backend} gather + rt_assemble_bands"
        if backend == "nccl" and os.environ.get("BENCH_SHARE_GPU") != "1":
            uid = [rt.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            err = ""
            try:
                comm = rt.Comm(gpu, uid[0], world, rank)
            except rt.RtError as e:
                err = str(e)
            ok = torch.tensor([1 if comm else 0], dtype=torch.int32, device="cuda")
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok.item()) == 1:
                gather_kind = "RCCL grouped send/recv to rank 0 + scatter (rt_comm_gather_bands)"
            else:
                if comm:
                    comm.close()
                comm = None
                gather_kind += f" (rt_comm unavailable: {err or 'on another rank'})"
                print(f"bench.py: {gather_kind}", file=sys.stderr)
    gbuf = full = None
    if world > 1 and rank == 0:
        full = torch.empty(H * W, dtype=torch.int32, device="cuda")
        if comm is None:
            gdev = "cuda" if backend == "nccl" else "cpu"
            gbuf = [torch.empty((world, maxr * W), dtype=torch.int32, device=gdev) for _ in range(2)]
    side = torch.cuda.Stream() if comm else None
    gathered = [None, None]  # per slot: event after its gather on the side stream
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    state = {"n": 0, "pending": None, "c": 0}

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
        if gathered[slot] is not None:  # the gather two frames back has read this slot
            stream.wait_event(gathered[slot])
        c = state["c"]
        state["c"] += 1
        if i is not None:
            ev[i][0].record(stream)
        dev.trace(cam, width=W, height=H, prev_ptr=prev.data_ptr(), cur_ptr=cur[slot].data_ptr(),
                  rays_ptr=ctr[c].data_ptr(), prev_count=0, frames=S, max_bounce=B, simd=not args.scalar,
                  band_rows=band_rows, band_count=bands, band_index=band_index, accum_zero=True,
                  stream=stream.cuda_stream)
        if i is not None:
            ev[i][1].record(stream)
        if world > 1 and comm is not None:
            traced = torch.cuda.Event()
            traced.record(stream)
            side.wait_event(traced)
            comm.gather_bands(cur[slot].data_ptr(), full.data_ptr() if rank == 0 else 0, W, H, 4, band_rows,
                              stream=side.cuda_stream)
            gathered[slot] = torch.cuda.Event()
            gathered[slot].record(side)
        elif world > 1:
            send = cur[slot] if backend == "nccl" else cur[slot].cpu()
            work = dist.gather(send, list(gbuf[slot].unbind(0)) if rank == 0 else None, dst=0, async_op=True)
            finish()
            state["pending"] = (work, slot)

    # Cold launch: the first launch for this camera / scene / geometry runs the
    # primary-ray cull pass and traces in the cull pass's live-first tile order
    # (the heaviest-first order is learned over the next launches).  A tiny
    # launch first loads the code objects, so cold_ms is the render's own cost.
    tiny_prev = torch.zeros((64 * 8, 4), dtype=torch.float32, device="cuda")
    tiny_cur = torch.zeros(64 * 8, dtype=torch.int32, device="cuda")
    dev.trace(cam, width=64, height=8, prev_ptr=tiny_prev.data_ptr(), cur_ptr=tiny_cur.data_ptr(),
              rays_ptr=rays.data_ptr(), frames=1, max_bounce=1, simd=not args.scalar, band_rows=8,
              accum_zero=True, stream=stream.cuda_stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t = time.perf_counter()
    step()
    finish()
    torch.cuda.synchronize()
    cold_ms = (time.perf_counter() - t) * 1e3
    cold_info = dev.last_info()
    for _ in range(max(args.warmup - 1, 0)):
        step()
    finish()
    torch.cuda.synchronize()
    rays_local = int(ctr[state["c"] - 1].item())  # this rank's segments per launch (last warm-up)
    first_timed = state["c"]
    rays_per_step = torch.tensor([rays_local, dev.last_info()["SegmentsFolded"]], dtype=torch.int64,
                                 device="cuda")
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
    info = dev.last_info()
    timed_counts = ctr[first_timed:first_timed + args.steps].tolist()
    if any(n != rays_local for n in timed_counts):
        raise SystemExit(f"bench.py: timed steps counted {timed_counts} segments, expected {rays_local} each")
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
    t = torch.tensor([elapsed, kern_ms, cold_ms], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms_max, cold_ms = float(t[0]), float(t[1]), float(t[2])
    seg_counted, seg_folded = int(rays_per_step[0].item()), int(rays_per_step[1].item())
    total_rays = seg_counted * args.steps
    value = total_rays / elapsed / 1e6

    if bands != world:
        if rank == 0:
            out = {"sim_ranks": bands, "sim_index": band_index, "rank0_rows": rows[band_index],
                   "rank0_kernel_ms": round(kern_ms, 3), "lanes_per_pixel": info["LanesPerPixel"],
                   "rank0_rays": rays_local, "ms_per_step": round(elapsed / args.steps * 1e3, 3)}
            stats = dev.debug_stats()
            if stats:
                out["sched_stats"] = stats
            print(json.dumps(out))
        if comm:
            comm.close()
        dev.close()
        return
    if rank == 0:
        ops = rays_local * ops_per_segment(N)
        achieved_alg = ops / (kern_ms / 1e3) / 1e12
        fb_bytes = rows[0] * W * (16 + 4)  # accumulation + RGBA8 written once per launch
        hbm_achieved = fb_bytes / (kern_ms / 1e3) / 1e9
        preset = all(getattr(args, k) == v for k, v in CONFIGS[args.config].items())
        tag = args.config.upper() if preset else "custom"
        view = "" if args.distance is None else f", camera {args.distance:g} from look-at"
        workload = (f"{tag}: {W}x{H}, {S} spp, {N} spheres, {B} bounces, {'scalar' if args.scalar else 'SIMD'} rules"
                    + ("" if args.scene == 1 else f", {SCENE_NAMES[args.scene]}") + view)
        pmc = pmc_record(workload)
        walks = {0: "any", 1: "groups", 2: "cl1", 3: "cl2", 4: "cl4", 5: "cl1rel", 6: "cl2rel", 7: "cl4rel"}
        kernel = (f"trace_kernel<{'SIMD' if not args.scalar else 'scalar'},SMEM,CULL,{info['LanesPerPixel']},"
                  f"{'one-wave' if info['OneWaveGroups'] else 'four-wave'},walk={walks.get(info['Walk'], '?')}>")
        roof = {"bound": "valu", "achieved": None, "peak": round(VALU_PEAK_TOPS, 1), "unit": "TFLOP/s",
                "frac": None, "traffic": None, "kernel": kernel, "kernel_ms": round(kern_ms, 3)}
        if pmc:
            ex = valu_roofline(pmc, kern_ms)
            roof["achieved"], roof["frac"] = ex.pop("achieved"), ex.pop("frac")
            roof["traffic"] = round(pmc["hbm_bytes_per_dispatch"]) if "hbm_bytes_per_dispatch" in pmc else None
            roof["executed"] = ex
            roof["source"] = pmc["file"]
            roof["note"] = ("frac = VALU issue occupancy of the trace kernel from the committed PMC record: "
                            "(SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) / (1024 SIMDs x GRBM_GUI_ACTIVE/8 / 4); "
                            "achieved = those quad-cycle slots x 128 f32 lane-ops / live kernel ms "
                            "(bench.py valu_roofline). traffic = FETCH_SIZE x2 + WRITE_SIZE (KiB), per launch.")
        roof["frac_algorithmic"] = round(achieved_alg / VALU_PEAK_TOPS, 4)
        roof["achieved_algorithmic"] = round(achieved_alg, 2)
        roof["work_per_launch"] = (f"{rays_local} segments x (21*{N}+70) f32 ops (SURVEY 8d brute force; the "
                                   "kernel skips most sphere tests exactly, so this rate can exceed the peak)")
        roof["hbm"] = {"achieved": round(hbm_achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": round(hbm_achieved / HBM_PEAK_GBS, 6), "bytes_per_launch": fb_bytes}
        seg_traced = seg_counted - seg_folded
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
            "data": f"synthetic ({'first ' + str(N) + ' spheres of ' if args.scene == 1 else ''}the reference's "
                    f"{SCENE_NAMES[args.scene]} scene, {'default camera' if args.distance is None else 'camera moved'}"
                    ", per-(pixel,frame) PCG seeds)",
            "config": {"workload": workload,
                       "width": W, "height": H, "spp": S, "spheres": N, "bounces": B, "scene": args.scene,
                       "parallelism": f"{world} GPU x interleaved {band_rows}-row bands",
                       **({"gather": gather_kind} if world > 1 else {}),
                       "rays_per_step": seg_counted},
            "segments": {"counted_per_step": seg_counted, "traced_per_step": seg_traced,
                         "counted_equal_every_timed_step": True,  # one counter per step, checked above
                         "folded_per_step": seg_folded,
                         "traced_mrays_per_s": round(seg_traced * args.steps / elapsed / 1e6, 1),
                         "note": "every segment is counted as the reference counts it (main.cpp:390); 'folded' "
                                 "ones belong to pixels whose every sample provably misses (dead tiles), folded "
                                 "by the empty-tile kernel instead of traced"},
            "cold_ms": round(cold_ms, 3),
            "cold": {"ms": round(cold_ms, 3), "cull_pass": bool(cold_info["CullPassRan"]),
                     "note": "first launch for this camera/scene/geometry (cull pass + untrained tile order), "
                             "wall clock incl. its host synchronisation; the timed steps reuse the cull masks "
                             "and the learned heaviest-first order"},
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
    if comm:
        comm.close()
    dev.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
