"""Multi-rank path on CPU (gloo, world_size 2 and 3): band ownership, the
padded rank-0 gather and the band assembly used by bench.py's N-GPU run,
with the oracle tracing each rank's bands.  The assembled image must equal a
single full render bit for bit (SURVEY §8e required check)."""
import os
import pathlib
import socket
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
W, H, S, B, N, BAND = 48, 100, 2, 6, 32, 32


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, str(ROOT))
    import __graft_entry__ as graft
    from oracle import oracle as orc
    graft.load_package()
    mg = __import__("simd_ray_tracer_amd.multigpu", fromlist=["x"])
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    o = orc.scene_builtin(1).prefix(N)
    cam = orc.camera(o, W, H)
    rows, maxr = mg.band_plan(H, BAND, world)
    local_cur = np.zeros((maxr, W), np.uint32)
    local_prev = np.zeros((maxr, W, 4), np.float32)
    rays = 0
    lr = 0
    for y0, y1 in mg.owned_rows(H, BAND, world, rank):
        p, c, r = orc.render(o, cam, W, H, frames=S, max_bounce=B, rows=(y0, y1))
        local_cur[lr:lr + y1 - y0] = c.reshape(H, W)[y0:y1]
        local_prev[lr:lr + y1 - y0] = p.reshape(H, W, 4)[y0:y1]
        lr += y1 - y0
        rays += r
    assert lr == rows[rank]
    cur_t = torch.from_numpy(local_cur.view(np.int32).reshape(-1))
    prev_t = torch.from_numpy(local_prev.reshape(-1, 4))
    g_cur = mg.gather_to_rank0(dist, cur_t, world, rank)
    g_prev = mg.gather_to_rank0(dist, prev_t, world, rank)
    tot = torch.tensor([rays], dtype=torch.int64)
    dist.all_reduce(tot)
    if rank == 0:
        cur = mg.assemble_numpy(torch.cat(g_cur).numpy().view(np.uint32), W, H, BAND, world, maxr)
        prev = mg.assemble_numpy(torch.cat(g_prev).numpy(), W, H, BAND, world, maxr)
        np.save(os.path.join(out_dir, "cur.npy"), cur)
        np.save(os.path.join(out_dir, "prev.npy"), prev)
        np.save(os.path.join(out_dir, "rays.npy"), tot.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_band_gather_matches_single_render(orc, tmp_path, world):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    o = orc.scene_builtin(1).prefix(N)
    prev, cur, rays = orc.render(o, orc.camera(o, W, H), W, H, frames=S, max_bounce=B)
    assert np.array_equal(np.load(tmp_path / "cur.npy"), cur)
    assert np.array_equal(np.load(tmp_path / "prev.npy").view(np.uint32), prev.view(np.uint32))
    assert int(np.load(tmp_path / "rays.npy")[0]) == rays
