"""Per-GPU band dispatch and the rank-0 gather.

The image is cut into row bands (bench.py uses 8 rows; the tests also use
the reference's 32-row TileSize, main.cpp:9) dealt round-robin to the
ranks: band b -> rank b % world.  Each rank traces its bands into a compact
local image (rt_band_local_rows x W), pads it to the largest rank's size,
and one collective gather (RCCL over xGMI on the GPU, gloo in the CPU tests)
brings every rank's buffer to rank 0, which scatters the bands back into
place (rt_assemble_bands on the GPU).  Samples are never split across
ranks: the running-mean fold is order dependent (main.cpp:487).
"""
from __future__ import annotations

import numpy as np


def band_plan(height: int, band_rows: int, world: int):
    """Rows per rank for the interleaved band deal, and the padded maximum."""
    bands = (height + band_rows - 1) // band_rows
    rows = [0] * world
    for b in range(bands):
        rows[b % world] += min(band_rows, height - b * band_rows)
    return rows, max(rows)


def row_owner_map(height: int, band_rows: int, world: int) -> np.ndarray:
    """For every image row y: (owner rank, row index inside the owner's compact image)."""
    out = np.zeros((height, 2), np.int64)
    for y in range(height):
        b = y // band_rows
        out[y, 0] = b % world
        out[y, 1] = (b // world) * band_rows + y % band_rows
    return out


def owned_rows(height: int, band_rows: int, world: int, rank: int):
    """Global row ranges [y0, y1) owned by `rank`, in compact-image order."""
    bands = (height + band_rows - 1) // band_rows
    return [(b * band_rows, min(height, (b + 1) * band_rows)) for b in range(rank, bands, world)]


def gather_to_rank0(dist, local, world: int, rank: int):
    """Collective gather of equally sized (padded) per-rank buffers to rank 0.
    Returns the list of per-rank buffers on rank 0, None elsewhere."""
    if world == 1:
        return [local]
    bufs = [local.new_empty(local.shape) for _ in range(world)] if rank == 0 else None
    dist.gather(local, bufs, dst=0)
    return bufs


def assemble_numpy(stacked: np.ndarray, width: int, height: int, band_rows: int, world: int, max_rows: int):
    """Reference (host) version of rt_assemble_bands: stacked is (world*max_rows*width, ...)."""
    m = row_owner_map(height, band_rows, world)
    per_rank = stacked.reshape(world, max_rows, width, *stacked.shape[1:])
    return per_rank[m[:, 0], m[:, 1]].reshape(height * width, *stacked.shape[1:])
