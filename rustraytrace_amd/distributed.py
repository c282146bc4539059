"""Multi-GPU image partitioning and the final gather.

One process per GPU. The scene and BVH are replicated (KB-sized); the work is split one of two
ways, with no data-path collective until the single final exchange:

* rows    (strong scaling, C3): row bands (`balanced_band`: 15 rows for C3 at 2/4/8 ranks)
          dealt round-robin over ranks (rank r owns bands b with b % n == r), which balances
          cheap sky rows against expensive ground rows.
          Rank 0 receives every rank's rows and places them — the image is bit-identical to a
          1-GPU render because every pixel is computed by the same lane program from the same
          (seed, pixel, sample) keys.
* samples (weak scaling, bench): every rank renders the whole frame over its own sample range
          [s_r, s_{r+1}); rank 0 sums the partial accums in rank order (deterministic).

The gather uses torch.distributed (backend "nccl" = RCCL over xGMI on the GPU box, "gloo" on
CPU in tests). RCCL has no Gather primitive: torch lowers dist.gather to grouped send/recv.
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

import numpy as np


def band_rows(height: int, band: int, rank: int, n_ranks: int) -> np.ndarray:
    """Global image rows owned by `rank` (mirror of rrt_tile_row_index, rrt_host.cpp)."""
    rows = []
    n_bands = (height + band - 1) // band
    for b in range(rank, n_bands, n_ranks):
        rows.extend(range(b * band, min((b + 1) * band, height)))
    return np.asarray(rows, dtype=np.int64)


def balanced_band(height: int, n_ranks: int, max_band: int = 16, min_band: int = 8) -> int:
    """Rows per band: the largest b in [min_band, max_band] with height % (b * n_ranks) == 0, so
    every rank owns the same number of bands and rows; max_band when no such b exists.

    C3 (2160 rows) at 16-row bands leaves 135 bands: at 2/4/8 ranks the busiest rank owns 0.74 %
    more rows than the mean, and the frame waits for it. 15-row bands give 144 = 8 x 18. The image
    does not depend on the band height (every pixel is keyed by its global index)."""
    for b in range(max_band, min_band - 1, -1):
        if height % (b * n_ranks) == 0:
            return b
    return max_band


def sample_range(spp_per_rank: int, rank: int) -> tuple:
    return rank * spp_per_rank, (rank + 1) * spp_per_rank


def gather_rows(local, height: int, band: int, dist, group=None, dst: int = 0):
    """Gather every rank's row-band accum (rows_r, W, 4) to `dst` and reassemble (H, W, 4).

    `local` is a torch tensor on the rank's device (cuda for RCCL, cpu for gloo). Ranks own
    different row counts; tiles are padded to the max so one gather moves them all."""
    import torch

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    counts = [len(band_rows(height, band, r, world)) for r in range(world)]
    rmax = max(counts)
    W = local.shape[1]
    padded = torch.zeros((rmax, W, 4), dtype=local.dtype, device=local.device)
    padded[: local.shape[0]] = local
    bufs = [torch.empty_like(padded) for _ in range(world)] if rank == dst else None
    dist.gather(padded, gather_list=bufs, dst=dst, group=group)
    if rank != dst:
        return None
    img = torch.empty((height, W, 4), dtype=local.dtype, device=local.device)
    for r in range(world):
        idx = torch.as_tensor(band_rows(height, band, r, world), device=local.device)
        img[idx] = bufs[r][: counts[r]]
    return img


def gather_sample_ranges(local, dist, group=None, dst: int = 0, out=None):
    """Gather every rank's full-frame partial accum to `dst` and sum them in rank order."""
    import torch

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    bufs = [torch.empty_like(local) for _ in range(world)] if rank == dst else None
    dist.gather(local, gather_list=bufs, dst=dst, group=group)
    if rank != dst:
        return None
    total = out if out is not None else torch.empty_like(local)
    total.copy_(bufs[0])
    for b in bufs[1:]:
        total += b  # fixed order: rank 0, 1, ..., n-1
    return total


def render_rows_distributed(render_tile: Callable[[int, int, int], "object"], height: int, band: int, dist,
                            group=None):
    """render_tile(band, rank, n_ranks) -> local (rows_r, W, 4) tensor; returns the image on rank 0."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    return gather_rows(render_tile(band, rank, world), height, band, dist, group)
