"""Multi-GPU image partitioning and the final gather.

One process per GPU. The scene and BVH are replicated (KB-sized); the work is split one of two
ways, with no data-path collective until the single final exchange:

* rows    (strong scaling, C3): row bands (`balanced_band`: 10 rows for C3 at 2/4/8 ranks)
          dealt over ranks in serpentine order (`band_owner`: period p = b // n holds one band
          per rank, ranks 0..n-1 in even periods and n-1..0 in odd ones), which balances cheap
          sky rows against expensive ground rows. Plain round-robin (b % n) gave every rank the
          same offset in every period, so rank n-1 always drew the lowest band of a period: C3's
          render time rose monotonically with rank, 1.96 % max over mean at 8 ranks.
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


def band_owner(b: int, n_ranks: int) -> int:
    """Rank owning row band b (include/rrt_hip.h RrtTile): serpentine over periods of n_ranks bands."""
    p, slot = divmod(b, n_ranks)
    return n_ranks - 1 - slot if p & 1 else slot


def band_rows(height: int, band: int, rank: int, n_ranks: int) -> np.ndarray:
    """Global image rows owned by `rank`, in the tile's local order (mirror of rrt_tile_row_index,
    rrt_host.cpp): its p-th band is band p * n + (rank, or n - 1 - rank in odd periods)."""
    rows = []
    n_bands = (height + band - 1) // band
    for p in range((n_bands + n_ranks - 1) // n_ranks):
        b = p * n_ranks + (n_ranks - 1 - rank if p & 1 else rank)
        if b < n_bands:
            rows.extend(range(b * band, min((b + 1) * band, height)))
    return np.asarray(rows, dtype=np.int64)


def balanced_band(height: int, n_ranks: int, max_band: int = 16, min_band: int = 10) -> int:
    """Rows per band: every rank must own the same number of bands and rows, so the candidates are
    the b with height % (b * n_ranks) == 0. Among those in [min_band, max_band] the smallest (the
    most bands per rank), else the largest in [8, min_band), else max_band.

    C3 (2160 rows) at 16-row bands left 135 bands: at 2/4/8 ranks the busiest rank owned 0.74 %
    more rows than the mean. With equal counts what is left is how evenly each rank's bands sample
    the image's row costs (sky rows are cheap, ground rows expensive): at 8 ranks, serpentine
    dealing, 15-row bands (18 per rank) put the slowest rank 1.17 % over the mean, 10-row bands
    (27 per rank) 0.21 %, 9-row 0.28 %; below 10 rows the 8-row work tiles straddle more band
    edges and the sum of the ranks' times grows (+0.2 % at 9, +0.3 % at 6, +0.7 % at 5;
    tools/c3_rank_balance.py). At 2 and 4 ranks every height from 9 to 15 is within 0.3 %. The
    image does not depend on the band height (every pixel is keyed by its global index)."""
    fits = [b for b in range(8, max_band + 1) if height % (b * n_ranks) == 0]
    upper = [b for b in fits if b >= min_band]
    if upper:
        return min(upper)
    return max(fits) if fits else max_band


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
