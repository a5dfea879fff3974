"""Sharded multi-GPU MSM: one process per GPU, partial points joined over RCCL/xGMI.

MSM is linear in the (point, scalar) vector, so every rank computes the MSM of a contiguous
1/world slice of the inputs on its own GPU (no data-path collective) and the per-rank partial
points (projective X|Y|T|Z, 128 B each) are all-gathered and added on rank 0 — the
generalisation of the reference's CPU/GPU co-compute split and its single affine join
(src/submission/submission.ts:116-154, msm-wasm/src/lib.rs:240-253).  The join is an elliptic
curve addition, not an RCCL reduction op, hence all_gather + host add.  The MSM is also a sum
over its signed-digit windows, so a points x windows split (P point shards times Q window ranges,
P Q = world: split_part) joins the same way and gives each GPU fewer buckets per entry
(DESIGN.md §6).
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) slice of n points owned by `rank` (sizes differ by at most 1)."""
    return n * rank // world, n * (rank + 1) // world


# Window width of a windows split (every GPU must cut the same windows): c = 15 measured best for
# 2^20 points as 4 point shards x 2 window ranges over 8 GPUs (slowest GPU 0.203 ms per MSM against
# 0.212 at c = 16 and 0.226 at c = 14; profiles/r4/split_probe.jsonl).
SPLIT_WINDOW_BITS = 15


# Window splits cut in half windows (MSM_FLAG_HALF_WINDOWS): c = 15's 17 main windows then split
# 8.5 / 8.5 instead of 8 / 9 between two ranges.
SPLIT_HALF_WINDOWS = True


def window_ranges(wm: int, q: int, halves: bool = False):
    """q contiguous ranges of an MSM's wm signed-digit windows: the wm - 1 main windows balanced,
    the overflow window (empty for canonical scalars) with the top range.  With `halves` the
    ranges are counted in half windows, (lo, hi, 2) over [0, 2 wm), so an odd number of main
    windows still splits evenly."""
    u = 2 if halves else 1
    main = u * (wm - 1)
    edges = [round(main * i / q) for i in range(q + 1)]
    edges[-1] = u * wm
    return [(a, b, 2) if halves else (a, b) for a, b in zip(edges[:-1], edges[1:])]


def parse_split(split: str, world: int) -> Tuple[int, int]:
    """"PxQ" -> (P, Q) with P * Q == world: P point shards times Q window ranges.
    "points" is world x 1 (every GPU a 1/world of the points, all windows)."""
    if split in ("", "points", "auto"):
        return world, 1
    p, q = (int(v) for v in split.lower().split("x"))
    if p < 1 or q < 1 or p * q != world:
        raise ValueError(f"split {split!r} does not factor {world} GPUs as points x windows")
    return p, q


def split_part(n: int, rank: int, world: int, split: str = "points"):
    """What GPU `rank` computes of an n-point MSM under a points x windows split: its point shard
    [lo, hi), its window range (None: all windows; (lo, hi, 2) in half windows) and the window
    width the range refers to (None: the library's own choice).  Rank r takes point shard r // Q and window range r % Q; the partials
    of all ranks sum to the MSM."""
    from . import window_count

    P, Q = parse_split(split, world)
    lo, hi = shard_range(n, rank // Q, P)
    if Q == 1:
        return lo, hi, None, None
    c = SPLIT_WINDOW_BITS
    return lo, hi, window_ranges(window_count(c), Q, SPLIT_HALF_WINDOWS)[rank % Q], c


def gather_partials(partial_xyzt_be: np.ndarray, device=None, group=None) -> np.ndarray:
    """all_gather this rank's partial(s) — one [32] or a batch [K, 32] — in ONE collective;
    returns [world, 32] (or [world, K, 32]) u32 on every rank."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    t = torch.from_numpy(np.ascontiguousarray(partial_xyzt_be, dtype=np.uint32).view(np.int32).copy())
    if device is not None:
        t = t.to(device)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t, group=group)
    return np.stack([o.cpu().numpy().view(np.uint32) for o in out])


def combine_batch_on_root(parts: np.ndarray, rank: int, root: int = 0):
    """parts [world, K, 32]: rank `root` joins each of the K MSMs' world partials in one libmsm
    call (one field inversion for the batch)."""
    if rank != root:
        return None
    from . import combine_partials_many

    return combine_partials_many(parts)


def combine_on_root(parts: np.ndarray, rank: int, root: int = 0) -> Optional[Tuple[int, int]]:
    """Rank `root` adds the gathered partials (libmsm host EC adds) into the affine result."""
    if rank != root:
        return None
    from . import combine_partials

    return combine_partials(parts)


def sharded_msm_device(d_points, d_scalars, n_local: int, rank: int, device=None, window_size=None,
                       group=None, windows=None) -> Optional[Tuple[int, int]]:
    """One sharded MSM step: local partial on this rank's GPU, gather, join on rank 0."""
    from . import compute_msm_device_partial

    part = compute_msm_device_partial(d_points, d_scalars, n_local, window_size=window_size, windows=windows)
    parts = gather_partials(part, device=device, group=group)
    return combine_on_root(parts, rank)


def sharded_msm_many_device(points_list, scalars_list, n_local: int, rank: int, device=None, window_size=None,
                            group=None, windows=None):
    """K sharded MSMs, pipelined: each rank computes its K partials through libmsm's pipelined
    entry (msm_compute_many_device_partial; `windows` = its window range under a points x windows
    split), then ONE all_gather ships all K x 128 B and rank 0 joins them — the exchange is batched
    across the K independent MSMs."""
    from . import compute_msm_many_device_partial

    parts = compute_msm_many_device_partial(points_list, scalars_list, n_local, window_size=window_size,
                                            windows=windows)
    gathered = gather_partials(parts, device=device, group=group)
    return combine_batch_on_root(gathered, rank)
