"""Multi-GPU sharding of a block batch (one process per GPU).

The batch is embarrassingly parallel: every block's CRC is independent
(util/crc32c.cc:487 takes one block; callers loop per block,
table/table_builder.cc:202).  So a batch is split into contiguous block ranges,
one per rank, with no data-path collective; RCCL (torch.distributed "nccl")
carries only the barrier and the max-over-ranks elapsed time, and optionally
a gather of the 4-byte CRCs for verification outside the timed region.
"""
from __future__ import annotations

import numpy as np


def shard_blocks(n_blocks: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous range [lo, hi) of ceil(n/world) blocks for `rank`."""
    per = (n_blocks + world - 1) // world
    lo = min(n_blocks, rank * per)
    return lo, min(n_blocks, lo + per)


def shard_by_bytes(lengths: np.ndarray, world: int, rank: int) -> tuple[int, int]:
    """Contiguous range balanced by cumulative bytes (variable-length batches):
    rank r takes the blocks whose byte prefix starts in [r*T/world, (r+1)*T/world)."""
    lengths = np.asarray(lengths, dtype=np.uint64)
    if lengths.size == 0:
        return 0, 0
    starts = np.concatenate(([0], np.cumsum(lengths)[:-1])).astype(np.uint64)
    total = int(lengths.sum())
    lo_b = total * rank // world
    hi_b = total * (rank + 1) // world
    lo = int(np.searchsorted(starts, lo_b, side="left"))
    hi = int(np.searchsorted(starts, hi_b, side="left")) if rank < world - 1 else lengths.size
    return lo, hi


def max_over_ranks(x: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_crcs(local: np.ndarray, counts: list[int], device=None) -> np.ndarray:
    """All-gather per-rank CRC slices (uint32) into the full batch order."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    m = max(counts)
    buf = np.zeros(m, dtype=np.uint32)
    buf[:local.size] = local
    t = torch.from_numpy(buf.view(np.int32)).to(device if device is not None else "cpu")
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return np.concatenate([p.cpu().numpy().view(np.uint32)[:c] for p, c in zip(parts, counts)])
