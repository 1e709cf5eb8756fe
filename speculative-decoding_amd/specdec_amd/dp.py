"""Data-parallel sharding of the verify path: one process per GPU, the global
batch split contiguously by row, no collective on the data path.

Rows are independent — the accept/resample of row b reads only row b's logits — and perf-mode
noise is keyed by (seed, call offset, GLOBAL row id), so a rank verifying rows [start, stop)
with ``row_base=start`` produces exactly the outputs a single call over the whole batch would
give for those rows.  The only cross-rank traffic is the reduction of the bench counters
(max wall time, summed tokens), done once after the timed region.
"""
from __future__ import annotations

from typing import Dict, Sequence, Tuple

import torch


def shard_rows(global_rows: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [start, stop) of rank `rank`; the first global_rows % world ranks get one extra row."""
    if world <= 0 or not 0 <= rank < world or global_rows < 0:
        raise ValueError(f"bad shard request: rows={global_rows} world={world} rank={rank}")
    base, extra = divmod(global_rows, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def aggregate(elapsed_s: float, counters: Dict[str, float], device, dist=None) -> Tuple[float, Dict[str, float]]:
    """(max over ranks of elapsed_s, per-counter sums over ranks).  dist: torch.distributed or None.
    Works with gloo (CPU tensors) and RCCL (device tensors)."""
    keys = sorted(counters)
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=device)
    c = torch.tensor([float(counters[k]) for k in keys], dtype=torch.float64, device=device)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t[0]), dict(zip(keys, c.tolist()))


def concat_shards(shards: Sequence[torch.Tensor]) -> torch.Tensor:
    """Per-rank row outputs (in rank order) -> the global batch's outputs."""
    return torch.cat(list(shards), dim=0)
