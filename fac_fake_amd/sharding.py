"""Frame sharding across the GPUs of one node (config 3 of BASELINE.json).

Every crop's forward is independent given its pos slot, so a
video's crops split contiguously by global index over the ranks (one process
per GPU, weights replicated), each rank scores its shard with no
communication, and the only exchange is one all-gather of the per-crop fp32
logits ([n_i, 2], padded to the largest shard) before the video-level mean
(cvit_prediction.py:240,258-281).  With backend "nccl" this is RCCL over xGMI;
the same code runs on "gloo" for CPU tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_bounds(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [lo, hi) of n crops for `rank` (sizes differ by at most one)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def max_shard(n: int, world: int) -> int:
    return -(-n // world)


def gather_logits(local: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """All-gather every rank's [n_i, 2] fp32 logits into [n_total, 2] in global crop order."""
    world = dist.get_world_size(group)
    cap = max_shard(n_total, world)
    buf = torch.zeros(cap, 2, dtype=torch.float32, device=local.device)
    buf[: local.shape[0]] = local
    out = torch.empty(world * cap, 2, dtype=torch.float32, device=local.device)
    dist.all_gather_into_tensor(out, buf, group=group)
    parts = [out[r * cap: r * cap + (shard_bounds(n_total, world, r)[1] - shard_bounds(n_total, world, r)[0])]
             for r in range(world)]
    return torch.cat(parts, 0)
