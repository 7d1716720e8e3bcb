"""Multi-GPU layout: target-pod rows sharded across ranks (one process per GPU).

Each rank computes the verdict planes for rows [row_range(P, world, rank)) of BOTH planes
(ingress rows keyed by destination, egress rows keyed by source).  Nothing on the data path
is exchanged; `assemble` is the optional RCCL all-gather (torch.distributed, backend "nccl" on
ROCm) that materialises the whole table on every rank.
"""
from __future__ import annotations


def row_range(P: int, world: int, rank: int):
    """Contiguous, balanced shard of P target rows for `rank` (differs by at most one row)."""
    return rank * P // world, (rank + 1) * P // world


def assemble(local_rows, P: int, group=None):
    """All-gather row shards [rows, K, W] into the full [P, K, W] table on every rank.

    Shards are padded to the largest shard so a single all_gather_into_tensor moves them.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    maxrows = max(hi - lo for lo, hi in (row_range(P, world, r) for r in range(world)))
    lo, hi = row_range(P, world, rank)
    K, W = local_rows.shape[1], local_rows.shape[2]
    send = local_rows.new_zeros((maxrows, K, W))
    send[: hi - lo] = local_rows[: hi - lo]
    out = local_rows.new_empty((world * maxrows, K, W))
    if dist.get_backend(group) == "gloo":
        parts = list(out.chunk(world))
        dist.all_gather(parts, send, group=group)
        out = torch.cat(parts)
    else:
        dist.all_gather_into_tensor(out, send, group=group)
    full = local_rows.new_empty((P, K, W))
    for r in range(world):
        a, b = row_range(P, world, r)
        full[a:b] = out[r * maxrows : r * maxrows + (b - a)]
    return full
