"""Multi-GPU layout: row shards across ranks (one process per GPU), two partitions.

* "source" (north_star): rank r owns SOURCE pods [lo, hi) — 64-pod aligned, so the
  ranks' 64-pod words tile every ingress row.  It computes every cell (s in [lo, hi), d, k): the
  egress rows of its sources and, for every destination, the words [lo/64, ceil(hi/64)) of the
  ingress row (include/cyclonus_hip.h, CYC_ROWS_SOURCE).  Table.Get(from, *) of a source is answered
  by one rank (pkg/connectivity/probe/table.go:54-56).
* "target": rank r owns target pods [lo, hi) of BOTH planes (ingress rows keyed by destination,
  egress rows keyed by source).

Every verdict depends only on replicated inputs: nothing on the data path is exchanged.  The whole
table on every rank is the library's own collective (cyc_comm_init + cyc_planes_allgather /
cyc_table_allgather, csrc/comm.hpp: RCCL broadcasts plus a HIP relayout kernel) — what a cgo host
calls and bench.py times.  `assemble` / `assemble_sources` below are the same assembly in
torch.distributed, for process groups the library's RCCL communicator cannot join (gloo: the CPU
tests and one-GPU rehearsals).  The ranges here must equal cyc_rows_shard's (test_gpu_assemble).
"""
from __future__ import annotations


def row_range(P: int, world: int, rank: int):
    """Target-row shard: contiguous, balanced shard of P rows for `rank` (differs by at most one row)."""
    return rank * P // world, (rank + 1) * P // world


def source_range(P: int, world: int, rank: int):
    """Source-row shard: the pods of a balanced share of the W = ceil(P/64) 64-pod words."""
    W = (P + 63) // 64
    return min(P, (rank * W // world) * 64), min(P, ((rank + 1) * W // world) * 64)


def shard_range(P: int, world: int, rank: int, partition: str = "target"):
    return source_range(P, world, rank) if partition == "source" else row_range(P, world, rank)


def _gather(send, world, group):
    """All-gather equal-shaped tensors into one [world, ...] buffer: a single all_gather_into_tensor
    (RCCL and gloo both take the concatenated [world * n0, ...] output form)."""
    import torch.distributed as dist

    out = send.new_empty((world * send.shape[0],) + tuple(send.shape[1:]))
    dist.all_gather_into_tensor(out, send, group=group)
    return out.view((world,) + tuple(send.shape))


def _send(local, n, shape, dim):
    """The all-gather's send buffer: `local` itself when it already has the padded shape, else a zero
    pad of `shape` with local's first n entries along `dim` copied in."""
    if tuple(local.shape) == tuple(shape) and local.is_contiguous():
        return local
    send = local.new_zeros(shape)
    send.narrow(dim, 0, n).copy_(local.narrow(dim, 0, n))
    return send


def assemble(local_rows, P: int, group=None, partition: str = "target"):
    """All-gather row shards [rows, K, W] (target rows of either plane, or a source partition's egress
    rows) into the full [P, K, W] plane on every rank.  Shards are padded to the largest shard so a
    single all-gather moves them.  The result may alias its inputs: at world 1 it is a view of
    `local_rows`, with equal shards a view of the gather buffer — clone() it if `local_rows` is reused."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    ranges = [shard_range(P, world, r, partition) for r in range(world)]
    maxrows = max(hi - lo for lo, hi in ranges)
    lo, hi = ranges[rank]
    K, W = local_rows.shape[1], local_rows.shape[2]
    if world == 1:  # the shard is the plane
        return local_rows[:P]
    parts = _gather(_send(local_rows, hi - lo, (max(maxrows, 1), K, W), 0), world, group)
    if all(b - a == maxrows for a, b in ranges):
        return parts.view(P, K, W)  # equal shards: the gathered buffer is already the plane's row order
    full = local_rows.new_empty((P, K, W))
    for r, (a, b) in enumerate(ranges):
        full[a:b] = parts[r][: b - a]
    return full


def assemble_sources(local_ingress, P: int, group=None):
    """All-gather a source partition's ingress slices [P, K, Wr] (each rank: the words of its
    sources in every destination's row) into the full [P, K, W] ingress plane on every rank.  At world 1
    the result is a view of `local_ingress` (clone() it if that buffer is reused)."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    W = (P + 63) // 64
    wr = [((r * W // world), ((r + 1) * W // world)) for r in range(world)]
    maxw = max(b - a for a, b in wr)
    K = local_ingress.shape[1]
    a, b = wr[rank]
    if world == 1:  # one rank computed every word of every row
        return local_ingress[:, :, :W]
    parts = _gather(_send(local_ingress, b - a, (P, K, max(maxw, 1)), 2), world, group)
    full = local_ingress.new_empty((P, K, W))
    for r, (a, b) in enumerate(wr):
        full[:, :, a:b] = parts[r][:, :, : b - a]
    return full
