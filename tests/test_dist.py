"""Row sharding + all-gather assembly on CPU (gloo, world_size 2), as bench.py uses them on RCCL."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cyclonus_amd.shard import assemble, assemble_sources, row_range, source_range


def test_row_range_partition():
    for P in (0, 1, 7, 64, 100_000, 100_003):
        for world in (1, 2, 3, 4, 8):
            spans = [row_range(P, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == P
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1


def test_source_range_partition():
    """Source shards: 64-pod aligned starts, tiling [0, P); their ingress windows tile the words."""
    for P in (0, 1, 7, 64, 65, 100_000, 100_003):
        W = (P + 63) // 64
        for world in (1, 2, 3, 4, 8):
            spans = [source_range(P, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == P
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            assert all(lo % 64 == 0 and (hi % 64 == 0 or hi == P) for lo, hi in spans)
            words = [(lo // 64, (hi + 63) // 64 if hi > lo else lo // 64) for lo, hi in spans]
            assert sum(b - a for a, b in words) == W
            assert max(b - a for a, b in words) - min(b - a for a, b in words) <= 1


def _worker(rank, world, port, P, K, W, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(1234)
    full = torch.randint(-(2**62), 2**62, (P, K, W), generator=g, dtype=torch.int64)
    lo, hi = row_range(P, world, rank)
    got = assemble(full[lo:hi].clone(), P)
    q.put((rank, bool(torch.equal(got, full))))
    dist.destroy_process_group()


@pytest.mark.parametrize("P", [5, 64, 131])
def test_assemble_gloo_world2(P):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + P
    procs = [ctx.Process(target=_worker, args=(r, 2, port, P, 3, (P + 63) // 64, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def _worker_src(rank, world, port, P, K, q):
    """Source partition: each rank holds its sources' egress rows and its word slice of every
    ingress row; the assembled planes equal the full ones."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    W = (P + 63) // 64
    g = torch.Generator().manual_seed(99)
    full_in = torch.randint(-(2**62), 2**62, (P, K, W), generator=g, dtype=torch.int64)
    full_eg = torch.randint(-(2**62), 2**62, (P, K, W), generator=g, dtype=torch.int64)
    lo, hi = source_range(P, world, rank)
    w0, w1 = lo // 64, (hi + 63) // 64 if hi > lo else lo // 64
    got_in = assemble_sources(full_in[:, :, w0:w1].clone(), P)
    got_eg = assemble(full_eg[lo:hi].clone(), P, partition="source")
    q.put((rank, bool(torch.equal(got_in, full_in) and torch.equal(got_eg, full_eg))))
    dist.destroy_process_group()


@pytest.mark.parametrize("P,world", [(5, 2), (130, 2), (300, 3), (256, 2), (70, 1)])
def test_assemble_sources_gloo(P, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + P + world
    procs = [ctx.Process(target=_worker_src, args=(r, world, port, P, 3, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}
