"""Multi-process shard path on the GPU: 2 ranks (spawned before they touch the GPU, gloo backend
for the collectives), each runs its shard of the engine — source rows (north_star's partition) or
target rows — and
* checks its own cells against the oracle: under the source partition, whole Combined rows
  Table.Get(from = s, *) of its sources (the rank holds both directions of those cells);
* all-gathers the shards with shard.assemble / assemble_sources and compares the assembled planes
  with a single-process full run and with oracle-sampled cells."""
import json
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("gpu")]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rank(rank, world, port, partition, q):
    import sys

    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    from cyclonus_amd import synth
    from cyclonus_amd.engine import Engine
    from cyclonus_amd.shard import assemble, assemble_sources, shard_range
    from oracle.oracle import Oracle

    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        data = synth.config3(n_ns=60)
        eng = Engine(0).build_policies(json.dumps(data["policies"])).load_resources(json.dumps(data["resources"]))
        sh = eng.prepare(data["probes"])
        P, K, W = sh["pods"], sh["slots"], sh["words"]
        lo, hi = shard_range(P, world, rank, partition)
        ri, wi, re_, we, w0 = eng.layout(lo, hi, partition)
        d_in = torch.empty((ri, K, wi), dtype=torch.int64, device="cuda")
        d_eg = torch.empty((re_, K, we), dtype=torch.int64, device="cuda")
        d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
        eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), torch.cuda.current_stream().cuda_stream, lo, hi,
                       partition)
        torch.cuda.synchronize()
        res = {"rank": rank, "rows": (lo, hi)}
        orc = Oracle(data["policies"], data["resources"])
        if partition == "source":
            # this rank's own Combined rows: sources at its ends and a few inside, every destination
            li, le = d_in.cpu().numpy().view(np.uint64), d_eg.cpu().numpy().view(np.uint64)
            st = d_st.cpu().numpy()
            bad = 0
            for s in sorted({lo, lo + 63, (lo + hi) // 2, hi - 1}):
                d = np.arange(P)
                for k in range(K):
                    gi = (li[d, k, s // 64 - w0] >> np.uint64(s % 64)) & np.uint64(1)
                    ge = (le[s - lo, k, d // 64] >> (d % 64).astype(np.uint64)) & np.uint64(1)
                    got = st[d, k].astype(np.uint8) | (gi.astype(np.uint8) << 4) | (ge.astype(np.uint8) << 5)
                    want = orc.cells(data["probes"], np.full(P, s), d, np.full(P, k), threads=8)
                    bad += int((got != want).sum())
            res["own_rows_mismatch"] = bad
            full_in = assemble_sources(d_in.cpu(), P)
            full_eg = assemble(d_eg.cpu(), P, partition="source")
        else:
            full_in = assemble(d_in.cpu(), P)
            full_eg = assemble(d_eg.cpu(), P)
        if rank == 0:
            st, ing, eg = eng.run_host()
            res["equal_full"] = bool(np.array_equal(full_in.numpy().view(np.uint64), ing)
                                     and np.array_equal(full_eg.numpy().view(np.uint64), eg)
                                     and np.array_equal(d_st.cpu().numpy(), st))
            rng = np.random.default_rng(3)
            s, d, k = rng.integers(0, P, 4000), rng.integers(0, P, 4000), rng.integers(0, K, 4000)
            want = orc.cells(data["probes"], s, d, k, threads=8)
            fi, fe = full_in.numpy().view(np.uint64), full_eg.numpy().view(np.uint64)
            gi = (fi[d, k, s // 64] >> (s % 64).astype(np.uint64)) & np.uint64(1)
            ge = (fe[s, k, d // 64] >> (d % 64).astype(np.uint64)) & np.uint64(1)
            got = st[d, k].astype(np.uint8) | (gi.astype(np.uint8) << 4) | (ge.astype(np.uint8) << 5)
            res["oracle_mismatch"] = int((got != want).sum())
        dist.destroy_process_group()
        q.put(res)
    except Exception as e:  # report, never hang the parent
        q.put({"rank": rank, "error": f"{type(e).__name__}: {e}"})


@pytest.mark.parametrize("partition,port", [("source", 29641), ("target", 29631)])
def test_two_rank_shards_assemble(partition, port):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, partition, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    for _ in procs:
        r = q.get(timeout=170)
        out[r["rank"]] = r
    for p in procs:
        p.join(timeout=30)
    assert all("error" not in r for r in out.values()), out
    assert out[0]["rows"][1] == out[1]["rows"][0]
    assert out[0]["equal_full"], "assembled shards differ from the single-process table"
    assert out[0]["oracle_mismatch"] == 0
    if partition == "source":
        assert out[0]["own_rows_mismatch"] == 0 and out[1]["own_rows_mismatch"] == 0
