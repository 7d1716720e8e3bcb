"""Table assembly behind the C ABI (include/cyclonus_hip.h, comm.hpp): the relayout of source shards'
ingress slices into whole rows, and the RCCL all-gather of row shards on a one-rank communicator.

* cyc_rows_merge_sources: every source shard of a world-N partition is run on this GPU (exactly what
  rank r of an N-GPU job computes), the library scatters the N ingress slices into one plane, and that
  plane must equal the whole-table run's ingress plane byte for byte (N = 2..8; config #2, a random
  problem whose pod count is not a multiple of 64, and config #3 at N = 8 — every shard's WHOLE
  ingress slice, the 12.5 KB rows k_emit_units copies a row per thread group, is compared).
* cyc_comm_init / cyc_planes_allgather / cyc_table_allgather with one rank (two ranks cannot share a
  GPU under RCCL): the broadcast groups, the chunked source-ingress path and the in-place row shares
  give the whole-table planes; the assembled device table answers cells like the whole table.
* cyc_rows_shard == cyclonus_amd.shard (the Python mirror bench.py uses).
The whole-table planes themselves are pinned to the oracle by test_gpu_parity / test_gpu_fullrows.
"""
import json

import pytest

from cyclonus_amd import synth
from cyclonus_amd.engine import Engine
from cyclonus_amd.shard import shard_range
from randgen import random_problem

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("gpu")]


def _engine(pols, res, probes):
    eng = Engine(0).build_policies(json.dumps(pols)).load_resources(json.dumps(res))
    sh = eng.prepare(probes)
    return eng, sh


def _whole(eng, sh):
    import torch

    P, K, W = sh["pods"], sh["slots"], sh["words"]
    d_in = torch.empty((P, K, W), dtype=torch.int64, device="cuda")
    d_eg = torch.empty((P, K, W), dtype=torch.int64, device="cuda")
    d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
    eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return d_in, d_eg, d_st


def _source_shard(eng, sh, world, rank):
    import torch

    P, K = sh["pods"], sh["slots"]
    lo, hi = eng.rows_shard(world, rank, "source")
    ri, wi, re_, we, _ = eng.layout(lo, hi, "source")
    d_in = torch.full((max(ri * K * wi, 1),), 0x5A5A, dtype=torch.int64, device="cuda")
    d_eg = torch.full((max(re_ * K * we, 1),), 0x5A5A, dtype=torch.int64, device="cuda")
    d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
    eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), torch.cuda.current_stream().cuda_stream, lo, hi,
                   "source")
    return d_in, d_eg, (lo, hi)


def _check_merge(eng, sh, worlds, whole_in):
    import torch

    for world in worlds:
        slices = [_source_shard(eng, sh, world, r)[0] for r in range(world)]
        full = torch.full_like(whole_in, 0x3C3C)
        eng.merge_sources([s.data_ptr() for s in slices], full.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        if not torch.equal(full, whole_in):
            bad = (full != whole_in).nonzero()
            raise AssertionError(f"world {world}: merged ingress plane differs from the whole table at "
                                 f"{bad.shape[0]} words, first (dst, slot, word) {tuple(bad[0].tolist())}")
        del slices, full
        torch.cuda.empty_cache()


def test_rows_shard_matches_python():
    pols, res, probes = random_problem(11, n_pods=40)
    eng, _ = _engine(pols, res, probes)
    P = eng.shape["pods"]  # (the library partitions its prepared pods)
    for world in (1, 2, 3, 5, 8):
        for r in range(world):
            for part in ("source", "target"):
                assert eng.rows_shard(world, r, part) == shard_range(P, world, r, part), (P, world, r, part)


@pytest.mark.parametrize("case", ["config2", "random"])
def test_merge_sources_equals_whole(case):
    if case == "config2":
        data = synth.config2()
        eng, sh = _engine(data["policies"], data["resources"], data["probes"])
    else:
        pols, res, probes = random_problem(7, n_pods=1000, n_pols=30)  # P % 64 != 0: a ragged last word
        eng, sh = _engine(pols, res, probes)
        assert sh["pods"] % 64
    whole_in, _, _ = _whole(eng, sh)
    _check_merge(eng, sh, range(2, 9), whole_in)


def test_merge_sources_config3_n8():
    """Config #3 at N = 8: each rank's whole ingress slice (every destination's 12.5 KB row slice, copied a
    row per 128-thread group by k_emit_units) lands exactly where the whole table has it."""
    data = synth.config3()
    from cyclonus_amd.flat import prepare_flat

    eng = Engine(0)
    sh = prepare_flat(eng, data["policies"], data["resources"], data["probes"])
    whole_in, _, _ = _whole(eng, sh)
    _check_merge(eng, sh, [8], whole_in)


def test_rccl_world1_allgather():
    """One-rank RCCL communicator owned by the context: both partitions' planes assembled by
    cyc_planes_allgather (separate full planes, and in place for row shares) equal the whole table,
    and cyc_table_allgather's table answers cells like the whole-table run."""
    import numpy as np
    import torch

    data = synth.config2()
    eng, sh = _engine(data["policies"], data["resources"], data["probes"])
    P, K = sh["pods"], sh["slots"]
    whole_in, whole_eg, whole_st = _whole(eng, sh)
    uid = Engine.comm_unique_id()
    assert len(uid) == 128
    eng.comm_init(1, 0, uid)
    stream = torch.cuda.current_stream().cuda_stream
    for part in ("source", "target"):
        d_in, d_eg, (lo, hi) = _source_shard(eng, sh, 1, 0) if part == "source" else (None, None, (0, P))
        if part == "target":
            d_in, d_eg, _ = _whole(eng, sh)
        f_in, f_eg = torch.full_like(whole_in, 7), torch.full_like(whole_eg, 7)
        eng.planes_allgather(d_in.data_ptr(), d_eg.data_ptr(), f_in.data_ptr(), f_eg.data_ptr(), stream, part)
        torch.cuda.synchronize()
        assert torch.equal(f_in, whole_in), part
        assert torch.equal(f_eg, whole_eg), part
    # in place: the shard already sits at its rows of the full planes
    f_in, f_eg, _ = _whole(eng, sh)
    eng.planes_allgather(f_in.data_ptr(), f_eg.data_ptr(), f_in.data_ptr(), f_eg.data_ptr(), stream, "target")
    torch.cuda.synchronize()
    assert torch.equal(f_in, whole_in) and torch.equal(f_eg, whole_eg)
    # the device-table form, from a source shard table
    shard = eng.table(0, P, "source")
    full = eng.table_allgather(shard)
    ref = eng.table(0, P)
    assert (full.row_lo, full.row_hi, full.partition) == (0, P, "target")
    rng = np.random.default_rng(3)
    for _ in range(4):
        s0, d0 = int(rng.integers(0, P - 64)), int(rng.integers(0, P - 200))
        a = full.cells(s0, s0 + 64, d0, d0 + 200)
        b = ref.cells(s0, s0 + 64, d0, d0 + 200)
        for k in a:
            assert np.array_equal(a[k], b[k]), k
    for t in (shard, full, ref):
        t.close()
    eng.comm_destroy()
    # without a communicator the collective refuses
    from cyclonus_amd import _lib

    with pytest.raises(_lib.CyclonusError):
        eng.planes_allgather(whole_in.data_ptr(), whole_eg.data_ptr(), f_in.data_ptr(), f_eg.data_ptr(), stream, "target")
    del whole_st
