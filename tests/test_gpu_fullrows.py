"""Whole plane rows at full size (configs #2, #3 and #4): complete ingress rows (one destination, every
source, every slot) and egress rows (one source, every destination, every slot) from the device
table equal the oracle's rows bit for bit — rows from the first / last positions, 64-pod word
edges, the most populous identities (largest classes) and random positions, on the whole table, on
target-row shards (row_lo > 0) and on source-row shards (the shard's egress rows, and its word slice
of every picked destination's ingress row).  Every check runs through both ingestion paths: the JSON
entry points and the flat tables bench.py times (flat.prepare_flat: cyc_policy_build_json +
cyc_resources_load + cyc_probe_prepare_configs); test_config3_flat_planes_equal_json compares the two
paths' whole planes at config #3's full size."""
import json
from collections import Counter

import numpy as np
import pytest

from cyclonus_amd import synth
from cyclonus_amd.engine import Engine
from cyclonus_amd.flat import prepare_flat
from cyclonus_amd.shard import row_range, source_range
from oracle.oracle import Oracle

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("gpu")]
THREADS = 16


def _pick_rows(res, lo, hi, n_random, seed):
    pods = res["Pods"][lo:hi]
    ident = [(p["Namespace"], tuple(sorted((p.get("Labels") or {}).items()))) for p in pods]
    top = [i for i, _ in Counter(ident).most_common(3)]
    rows = {0, 1, 63, 64, 65, len(pods) // 2, len(pods) - 64, len(pods) - 1}
    for t in top:  # first and last pod of the largest identities
        idx = [i for i, x in enumerate(ident) if x == t]
        rows |= {idx[0], idx[-1]}
    rng = np.random.default_rng(seed)
    rows |= set(int(x) for x in rng.integers(0, len(pods), n_random))
    return sorted(lo + r for r in rows if 0 <= r < len(pods))


INGEST = pytest.mark.parametrize("ingest", ["json", "flat"])


def _prepared(data, ingest):
    """An engine prepared through the JSON entry points or through bench.py's flat path."""
    if ingest == "flat":
        eng = Engine(0)
        return eng, prepare_flat(eng, data["policies"], data["resources"], data["probes"])
    eng = Engine(0).build_policies(json.dumps(data["policies"])).load_resources(json.dumps(data["resources"]))
    return eng, eng.prepare(data["probes"])


def _check(name, kw, shards, source_shards=(), ingest="json"):
    import torch

    data = synth.CONFIGS[name](**kw)
    eng, sh = _prepared(data, ingest)
    P, K, W = sh["pods"], sh["slots"], sh["words"]
    orc = Oracle(data["policies"], data["resources"])
    for world, rank in source_shards:
        lo, hi = source_range(P, world, rank)
        ri, wi, re_, we, w0 = eng.layout(lo, hi, "source")
        d_in = torch.empty((ri, K, wi), dtype=torch.int64, device="cuda")
        d_eg = torch.empty((re_, K, we), dtype=torch.int64, device="cuda")
        d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
        eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), torch.cuda.current_stream().cuda_stream, lo, hi,
                       "source")
        torch.cuda.synchronize()
        assert eng.last_emit() == ("k_emit_units<1024,7>", 1), eng.last_emit()  # one launch over both planes
        dsts = _pick_rows(data["resources"], 0, P, 6, seed=world * 1000 + rank)  # any destination
        srcs = _pick_rows(data["resources"], lo, hi, 4, seed=world * 1000 + rank + 1)  # the shard's sources
        g_in = d_in[torch.as_tensor(dsts, device="cuda")].cpu().numpy().view(np.uint64)
        g_eg = d_eg[torch.as_tensor([p - lo for p in srcs], device="cuda")].cpu().numpy().view(np.uint64)
        del d_in, d_eg
        torch.cuda.empty_cache()
        for k in range(K):
            for x, pod in enumerate(dsts):
                want = orc.row(data["probes"], "ingress", pod, k, threads=THREADS)[w0:w0 + wi]
                bad = np.nonzero(g_in[x, k] != want)[0]
                assert bad.size == 0, (f"{name} source shard {rank}/{world} ingress row {pod} slot {k}: {bad.size} words "
                                       f"of the slice differ, first at word {w0 + int(bad[0])}")
            for x, pod in enumerate(srcs):
                want = orc.row(data["probes"], "egress", pod, k, threads=THREADS)
                bad = np.nonzero(g_eg[x, k] != want)[0]
                assert bad.size == 0, (f"{name} source shard {rank}/{world} egress row {pod} slot {k}: {bad.size} words "
                                       f"differ, first at word {int(bad[0])}")
    for world, rank in shards:
        lo, hi = row_range(P, world, rank)
        rows = hi - lo
        d_in = torch.empty((rows, K, W), dtype=torch.int64, device="cuda")
        d_eg = torch.empty((rows, K, W), dtype=torch.int64, device="cuda")
        d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
        eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), torch.cuda.current_stream().cuda_stream, lo, hi)
        torch.cuda.synchronize()
        picks = _pick_rows(data["resources"], lo, hi, 6, seed=world * 100 + rank)
        idx = torch.as_tensor([p - lo for p in picks], device="cuda")
        g_in = d_in[idx].cpu().numpy().view(np.uint64)
        g_eg = d_eg[idx].cpu().numpy().view(np.uint64)
        del d_in, d_eg
        torch.cuda.empty_cache()
        for x, pod in enumerate(picks):
            for k in range(K):
                want_in = orc.row(data["probes"], "ingress", pod, k, threads=THREADS)
                want_eg = orc.row(data["probes"], "egress", pod, k, threads=THREADS)
                for plane, got, want in (("ingress", g_in[x, k], want_in), ("egress", g_eg[x, k], want_eg)):
                    bad = np.nonzero(got != want)[0]
                    assert bad.size == 0, (f"{name} shard {rank}/{world} {plane} row {pod} slot {k}: "
                                           f"{bad.size} words differ, first at word {int(bad[0])}")


@INGEST
def test_config2_full_rows(ingest):
    """Config #2 (per-pod PM rows, in-place class rows, the flat emit): whole table, a target shard
    and a source shard."""
    _check("config2", {}, [(1, 0), (4, 2)], [(8, 5)], ingest)


def test_config3_full_rows():
    """Config #3 through bench.py's flat path (the JSON path's whole planes equal these byte for byte:
    test_config3_flat_planes_equal_json): the whole table (two row phases), a target and a source shard."""
    _check("config3", {}, [(1, 0), (8, 3)], [(8, 3)], "flat")


@INGEST
def test_config4_full_rows(ingest):
    _check("config4", {}, [(1, 0), (4, 3)], [(4, 1)], ingest)


def test_config3_flat_planes_equal_json():
    """The headline's exact preparation (bench.py: flat tables) and the JSON one give byte-identical
    whole planes and status plane at config #3's full size (2 x 10 GB per path), the same shape and
    classes; cyc_last_emit names the emit (k_emit_wide_buf<1024,7>, one launch per row phase)."""
    import torch

    data = synth.CONFIGS["config3"]()
    outs, shapes = [], []
    for ingest in ("flat", "json"):
        eng, sh = _prepared(data, ingest)
        sh = {k: v for k, v in sh.items() if k != "prepare_s"}
        P, K, W = sh["pods"], sh["slots"], sh["words"]
        d_in = torch.full((P, K, W), 0x5A5A, dtype=torch.int64, device="cuda")
        d_eg = torch.full((P, K, W), 0x5A5A, dtype=torch.int64, device="cuda")
        d_st = torch.full((P, K), 0x5A, dtype=torch.uint8, device="cuda")
        eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        # (a whole table of >= 8 GB planes runs as two row phases: one emit launch each)
        assert eng.get_option("row_phases_active") == 2
        assert eng.last_emit() == ("k_emit_wide_buf<1024,7>", 2), eng.last_emit()
        if outs:
            for plane, a, b in zip(("ingress", "egress", "status"), outs[0], (d_in, d_eg, d_st)):
                assert torch.equal(a, b), f"config #3 {plane} plane: flat-prepared != JSON-prepared"
        outs.append((d_in, d_eg, d_st))
        shapes.append((sh, eng.classes()))
        eng.close()
        if len(outs) == 2:
            del outs[1]
    assert shapes[0] == shapes[1]


def test_config3u_full_rows():
    """Class explosion: config #3's shape with every pod identity distinct (synth.config3u)."""
    _check("config3u", {}, [(1, 0)])
