"""Device-resident tables (cyc_table_*): the lazy probe.Table's Connectivity values computed on the
GPU from the resident planes, bit-exact vs the oracle's table (jobrunner.go:36-55,85-93 mapping
applied to the oracle planes by probe.PlaneCells)."""
import json
import os

import numpy as np
import pytest

from cyclonus_amd import _lib
from cyclonus_amd._lib import CyclonusError, CyclonusPanic
from cyclonus_amd.engine import Engine
from cyclonus_amd.probe import PlaneCells
from cyclonus_amd.shard import row_range, source_range
from oracle.oracle import Oracle, OraclePanic
from randgen import random_problem

GOLD = os.path.join(os.path.dirname(__file__), "golden")
pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("gpu")]


def _same(dt, want, P, K, ctx):
    got = dt.cells(0, P, 0, P, 0, K)
    exp = want.cells(0, P, 0, P, 0, K)
    for n in ("ingress", "egress", "combined"):
        assert got[n].shape == exp[n].shape, (ctx, n)
        bad = np.argwhere(got[n] != exp[n])
        assert bad.size == 0, f"{ctx}: {n} differs at {bad[:5].tolist()}"


def test_table_cells_config1():
    c = json.load(open(os.path.join(GOLD, "config1.json")))
    eng = Engine(0).build_policies(c["policies"]).load_resources(c["resources"])
    sh = eng.prepare(c["probes"])
    dt = eng.table()
    want = PlaneCells(*Oracle(c["policies"], c["resources"]).probe(c["probes"]))
    _same(dt, want, sh["pods"], sh["slots"], "config1")
    # single cells and sub-blocks, optional outputs
    P, K = sh["pods"], sh["slots"]
    for s_lo, s_hi, d_lo, d_hi, k_lo, k_hi in ((0, 1, 0, 1, 0, 1), (3, 7, 2, 9, 1, 3), (8, 9, 0, 9, 2, 3), (4, 4, 0, 9, 0, 3)):
        g = dt.cells(s_lo, s_hi, d_lo, d_hi, k_lo, k_hi, want=("combined",))
        w = want.cells(s_lo, s_hi, d_lo, d_hi, k_lo, k_hi, want=("combined",))
        assert np.array_equal(g["combined"], w["combined"])
    with pytest.raises(CyclonusError):
        dt.cells(0, P + 1, 0, P, 0, K)


@pytest.mark.parametrize("block", range(3))
def test_table_cells_random(block):
    """Random problems (AllAvailable, named / numbered probes, invalid named ports and protocols)."""
    eng = Engine(0)
    n = 0
    for seed in range(5000 + block * 40, 5000 + block * 40 + 40):
        pols, res, probes = random_problem(seed)
        try:
            want = PlaneCells(*Oracle(pols, res).probe(probes))
        except OraclePanic:
            continue
        eng.build_policies(pols).load_resources(res)
        sh = eng.prepare(probes)
        _same(eng.table(), want, sh["pods"], sh["slots"], f"seed {seed}")
        n += 1
    assert n > 20


def test_table_row_shards_and_wrap():
    """Row-shard tables answer their own rows: ingress for their destinations, egress for their
    sources; a table over run_device planes (cyc_table_wrap) equals an owned one."""
    import torch

    pols, res, probes = random_problem(6100, n_pods=150, n_pols=30)
    want = PlaneCells(*Oracle(pols, res).probe(probes))
    eng = Engine(0).build_policies(pols).load_resources(res)
    sh = eng.prepare(probes)
    P, K, W = sh["pods"], sh["slots"], sh["words"]
    for world in (2, 3):
        for rank in range(world):
            lo, hi = row_range(P, world, rank)
            t = eng.table(lo, hi)
            g = t.cells(0, P, lo, hi, 0, K, want=("ingress",))["ingress"]
            assert np.array_equal(g, want.cells(0, P, lo, hi, 0, K, want=("ingress",))["ingress"]), (world, rank)
            g = t.cells(lo, hi, 0, P, 0, K, want=("egress",))["egress"]
            assert np.array_equal(g, want.cells(lo, hi, 0, P, 0, K, want=("egress",))["egress"]), (world, rank)
            g = t.cells(lo, hi, lo, hi, 0, K)
            w = want.cells(lo, hi, lo, hi, 0, K)
            assert all(np.array_equal(g[n], w[n]) for n in g), (world, rank)
            if hi < P:
                with pytest.raises(CyclonusError):
                    t.cells(0, P, 0, P, 0, K, want=("combined",))
    d_in = torch.zeros((P, K, W), dtype=torch.int64, device="cuda")
    d_eg = torch.zeros((P, K, W), dtype=torch.int64, device="cuda")
    d_st = torch.zeros((P, K), dtype=torch.uint8, device="cuda")
    eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    _same(eng.wrap_table(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr()), want, P, K, "wrap")


def test_table_source_shards():
    """Source-row tables (CYC_ROWS_SOURCE) answer Table.Get(from, *) for their sources: every
    Ingress / Egress / Combined value of (s in shard, any d, k), from owned planes and from wrapped
    run_device planes; cells of other sources are refused."""
    import torch

    for seed in (6300, 6301, 6302):
        pols, res, probes = random_problem(seed, n_pods=190, n_pols=30)
        want = PlaneCells(*Oracle(pols, res).probe(probes))
        eng = Engine(0).build_policies(pols).load_resources(res)
        sh = eng.prepare(probes)
        P, K = sh["pods"], sh["slots"]
        for world in (2, 3):
            for rank in range(world):
                lo, hi = source_range(P, world, rank)
                t = eng.table(lo, hi, "source")
                assert t.partition == "source" and t.window[0] == lo // 64
                g = t.cells(lo, hi, 0, P, 0, K)
                w = want.cells(lo, hi, 0, P, 0, K)
                assert all(np.array_equal(g[n], w[n]) for n in g), (seed, world, rank)
                if hi < P:
                    with pytest.raises(CyclonusError):
                        t.cells(hi, P, 0, P, 0, K, want=("ingress",))
                ri, wi, re_, we, _ = eng.layout(lo, hi, "source")
                d_in = torch.zeros((ri, K, max(wi, 1)), dtype=torch.int64, device="cuda")
                d_eg = torch.zeros((max(re_, 1), K, we), dtype=torch.int64, device="cuda")
                d_st = torch.zeros((P, K), dtype=torch.uint8, device="cuda")
                eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), torch.cuda.current_stream().cuda_stream,
                               lo, hi, "source")
                torch.cuda.synchronize()
                t2 = eng.wrap_table(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), lo, hi, "source")
                g2 = t2.cells(lo, hi, 0, P, 0, K)
                assert all(np.array_equal(g2[n], w[n]) for n in g2), (seed, world, rank, "wrap")


def test_table_panics_and_lifetime():
    """A panicking build reports the reference's panic from cyc_table_run; a table outlives its context."""
    eng = Engine(0)
    hit = False
    for seed in range(10_000, 10_060):
        pols, res, probes = random_problem(seed, bad=True)
        try:
            Oracle(pols, res).probe(probes)
            continue
        except OraclePanic as e:
            msg = str(e)
        try:
            eng.build_policies(pols).load_resources(res)
            eng.prepare(probes)
            eng.table()
        except CyclonusPanic as p:
            assert p.msg == msg, seed
            hit = True
            break
    assert hit
    pols, res, probes = random_problem(6200, n_pods=40)
    want = PlaneCells(*Oracle(pols, res).probe(probes))
    e2 = Engine(0).build_policies(pols).load_resources(res)
    sh = e2.prepare(probes)
    t = e2.table()
    e2.close()
    _same(t, want, sh["pods"], sh["slots"], "after ctx destroy")
    assert _lib.CONNECTIVITY[_lib.CONN_ALLOWED] == "allowed"


def test_cpp_driver_tables(tmp_path):
    """The C++ C-ABI driver (tests/native/capi_driver.cpp) prints every cell's Connectivity through
    cyc_table_run / cyc_table_cells, from the JSON and from the flat-table entry points: equal to the
    oracle's table on config1 and random problems."""
    import subprocess

    from cyclonus_amd import build, flat

    drv = build.DRIVER
    assert os.path.exists(drv), "build the driver first (cyclonus_amd.build)"
    short = {0: "?", 1: "!", 2: "P", 3: "N", 4: "X", 5: ".", 255: "-"}
    cases = [json.load(open(os.path.join(GOLD, "config1.json")))]
    cases = [(c["policies"], c["resources"], c["probes"]) for c in cases]
    cases += [random_problem(seed) for seed in range(7000, 7012)]
    for n, (pols, res, probes) in enumerate(cases):
        try:
            want = PlaneCells(*Oracle(pols, res).probe(probes))
        except OraclePanic:
            continue
        paths = []
        for name, doc in (("pols", pols), ("res", res), ("probes", probes)):
            p = tmp_path / f"{name}{n}.json"
            p.write_text(json.dumps(doc))
            paths.append(str(p))
        # the JSON entry points, then the flat-table ones (cyc_policy_load of the built policy,
        # cyc_resources_load, cyc_probe_prepare_configs: the cgo binding's no-JSON form)
        ir = Engine(0).build_policies(pols).policy_ir()
        fpaths = [str(tmp_path / f"{n}.{x}") for x in ("pol.tab", "res.tab", "probes.txt")]
        flat.dump_tables(flat.PolicyTables(ir), fpaths[0])
        flat.dump_tables(flat.ResourceTables(res), fpaths[1])
        flat.dump_probe_configs(probes, fpaths[2])
        for argv in ([drv, *paths], [drv, "--flat", *fpaths]):
            r = subprocess.run(argv, capture_output=True, text=True, timeout=100)
            assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
            lines = r.stdout.splitlines()
            P, K = (int(x) for x in lines[0].split()[1:])
            w = want.cells(0, P, 0, P, 0, K)
            for line in lines[1:]:
                s, d, cells = line.split(" ")
                s, d = int(s), int(d)
                exp = "".join(short[int(w["ingress"][s, d, k])] + short[int(w["egress"][s, d, k])] +
                              short[int(w["combined"][s, d, k])] for k in range(K))
                assert cells == exp, (n, argv[1], s, d, cells, exp)
            assert len(lines) == 1 + P * P
