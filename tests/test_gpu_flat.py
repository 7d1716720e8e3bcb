"""GPU: the flat-table entry points (cyc_policy_load / cyc_resources_load / cyc_probe_prepare_configs,
include/cyclonus_hip.h) produce the same verdict tables as the JSON ones and the oracle — whole tables
on random problems (panics and duplicate job keys included), and a shared prepare serving several
probe configs (analyze.go:241-243 runs one RunProbeForConfig per probe over the same Resources)."""
import numpy as np
import pytest

from cyclonus_amd._lib import CyclonusPanic
from cyclonus_amd.engine import Engine
from oracle.oracle import Oracle, OraclePanic
from randgen import random_problem

pytestmark = pytest.mark.gpu


def _run(eng):
    try:
        return eng.run_host()
    except CyclonusPanic as e:
        return ("panic", e.code, e.msg)


def _same(a, b, ctx):
    if isinstance(a, tuple) and isinstance(a[0], str) or isinstance(b, tuple) and isinstance(b[0], str):
        assert a == b, ctx
        return
    for x, y in zip(a, b):
        assert np.array_equal(x, y), ctx


def test_flat_equals_json_random(gpu):
    n = 0
    for seed in range(90):
        pols, res, probes = random_problem(400_000 + seed, bad=seed % 4 == 0, dups=seed % 3 == 0)
        a = Engine(0).build_policies(pols).load_resources(res)
        a.prepare(probes)
        ir = a.policy_ir()
        b = Engine(0).load_policy_tables(ir).load_resources_tables(res)
        b.prepare_configs(probes)
        assert b.shape == a.shape, seed
        _same(_run(a), _run(b), f"seed {seed}")
        n += 1
    assert n == 90


def test_flat_tables_vs_oracle(gpu):
    """Flat path against the oracle directly (not only against the JSON path)."""
    for seed in range(40):
        pols, res, probes = random_problem(410_000 + seed)
        try:
            want = Oracle(pols, res).probe(probes)
        except OraclePanic:
            continue
        e = Engine(0).build_policies(pols).load_resources_tables(res)
        e.prepare_configs(probes)
        st, ing, eg = e.run_host()
        wst, wing, weg = want
        assert np.array_equal(st, wst) and np.array_equal(ing, wing) and np.array_equal(eg, weg), seed


def test_one_prepare_serves_every_probe(gpu):
    """One cyc_probe_prepare_configs over every probe config, one run: each config's slots equal its
    own stand-alone prepare and run (the resident Resources and policy are loaded once)."""
    for seed in range(20):
        pols, res, probes = random_problem(420_000 + seed)
        if len(probes) < 2:
            probes = probes + [{"Port": 81, "Protocol": "TCP"}, {"AllAvailable": True}]
        e = Engine(0).build_policies(pols).load_resources_tables(res)
        e.prepare_configs(probes)
        try:
            st, ing, eg = e.run_host()
        except CyclonusPanic:
            continue
        k0 = 0
        for pr in probes:
            one = Engine(0).build_policies(pols).load_resources_tables(res)
            one.prepare_configs([pr])
            s1, i1, e1 = one.run_host()
            k = s1.shape[1]
            assert np.array_equal(st[:, k0:k0 + k], s1), (seed, pr)
            assert np.array_equal(ing[:, k0:k0 + k], i1) and np.array_equal(eg[:, k0:k0 + k], e1), (seed, pr)
            k0 += k
        assert k0 == st.shape[1]
