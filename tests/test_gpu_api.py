"""GPU tests of the reference-shaped API: matcher.IsTrafficAllowed (cyc_query_traffic) and the
probe Runner / Table view, against the oracle."""
import json
import os
import random

import numpy as np
import pytest

from cyclonus_amd._lib import CyclonusPanic
from cyclonus_amd.matcher import build_network_policies
from cyclonus_amd.probe import PlaneCells, Resources, Table, new_all_available, new_probe_config, new_simulated_runner
from oracle.oracle import Oracle, OraclePanic
from randgen import KEYS, NS, VALS, random_problem

GOLD = os.path.join(os.path.dirname(__file__), "golden")
KAT = json.load(open(os.path.join(GOLD, "kat.json")))
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", KAT["policy"]["cases"], ids=lambda c: c["name"])
def test_policy_tests_kats_gpu(gpu, case):
    pol = build_network_policies(True, case["policies"])
    assert pol.is_traffic_allowed(case["traffic"]).is_allowed() == case["allowed"]


def _random_traffic(r, bad):
    def end():
        if r.random() < 0.25:
            ip = r.choice(["1.2.3.4", "10.1.2.3", "fd00:10::1", "::ffff:10.1.2.9", "192.168.1.5"])
            if bad and r.random() < 0.2:
                ip = r.choice(["", "nope"])
            return {"Internal": None, "IP": ip}
        labels = {k: r.choice(VALS) for k in r.sample(KEYS, r.randint(0, 3))} if r.random() < 0.9 else None
        nsl = {"ns": r.choice(NS)} if r.random() < 0.8 else None
        ip = r.choice(["10.1.2.%d" % r.randint(0, 255), "192.168.1.%d" % r.randint(0, 20), "fd00:10::%x" % r.randint(0, 300)])
        if bad and r.random() < 0.1:
            ip = "TODO"
        return {"Internal": {"PodLabels": labels, "NamespaceLabels": nsl, "Namespace": r.choice(NS)}, "IP": ip}

    return {"Source": end(), "Destination": end(), "ResolvedPort": r.choice([80, 81, 53, 443, 9000]),
            "ResolvedPortName": r.choice(["", "serve-80-tcp", "serve-53-udp", "http"]),
            "Protocol": r.choice(["TCP", "UDP", "SCTP", "tcp"])}


@pytest.mark.parametrize("bad", [False, True])
def test_query_traffic_random(gpu, bad):
    r = random.Random(99 + bad)
    for seed in range(120):
        pols, _, _ = random_problem(20_000 + seed + 1000 * bad, bad=bad)
        traffics = [_random_traffic(r, bad) for _ in range(50)]
        try:
            orc = Oracle(pols)
        except OraclePanic:
            continue
        want = []
        want_panic = None
        for t in traffics:  # analyze.go:209-225 stops at the first panicking traffic
            (res,) = orc.query_traffic([t])
            if isinstance(res, OraclePanic):
                want_panic = str(res)
                break
            want.append(res)
        pol = build_network_policies(True, pols)
        for query in (pol.engine.query_traffic, pol.engine.query_traffic_tables):  # JSON and flat tables
            if want_panic is not None:
                with pytest.raises(CyclonusPanic) as e:
                    query(traffics)
                assert e.value.msg == want_panic, seed
            else:
                assert query(traffics) == want, seed


def test_readme_queries_gpu(gpu):
    """README.md:218-287 query-traffic / query-target examples through the GPU entry points."""
    from test_oracle_golden import check_readme_queries

    c = json.load(open(os.path.join(GOLD, "config1.json")))
    q = c["readme_queries"]
    pol = build_network_policies(True, c["policies"])
    ir = pol.to_json()
    (tr,) = pol.engine.query_traffic_targets([q["query_traffic"]["traffic"]])
    (tg,) = pol.query_targets([q["query_target"]["pod"]])
    check_readme_queries(ir, tr, tg, q)
    res = pol.is_traffic_allowed(q["query_traffic"]["traffic"])
    assert not res.is_allowed() and res.ingress.is_allowed() and not res.egress.is_allowed()
    orc = Oracle(c["policies"], c["resources"])
    assert pol.engine.query_traffic_targets(q["examples_traffic"]) == orc.query_traffic_targets(q["examples_traffic"])
    assert pol.query_targets(q["examples_targets"]) == orc.query_targets(q["examples_targets"])


@pytest.mark.parametrize("bad", [False, True])
def test_query_targets_random(gpu, bad):
    """Target lists (query-traffic) and TargetsApplyingToPod (query-target) vs the oracle,
    including the first panicking traffic / pod."""
    r = random.Random(7 + bad)
    for seed in range(80):
        pols, _, _ = random_problem(40_000 + seed + 1000 * bad, bad=bad)
        try:
            orc = Oracle(pols)
        except OraclePanic:
            continue
        pol = build_network_policies(True, pols)
        traffics = [_random_traffic(r, bad) for _ in range(30)]
        try:
            want = orc.query_traffic_targets(traffics)
        except OraclePanic as e:
            with pytest.raises(CyclonusPanic) as g:
                pol.engine.query_traffic_targets(traffics)
            assert g.value.msg == str(e), seed
        else:
            assert pol.engine.query_traffic_targets(traffics) == want, seed
        pods = [{"Namespace": r.choice(NS), "Labels": {k: r.choice(VALS) for k in r.sample(KEYS, r.randint(0, 3))}}
                for _ in range(20)]
        try:
            want = orc.query_targets(pods)
        except OraclePanic as e:
            with pytest.raises(CyclonusPanic) as g:
                pol.query_targets(pods)
            assert g.value.msg == str(e), seed
        else:
            assert pol.query_targets(pods) == want, seed


def test_runner_tables_match_oracle_render(gpu):
    c = json.load(open(os.path.join(GOLD, "config1.json")))
    pol = build_network_policies(True, c["policies"])
    runner = new_simulated_runner(pol)
    res = Resources.from_json(c["resources"])
    tables = runner.run_probes(c["probes"], res)
    st, inp, egp = Oracle(c["policies"], c["resources"]).probe(c["probes"])
    for i, (t, p) in enumerate(zip(tables, c["probes"])):
        o = Table(res, new_probe_config(p["Port"], p["Protocol"]), PlaneCells(st, inp, egp), i, i + 1)
        for fn in ("render_ingress", "render_egress", "render_table"):
            assert getattr(t, fn)() == getattr(o, fn)()
    assert tables[0].render_table() == c["readme_combined_tcp80"]["text"]


def test_runner_all_available_and_named(gpu):
    pols, resd, _ = random_problem(4242, n_pods=12, n_pols=8)
    pol = build_network_policies(True, pols)
    runner = new_simulated_runner(pol)
    res = Resources.from_json(resd)
    probes = [new_all_available(), new_probe_config("serve-80-tcp", "TCP"), new_probe_config(81, "UDP")]
    tables = runner.run_probes(probes, res)
    st, inp, egp = Oracle(pols, resd).probe([p.to_json() for p in probes])
    maxc = max(len(p.containers) for p in res.pods)
    lo = 0
    for t, p in zip(tables, probes):
        n = maxc if p.all_available else 1
        o = Table(res, p, PlaneCells(st, inp, egp), lo, lo + n)
        lo += n
        for fr, to in t.keys():
            assert t.get(fr, to) == o.get(fr, to)
        try:
            want = o.render_table()
        except CyclonusPanic:
            with pytest.raises(CyclonusPanic):
                t.render_table()
            continue
        assert t.render_table() == want


def test_config1_through_yaml_loader(gpu):
    """analyze --mode probe's input path on the reference's own files: the policy directory
    networkpolicies/simple-example (copied byte for byte to tests/golden/yaml/, read as
    cli/utils.go:14-60 does) -> BuildNetworkPolicies -> GPU table -> README.md:294-313 byte for byte."""
    from cyclonus_amd.loader import read_policies_from_path

    c = json.load(open(os.path.join(GOLD, "config1.json")))
    pols = read_policies_from_path(os.path.join(GOLD, "yaml", "simple-example"))
    assert json.dumps(pols, sort_keys=True) == json.dumps(c["policies"], sort_keys=True)
    runner = new_simulated_runner(build_network_policies(True, pols))
    table = runner.run_probe_for_config(new_probe_config(80, "TCP"), Resources.from_json(c["resources"]))
    assert table.render_table() == c["readme_combined_tcp80"]["text"]
