"""Pin the CPU oracle to the reference's own golden vectors (tests/golden/, see make_fixtures.py).

README.md:294-313 (combined table), pkg/kube/ipaddress_tests.go, labelselector_tests.go,
pkg/matcher/policy_tests.go, builder_tests.go and simplifier_tests.go.
"""
import json
import os

import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")
KAT = json.load(open(os.path.join(GOLD, "kat.json")))


def test_readme_combined_table():
    c = json.load(open(os.path.join(GOLD, "config1.json")))
    orc = O.Oracle(c["policies"], c["resources"], True)
    status, inp, egp = orc.probe(c["probes"])
    ing, eg = O.combined_table(status, inp, egp)
    names = [p["Namespace"] + "/" + p["Name"] for p in c["resources"]["Pods"]]
    exp = c["readme_combined_tcp80"]
    assert exp["header"] == sorted(n.upper() for n in names)
    for s, fr in enumerate(names):
        for d, to in enumerate(names):
            assert status[d, 0] == O.ST_VALID
            got = "." if (ing[s, d, 0] and eg[s, d, 0]) else "X"
            assert got == exp["rows"][fr][to.upper()], (fr, to)
    # probe 3 is TCP/82: no container serves it -> invalidportprotocol everywhere (resources.go:320-323)
    assert (status[:, 2] == O.ST_BAD_PORT_PROTOCOL).all()


@pytest.mark.parametrize("ip,cidr,member", KAT["ip"]["in_cidr"])
def test_ip_in_cidr(ip, cidr, member):
    assert O.ip_in_cidr(ip, cidr) == member


@pytest.mark.parametrize("ip,cidr,excepts,match", KAT["ip"]["ipblock"])
def test_ipblock(ip, cidr, excepts, match):
    assert O.ipblock_match(ip, cidr, []) is True or excepts == [] and not match
    assert O.ipblock_match(ip, cidr, excepts) == match


@pytest.mark.parametrize("ip,cidr,excepts", KAT["ip"]["errors"])
def test_ip_errors(ip, cidr, excepts):
    assert O.ipblock_match(ip, cidr, excepts) is None


@pytest.mark.parametrize("ip,bits,expected", KAT["ip"]["make_ipv4_cidr"])
def test_make_ipv4_cidr(ip, bits, expected):
    assert O.make_ipv4_cidr(ip, bits) == expected


@pytest.mark.parametrize("labels,selector,match", KAT["selector"]["cases"])
def test_selector(labels, selector, match):
    assert O.selector_match(labels, selector) == match


def test_selector_quirks():
    # labelselector.go:70 labels[k] != v: matchLabels {k: ""} matches a pod WITHOUT k
    assert O.selector_match({}, {"matchLabels": {"a": ""}})
    # :37-42 NotIn with the key absent is NOT a match (differs from upstream k8s)
    assert not O.selector_match({}, {"matchExpressions": [{"key": "a", "operator": "NotIn", "values": ["x"]}]})
    assert O.selector_match({"a": "y"}, {"matchExpressions": [{"key": "a", "operator": "NotIn", "values": ["x"]}]})
    assert O.selector_match({"a": ""}, {"matchExpressions": [{"key": "a", "operator": "Exists"}]})
    assert O.selector_match({}, {"matchExpressions": [{"key": "a", "operator": "DoesNotExist"}]})
    with pytest.raises(O.OraclePanic):
        O.selector_match({"a": "b"}, {"matchExpressions": [{"key": "a", "operator": "Bogus"}]})
    # a failed matchLabels short-circuits before a bad operator is reached
    assert not O.selector_match({}, {"matchLabels": {"a": "b"}, "matchExpressions": [{"key": "a", "operator": "Bogus"}]})


def test_go_net_semantics():
    # Go 1.16 net: v4-mapped addresses collapse to IPv4; ::/0 matches no IPv4; ::ffff:0:0/96 every IPv4
    assert O.ip_in_cidr("::ffff:10.1.2.3", "10.0.0.0/8") is True
    assert O.ip_in_cidr("10.1.2.3", "::/0") is False
    assert O.ip_in_cidr("10.1.2.3", "::ffff:0:0/96") is True
    assert O.ip_in_cidr("10.1.2.3", "::ffff:0:0/80") is False
    assert O.ip_in_cidr("fd00::1", "::/0") is True
    assert O.ip_in_cidr("010.001.002.003", "10.1.2.0/24") is True  # Go 1.16 accepts leading zeros
    assert O.ip_in_cidr("1.2.3.4", "1.2.3.4/33") is None
    assert O.ip_in_cidr("1.2.3", "1.2.3.0/24") is None


@pytest.mark.parametrize("case", KAT["policy"]["cases"], ids=lambda c: c["name"])
def test_policy_tests(case):
    orc = O.Oracle(case["policies"], None, True)
    (res,) = orc.query_traffic([case["traffic"]])
    assert (res[0] and res[1]) == case["allowed"]


def _single_target_peers(ir, direction):
    d = ir["Ingress" if direction == "ingress" else "Egress"]
    if not d:
        return "absent", None
    assert len(d) == 1
    (t,) = d.values()
    return t["Peers"], t


@pytest.mark.parametrize("case", KAT["builder"]["cases"], ids=lambda c: c["name"])
def test_builder_tests(case):
    ir = O.Oracle(case["policies"], None, case.get("simplify", True)).policy_json()
    for direction in ("ingress", "egress"):
        peers, t = _single_target_peers(ir, direction)
        assert peers == case[direction], direction
        if "namespace" in case and t is not None:
            assert t["Namespace"] == case["namespace"]


def test_compile_panics():
    bad_types = [{"metadata": {"name": "a", "namespace": "x"}, "spec": {"podSelector": {}}}]
    with pytest.raises(O.OraclePanic, match="need at least 1 type"):
        O.Oracle(bad_types)
    bad_range = [{"metadata": {"name": "a"}, "spec": {"podSelector": {}, "policyTypes": ["Ingress"],
                                                       "ingress": [{"ports": [{"port": 90, "endPort": 80}]}]}}]
    with pytest.raises(O.OraclePanic, match="end port < start port"):
        O.Oracle(bad_range)


def _describe(ir, direction, pks):
    """Primary keys -> {namespace, selector} of the targets (the README tables' TARGET column)."""
    return [{"namespace": ir[direction][pk]["Namespace"], "selector": ir[direction][pk]["PodSelector"]} for pk in pks]


def _source_rules(ir, direction, pks):
    out = set()
    for pk in pks:
        t = ir[direction][pk]
        for r in t["SourceRules"]:  # a target's rules all live in the target's namespace
            out.add(f"{t['Namespace']}/{r['metadata']['name']}")
    return out


def _key(d):
    return json.dumps(d, sort_keys=True)


def check_readme_queries(ir, traffic_result, target_result, q):
    """README.md:218-287 query-traffic / query-target examples against a result in the shape of
    cyc_query_traffic_targets / cyc_query_targets (target lists as primary keys)."""
    exp = q["query_traffic"]["expected"]
    for d in ("Ingress", "Egress"):
        for lst in ("AllowingTargets", "DenyingTargets"):
            got = sorted(map(_key, _describe(ir, d, traffic_result[d][lst])))
            assert got == sorted(map(_key, exp[d][lst])), (d, lst)
    assert traffic_result["IsAllowed"] == exp["IsAllowed"]
    for d in ("Ingress", "Egress"):
        assert _source_rules(ir, d, target_result[d]) == set(q["query_target"]["expected_source_rules"][d]), d


def test_readme_queries_oracle():
    c = json.load(open(os.path.join(GOLD, "config1.json")))
    q = c["readme_queries"]
    orc = O.Oracle(c["policies"], c["resources"])
    ir = orc.policy_json()
    (tr,) = orc.query_traffic_targets([q["query_traffic"]["traffic"]])
    (tg,) = orc.query_targets([q["query_target"]["pod"]])
    check_readme_queries(ir, tr, tg, q)
    # the lists agree with the pinned per-direction verdicts (policy.go:89-91)
    for t, (i, e) in zip(orc.query_traffic_targets(q["examples_traffic"]), orc.query_traffic(q["examples_traffic"])):
        assert t["Ingress"]["IsAllowed"] == i and t["Egress"]["IsAllowed"] == e
        for d in ("Ingress", "Egress"):
            assert t[d]["IsAllowed"] == (bool(t[d]["AllowingTargets"]) or not t[d]["DenyingTargets"])
    assert len(orc.query_targets(q["examples_targets"])) == len(q["examples_targets"])
