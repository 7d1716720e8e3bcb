#!/usr/bin/env python3
"""Regenerate the committed golden fixtures from the reference's own data files and tests.

Run in the build container only (it reads /root/reference, which does not exist on the GPU
box).  Everything written here is DATA: inputs and expected outputs.

  config1.json        networkpolicies/simple-example/*.yaml (filepath.Walk = lexical order),
                      examples/probe.json, and the Combined table of README.md:294-313.
  policy_fixtures.json  other YAML policy fixtures (upstream_test_cases, features/portrange1,
                      allow-all*.yaml) converted to k8s JSON.
  kat.json            known-answer vectors transcribed from the reference's Ginkgo tests:
                      pkg/kube/ipaddress_tests.go:14-203, labelselector_tests.go:11-15,
                      pkg/matcher/policy_tests.go:12-223, builder_tests.go:23-342,
                      simplifier_tests.go (structural cases restated as end-to-end policies).
"""
import glob
import json
import os
import re

import yaml

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def load_yaml_policies(path):
    with open(path) as f:
        doc = yaml.safe_load(f)
    return doc if isinstance(doc, list) else [doc]


def readme_combined_table():
    """Transcribe README.md:294-313 (analyze --mode probe, simple-example, TCP/80)."""
    lines = open(os.path.join(REF, "README.md")).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.strip() == "Combined:" and i > 280)
    rows = [l for l in lines[start + 1 : start + 20] if l.startswith("|")]
    header = [c.strip() for c in rows[0].strip("|").split("|")]
    table = {}
    for r in rows[1:]:
        cells = [c.strip() for c in r.strip("|").split("|")]
        table[cells[0]] = dict(zip(header[1:], cells[1:]))
    raw = [l for l in lines[start + 1 : start + 20] if l.startswith("+") or l.startswith("|")]
    return {"header": header[1:], "rows": table, "text": "\n".join(raw) + "\n"}


def readme_queries():
    """README.md:218-287 (analyze --mode query-target / query-traffic on simple-example),
    transcribed: the query-traffic example's traffic (its Traffic table, :262-268) with the
    Type / Action / Target rows of its result table (:271-287), and the query-target example
    (:229-246) as the SOURCE RULES of the targets combined per direction."""
    lines = open(os.path.join(REF, "README.md")).read().splitlines()
    assert "192.168.1.99" in lines[264] and "192.168.1.100" in lines[266] and "IS ALLOWED?" in lines[285]
    traffic = {
        "Source": {"Internal": {"PodLabels": {"app": "c"}, "NamespaceLabels": {"ns": "y"}, "Namespace": "y"},
                   "IP": "192.168.1.99"},
        "Destination": {"Internal": {"PodLabels": {"pod": "b"}, "NamespaceLabels": {"ns": "y"}, "Namespace": "y"},
                        "IP": "192.168.1.100"},
        "ResolvedPort": 80, "ResolvedPortName": "serve-80-tcp", "Protocol": "TCP",
    }
    all_pods = {"namespace": "y", "selector": {}}
    pod_b = {"namespace": "y", "selector": {"matchLabels": {"pod": "b"}}}
    return {
        "query_traffic": {
            "source": "README.md:251-287",
            "traffic": traffic,
            "expected": {"Ingress": {"AllowingTargets": [pod_b], "DenyingTargets": [all_pods]},
                         "Egress": {"AllowingTargets": [], "DenyingTargets": [all_pods]},
                         "IsAllowed": False},
        },
        "query_target": {
            "source": "README.md:218-246",
            "pod": {"Namespace": "y", "Labels": {"pod": "a"}},
            "expected_source_rules": {
                "Ingress": ["y/allow-label-to-label", "y/deny-all-for-label", "y/deny-all"],
                "Egress": ["y/deny-all-egress", "y/allow-all-egress-by-label"],
            },
        },
        "examples_targets": json.load(open(os.path.join(REF, "examples/targets.json"))),
        "examples_traffic": json.load(open(os.path.join(REF, "examples/traffic.json"))),
    }


def config1():
    files = sorted(glob.glob(os.path.join(REF, "networkpolicies/simple-example/*.yaml")))
    policies = []
    for f in files:
        policies += load_yaml_policies(f)
    probe = json.load(open(os.path.join(REF, "examples/probe.json")))
    return {
        "source": "networkpolicies/simple-example/*.yaml + examples/probe.json; expected = README.md:294-313",
        "policies": policies,
        "resources": probe["Resources"],
        "probes": probe["Probes"],
        "readme_combined_tcp80": readme_combined_table(),
        "readme_queries": readme_queries(),
    }


def policy_fixtures():
    out = {}
    for rel in [
        "networkpolicies/upstream_test_cases/allow-to-ns-y-pod-a.yaml",
        "networkpolicies/features/portrange1.yaml",
        "networkpolicies/allow-all.yaml",
        "networkpolicies/allow-all-internal.yaml",
    ]:
        out[rel] = load_yaml_policies(os.path.join(REF, rel))
    return out


# ----------------------------------------------------------------------------- KATs
def ip_kats():
    # ipaddress_tests.go:14-47 IsIPInCIDR
    in_cidr = [
        ["1.2.3.3", "1.2.3.0/24", True],
        ["1.2.3.3", "1.2.3.0/28", True],
        ["1.2.3.3", "1.2.3.0/30", True],
        ["1.2.3.3", "1.2.3.0/31", False],
    ]
    # :63-107 IPBlocks without except; :109-155 with except (and without-except must match)
    block = [
        ["1.2.3.3", "1.2.3.0/24", [], True],
        ["1.2.3.3", "1.2.3.0/28", [], True],
        ["1.2.3.3", "1.2.3.0/30", [], True],
        ["1.2.3.3", "1.2.3.0/31", [], False],
        ["1.2.3.3", "1.2.3.0/28", ["1.2.3.0/30"], False],
        ["1.2.3.4", "1.2.3.0/28", ["1.2.3.4/30"], False],
        ["1.2.3.3", "1.2.3.0/28", ["1.2.3.4/30"], True],
    ]
    # :55-61 malformed IP / CIDR must error
    errors = [["abc", "1.2.3.4", []]]
    # :158-201 MakeIPV4CIDR
    make = [
        ["255.255.255.255", 32, "255.255.255.255/32"],
        ["255.255.255.255", 31, "255.255.255.254/31"],
        ["255.255.255.255", 30, "255.255.255.252/30"],
        ["255.255.255.255", 28, "255.255.255.240/28"],
        ["255.255.255.255", 24, "255.255.255.0/24"],
        ["255.255.255.255", 16, "255.255.0.0/16"],
    ]
    return {"source": "pkg/kube/ipaddress_tests.go", "in_cidr": in_cidr, "ipblock": block, "errors": errors, "make_ipv4_cidr": make}


def selector_kats():
    # labelselector_tests.go:11-15
    return {"source": "pkg/kube/labelselector_tests.go:11-15", "cases": [[{}, {"matchLabels": {"pod": "b"}}, False]]}


def traffic(src_ns, src_labels, src_nslabels, src_ip, dst_ns, dst_labels, dst_nslabels, dst_ip, port, name, proto, src_external=False):
    def peer(ns, labels, nslabels, ip, external):
        return {"Internal": None if external else {"PodLabels": labels, "NamespaceLabels": nslabels, "Namespace": ns}, "IP": ip}

    return {
        "Source": peer(src_ns, src_labels, src_nslabels, src_ip, src_external),
        "Destination": peer(dst_ns, dst_labels, dst_nslabels, dst_ip, False),
        "ResolvedPort": port,
        "ResolvedPortName": name,
        "Protocol": proto,
    }


def policy_test_kats():
    """pkg/matcher/policy_tests.go:12-223 — BuildNetworkPolicies(true) + IsTrafficAllowed."""
    sctp = yaml.safe_load(
        """
apiVersion: networking.k8s.io/v1
kind: NetworkPolicy
metadata:
  name: policy-207
  namespace: x
spec:
  ingress:
  - ports:
    - protocol: SCTP
  podSelector: {}
  policyTypes:
  - Ingress"""
    )
    egress_ips = yaml.safe_load(
        """
apiVersion: networking.k8s.io/v1
kind: NetworkPolicy
metadata:
  creationTimestamp: null
  name: vary-egress-37-0-0-0-19
  namespace: x
spec:
  egress:
  - ports:
    - port: 80
      protocol: TCP
    to:
    - podSelector: {}
    - ipBlock:
        cidr: 192.168.242.213/24
  - ports:
    - port: 53
      protocol: UDP
  podSelector:
    matchLabels:
      pod: a
  policyTypes:
  - Egress"""
    )
    named = yaml.safe_load(
        """
apiVersion: networking.k8s.io/v1
kind: NetworkPolicy
metadata:
  name: abc
  namespace: x
spec:
  ingress:
  - ports:
    - port: port-hello
      protocol: TCP
  podSelector:
    matchLabels:
      pod: a
  policyTypes:
  - Ingress"""
    )
    t_tcp = traffic("y", None, None, "1.2.3.4", "x", None, None, "1.2.3.5", 103, "", "TCP")
    t_sctp = traffic("y", None, None, "1.2.3.4", "x", None, None, "1.2.3.5", 103, "", "SCTP")
    t_tcp_ext = traffic("", None, None, "1.2.3.4", "x", None, None, "1.2.3.5", 103, "", "TCP", src_external=True)
    t_sctp_ext = traffic("", None, None, "1.2.3.4", "x", None, None, "1.2.3.5", 103, "", "SCTP", src_external=True)
    t_ips = traffic("x", {"pod": "a"}, {"ns": "x"}, "1.2.3.4", "y", {"pod": "b"}, {"ns": "y"}, "192.168.242.249", 80, "", "TCP")
    t_named = traffic("", None, None, "1.2.3.4", "x", {"pod": "a"}, {"ns": "x"}, "192.168.242.249", 0, "port-hello", "TCP", src_external=True)
    return {
        "source": "pkg/matcher/policy_tests.go",
        "cases": [
            {"name": "sctp-only: TCP from pod denied (:31-56)", "policies": [sctp], "traffic": t_tcp, "allowed": False},
            {"name": "sctp-only: SCTP from pod allowed (:58-81)", "policies": [sctp], "traffic": t_sctp, "allowed": True},
            {"name": "sctp-only: TCP from ip denied (:85-103)", "policies": [sctp], "traffic": t_tcp_ext, "allowed": False},
            {"name": "sctp-only: SCTP from ip allowed (:105-123)", "policies": [sctp], "traffic": t_sctp_ext, "allowed": True},
            {"name": "egress to ips in cidr (:155-179)", "policies": [egress_ips], "traffic": t_ips, "allowed": True},
            {"name": "ingress to named port (:201-221)", "policies": [named], "traffic": t_named, "allowed": True},
        ],
    }


NS = "pathological-namespace"


def np_(name, types, ingress=None, egress=None, ns=NS):
    spec = {"podSelector": {}, "policyTypes": types}
    if ingress is not None:
        spec["ingress"] = ingress
    if egress is not None:
        spec["egress"] = egress
    md = {"name": name}
    if ns is not None:
        md["namespace"] = ns
    return {"metadata": md, "spec": spec}


def builder_kats():
    """pkg/matcher/builder_tests.go — compiled peer structure in json.Marshal(*matcher.Policy) form.

    Each case: policies (k8s JSON), simplify flag, and for each direction the expected Peers list
    (None == Go nil) of the single target, in the matcher JSON encoding."""
    ALLP = {"Type": "all peers"}
    ALLPORTS = {"Type": "all ports"}

    def sp(ports=None, ranges=None):
        return {"PortRanges": ranges, "Ports": ports, "Type": "specific ports"}

    cases = [
        # :24-58 nil ingress/egress
        {"name": "allow-no-ingress", "policies": [np_("allow-no-ingress", ["Ingress"])], "ingress": None, "egress": "absent"},
        {"name": "allow-no-egress", "policies": [np_("allow-no-egress", ["Egress"])], "ingress": "absent", "egress": None},
        {"name": "allow-neither", "policies": [np_("allow-no-ingress-allow-no-egress", ["Egress", "Ingress"])], "ingress": None, "egress": None},
        # :72-99 empty ingress/egress
        {"name": "allow-no-ingress-empty", "policies": [np_("a", ["Ingress"], ingress=[])], "ingress": None, "egress": "absent"},
        {"name": "allow-no-egress-empty", "policies": [np_("a", ["Egress"], egress=[])], "ingress": "absent", "egress": None},
        {"name": "allow-neither-empty", "policies": [np_("a", ["Egress", "Ingress"], ingress=[], egress=[])], "ingress": None, "egress": None},
        # :102-125 allow all
        {"name": "allow-all-ingress", "policies": [np_("a", ["Ingress"], ingress=[{}])], "ingress": [ALLP], "egress": "absent"},
        {"name": "allow-all-egress", "policies": [np_("a", ["Egress"], egress=[{}])], "ingress": "absent", "egress": [ALLP]},
        {"name": "allow-all-both", "policies": [np_("a", ["Egress", "Ingress"], ingress=[{}], egress=[{}])], "ingress": [ALLP], "egress": [ALLP]},
        # :60-70 missing namespace -> "default"
        {"name": "missing-namespace", "policies": [np_("abc", ["Ingress", "Egress"], ingress=[], ns=None)], "ingress": None, "egress": None, "namespace": "default"},
        # :147-182 egress rules -> [pod(exact abc, all pods, 80/TCP), ip(80/TCP), portsForAll(53/UDP)]  (unsimplified)
        {
            "name": "dns-and-ipblock (unsimplified)",
            "simplify": False,
            "policies": [
                np_(
                    "dns",
                    ["Egress"],
                    egress=[
                        {"ports": [{"port": 80, "protocol": "TCP"}], "to": [{"podSelector": {}}, {"ipBlock": {"cidr": "192.168.242.213/24"}}]},
                        {"ports": [{"port": 53, "protocol": "UDP"}]},
                    ],
                    ns="abc",
                )
            ],
            "ingress": "absent",
            "egress": [
                {"Namespace": {"Namespace": "abc", "Type": "specific namespace"}, "Pod": {"Type": "all pods"}, "Port": sp([{"Port": 80, "Protocol": "TCP"}])},
                {"CIDR": "192.168.242.213/24", "Except": None, "Port": sp([{"Port": 80, "Protocol": "TCP"}]), "Type": "IPBlock"},
                {"Port": sp([{"Port": 53, "Protocol": "UDP"}]), "Type": "all peers for port"},
            ],
        },
        # :186-236 BuildPeerMatcher cases
        {"name": "ports-for-all sctp/103", "simplify": False,
         "policies": [np_("a", ["Ingress"], ingress=[{"ports": [{"protocol": "SCTP", "port": 103}]}], ns="abc")],
         "ingress": [{"Port": sp([{"Port": 103, "Protocol": "SCTP"}]), "Type": "all peers for port"}], "egress": "absent"},
        {"name": "single ipblock", "simplify": False,
         "policies": [np_("a", ["Ingress"], ingress=[{"from": [{"ipBlock": {"cidr": "10.0.0.1/24", "except": ["10.0.0.2/30"]}}]}], ns="abc")],
         "ingress": [{"CIDR": "10.0.0.1/24", "Except": ["10.0.0.2/30"], "Port": ALLPORTS, "Type": "IPBlock"}], "egress": "absent"},
        {"name": "empty pod+ns selectors", "simplify": False,
         "policies": [np_("a", ["Ingress"], ingress=[{"from": [{"podSelector": {}, "namespaceSelector": {}}]}], ns="abc")],
         "ingress": [{"Namespace": {"Type": "all namespaces"}, "Pod": {"Type": "all pods"}, "Port": ALLPORTS}], "egress": "absent"},
        {"name": "empty pod selector only", "simplify": False,
         "policies": [np_("a", ["Ingress"], ingress=[{"from": [{"podSelector": {}}]}], ns="abc")],
         "ingress": [{"Namespace": {"Namespace": "abc", "Type": "specific namespace"}, "Pod": {"Type": "all pods"}, "Port": ALLPORTS}], "egress": "absent"},
        # :239-318 BuildIPBlockNamespacePodMatcher (6 ns x pod combos)
        {"name": "ns/pod combos", "simplify": False,
         "policies": [np_("a", ["Ingress"], ns=NS, ingress=[{"from": [
             {"podSelector": {"matchLabels": {"b": "d"}}},
             {"podSelector": {"matchLabels": {"e": "f"}}, "namespaceSelector": {}},
             {"podSelector": {"matchLabels": {"g": "g"}}, "namespaceSelector": {"matchLabels": {"a": "b"}}},
             {"namespaceSelector": {"matchLabels": {"a": "b"}}},
             {"podSelector": {}, "namespaceSelector": {"matchLabels": {"a": "b"}}},
         ]}])],
         "ingress": [
             {"Namespace": {"Namespace": NS, "Type": "specific namespace"}, "Pod": {"Selector": {"matchLabels": {"b": "d"}}, "Type": "matching pods by label"}, "Port": ALLPORTS},
             {"Namespace": {"Type": "all namespaces"}, "Pod": {"Selector": {"matchLabels": {"e": "f"}}, "Type": "matching pods by label"}, "Port": ALLPORTS},
             {"Namespace": {"Selector": {"matchLabels": {"a": "b"}}, "Type": "matching namespace by label"}, "Pod": {"Selector": {"matchLabels": {"g": "g"}}, "Type": "matching pods by label"}, "Port": ALLPORTS},
             {"Namespace": {"Selector": {"matchLabels": {"a": "b"}}, "Type": "matching namespace by label"}, "Pod": {"Type": "all pods"}, "Port": ALLPORTS},
             {"Namespace": {"Selector": {"matchLabels": {"a": "b"}}, "Type": "matching namespace by label"}, "Pod": {"Type": "all pods"}, "Port": ALLPORTS},
         ], "egress": "absent"},
        # :321-341 Port from NetworkPolicyPort
        {"name": "port matchers", "simplify": False,
         "policies": [np_("a", ["Ingress"], ns="abc", ingress=[
             {"ports": [{"protocol": "SCTP"}], "from": [{"podSelector": {}}]},
             {"ports": [{"protocol": "TCP", "port": 9001}], "from": [{"podSelector": {}}]},
             {"ports": [{"protocol": "UDP", "port": "hello"}], "from": [{"podSelector": {}}]},
         ])],
         "ingress": [
             {"Namespace": {"Namespace": "abc", "Type": "specific namespace"}, "Pod": {"Type": "all pods"}, "Port": sp([{"Port": None, "Protocol": "SCTP"}])},
             {"Namespace": {"Namespace": "abc", "Type": "specific namespace"}, "Pod": {"Type": "all pods"}, "Port": sp([{"Port": 9001, "Protocol": "TCP"}])},
             {"Namespace": {"Namespace": "abc", "Type": "specific namespace"}, "Pod": {"Type": "all pods"}, "Port": sp([{"Port": "hello", "Protocol": "UDP"}])},
         ], "egress": "absent"},
        # simplifier_tests.go:36-56 — Simplify([all, allOnTCP80, ip, allPodsAllPorts, allPodsTCP103]) == [all]
        {"name": "simplify: all wins", "simplify": True,
         "policies": [np_("a", ["Ingress"], ns="abc", ingress=[
             {},
             {"ports": [{"port": 80, "protocol": "TCP"}]},
             {"from": [{"ipBlock": {"cidr": "10.0.0.1/24", "except": ["10.0.0.2/30"]}}]},
             {"from": [{"podSelector": {}, "namespaceSelector": {}}]},
             {"ports": [{"port": 103, "protocol": "TCP"}], "from": [{"podSelector": {}, "namespaceSelector": {}}]},
         ])],
         "ingress": [ALLP], "egress": "absent"},
        # simplifier_tests.go:55 — Simplify([allOnTCP80, allPodsAllPorts]) == same
        {"name": "simplify: ports-for-all + all pods", "simplify": True,
         "policies": [np_("a", ["Ingress"], ns="abc", ingress=[
             {"ports": [{"port": 80, "protocol": "TCP"}]},
             {"from": [{"podSelector": {}, "namespaceSelector": {}}]},
         ])],
         "ingress": [{"Port": sp([{"Port": 80, "Protocol": "TCP"}]), "Type": "all peers for port"},
                     {"Namespace": {"Type": "all namespaces"}, "Pod": {"Type": "all pods"}, "Port": ALLPORTS}], "egress": "absent"},
        # simplifier_tests.go:71-74 — simplifyPortsForAllPeers([tcp80, tcp103]) == [80/TCP, 103/TCP]
        {"name": "simplify: combine ports-for-all", "simplify": True,
         "policies": [np_("a", ["Ingress"], ns="abc", ingress=[
             {"ports": [{"port": 103, "protocol": "TCP"}]},
             {"ports": [{"port": 80, "protocol": "TCP"}]},
         ])],
         "ingress": [{"Port": sp([{"Port": 80, "Protocol": "TCP"}, {"Port": 103, "Protocol": "TCP"}]), "Type": "all peers for port"}], "egress": "absent"},
        # simplifier_tests.go:76-93 — dns + pod with port range are not mixed
        {"name": "simplify: dns + port range pod", "simplify": True,
         "policies": [np_("a", ["Ingress"], ns="abc", ingress=[
             {"ports": [{"port": 53, "protocol": "UDP"}]},
             {"ports": [{"port": 80, "endPort": 103, "protocol": "TCP"}], "from": [{"podSelector": {"matchLabels": {"app": "x"}}, "namespaceSelector": {}}]},
         ])],
         "ingress": [{"Port": sp([{"Port": 53, "Protocol": "UDP"}]), "Type": "all peers for port"},
                     {"Namespace": {"Type": "all namespaces"}, "Pod": {"Selector": {"matchLabels": {"app": "x"}}, "Type": "matching pods by label"},
                      "Port": sp(None, [{"From": 80, "Protocol": "TCP", "To": 103, "Type": "port range"}])}], "egress": "absent"},
    ]
    return {"source": "pkg/matcher/builder_tests.go, simplifier_tests.go", "cases": cases}


def policy_yaml_files():
    """networkpolicies/**/*.yaml copied byte for byte (data: the policy inputs config #1 and the
    policy fixtures are read from, cli/utils.go:14-60) into tests/golden/yaml/, so the product's YAML
    loader is tested on the reference's own policy text."""
    import shutil

    src_root = os.path.join(REF, "networkpolicies")
    dst_root = os.path.join(OUT, "yaml")
    for f in sorted(glob.glob(os.path.join(src_root, "**", "*.yaml"), recursive=True)):
        dst = os.path.join(dst_root, os.path.relpath(f, src_root))
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        shutil.copyfile(f, dst)


def main():
    policy_yaml_files()
    json.dump(config1(), open(os.path.join(OUT, "config1.json"), "w"), indent=1, sort_keys=True)
    json.dump(policy_fixtures(), open(os.path.join(OUT, "policy_fixtures.json"), "w"), indent=1, sort_keys=True)
    kat = {"ip": ip_kats(), "selector": selector_kats(), "policy": policy_test_kats(), "builder": builder_kats()}
    json.dump(kat, open(os.path.join(OUT, "kat.json"), "w"), indent=1, sort_keys=True)
    print("wrote fixtures to", OUT)


if __name__ == "__main__":
    main()
