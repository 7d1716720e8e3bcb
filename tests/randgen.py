"""Seeded random NetworkPolicy / Resources generator for parity tests.

Covers every matcher feature of the reference's verdict path: nil vs empty rule lists, all six
namespace x pod selector combinations, matchLabels (incl. empty-string values) and every
matchExpressions operator, IPBlock with nested excepts (IPv4, IPv6, v4-mapped, edge prefixes),
numbered / named / nil ports, endPort ranges, TCP/UDP/SCTP and raw lower-case protocols,
duplicate rules (simplifier merges), pods with duplicated IPs, missing namespaces, AllAvailable
and PortProtocol probes.  `panics=True` also mixes in inputs that make the reference panic.
"""
from __future__ import annotations

import random

NS = ["x", "y", "z", "w"]
KEYS = ["pod", "app", "tier", "env"]
VALS = ["a", "b", "c", "d", ""]
PROTOS = ["TCP", "UDP", "SCTP"]


def _labels(r: random.Random, maxn=3):
    n = r.randint(0, maxn)
    return {k: r.choice(VALS) for k in r.sample(KEYS, n)}


def _selector(r: random.Random, allow_empty=True):
    if allow_empty and r.random() < 0.25:
        return {}
    s = {}
    if r.random() < 0.6:
        s["matchLabels"] = {k: r.choice(VALS) for k in r.sample(KEYS, r.randint(1, 2))}
    if r.random() < 0.5 or not s:
        exprs = []
        for _ in range(r.randint(1, 2)):
            op = r.choice(["In", "NotIn", "Exists", "DoesNotExist"])
            e = {"key": r.choice(KEYS), "operator": op}
            if op in ("In", "NotIn"):
                e["values"] = r.sample(VALS, r.randint(1, 3))
            exprs.append(e)
        s["matchExpressions"] = exprs
    return s


V4_CIDRS = ["10.0.0.0/8", "10.1.0.0/16", "10.1.2.0/24", "10.1.2.8/29", "10.1.2.3/32", "0.0.0.0/0", "192.168.1.0/24",
            "192.168.1.0/28", "10.1.2.128/25", "172.16.0.0/12"]
V6_CIDRS = ["fd00::/8", "fd00:10::/64", "fd00:10::/120", "::/0", "::ffff:0:0/96", "::ffff:10.1.0.0/112",
            "::ffff:0:0/80", "2001:db8::/32", "fd00:10::5/128"]
BAD_CIDRS = ["10.0.0.1", "10.0.0.0/33", "abc/8", "fd00::/129", "1.2.3.4/-1"]


def _cidr(r: random.Random, v6: bool, bad: bool):
    if bad and r.random() < 0.15:
        return r.choice(BAD_CIDRS)
    if v6 and r.random() < 0.4:
        return r.choice(V6_CIDRS)
    return r.choice(V4_CIDRS)


def _ports(r: random.Random, bad: bool):
    n = r.choice([0, 0, 1, 1, 2, 3])
    out = []
    for _ in range(n):
        p = {}
        if r.random() < 0.7:
            p["protocol"] = r.choice(PROTOS)
        kind = r.random()
        if kind < 0.45:
            p["port"] = r.choice([80, 81, 53, 443, 8080])
        elif kind < 0.7:
            p["port"] = r.choice(["serve-80-tcp", "serve-81-udp", "serve-53-udp", "http", "dns"])
        elif kind < 0.9:
            lo = r.choice([50, 80, 81, 100])
            p["port"] = lo
            p["endPort"] = lo + r.choice([0, 1, 5, 400])
        out.append(p)
    return out


def _peer(r: random.Random, v6: bool, bad: bool):
    k = r.random()
    if k < 0.25:
        ib = {"cidr": _cidr(r, v6, bad)}
        if r.random() < 0.5:
            ib["except"] = [_cidr(r, v6, bad) for _ in range(r.randint(1, 3))]
        return {"ipBlock": ib}
    p = {}
    c = r.randint(0, 5)
    if c in (1, 3, 5):
        p["podSelector"] = _selector(r)
    if c in (2, 3, 4, 5):
        p["namespaceSelector"] = _selector(r) if c != 4 else {}
    if not p:
        p["podSelector"] = {}
    return p


def random_policy(r: random.Random, i: int, v6=False, bad=False):
    types = r.choice([["Ingress"], ["Egress"], ["Ingress", "Egress"], ["Egress", "Ingress"]])
    spec = {"podSelector": _selector(r), "policyTypes": types}
    for t in types:
        key = "ingress" if t == "Ingress" else "egress"
        pk = "from" if t == "Ingress" else "to"
        c = r.random()
        if c < 0.1:
            continue  # nil rules
        if c < 0.2:
            spec[key] = []
            continue
        rules = []
        for _ in range(r.randint(1, 3)):
            rule = {}
            ports = _ports(r, bad)
            if ports:
                rule["ports"] = ports
            if r.random() < 0.8:
                peers = [_peer(r, v6, bad) for _ in range(r.randint(1, 3))]
                if r.random() < 0.15 and peers:
                    peers.append(dict(peers[0]))  # duplicate peer -> simplifier merge
                rule[pk] = peers
            rules.append(rule)
        spec[key] = rules
    md = {"name": f"p{i}"}
    if r.random() < 0.95:
        md["namespace"] = r.choice(NS)
    if bad and r.random() < 0.05:
        spec["podSelector"] = {"matchExpressions": [{"key": "pod", "operator": "Bogus"}]}
    return {"apiVersion": "networking.k8s.io/v1", "kind": "NetworkPolicy", "metadata": md, "spec": spec}


def random_resources(r: random.Random, n_pods: int, v6=False, bad=False, dups=False):
    nss = {}
    for ns in NS[:3]:
        nss[ns] = {"ns": ns, **_labels(r, 2)} if r.random() < 0.9 else None
    pods = []
    for i in range(n_pods):
        ns = r.choice(NS)  # "w" has no Namespaces entry -> nil namespace labels
        if v6 and r.random() < 0.3:
            ip = r.choice([f"fd00:10::{i + 1:x}", f"::ffff:10.1.2.{i % 250}", f"2001:db8::{i:x}"])
        else:
            ip = r.choice([f"10.1.2.{i % 250}", f"10.1.{r.randint(0, 3)}.{i % 250}", f"192.168.1.{i % 250}"])
        if bad and r.random() < 0.05:
            ip = r.choice(["", "TODO", "10.1.2"])
        conts = []
        used = set()
        for j in range(r.randint(1, 4)):
            port = r.choice([80, 81, 53, 443, 8080, 9000])
            proto = r.choice(PROTOS + ["tcp"])
            if (proto, port) in used and not (dups and r.random() < 0.3):
                continue
            used.add((proto, port))
            conts.append({"Name": f"c{j}", "Port": port, "Protocol": proto, "PortName": f"serve-{port}-{proto.lower()}"})
        name = f"p{i}"
        if dups and pods and r.random() < 0.08:  # a second pod with an earlier pod's ns/name (one table Item)
            twin = r.choice(pods)
            ns, name = twin["Namespace"], twin["Name"]
        pods.append({"Namespace": ns, "Name": name, "Labels": _labels(r), "IP": ip, "Containers": conts})
    return {"Namespaces": {k: v for k, v in nss.items()}, "Pods": pods}


def random_probes(r: random.Random):
    out = []
    for _ in range(r.randint(1, 3)):
        c = r.random()
        if c < 0.3:
            out.append({"AllAvailable": True})
        elif c < 0.7:
            out.append({"Port": r.choice([80, 81, 53, 443, 8080, 82]), "Protocol": r.choice(PROTOS)})
        else:
            out.append({"Port": r.choice(["serve-80-tcp", "serve-81-udp", "serve-53-udp", "nope"]), "Protocol": r.choice(PROTOS)})
    return out


def random_problem(seed: int, n_pods=None, n_pols=None, v6=None, bad=False, dups=False):
    """dups=True: pods may repeat an earlier pod's ns/name and containers may repeat a (protocol, port):
    the reference's table build then dies on a duplicate job key (table.go:16-22, 38-48)."""
    r = random.Random(seed)
    if v6 is None:
        v6 = r.random() < 0.5
    n_pods = n_pods or r.randint(1, 40)
    n_pols = n_pols if n_pols is not None else r.randint(0, 12)
    pols = [random_policy(r, i, v6, bad) for i in range(n_pols)]
    return pols, random_resources(r, n_pods, v6, bad, dups), random_probes(r)
