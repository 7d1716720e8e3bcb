"""Deterministic synthetic workloads for the BASELINE.json configs.

All randomness comes from xoshiro256** (seed 20250217 unless stated), so every rank of a
multi-GPU run and the CPU baseline build byte-identical inputs.  Outputs are the reference's
own wire formats: a list of k8s NetworkPolicy objects, a probe.Resources document and a list
of generator.ProbeConfig values.

  config2()  10k pods (100 ns x 100) x 1k policies (upstream e2e test-case shapes) x 4 ports
  config3()  100k pods (1000 ns x 2 deployments x 50 replicas) x 10k policies x 8 ports
  config4()  50k pods (IPv4 / IPv6 / v4-mapped) x 5k IPBlock-heavy policies x 4 ports
"""
from __future__ import annotations

MASK64 = (1 << 64) - 1


class Xoshiro256ss:
    """xoshiro256** 1.0 (Blackman & Vigna), seeded through splitmix64."""

    def __init__(self, seed: int):
        s = []
        z = seed & MASK64
        for _ in range(4):
            z = (z + 0x9E3779B97F4A7C15) & MASK64
            x = z
            x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
            x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & MASK64
            s.append(x ^ (x >> 31))
        self.s = s

    def next(self) -> int:
        s = self.s
        r = (((s[1] * 5) & MASK64) << 7 | ((s[1] * 5) & MASK64) >> 57) & MASK64
        r = (r * 9) & MASK64
        t = (s[1] << 17) & MASK64
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = ((s[3] << 45) | (s[3] >> 19)) & MASK64
        return r

    def below(self, n: int) -> int:
        return (self.next() >> 11) * n >> 53

    def random(self) -> float:
        return (self.next() >> 11) / float(1 << 53)

    def choice(self, seq):
        return seq[self.below(len(seq))]

    def weighted(self, weights):
        x = self.random() * sum(weights)
        for i, w in enumerate(weights):
            x -= w
            if x < 0:
                return i
        return len(weights) - 1

    def sample(self, seq, k):
        pool = list(seq)
        out = []
        for _ in range(min(k, len(pool))):
            out.append(pool.pop(self.below(len(pool))))
        return out


def _ipv4(n: int) -> str:
    return f"{(n >> 24) & 255}.{(n >> 16) & 255}.{(n >> 8) & 255}.{n & 255}"


def _containers(specs):
    return [{"Name": f"cont-{p}-{pr.lower()}", "Port": p, "Protocol": pr, "PortName": f"serve-{p}-{pr.lower()}"} for p, pr in specs]


def _netpol(name, ns, pod_selector, types, ingress=None, egress=None):
    spec = {"podSelector": pod_selector, "policyTypes": types}
    if ingress is not None:
        spec["ingress"] = ingress
    if egress is not None:
        spec["egress"] = egress
    return {"apiVersion": "networking.k8s.io/v1", "kind": "NetworkPolicy", "metadata": {"name": name, "namespace": ns}, "spec": spec}


# ============================================================================ config #3
C3_PORTS = [(80, "TCP"), (81, "TCP"), (443, "TCP"), (8080, "TCP"), (53, "UDP"), (80, "UDP"), (81, "SCTP"), (9000, "SCTP")]
TIERS = ["web", "api", "db", "cache", "queue"]
VERSIONS = ["v1", "v2", "v3", "v4"]
ROLES = [f"r{i}" for i in range(10)]
ENVS = ["prod", "staging", "dev"]
TEAMS = [f"t{i:02d}" for i in range(50)]


def config3(n_ns=1000, templates_per_ns=2, replicas=50, policies_per_ns=10, seed=20250217):
    """Synthetic 100k pods x 10k policies x 8 port/protocols."""
    r = Xoshiro256ss(seed)
    apps = [f"app-{i:04d}" for i in range(2000)]
    namespaces, pods, templates = {}, [], {}
    for i in range(n_ns):
        ns = f"ns-{i:04d}"
        namespaces[ns] = {"ns": ns, "env": r.choice(ENVS), "team": r.choice(TEAMS)}
        tl = []
        for t in range(templates_per_ns):
            labels = {"app": r.choice(apps), "tier": r.choice(TIERS), "version": r.choice(VERSIONS), "role": r.choice(ROLES)}
            if r.random() < 0.10:
                del labels[r.choice(sorted(labels))]
            tl.append(labels)
            for j in range(replicas):
                ipn = (10 << 24) + i * 128 + t * replicas + j
                pods.append({"Namespace": ns, "Name": f"{labels.get('app', 'x')}-{t}-{j:03d}", "Labels": labels,
                             "IP": _ipv4(ipn), "Containers": _containers(C3_PORTS)})
        templates[ns] = tl
    ns_names = sorted(namespaces)

    def pod_selector(ns):
        k = r.weighted([10, 60, 30])
        if k == 0:
            return {}
        tl = r.choice(templates[ns])
        if k == 1:
            keys = r.sample(sorted(tl), 1 + r.below(2)) if tl else []
            return {"matchLabels": {kk: tl[kk] for kk in keys}} if keys else {}
        exprs = []
        for _ in range(1 + r.below(2)):
            op = r.choice(["In", "NotIn", "Exists", "DoesNotExist"])
            key = r.choice(["app", "tier", "version", "role"])
            e = {"key": key, "operator": op}
            if op in ("In", "NotIn"):
                vocab = {"app": [tl.get("app", apps[0]), r.choice(apps)], "tier": TIERS, "version": VERSIONS, "role": ROLES}[key]
                e["values"] = r.sample(vocab, 1 + r.below(2))
            exprs.append(e)
        return {"matchExpressions": exprs}

    def ns_selector():
        k = r.below(3)
        if k == 0:
            return {"matchLabels": {"env": r.choice(ENVS)}}
        if k == 1:
            return {"matchLabels": {"team": r.choice(TEAMS)}}
        return {"matchLabels": {"ns": r.choice(ns_names)}}

    def ipblock():
        plen = 16 + r.below(13)  # /16 .. /28
        base = (10 << 24) + r.below(n_ns * 128)
        net = base & (~((1 << (32 - plen)) - 1) & 0xFFFFFFFF)
        ib = {"cidr": f"{_ipv4(net)}/{plen}"}
        nex = r.below(3)
        if nex and plen < 30:
            ex = []
            for _ in range(nex):
                elen = min(32, plen + 1 + r.below(6))
                off = r.below(1 << (32 - plen)) & (~((1 << (32 - elen)) - 1) & 0xFFFFFFFF)
                ex.append(f"{_ipv4(net + off)}/{elen}")
            ib["except"] = ex
        return {"ipBlock": ib}

    def peer(ns):
        if r.random() < 0.2:
            return ipblock()
        p = {}
        podk = r.below(2)  # empty | label
        nsk = r.below(3)  # nil | empty | label
        if podk == 0:
            p["podSelector"] = {}
        else:
            src = r.choice(templates[r.choice(ns_names)] if r.random() < 0.5 else templates[ns])
            p["podSelector"] = {"matchLabels": {"app": src.get("app", "none")}}
        if nsk == 1:
            p["namespaceSelector"] = {}
        elif nsk == 2:
            p["namespaceSelector"] = ns_selector()
        return p

    def ports():
        n = r.weighted([30, 50, 20])
        out, n_ranges = [], 0
        for _ in range(n):
            pp = {}
            proto = r.choice([None, "TCP", "UDP", "SCTP"])
            if proto:
                pp["protocol"] = proto
            kind = r.weighted([60, 25, 15])
            if kind == 2 and n_ranges >= 2:
                kind = 0
            port, cproto = r.choice(C3_PORTS)
            if kind == 0:
                pp["port"] = port
            elif kind == 1:
                pp["port"] = f"serve-{port}-{cproto.lower()}"
            else:
                pp["port"] = port
                pp["endPort"] = port + r.choice([0, 1, 10, 400, 9000])
                n_ranges += 1
            out.append(pp)
        return out

    def rules(ns, key):
        out = []
        for _ in range(r.weighted([10, 60, 20, 10])):
            rule = {}
            ps = ports()
            if ps:
                rule["ports"] = ps
            npeer = r.weighted([15, 50, 25, 10])
            if npeer:
                rule[key] = [peer(ns) for _ in range(npeer)]
            out.append(rule)
        return out

    policies = []
    for ns in ns_names:
        for j in range(policies_per_ns):
            types = [["Ingress"], ["Egress"], ["Ingress", "Egress"]][r.weighted([40, 30, 30])]
            ing = rules(ns, "from") if "Ingress" in types else None
            eg = rules(ns, "to") if "Egress" in types else None
            policies.append(_netpol(f"np-{ns}-{j}", ns, pod_selector(ns), types, ing, eg))
    resources = {"Namespaces": namespaces, "Pods": pods}
    return {"name": "config3", "policies": policies, "resources": resources, "probes": [{"AllAvailable": True}],
            "description": f"{len(pods)} pods x {len(policies)} policies x {len(C3_PORTS)} port/protocols"}


# ============================================================================ config #2
C2_PORTS = [(80, "TCP"), (81, "TCP"), (53, "UDP"), (80, "SCTP")]


def _upstream_policies(ns, other_ns, pod, app, r: Xoshiro256ss, i):
    """Shapes of networkpolicies/upstream_test_cases/allow-to-ns-y-pod-a.yaml and the upstream
    e2e cases of pkg/generator/upstreame2ecases.go, with namespace / label substitution."""
    k = i % 14
    sel = {"matchLabels": {"pod": pod}}
    if k == 0:  # allow-to-ns-y-pod-a.yaml
        return _netpol(f"allow-to-{other_ns}-{pod}-{i}", ns, sel, ["Egress"], egress=[
            {"to": [{"namespaceSelector": {"matchLabels": {"ns": other_ns}}, "podSelector": {"matchLabels": {"pod": pod}}}],
             "ports": [{"port": 80, "protocol": "TCP"}]},
            {"ports": [{"port": 53, "protocol": "UDP"}]}])
    if k == 1:  # deny all ingress
        return _netpol(f"deny-all-{i}", ns, {}, ["Ingress"], ingress=[])
    if k == 2:  # allow ingress from same namespace pods
        return _netpol(f"allow-same-ns-{i}", ns, {}, ["Ingress"], ingress=[{"from": [{"podSelector": {}}]}])
    if k == 3:  # allow from other namespace by label
        return _netpol(f"allow-from-ns-{i}", ns, sel, ["Ingress"], ingress=[{"from": [{"namespaceSelector": {"matchLabels": {"ns": other_ns}}}]}])
    if k == 4:  # pod + ns selector combined
        return _netpol(f"allow-pod-ns-{i}", ns, sel, ["Ingress"], ingress=[
            {"from": [{"namespaceSelector": {"matchLabels": {"ns": other_ns}}, "podSelector": {"matchLabels": {"app": app}}}]}])
    if k == 5:  # numbered port
        return _netpol(f"allow-port-81-{i}", ns, sel, ["Ingress"], ingress=[{"ports": [{"port": 81, "protocol": "TCP"}], "from": [{"namespaceSelector": {}}]}])
    if k == 6:  # named port
        return _netpol(f"allow-named-{i}", ns, sel, ["Ingress"], ingress=[{"ports": [{"port": "serve-80-tcp", "protocol": "TCP"}], "from": [{"podSelector": {}}]}])
    if k == 7:  # deny all egress
        return _netpol(f"deny-egress-{i}", ns, sel, ["Egress"], egress=[])
    if k == 8:  # allow egress to same-ns app on a port
        return _netpol(f"egress-app-{i}", ns, {"matchLabels": {"app": app}}, ["Egress"], egress=[
            {"to": [{"podSelector": {"matchLabels": {"app": app}}}], "ports": [{"port": 80, "protocol": "TCP"}]}])
    if k == 9:  # ipBlock with except
        third = r.below(100)
        return _netpol(f"ipblock-{i}", ns, sel, ["Ingress"], ingress=[{"from": [{"ipBlock": {"cidr": f"10.{third}.0.0/16", "except": [f"10.{third}.{r.below(100)}.0/24"]}}]}])
    if k == 10:  # matchExpressions NotIn / In
        return _netpol(f"expr-{i}", ns, {"matchExpressions": [{"key": "app", "operator": "NotIn", "values": [app]}]}, ["Ingress"],
                       ingress=[{"from": [{"podSelector": {"matchExpressions": [{"key": "pod", "operator": "In", "values": [pod, "a"]}]}}]}])
    if k == 11:  # allow all ingress + egress
        return _netpol(f"allow-all-{i}", ns, sel, ["Ingress", "Egress"], ingress=[{}], egress=[{}])
    if k == 12:  # SCTP / UDP only
        return _netpol(f"proto-{i}", ns, sel, ["Ingress"], ingress=[{"ports": [{"protocol": "SCTP"}, {"port": 53, "protocol": "UDP"}]}])
    # k == 13: endPort range
    return _netpol(f"range-{i}", ns, {}, ["Egress"], egress=[{"ports": [{"port": 80, "endPort": 81, "protocol": "TCP"}], "to": [{"namespaceSelector": {}}]}])


def config2(n_ns=100, pods_per_ns=100, n_policies=1000, seed=20250217):
    """networkpolicies/upstream_test_cases shapes over 10k pods x 1k policies x 4 ports."""
    r = Xoshiro256ss(seed)
    names = [f"p{j:03d}" for j in range(pods_per_ns)]
    namespaces, pods = {}, []
    for i in range(n_ns):
        ns = f"ns-{i:03d}"
        namespaces[ns] = {"ns": ns}
        for j in range(pods_per_ns):
            pods.append({"Namespace": ns, "Name": names[j], "Labels": {"pod": names[j], "app": f"app{j % 20:02d}"},
                         "IP": f"10.{i}.{j}.1", "Containers": _containers(C2_PORTS)})
    policies = []
    for i in range(n_policies):
        ns = f"ns-{r.below(n_ns):03d}"
        other = f"ns-{r.below(n_ns):03d}"
        policies.append(_upstream_policies(ns, other, r.choice(names), f"app{r.below(20):02d}", r, i))
    return {"name": "config2", "policies": policies, "resources": {"Namespaces": namespaces, "Pods": pods},
            "probes": [{"AllAvailable": True}], "description": f"{len(pods)} pods x {len(policies)} policies x 4 ports"}


# ============================================================================ config #4
C4_PORTS = [(80, "TCP"), (443, "TCP"), (53, "UDP"), (9000, "SCTP")]


def config4(n_pods=50_000, n_policies=5000, n_ns=500, seed=20250217):
    """IPBlock-heavy: IPv4 10.0.0.0/16, IPv6 fd00:10::/64 and ::ffff:10.x.y.z pods; every policy
    has ingress and egress with 1-4 IPBlock peers (1-3 nested excepts, mixed families)."""
    r = Xoshiro256ss(seed)
    namespaces, pods = {}, []
    for i in range(n_ns):
        namespaces[f"ns-{i:03d}"] = {"ns": f"ns-{i:03d}"}
    per_ns = n_pods // n_ns
    for n in range(n_pods):
        ns = f"ns-{n // per_ns:03d}" if n // per_ns < n_ns else f"ns-{n_ns - 1:03d}"
        u = r.random()
        if u < 0.50:
            ip = f"10.0.{(n >> 8) & 255}.{n & 255}"
        elif u < 0.99:
            ip = f"fd00:10::{n:x}"
        else:
            ip = f"::ffff:10.0.{(n >> 8) & 255}.{n & 255}"
        pods.append({"Namespace": ns, "Name": f"pod-{n:05d}", "Labels": {"app": f"a{n % 50}", "ip": "v4" if u < 0.5 else "v6"},
                     "IP": ip, "Containers": _containers(C4_PORTS)})
    edge = ["0.0.0.0/0", "::/0", "::ffff:0:0/96", "10.0.1.7/32", "fd00:10::7/128"]

    def v4_cidr():
        plen = 16 + r.below(13)
        base = (10 << 24) + r.below(1 << 16)
        net = base & (~((1 << (32 - plen)) - 1) & 0xFFFFFFFF)
        return net, plen

    def block():
        if r.random() < 0.1:
            return {"ipBlock": {"cidr": r.choice(edge)}}
        if r.random() < 0.6:
            net, plen = v4_cidr()
            ex = []
            for _ in range(1 + r.below(3)):
                elen = min(32, plen + 1 + r.below(8))
                off = r.below(1 << (32 - plen)) & (~((1 << (32 - elen)) - 1) & 0xFFFFFFFF)
                ex.append(f"{_ipv4(net + off)}/{elen}")
            return {"ipBlock": {"cidr": f"{_ipv4(net)}/{plen}", "except": ex}}
        plen = 112 + r.below(15)
        host = r.below(n_pods) & ~((1 << (128 - plen)) - 1)
        ex = []
        for _ in range(1 + r.below(3)):
            elen = min(128, plen + 1 + r.below(6))
            off = r.below(1 << (128 - plen)) & ~((1 << (128 - elen)) - 1)
            ex.append(f"fd00:10::{host + off:x}/{elen}")
        return {"ipBlock": {"cidr": f"fd00:10::{host:x}/{plen}", "except": ex}}

    policies = []
    for i in range(n_policies):
        ns = f"ns-{r.below(n_ns):03d}"
        sel = {"matchLabels": {"app": f"a{r.below(50)}"}} if r.random() < 0.7 else {}
        ports = [{"port": r.choice(C4_PORTS)[0], "protocol": r.choice(C4_PORTS)[1]}] if r.random() < 0.5 else None
        ing = {"from": [block() for _ in range(1 + r.below(4))]}
        eg = {"to": [block() for _ in range(1 + r.below(4))]}
        if ports:
            ing["ports"] = ports
            eg["ports"] = ports
        policies.append(_netpol(f"ipb-{i}", ns, sel, ["Ingress", "Egress"], [ing], [eg]))
    return {"name": "config4", "policies": policies, "resources": {"Namespaces": namespaces, "Pods": pods},
            "probes": [{"AllAvailable": True}], "description": f"{n_pods} pods x {n_policies} IPBlock policies x 4 ports"}


def config3u(n_ns=1000, seed=20250217):
    """Class-explosion variant of config #3 (SURVEY §7 "class explosion"): the
    same 100k pods x 10k policies x 8 port/protocols, but every pod has its own label set (100
    templates per namespace, one replica each), so pod identities are all distinct and the
    policies' selectors split each namespace into many target classes.  A stress workload for the
    class rows, not a BASELINE config."""
    d = config3(n_ns=n_ns, templates_per_ns=100, replicas=1, seed=seed)
    d["name"] = "config3u"
    d["description"] += " (all pod identities distinct)"
    return d


CONFIGS = {"config2": config2, "config3": config3, "config4": config4, "config3u": config3u}
