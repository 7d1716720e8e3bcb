"""Config #5 input producer: the reference's test-case generator and simulated interpreter state.

Restates pkg/generator (testcasegenerator.go:64-84 GenerateAllTestCases: Target, Rules, Peers,
PortProtocol, Example, Action, Conflict, UpstreamE2E cases; netpol.go builders; constants.go)
and the simulated half of pkg/connectivity/interpreter.go:64-148 (TestCaseState actions,
testcasestate.go:19-173) on top of `cyclonus generate --mock` defaults (cli/generate.go:49-69):
namespaces x,y,z x pods a,b,c, containers {80,81} x {TCP,UDP,SCTP}, allow-dns on, MockKubernetes
pod IPs 192.168.1.<n> with n counting up from 1 across the whole run (kube/ikubernetes.go:292-298).

This is host-side input generation only; every verdict is computed by libcyclonus_hip.
`sweep()` returns one record per probe step: the policies in force, the Resources after the
step's actions, and the step's probe config, in the reference's execution order.
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field
from typing import List, Optional

# constants.go
TCP, UDP, SCTP = "TCP", "UDP", "SCTP"
EMPTY = {}
POD_A = {"matchLabels": {"pod": "a"}}
POD_C = {"matchLabels": {"pod": "c"}}
POD_AB = {"matchExpressions": [{"key": "pod", "operator": "In", "values": ["a", "b"]}]}
POD_BC = {"matchExpressions": [{"key": "pod", "operator": "In", "values": ["b", "c"]}]}
NS_X = {"matchLabels": {"ns": "x"}}
NS_XY = {"matchExpressions": [{"key": "ns", "operator": "In", "values": ["x", "y"]}]}
NS_YZ = {"matchExpressions": [{"key": "ns", "operator": "In", "values": ["y", "z"]}]}

PROBE_ALL = {"AllAvailable": True}
PROBE_80_TCP = {"Port": 80, "Protocol": TCP}
PROBE_81_TCP = {"Port": 81, "Protocol": TCP}
PROBE_SERVE_80_TCP = {"Port": "serve-80-tcp", "Protocol": TCP}
PROBE_SERVE_81_TCP = {"Port": "serve-81-tcp", "Protocol": TCP}


def port(p=None, proto=None):
    d = {}
    if proto is not None:
        d["protocol"] = proto
    if p is not None:
        d["port"] = p
    return d


ALLOW_DNS_RULE = {"ports": [port(53, UDP)], "peers": []}


@dataclass
class Netpol:  # netpol.go:10-16 (Ingress/Egress None == nil NetpolPeers)
    name: str
    namespace: str
    pod_selector: dict
    ingress: Optional[List[dict]] = None  # list of rules {"ports": [...], "peers": [...]}
    egress: Optional[List[dict]] = None

    def network_policy(self) -> dict:  # netpol.go:39-80
        spec = {"podSelector": copy.deepcopy(self.pod_selector)}
        types = []
        if self.ingress is not None:
            types.append("Ingress")
            rules = [_rule_json(r, "from") for r in self.ingress]
            if rules:
                spec["ingress"] = rules
        if self.egress is not None:
            types.append("Egress")
            rules = [_rule_json(r, "to") for r in self.egress]
            if rules:
                spec["egress"] = rules
        if not types:
            raise ValueError("cannot have 0 policy types")
        spec["policyTypes"] = types
        return {"kind": "NetworkPolicy", "apiVersion": "networking.k8s.io/v1",
                "metadata": {"name": self.name, "namespace": self.namespace}, "spec": spec}


def _rule_json(rule, peers_key):
    out = {}
    if rule.get("ports"):
        out["ports"] = copy.deepcopy(rule["ports"])
    if rule.get("peers"):
        out[peers_key] = copy.deepcopy(rule["peers"])
    return out


def base_policy() -> Netpol:  # netpol.go:184-226 baseTestPolicy
    return Netpol(
        "base", "x", copy.deepcopy(POD_A),
        ingress=[{"ports": [port(80, TCP)], "peers": [{"podSelector": POD_BC, "namespaceSelector": NS_XY}]}],
        egress=[{"ports": [port(80, TCP)], "peers": [{"podSelector": POD_AB, "namespaceSelector": NS_YZ}]}, ALLOW_DNS_RULE],
    )


def build_policy(*setters) -> Netpol:  # netpol.go:176-182
    p = base_policy()
    for s in setters:
        s(p)
    return p


def set_namespace(ns):
    def f(p):
        p.namespace = ns
    return f


def set_pod_selector(sel):
    def f(p):
        p.pod_selector = copy.deepcopy(sel)
    return f


def set_rules(is_ingress, rules):
    def f(p):
        if is_ingress:
            p.ingress = copy.deepcopy(rules)
        else:
            p.egress = copy.deepcopy(rules)
    return f


def set_ports(is_ingress, ports):
    def f(p):
        (p.ingress if is_ingress else p.egress)[0] = dict((p.ingress if is_ingress else p.egress)[0], ports=copy.deepcopy(ports))
    return f


def set_peers(is_ingress, peers):
    def f(p):
        (p.ingress if is_ingress else p.egress)[0] = dict((p.ingress if is_ingress else p.egress)[0], peers=copy.deepcopy(peers))
    return f


# action.go
def create_policy(pol):
    return ("create_policy", pol)


def update_policy(pol):
    return ("update_policy", pol)


def delete_policy(ns, name):
    return ("delete_policy", ns, name)


def create_namespace(ns, labels):
    return ("create_namespace", ns, labels)


def set_namespace_labels(ns, labels):
    return ("set_namespace_labels", ns, labels)


def delete_namespace(ns):
    return ("delete_namespace", ns)


def create_pod(ns, pod, labels):
    return ("create_pod", ns, pod, labels)


def set_pod_labels(ns, pod, labels):
    return ("set_pod_labels", ns, pod, labels)


def delete_pod(ns, pod):
    return ("delete_pod", ns, pod)


@dataclass
class TestCase:  # testcase.go:12-45
    description: str
    tags: set
    steps: list = field(default_factory=list)  # [(probe, [actions])]


def single(desc, tags, probe, *actions):
    if not desc:
        desc = ",".join(sorted(tags))
    return TestCase(desc, set(tags), [(probe, list(actions))])


def direction(is_ingress):
    return "ingress" if is_ingress else "egress"


def make_ipv4_cidr(ip, bits):  # kube/ipaddress.go:42-46
    a = [int(x) for x in ip.split(".")]
    n = (a[0] << 24) | (a[1] << 16) | (a[2] << 8) | a[3]
    n &= (0xFFFFFFFF << (32 - bits)) & 0xFFFFFFFF
    return f"{n >> 24}.{(n >> 16) & 255}.{(n >> 8) & 255}.{n & 255}/{bits}"


class Generator:
    def __init__(self, pod_ip: str, allow_dns: bool = True, namespaces=("x", "y", "z")):
        self.pod_ip = pod_ip
        self.allow_dns = allow_dns
        self.namespaces = list(namespaces)

    # targetcases.go
    def target_cases(self):
        cases = [single(f"set namespace to {ns}", {"target-namespace"}, PROBE_ALL,
                        create_policy(build_policy(set_namespace(ns)).network_policy())) for ns in self.namespaces]
        for sel in (EMPTY, POD_A, POD_AB):
            cases.append(single("set pod selector", {"target-pod-selector"}, PROBE_ALL,
                                create_policy(build_policy(set_pod_selector(sel)).network_policy())))
        return cases

    # rulescases.go
    def rules_cases(self):
        cases = []
        for ing in (False, True):
            d = direction(ing)
            cases.append(single(f"{d}: deny all", {d, "deny-all"}, PROBE_ALL, create_policy(build_policy(set_rules(ing, [])).network_policy())))
            cases.append(single(f"{d}: allow all", {d, "allow-all"}, PROBE_ALL, create_policy(build_policy(set_rules(ing, [{}])).network_policy())))
        return cases

    # peerscases.go
    def peers(self):
        pod = [
            ("empty pods + nil ns", {"podSelector": EMPTY}),
            ("pods by label + nil ns", {"podSelector": POD_C}),
            ("nil pods + empty ns", {"namespaceSelector": EMPTY}),
            ("empty pods + empty ns", {"podSelector": EMPTY, "namespaceSelector": EMPTY}),
            ("pods by label + empty ns", {"podSelector": POD_C, "namespaceSelector": EMPTY}),
            ("nil pods + ns by label", {"namespaceSelector": NS_X}),
            ("empty pods + ns by label", {"podSelector": EMPTY, "namespaceSelector": NS_X}),
            ("pods by label + ns by label", {"podSelector": POD_C, "namespaceSelector": NS_X}),
        ]
        c24, c28 = make_ipv4_cidr(self.pod_ip, 24), make_ipv4_cidr(self.pod_ip, 28)
        ip = [("simple ipblock", {"ipBlock": {"cidr": c24}}), ("ipblock with except", {"ipBlock": {"cidr": c24, "except": [c28]}})]
        return copy.deepcopy(pod + ip)

    def peers_cases(self):
        cases = []
        for ing in (True, False):
            d = direction(ing)
            cases.append(single(f"{d}: empty peers", {d, "any-peer"}, PROBE_ALL, create_policy(build_policy(set_peers(ing, [])).network_policy())))
        for ing in (True, False):
            for desc, p in self.peers():
                cases.append(single(desc, {direction(ing)}, PROBE_ALL, create_policy(build_policy(set_peers(ing, [p])).network_policy())))
        for ing in (True, False):
            ps = self.peers()
            for i, (d1, p1) in enumerate(ps):
                for j, (d2, p2) in enumerate(ps):
                    if i < j:
                        cases.append(single(f"{direction(ing)}, 2-peer: {d1}, {d2}", {direction(ing), "multi-peer"}, PROBE_ALL,
                                            create_policy(build_policy(set_peers(ing, [p1, p2])).network_policy())))
        return cases

    # portprotocolcases.go
    def port_protocol_cases(self):
        cases = []
        for ing in (False, True):
            d = direction(ing)
            cases.append(single(f"{d}: empty port/protocol", {d, "any-port-protocol"}, PROBE_ALL,
                                create_policy(build_policy(set_ports(ing, [])).network_policy())))
        npps = [port(p, proto) for proto in (None, TCP, UDP, SCTP) for p in (None, 80, 81)]
        npps += [port("serve-80-tcp", TCP), port("serve-81-tcp", TCP), port("serve-80-udp", UDP), port("serve-81-udp", UDP),
                 port("serve-80-sctp", SCTP), port("serve-81-sctp", SCTP)]
        for ing in (False, True):
            d = direction(ing)
            for npp in npps:
                cases.append(single("", {d}, PROBE_ALL, create_policy(build_policy(set_ports(ing, [npp])).network_policy())))
            for desc, npp in (("open a named port that doesn't match its protocol", port("serve-81-udp", TCP)),
                              ("open a named port that isn't served", port("serve-7981-udp", TCP)),
                              ("open a numbered port that isn't served", port(7981, TCP))):
                cases.append(single(desc, {"pathological", d}, PROBE_ALL, create_policy(build_policy(set_ports(ing, [npp])).network_policy())))
        pairs = [
            [port(), port(80)],
            [port(), port("serve-80-tcp")],
            [port(), port(proto=UDP)],
            [port(80), port(81)],
            [port(80), port("serve-81-tcp")],
            [port(80), port("serve-81-udp", UDP)],
            [port(80, UDP), port("serve-81-udp", UDP)],
        ]
        for ing in (False, True):
            for pr in pairs:
                cases.append(single("", {"multi-port/protocol", direction(ing)}, PROBE_ALL,
                                    create_policy(build_policy(set_ports(ing, pr)).network_policy())))
        return cases

    # examplecases.go
    def example_cases(self):
        allow81 = {"kind": "NetworkPolicy", "apiVersion": "networking.k8s.io/v1", "metadata": {"name": "allow-all", "namespace": "x"},
                   "spec": {"podSelector": {}, "ingress": [{"ports": [{"port": "serve-81-tcp"}]}], "policyTypes": ["Ingress"]}}
        return [TestCase("should allow ingress access on one named port", {"example"}, [
            (PROBE_ALL, [create_policy(allow81)]),
            (PROBE_ALL, [create_namespace("w", {"ns": "w"}), create_pod("w", "a", {"pod": "a"})]),
            (PROBE_ALL, [delete_pod("w", "a")]),
            (PROBE_ALL, [delete_namespace("w")]),
            (PROBE_ALL, []),
            (PROBE_81_TCP, []),
            (PROBE_SERVE_81_TCP, []),
        ])]

    # actioncases.go
    def action_cases(self):
        base = base_policy()
        return [
            TestCase("Create/delete policy", {"create-policy", "delete-policy"}, [
                (PROBE_ALL, [create_policy(base.network_policy())]),
                (PROBE_ALL, [delete_policy(base.namespace, base.name)])]),
            TestCase("Create/update policy", {"create-policy", "update-policy"}, [
                (PROBE_ALL, [create_policy(base.network_policy())]),
                (PROBE_ALL, [update_policy(build_policy(set_ports(True, [port("serve-81-udp", UDP)])).network_policy())])]),
            TestCase("Create/delete namespace", {"create-namespace", "delete-namespace"}, [
                (PROBE_ALL, [create_policy(base.network_policy())]),
                (PROBE_ALL, [create_namespace("y-2", {"ns": "y"}), create_pod("y-2", "a", {"pod": "a"}), create_pod("y-2", "b", {"pod": "b"})]),
                (PROBE_ALL, [delete_namespace("y-2")])]),
            TestCase("Update namespace so that policy applies, then again so it no longer applies", {"set-namespace-labels"}, [
                (PROBE_ALL, [create_policy(build_policy(set_peers(True, [{"namespaceSelector": {"matchLabels": {"new-ns": "qrs"}}}])).network_policy())]),
                (PROBE_ALL, [set_namespace_labels("y", {"ns": "y", "new-ns": "qrs"})]),
                (PROBE_ALL, [set_namespace_labels("y", {"ns": "y"})])]),
            TestCase("Create/delete pod", {"create-pod", "delete-pod"}, [
                (PROBE_ALL, [create_policy(base.network_policy())]),
                (PROBE_ALL, [create_pod("x", "d", {"pod": "d"})]),
                (PROBE_ALL, [delete_pod("x", "d")])]),
            TestCase("Update pod so that policy applies, then again so it no longer applies", {"set-pod-labels"}, [
                (PROBE_ALL, [create_policy(build_policy(set_peers(True, [{"podSelector": {"matchLabels": {"new-label": "abc"}},
                                                                          "namespaceSelector": NS_YZ}])).network_policy())]),
                (PROBE_ALL, [set_pod_labels("y", "b", {"pod": "b", "new-label": "abc"})]),
                (PROBE_ALL, [set_pod_labels("y", "b", {"pod": "b"})])]),
        ]

    # conflictcases.go
    def conflict_cases(self):
        src = ("x", {"matchLabels": {"pod": "b"}})
        dst = ("y", {"matchLabels": {"pod": "c"}})
        allow_all = [{}]
        deny_all = None  # NetpolPeers{Rules: nil}: the direction is set, with no rules
        by_pod = [{"peers": [{"namespaceSelector": {}}]}]
        by_ip = [{"peers": [{"ipBlock": {"cidr": "0.0.0.0/0"}}]}]
        deny_by_ip = [{"peers": [{"ipBlock": {"cidr": "0.0.0.0/31"}}]}]
        deny_by_pod = [{"peers": [{"namespaceSelector": {"matchLabels": {"this-will-never-happen": "qrs123"}}}]}]

        def np(name, target, ingress="unset", egress="unset"):
            n = Netpol(name, target[0], copy.deepcopy(target[1]))
            if ingress != "unset":
                n.ingress = [] if ingress is None else copy.deepcopy(ingress)
            if egress != "unset":
                n.egress = [] if egress is None else copy.deepcopy(egress)
            return n

        S, D = src, dst
        conf = [
            ("deny all from source, allow all to dest", {"deny-all", "allow-all", "ingress", "egress"},
             [np("deny-all-egress", S, egress=deny_all), np("allow-all-ingress", D, ingress=allow_all)]),
            ("allow all from source, deny all to dest", {"deny-all", "allow-all", "ingress", "egress"},
             [np("allow-all-egress", S, egress=allow_all), np("deny-all-ingress", D, ingress=deny_all)]),
            ("deny all + allow all from same source", {"deny-all", "allow-all", "egress"},
             [np("deny-all-egress", S, egress=deny_all), np("allow-all-egress", S, egress=allow_all)]),
            ("deny all + allow all to same dest", {"deny-all", "allow-all", "ingress"},
             [np("deny-all-ingress", D, ingress=deny_all), np("allow-all-ingress", D, ingress=allow_all)]),
            ("deny all + allow all by pod from same source", {"deny-all", "all-pods", "all-namespaces", "egress"},
             [np("deny-all-egress", S, egress=deny_all), np("allow-all-egress-by-pod", S, egress=by_pod)]),
            ("deny all + allow all by IP from same source", {"deny-all", "egress"},
             [np("deny-all-egress", S, egress=deny_all), np("allow-all-egress-by-ip", S, egress=by_ip)]),
            ("deny all by IP + allow all by pod from same source", {"all-pods", "all-namespaces", "egress"},
             [np("deny-all-egress-by-ip", S, egress=deny_by_ip), np("allow-all-egress-by-pod", S, egress=by_pod)]),
            ("deny all by pod + allow all by IP from same source", {"egress"},
             [np("deny-all-egress-by-pod", S, egress=deny_by_pod), np("allow-all-egress-by-ip", S, egress=by_ip)]),
            # the reference passes `source` as the destination target of the next four (conflictcases.go:286-289)
            ("deny all + allow all by pod to same source", {"deny-all", "ingress", "all-pods", "all-namespaces"},
             [np("deny-all-ingress", S, ingress=deny_all), np("allow-all-ingress-by-pod", S, ingress=by_pod)]),
            ("deny all + allow all by IP to same source", {"deny-all", "ingress"},
             [np("deny-all-ingress", S, ingress=deny_all), np("allow-all-ingress-by-ip", S, ingress=by_ip)]),
            ("deny all by IP + allow all by pod to same source", {"ingress", "all-pods", "all-namespaces"},
             [np("deny-all-ingress-by-ip", S, ingress=deny_by_ip), np("allow-all-ingress-by-pod", S, ingress=by_pod)]),
            ("deny all by pod + allow all by IP to same source", {"ingress"},
             [np("deny-all-ingress-by-pod", S, ingress=deny_by_pod), np("allow-all-ingress-by-ip", S, ingress=by_ip)]),
            ("egress: deny all by IP", {"egress"}, [np("deny-all-egress-by-ip", S, egress=deny_by_ip)]),
            ("egress: deny all by pod", {"egress"}, [np("deny-all-egress-by-ip", S, egress=deny_by_pod)]),
            ("ingress: deny all by IP", {"ingress"}, [np("deny-all-ingress-by-ip", S, ingress=deny_by_ip)]),
            ("ingress: deny all by pod", {"ingress"}, [np("deny-all-ingress-by-ip", S, ingress=deny_by_pod)]),
        ]
        cases = []
        for desc, tags, pols in conf:
            actions = [create_policy(p.network_policy()) for p in pols]
            if any(p.egress is not None for p in pols) and self.allow_dns:
                dns = Netpol("allow-dns", S[0], copy.deepcopy(S[1]), egress=[copy.deepcopy(ALLOW_DNS_RULE)])
                actions.append(create_policy(dns.network_policy()))
            cases.append(single(desc, tags | {"conflict"}, PROBE_ALL, *actions))
        return cases

    # upstreame2ecases.go
    def upstream_cases(self):
        def np(name, ns, sel, types, ingress=None, egress=None):
            spec = {"podSelector": sel, "policyTypes": types}
            if ingress is not None:
                spec["ingress"] = ingress
            if egress is not None:
                spec["egress"] = egress
            return {"kind": "NetworkPolicy", "apiVersion": "networking.k8s.io/v1", "metadata": {"name": name, "namespace": ns}, "spec": spec}

        dns_egress = {"ports": [{"protocol": UDP, "port": 53}]}
        a = {"matchLabels": {"pod": "a"}}
        T = TestCase
        return [
            single("should support a 'default-deny-ingress' policy", {"upstream-e2e", "ingress", "deny-all"}, PROBE_ALL,
                   create_policy(np("deny-ingress", "x", {}, ["Ingress"]))),
            single("should support a 'default-deny-all' policy", {"upstream-e2e", "deny-all"}, PROBE_ALL,
                   create_policy(np("deny-all-allow-dns", "x", {}, ["Egress", "Ingress"], egress=[dns_egress]))),
            single("should enforce policy based on Multiple PodSelectors and NamespaceSelectors", {"upstream-e2e"}, PROBE_ALL,
                   create_policy(np("allow-ns-y-z-pod-b-c", "x", a, ["Ingress"], ingress=[{"from": [{
                       "namespaceSelector": {"matchExpressions": [{"key": "ns", "operator": "NotIn", "values": ["x"]}]},
                       "podSelector": {"matchExpressions": [{"key": "pod", "operator": "In", "values": ["b", "c"]}]}}]}]))),
            T("should enforce multiple, stacked policies with overlapping podSelectors [Feature:NetworkPolicy]", {"upstream-e2e"}, [
                (PROBE_ALL, [create_policy(np("allow-client-a-via-ns-selector-81", "x", a, ["Ingress"], ingress=[
                    {"from": [{"namespaceSelector": {"matchLabels": {"ns": "y"}}}], "ports": [{"port": 81, "protocol": TCP}]}]))]),
                (PROBE_ALL, []),
                (PROBE_ALL, [create_policy(np("allow-client-a-via-ns-selector-80", "x", a, ["Ingress"], ingress=[
                    {"from": [{"namespaceSelector": {"matchLabels": {"ns": "y"}}}], "ports": [{"port": 80, "protocol": TCP}]}]))])]),
            T("should support allow-all policy", {"upstream-e2e", "allow-all"}, [
                (PROBE_ALL, [create_policy(np("allow-all", "x", {}, ["Ingress"], ingress=[{}]))]),
                (PROBE_ALL, [])]),
            T("should allow ingress access on one named port", {"upstream-e2e", "ingress", "named-port"}, [
                (PROBE_SERVE_81_TCP, [create_policy(np("allow-all", "x", {}, ["Ingress"], ingress=[{"ports": [{"port": "serve-81-tcp"}]}]))]),
                (PROBE_ALL, [])]),
            T("should enforce updated policy", {"upstream-e2e"}, [
                (PROBE_ALL, [create_policy(np("allow-all-mutate-to-deny-all", "x", {}, ["Ingress"], ingress=[{}]))]),
                (PROBE_ALL, [update_policy(np("allow-all-mutate-to-deny-all", "x", {}, ["Ingress"]))])]),
            T("should allow ingress access from updated namespace", {"upstream-e2e"}, [
                (PROBE_ALL, [create_policy(np("allow-client-a-via-ns-selector", "x", a, ["Ingress"], ingress=[
                    {"from": [{"namespaceSelector": {"matchLabels": {"ns2": "updated"}}}]}]))]),
                (PROBE_ALL, [set_namespace_labels("y", {"ns": "y", "ns2": "updated"})])]),
            T("should allow ingress access from updated pod", {"upstream-e2e"}, [
                (PROBE_ALL, [create_policy(np("allow-client-a-via-pod-selector", "x", a, ["Ingress"], ingress=[
                    {"from": [{"podSelector": {"matchLabels": {"pod": "b", "pod2": "updated"}}}]}]))]),
                (PROBE_ALL, [set_pod_labels("x", "b", {"pod": "b", "pod2": "updated"})])]),
            T("should deny ingress access to updated pod", {"upstream-e2e"}, [
                (PROBE_ALL, [create_policy(np("deny-ingress-via-label-selector", "x", {"matchLabels": {"target": "isolated"}}, ["Ingress"]))]),
                (PROBE_ALL, [set_pod_labels("x", "a", {"target": "isolated"})])]),
            T("should work with Ingress, Egress specified together", {"upstream-e2e"}, [
                (PROBE_ALL, [create_policy(np("allow-client-a-via-pod-selector", "x", a, ["Ingress", "Egress"],
                                              ingress=[{"from": [{"podSelector": {"matchLabels": {"pod": "b"}}}]}],
                                              egress=[{"ports": [{"port": 80}, {"protocol": UDP, "port": 53}]}]))]),
                (PROBE_ALL, [])]),
            single("should support denying of egress traffic on the client side (even if the server explicitly allows this traffic)",
                   {"upstream-e2e", "conflict"}, PROBE_ALL,
                   create_policy(np("allow-to-ns-y-pod-a", "x", a, ["Egress"], egress=[
                       {"to": [{"namespaceSelector": {"matchLabels": {"ns": "y"}}, "podSelector": {"matchLabels": {"pod": "a"}}}]},
                       {"ports": [{"protocol": UDP, "port": 53}]}])),
                   create_policy(np("allow-from-xa-on-ya-match-selector", "y", a, ["Ingress"], ingress=[
                       {"from": [{"namespaceSelector": {"matchLabels": {"ns": "x"}}, "podSelector": {"matchLabels": {"pod": "a"}}}]}])),
                   create_policy(np("allow-from-xa-on-yb-match-selector", "y", {"matchLabels": {"pod": "b"}}, ["Ingress"], ingress=[
                       {"from": [{"namespaceSelector": {"matchLabels": {"ns": "x"}}, "podSelector": {"matchLabels": {"pod": "a"}}}]}]))),
            T("should stop enforcing policies after they are deleted", {"upstream-e2e", "deny-all", "delete-policy"}, [
                (PROBE_ALL, [create_policy(np("deny-all", "x", {}, ["Ingress", "Egress"]))]),
                (PROBE_ALL, [delete_policy("x", "deny-all")])]),
        ]

    def all_cases(self):  # testcasegenerator.go:64-74 order
        return (self.target_cases() + self.rules_cases() + self.peers_cases() + self.port_protocol_cases() +
                self.example_cases() + self.action_cases() + self.conflict_cases() + self.upstream_cases())


# ----------------------------------------------------------------------------- interpreter state
DEFAULT_NAMESPACES = ("x", "y", "z")
DEFAULT_PODS = ("a", "b", "c")
DEFAULT_PORTS = (80, 81)
DEFAULT_PROTOCOLS = (TCP, UDP, SCTP)


class MockIPs:  # kube/ikubernetes.go:292-298: 192.168.1.<n>, n = 1, 2, ... across the whole run
    def __init__(self):
        self.next_id = 1

    def take(self):
        if self.next_id >= 255:
            raise RuntimeError("unable to handle more than 254 pods in mock")
        ip = f"192.168.1.{self.next_id}"
        self.next_id += 1
        return ip


def default_resources(ips: MockIPs):  # resources.go:21-46 + pod.go:28-42, 181-189
    conts = [{"Name": f"cont-{p}-{pr.lower()}", "Port": p, "Protocol": pr, "PortName": f"serve-{p}-{pr.lower()}"}
             for p in DEFAULT_PORTS for pr in DEFAULT_PROTOCOLS]
    pods = [{"Namespace": ns, "Name": n, "Labels": {"pod": n}, "IP": ips.take(), "Containers": conts}
            for ns in DEFAULT_NAMESPACES for n in DEFAULT_PODS]
    return {"Namespaces": {ns: {"ns": ns} for ns in DEFAULT_NAMESPACES}, "Pods": pods}


class CaseState:  # connectivity/testcasestate.go:19-173 (simulated half)
    def __init__(self, resources, ips):
        self.resources = copy.deepcopy(resources)
        self.policies = []
        self.ips = ips

    def _find_pod(self, ns, name):
        for i, p in enumerate(self.resources["Pods"]):
            if p["Namespace"] == ns and p["Name"] == name:
                return i
        raise KeyError(f"pod {ns}/{name} not found")

    def apply(self, action):
        kind, args = action[0], action[1:]
        r = self.resources
        if kind == "create_policy":
            (pol,) = args
            md = pol["metadata"]
            if any(p["metadata"]["namespace"] == md["namespace"] and p["metadata"]["name"] == md["name"] for p in self.policies):
                raise ValueError(f"cannot create policy {md['namespace']}/{md['name']}: already exists")
            self.policies.append(pol)
        elif kind == "update_policy":
            (pol,) = args
            md = pol["metadata"]
            for i, p in enumerate(self.policies):
                if p["metadata"]["namespace"] == md["namespace"] and p["metadata"]["name"] == md["name"]:
                    self.policies[i] = pol
                    break
            else:
                raise ValueError("cannot update policy: not found")
        elif kind == "delete_policy":
            ns, name = args
            idx = [i for i, p in enumerate(self.policies) if p["metadata"]["namespace"] == ns and p["metadata"]["name"] == name]
            if not idx:
                raise ValueError("cannot delete policy: not found")
            del self.policies[idx[-1]]
        elif kind == "create_namespace":
            ns, labels = args
            if ns in r["Namespaces"]:
                raise ValueError(f"namespace {ns} already found")
            r["Namespaces"][ns] = dict(labels)
        elif kind == "set_namespace_labels":
            ns, labels = args
            if ns not in r["Namespaces"]:
                raise ValueError(f"namespace {ns} not found")
            r["Namespaces"][ns] = dict(labels)
        elif kind == "delete_namespace":
            (ns,) = args
            if ns not in r["Namespaces"]:
                raise ValueError(f"namespace {ns} not found")
            del r["Namespaces"][ns]
            r["Pods"] = [p for p in r["Pods"] if p["Namespace"] != ns]
        elif kind == "create_pod":  # resources.go:165-178: containers copied from the first pod
            ns, name, labels = args
            if ns not in r["Namespaces"]:
                raise ValueError(f"can't find namespace {ns}")
            r["Pods"].append({"Namespace": ns, "Name": name, "Labels": dict(labels), "IP": self.ips.take(),
                              "Containers": copy.deepcopy(r["Pods"][0]["Containers"])})
        elif kind == "set_pod_labels":
            ns, name, labels = args
            r["Pods"][self._find_pod(ns, name)]["Labels"] = dict(labels)
        elif kind == "delete_pod":
            ns, name = args
            del r["Pods"][self._find_pod(ns, name)]
        else:
            raise ValueError(f"invalid Action {kind}")


def sweep(allow_dns: bool = True):
    """Every probe step of `cyclonus generate --mock --exclude ''`, in execution order."""
    ips = MockIPs()
    base = default_resources(ips)
    zc = next(p for p in base["Pods"] if p["Namespace"] == "z" and p["Name"] == "c")
    gen = Generator(zc["IP"], allow_dns)
    steps = []
    for ci, case in enumerate(gen.all_cases()):
        state = CaseState(base, ips)
        for si, (probe, actions) in enumerate(case.steps):
            for a in actions:
                state.apply(a)
            steps.append({"case": ci, "step": si, "description": case.description, "policies": copy.deepcopy(state.policies),
                          "resources": copy.deepcopy(state.resources), "probe": probe})
    return steps
