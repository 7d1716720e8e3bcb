"""Host-side mirror of the reference's pkg/matcher API, backed by libcyclonus_hip.

    policy = build_network_policies(True, netpols)       # builder.go:11-26
    result = policy.is_traffic_allowed(traffic)           # policy.go:131-136
    result.is_allowed(), result.ingress.is_allowed()      # policy.go:89-91, :123-125

Traffic objects are the reference's matcher.Traffic JSON shape (traffic.go:11-81): dicts with
Source / Destination {"Internal": {"PodLabels", "NamespaceLabels", "Namespace"} | None, "IP"},
"ResolvedPort", "ResolvedPortName", "Protocol".  Evaluation runs on the GPU (cyc_query_traffic_tables,
or cyc_query_traffic_targets for the target lists); a Go panic of the reference surfaces as cyclonus_amd.CyclonusPanic with the same message.
"""
from __future__ import annotations

import json
from dataclasses import dataclass
from typing import List, Optional

from .engine import Engine


@dataclass
class InternalPeer:  # traffic.go:75-81
    pod_labels: Optional[dict]
    namespace_labels: Optional[dict]
    namespace: str

    def to_json(self):
        return {"PodLabels": self.pod_labels, "NamespaceLabels": self.namespace_labels, "Namespace": self.namespace}


@dataclass
class TrafficPeer:  # traffic.go:58-73
    internal: Optional[InternalPeer]
    ip: str

    def is_external(self) -> bool:
        return self.internal is None

    def to_json(self):
        return {"Internal": self.internal.to_json() if self.internal else None, "IP": self.ip}


@dataclass
class Traffic:  # traffic.go:11-18
    source: TrafficPeer
    destination: TrafficPeer
    resolved_port: int = 0
    resolved_port_name: str = ""
    protocol: str = "TCP"

    def to_json(self):
        return {"Source": self.source.to_json(), "Destination": self.destination.to_json(), "ResolvedPort": self.resolved_port,
                "ResolvedPortName": self.resolved_port_name, "Protocol": self.protocol}


def _traffic_json(t):
    return t.to_json() if isinstance(t, Traffic) else t


@dataclass
class DirectionResult:  # policy.go:84-91
    allowed: bool
    # primary keys of the matching targets that allow / deny (None when not requested); the
    # reference walks a Go map, so its order is random — these are in primary-key order
    allowing_targets: Optional[List[str]] = None
    denying_targets: Optional[List[str]] = None

    def is_allowed(self) -> bool:
        return self.allowed


@dataclass
class AllowedResult:  # policy.go:93-125
    ingress: DirectionResult
    egress: DirectionResult

    def is_allowed(self) -> bool:
        return self.ingress.is_allowed() and self.egress.is_allowed()


class Policy:
    """*matcher.Policy: compiled targets held by a libcyclonus_hip context on `device`."""

    def __init__(self, engine: Engine):
        self.engine = engine

    def to_json(self) -> dict:
        """json.Marshal(*matcher.Policy)."""
        return self.engine.policy_ir()

    @property
    def ingress(self) -> dict:
        return self.to_json()["Ingress"]

    @property
    def egress(self) -> dict:
        return self.to_json()["Egress"]

    def is_traffic_allowed(self, traffic) -> AllowedResult:
        """policy.go:131-136, with the allowing / denying target lists."""
        return self.is_traffic_allowed_batch([traffic], targets=True)[0]

    def is_traffic_allowed_batch(self, traffics, targets: bool = False):
        """One GPU batch; targets=True also returns the DirectionResult target lists."""
        docs = [_traffic_json(t) for t in traffics]
        if not targets:  # the flat tables a Go JobRunner passes (cyc_query_traffic_tables), no JSON
            res = self.engine.query_traffic_tables(docs)
            return [AllowedResult(DirectionResult(i), DirectionResult(e)) for i, e in res]
        out = []
        for r in self.engine.query_traffic_targets(docs):
            dirs = [DirectionResult(r[k]["IsAllowed"], r[k]["AllowingTargets"], r[k]["DenyingTargets"])
                    for k in ("Ingress", "Egress")]
            out.append(AllowedResult(*dirs))
        return out

    def targets_applying_to_pod(self, is_ingress: bool, namespace: str, pod_labels) -> List[str]:
        """policy.go:68-82 (primary keys, in primary-key order)."""
        r = self.engine.query_targets([{"Namespace": namespace, "Labels": pod_labels}])[0]
        return r["Ingress" if is_ingress else "Egress"]

    def query_targets(self, pods):
        """analyze --mode query-target (analyze.go:163-187): per QueryTargetPod {Namespace, Labels},
        the targets applying to it per direction."""
        return self.engine.query_targets(list(pods))


def build_network_policies(simplify: bool, netpols, device: int = 0) -> Policy:
    """matcher.BuildNetworkPolicies(simplify, netpols) (builder.go:11-26)."""
    return Policy(Engine(device).build_policies(json.dumps(list(netpols)), simplify))


def load_policy(policy_json, device: int = 0) -> Policy:
    """A Policy from json.Marshal(*matcher.Policy) produced by the Go reference."""
    doc = policy_json if isinstance(policy_json, str) else json.dumps(policy_json)
    return Policy(Engine(device).load_policy_ir(doc))
