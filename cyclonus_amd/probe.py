"""Host-side mirror of the reference's pkg/connectivity/probe simulated path, on libcyclonus_hip.

    runner = new_simulated_runner(policy)                          # jobrunner.go:17-19
    table = runner.run_probe_for_config(new_probe_config(80, "TCP"), resources)   # :29-31
    print(table.render_table())                                    # table.go:66-68

`Table` is a lazy view over the packed verdict planes (it never materialises the P^2 Item
maps of truthtable.go:28-48); `Table.get(from, to)` builds one Item on demand.  Job keys,
statuses and the Connectivity values follow job.go:23-25 and jobrunner.go:33-94.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from . import _lib
from .engine import Engine
from .matcher import Policy, _traffic_json
from .tablewriter import render

# connectivity.go:7-14 and ShortString :27-42
UNKNOWN, CHECK_FAILED, INVALID_NAMED_PORT, INVALID_PORT_PROTOCOL, BLOCKED, ALLOWED = (
    "unknown", "checkfailed", "invalidnamedport", "invalidportprotocol", "blocked", "allowed")
SHORT = {UNKNOWN: "?", CHECK_FAILED: "!", BLOCKED: "X", ALLOWED: ".", INVALID_NAMED_PORT: "P", INVALID_PORT_PROTOCOL: "N"}


def short_string(c: str) -> str:
    if c not in SHORT:
        raise ValueError(f"invalid Connectivity value: {c}")
    return SHORT[c]


# ----------------------------------------------------------------------------- model
@dataclass
class Container:  # pod.go:173-179
    name: str
    port: int
    protocol: str
    port_name: str

    def to_json(self):
        return {"Name": self.name, "Port": self.port, "Protocol": self.protocol, "PortName": self.port_name}


@dataclass
class Pod:  # pod.go:44-51
    namespace: str
    name: str
    labels: Optional[Dict[str, str]]
    ip: str
    containers: List[Container] = field(default_factory=list)

    def pod_string(self) -> str:  # podstring.go:11-14
        return f"{self.namespace}/{self.name}"

    def to_json(self):
        return {"Namespace": self.namespace, "Name": self.name, "Labels": self.labels, "IP": self.ip,
                "Containers": [c.to_json() for c in self.containers]}


@dataclass
class Resources:  # resources.go:15-19
    namespaces: Dict[str, Optional[Dict[str, str]]]
    pods: List[Pod]

    @staticmethod
    def from_json(doc) -> "Resources":
        doc = json.loads(doc) if isinstance(doc, (str, bytes)) else doc
        pods = [Pod(p.get("Namespace", ""), p.get("Name", ""), p.get("Labels"), p.get("IP", ""),
                    [Container(c.get("Name", ""), int(c.get("Port", 0)), c.get("Protocol", ""), c.get("PortName", ""))
                     for c in p.get("Containers") or []]) for p in doc.get("Pods") or []]
        return Resources(dict(doc.get("Namespaces") or {}), pods)

    def to_json(self):
        return {"Namespaces": self.namespaces, "Pods": [p.to_json() for p in self.pods]}

    def sorted_pod_names(self) -> List[str]:  # resources.go:223-230
        return sorted(p.pod_string() for p in self.pods)


@dataclass
class ProbeConfig:  # generator/testcase.go:139-156
    all_available: bool = False
    port: Optional[object] = None  # int or str (intstr.IntOrString)
    protocol: str = ""

    def to_json(self):
        if self.all_available:
            return {"AllAvailable": True}
        return {"Port": self.port, "Protocol": self.protocol}


def new_probe_config(port, protocol) -> ProbeConfig:
    return ProbeConfig(False, port, protocol)


def new_all_available() -> ProbeConfig:
    return ProbeConfig(True)


def _as_resources(r) -> Resources:
    return r if isinstance(r, Resources) else Resources.from_json(r)


def _as_probe(c) -> ProbeConfig:
    if isinstance(c, ProbeConfig):
        return c
    if c.get("AllAvailable"):
        return ProbeConfig(True)
    pp = c.get("PortProtocol", c)
    return ProbeConfig(False, pp.get("Port"), pp.get("Protocol", ""))


@dataclass
class JobResult:  # job.go:16-25
    key: str
    ingress: str
    egress: str
    combined: str


@dataclass
class Item:  # table.go:10-23
    from_: str
    to: str
    job_results: Dict[str, JobResult]


# ----------------------------------------------------------------------------- table view
_CONN = {_lib.CONN_UNKNOWN: UNKNOWN, _lib.CONN_CHECK_FAILED: CHECK_FAILED, _lib.CONN_INVALID_NAMED_PORT: INVALID_NAMED_PORT,
         _lib.CONN_INVALID_PORT_PROTOCOL: INVALID_PORT_PROTOCOL, _lib.CONN_BLOCKED: BLOCKED, _lib.CONN_ALLOWED: ALLOWED}


class PlaneCells:
    """Cells source over packed planes held on the host (status[P,K], ingress[P,K,W], egress[P,K,W]),
    e.g. the oracle's: the same Connectivity mapping as cyc_table_cells (jobrunner.go:36-55,85-93)."""

    def __init__(self, status, ingress, egress):
        self.status, self.ingress, self.egress = status, ingress, egress

    def cells(self, s_lo, s_hi, d_lo, d_hi, k_lo, k_hi, want=("ingress", "egress", "combined")):
        s = np.arange(s_lo, s_hi)[:, None, None]
        d = np.arange(d_lo, d_hi)[None, :, None]
        k = np.arange(k_lo, k_hi)[None, None, :]
        st = self.status[d, k]
        ai = ((self.ingress[d, k, s // 64] >> (s % 64).astype(np.uint64)) & np.uint64(1)).astype(bool)
        ae = ((self.egress[s, k, d // 64] >> (d % 64).astype(np.uint64)) & np.uint64(1)).astype(bool)
        valid, bpp, bnp = st == _lib.JOB_VALID, st == _lib.JOB_BAD_PORT_PROTOCOL, st == _lib.JOB_BAD_NAMED_PORT
        inv = np.where(bpp, _lib.CONN_INVALID_PORT_PROTOCOL, np.where(bnp, _lib.CONN_INVALID_NAMED_PORT, _lib.CONN_NO_JOB))
        allowed = lambda b: np.where(b, _lib.CONN_ALLOWED, _lib.CONN_BLOCKED)  # noqa: E731
        out = {"ingress": np.where(valid, allowed(ai), inv),
               "egress": np.where(valid, allowed(ae), np.where(bpp | bnp, _lib.CONN_UNKNOWN, _lib.CONN_NO_JOB)),
               "combined": np.where(valid, allowed(ai & ae), inv)}
        return {n: np.broadcast_to(out[n], (s_hi - s_lo, d_hi - d_lo, k_hi - k_lo)).astype(np.uint8) for n in want}


class Table:
    """Lazy probe.Table over one probe config's slots of a verdict table (table.go:24-56).

    `cells` is a cells source: the product's DeviceTable (cyc_table: planes resident on the GPU,
    Connectivity computed on the device per block of cells) or a PlaneCells view.  Items
    (table.go:10-23) are built on demand; the P^2 Item maps of truthtable.go:28-48 never exist."""

    CACHE_CELLS = 1 << 24  # whole-table Connectivity cache for rendering small tables

    def __init__(self, resources: Resources, config: ProbeConfig, cells, slot_lo: int, slot_hi: int):
        self.resources = resources
        self.config = config
        self.src = cells
        self.slots = range(slot_lo, slot_hi)
        self.items = resources.sorted_pod_names()
        self.index = {p.pod_string(): i for i, p in enumerate(resources.pods)}
        self._all = None
        self._rows = {}

    def _job_key(self, d: int, j: int) -> str:
        pod = self.resources.pods[d]
        if self.config.all_available:
            c = pod.containers[j]
            return f"{c.protocol}/{c.port}"
        port = self.config.port
        if isinstance(port, str):  # named port: ResolvedPort is -1 when it does not resolve
            hit = next((c for c in pod.containers if c.port_name == port), None)
            resolved = hit.port if hit is not None else -1
        else:
            resolved = int(port)
        return f"{self.config.protocol}/{resolved}"

    def _row(self, s: int):
        """Connectivity codes of source row s: {name: [P, nk]}."""
        P, lo, hi = len(self.resources.pods), self.slots.start, self.slots.stop
        if self._all is None and P * P * max(hi - lo, 1) <= self.CACHE_CELLS:
            self._all = self.src.cells(0, P, 0, P, lo, hi)
        if self._all is not None:
            return {n: a[s] for n, a in self._all.items()}
        if s not in self._rows:
            if len(self._rows) > 64:
                self._rows.clear()
            self._rows[s] = {n: a[0] for n, a in self.src.cells(s, s + 1, 0, P, lo, hi).items()}
        return self._rows[s]

    def get(self, fr: str, to: str) -> Item:
        s, d = self.index[fr], self.index[to]
        row = self._row(s)
        out = {}
        for j in range(len(self.slots)):
            ci = int(row["combined"][d, j])
            if ci == _lib.CONN_NO_JOB:
                continue
            key = self._job_key(d, j)
            out[key] = JobResult(key, _CONN[int(row["ingress"][d, j])], _CONN[int(row["egress"][d, j])], _CONN[ci])
        return Item(fr, to, out)

    def keys(self):
        return [(a, b) for a in self.items for b in self.items]

    # table.go:58-156
    def render_ingress(self) -> str:
        return self._render(lambda r: short_string(r.ingress))

    def render_egress(self) -> str:
        return self._render(lambda r: short_string(r.egress))

    def render_table(self) -> str:
        return self._render(lambda r: short_string(r.combined))

    def _render(self, fn) -> str:
        uniform, single = True, True
        schema = set()
        for fr, to in self.keys():
            d = self.get(fr, to).job_results
            if len(d) != 1:
                single = False
                break
            schema.add("_".join(sorted(d)))
            if len(schema) > 1:
                uniform = False
                break
        if uniform and single:  # renderSimpleTable :96-105
            rows = [[fr] + [fn(next(iter(self.get(fr, to).job_results.values()))) for to in self.items] for fr in self.items]
            return render([""] + self.items, rows, row_line=False)
        if uniform:  # renderUniformMultiTable :107-123 (schema of the first cell)
            first = self.get(self.items[0], self.items[0]).job_results
            keys = sorted(first)
            rows = []
            for fr in self.items:
                row = [fr]
                for to in self.items:
                    d = self.get(fr, to).job_results
                    if any(k not in d for k in keys):
                        raise _lib.CyclonusPanic(0, "runtime error: invalid memory address or nil pointer dereference")
                    row.append("\n".join(fn(d[k]) for k in keys))
                rows.append(row)
            return render(["\n".join(keys)] + self.items, rows, row_line=True)
        rows = []  # renderNonuniformTable :125-140
        for fr in self.items:
            row = [fr]
            for to in self.items:
                d = self.get(fr, to).job_results
                row.append("\n".join(f"{k}: {fn(d[k])}" for k in sorted(d)))
            rows.append(row)
        return render([""] + self.items, rows, row_line=True)


# ----------------------------------------------------------------------------- runners
class Runner:
    """probe.Runner over the GPU engine (jobrunner.go:13-58)."""

    def __init__(self, policy: Policy):
        self.policy = policy
        self.job_runner = SimulatedJobRunner(policy)

    def run_probe_for_config(self, probe_config, resources) -> Table:
        return self.run_probes([probe_config], resources)[0]

    def run_probes(self, probe_configs, resources) -> List[Table]:
        """All configs in one batched GPU pass; one Table per config."""
        res = _as_resources(resources)
        cfgs = [_as_probe(c) for c in probe_configs]
        eng: Engine = self.policy.engine
        eng.load_resources(json.dumps(res.to_json()))
        eng.prepare([c.to_json() for c in cfgs])
        dt = eng.table()  # planes stay on the GPU; Items are built from device-computed cells
        maxc = max((len(p.containers) for p in res.pods), default=0)
        tables, lo = [], 0
        for c in cfgs:
            n = maxc if c.all_available else 1
            tables.append(Table(res, c, dt, lo, lo + n))
            lo += n
        return tables


class SimulatedJobRunner:
    """JobRunner.RunJobs (jobrunner.go:60-94) for explicit job lists: every job's Traffic
    (job.go:81-103) is evaluated on the GPU in one batch."""

    def __init__(self, policy: Policy):
        self.policies = policy

    def run_jobs(self, jobs) -> List[JobResult]:
        traffics = []
        for j in jobs:
            traffics.append({
                "Source": {"Internal": {"PodLabels": j.get("FromPodLabels"), "NamespaceLabels": j.get("FromNamespaceLabels"),
                                        "Namespace": j.get("FromNamespace", "")}, "IP": j.get("FromIP", "")},
                "Destination": {"Internal": {"PodLabels": j.get("ToPodLabels"), "NamespaceLabels": j.get("ToNamespaceLabels"),
                                             "Namespace": j.get("ToNamespace", "")}, "IP": j.get("ToIP", "")},
                "ResolvedPort": j.get("ResolvedPort", 0), "ResolvedPortName": j.get("ResolvedPortName", ""),
                "Protocol": j.get("Protocol", "")})
        out = []
        for j, r in zip(jobs, self.policies.is_traffic_allowed_batch([_traffic_json(t) for t in traffics])):
            ing = ALLOWED if r.ingress.is_allowed() else BLOCKED
            eg = ALLOWED if r.egress.is_allowed() else BLOCKED
            out.append(JobResult(f"{j.get('Protocol', '')}/{j.get('ResolvedPort', 0)}", ing, eg,
                                 ALLOWED if r.is_allowed() else BLOCKED))
        return out


def new_simulated_runner(policy: Policy) -> Runner:
    return Runner(policy)
