"""Flat-table ingestion (include/cyclonus_hip.h: cyc_resource_tables, cyc_policy_tables,
cyc_probe_config): the inputs as POD arrays plus one string table, the form a cgo binding hands over
from its Go values without any JSON.

This module is the Python counterpart of that binding: it walks a probe.Resources value
(pkg/connectivity/probe/resources.go:15-19, pod.go:44-51,173-179), an already-built *matcher.Policy
(as json.Marshal renders it, pkg/matcher/*.go MarshalJSON) or a list of generator.ProbeConfig values
and fills the arrays.  The library copies everything during the call; the arrays live as long as the
table object.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

i32p, i64p, u8p = ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_uint8)


class Strings(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("bytes", ctypes.c_void_p), ("off", i64p)]


class ResourceTablesC(ctypes.Structure):
    _fields_ = [("str", Strings), ("n_namespaces", ctypes.c_int64), ("ns_name", i32p), ("ns_nil", u8p),
                ("ns_label_off", i64p), ("ns_label_key", i32p), ("ns_label_val", i32p), ("n_pods", ctypes.c_int64),
                ("pod_ns", i32p), ("pod_name", i32p), ("pod_ip", i32p), ("pod_label_off", i64p), ("label_key", i32p),
                ("label_val", i32p), ("pod_cont_off", i64p), ("cont_name", i32p), ("cont_port", i32p),
                ("cont_proto", i32p), ("cont_port_name", i32p), ("pod_nil", u8p)]


class TrafficTablesC(ctypes.Structure):
    _fields_ = [("str", Strings), ("n", ctypes.c_int64), ("internal", u8p), ("ip", i32p), ("ns", i32p),
                ("label_off", i64p), ("label_key", i32p), ("label_val", i32p), ("ns_label_off", i64p),
                ("ns_label_key", i32p), ("ns_label_val", i32p), ("port", i32p), ("port_name", i32p), ("protocol", i32p)]


class ProbeConfigC(ctypes.Structure):
    _fields_ = [("all_available", ctypes.c_int32), ("port_is_name", ctypes.c_int32), ("port", ctypes.c_int32),
                ("port_name_ptr", ctypes.c_char_p), ("port_name_len", ctypes.c_int64),
                ("protocol_ptr", ctypes.c_char_p), ("protocol_len", ctypes.c_int64)]


class PolicyTablesC(ctypes.Structure):
    _fields_ = [("str", Strings), ("n_selectors", ctypes.c_int64), ("sel_label_off", i64p), ("sel_label_key", i32p),
                ("sel_label_val", i32p), ("sel_expr_off", i64p), ("expr_key", i32p), ("expr_op", i32p),
                ("expr_value_off", i64p), ("expr_value", i32p), ("n_port_matchers", ctypes.c_int64), ("pm_all", u8p),
                ("pm_ports_nil", u8p), ("pm_ranges_nil", u8p), ("pm_port_off", i64p), ("port_kind", u8p),
                ("port_value", i32p), ("port_proto", i32p), ("pm_range_off", i64p), ("range_from", i32p),
                ("range_to", i32p), ("range_proto", i32p), ("n_targets", ctypes.c_int64 * 2), ("target_ns", i32p),
                ("target_sel", i32p), ("target_peers_nil", u8p), ("target_peer_off", i64p), ("target_rule_off", i64p),
                ("rule_name", i32p), ("peer_kind", u8p), ("peer_port", i32p), ("peer_ns_kind", u8p), ("peer_ns", i32p),
                ("peer_pod_sel", i32p), ("peer_cidr", i32p), ("peer_except_off", i64p), ("peer_except_nil", u8p),
                ("except_cidr", i32p)]


class _Interner:
    """One string table: index per distinct string, bytes concatenated (UTF-8: Go strings are bytes)."""

    def __init__(self):
        self.ids = {}

    def __call__(self, s) -> int:
        s = "" if s is None else s
        i = self.ids.get(s)
        if i is None:
            i = self.ids[s] = len(self.ids)
        return i

    def table(self, keep):
        enc = [s.encode() for s in self.ids]
        off = np.zeros(len(enc) + 1, np.int64)
        np.cumsum([len(b) for b in enc], out=off[1:])
        blob = ctypes.create_string_buffer(b"".join(enc), max(int(off[-1]), 1))
        keep += [blob, off]
        return Strings(len(enc), ctypes.cast(blob, ctypes.c_void_p), off.ctypes.data_as(i64p))


def _arr(keep, xs, dtype, ptr):
    a = np.ascontiguousarray(np.asarray(xs, dtype=dtype))
    if a.size == 0:
        a = np.zeros(1, dtype)  # a valid pointer for empty ranges
    keep.append(a)
    return a.ctypes.data_as(ptr)


def _offsets(counts):
    off = np.zeros(len(counts) + 1, np.int64)
    if len(counts):
        np.cumsum(counts, out=off[1:])
    return off


class ResourceTables:
    """cyc_resource_tables of a probe.Resources value {"Namespaces": {ns: labels | None}, "Pods": [...]}
    (the exported Go field names; the pod fields Namespace, Name, Labels, IP, Containers[Name, Port,
    Protocol, PortName])."""

    def __init__(self, resources: dict):
        S, keep = _Interner(), []
        nss = resources.get("Namespaces") or {}
        ns_name, ns_nil, ns_cnt, ns_k, ns_v = [], [], [], [], []
        for ns, labels in nss.items():
            ns_name.append(S(ns))
            ns_nil.append(1 if labels is None else 0)
            labels = labels or {}
            ns_cnt.append(len(labels))
            ns_k += [S(k) for k in labels]
            ns_v += [S(v) for v in labels.values()]
        pods = resources.get("Pods") or []
        pns, pname, pip, lcnt, lk, lv, ccnt, cn, cp, cpr, cpn, pnil = ([] for _ in range(12))
        for p in pods:
            pns.append(S(p.get("Namespace")))
            pname.append(S(p.get("Name")))
            pip.append(S(p.get("IP")))
            pnil.append((1 if p.get("Labels") is None else 0) | (2 if p.get("Containers") is None else 0))
            labels = p.get("Labels") or {}
            lcnt.append(len(labels))
            lk += [S(k) for k in labels]
            lv += [S(v) for v in labels.values()]
            cs = p.get("Containers") or []
            ccnt.append(len(cs))
            for c in cs:
                cn.append(S(c.get("Name")))
                cp.append(int(c.get("Port") or 0))
                cpr.append(S(c.get("Protocol")))
                cpn.append(S(c.get("PortName")))
        t = ResourceTablesC()
        t.str = S.table(keep)
        t.n_namespaces = len(ns_name)
        t.ns_name = _arr(keep, ns_name, np.int32, i32p)
        t.ns_nil = _arr(keep, ns_nil, np.uint8, u8p)
        t.ns_label_off = _arr(keep, _offsets(ns_cnt), np.int64, i64p)
        t.ns_label_key = _arr(keep, ns_k, np.int32, i32p)
        t.ns_label_val = _arr(keep, ns_v, np.int32, i32p)
        t.n_pods = len(pods)
        t.pod_ns = _arr(keep, pns, np.int32, i32p)
        t.pod_name = _arr(keep, pname, np.int32, i32p)
        t.pod_ip = _arr(keep, pip, np.int32, i32p)
        t.pod_label_off = _arr(keep, _offsets(lcnt), np.int64, i64p)
        t.label_key = _arr(keep, lk, np.int32, i32p)
        t.label_val = _arr(keep, lv, np.int32, i32p)
        t.pod_cont_off = _arr(keep, _offsets(ccnt), np.int64, i64p)
        t.cont_name = _arr(keep, cn, np.int32, i32p)
        t.cont_port = _arr(keep, cp, np.int32, i32p)
        t.cont_proto = _arr(keep, cpr, np.int32, i32p)
        t.cont_port_name = _arr(keep, cpn, np.int32, i32p)
        t.pod_nil = _arr(keep, pnil, np.uint8, u8p)
        self.c, self._keep = t, keep


def _field(d, name, default=None, nullable=False):
    """A struct field of a decoded JSON object as encoding/json fills it: keys match the field name
    case-insensitively and, among several keys naming the field, the last one wins; a JSON null
    leaves a scalar field unchanged and sets a pointer / map field (nullable) to nil — the JSON entry
    points' rule (csrc/cjson.hpp)."""
    got = default
    if isinstance(d, dict):
        low = name.lower()
        for k, v in d.items():
            if isinstance(k, str) and k.lower() == low and (v is not None or nullable):
                got = v
    return got


def _go_int32(x) -> int:
    """int32(x) of a Go int (two's-complement wrap), as the JSON path stores ResolvedPort."""
    return ((int(x) + (1 << 31)) & 0xFFFFFFFF) - (1 << 31)


class TrafficTables:
    """cyc_traffic_tables of matcher.Traffic values {"Source": peer, "Destination": peer, "ResolvedPort",
    "ResolvedPortName", "Protocol"}, peer = {"Internal": None | {"PodLabels", "NamespaceLabels",
    "Namespace"}, "IP"} (pkg/matcher/traffic.go:11-18): what a Go JobRunner passes per []*Job."""

    def __init__(self, traffics):
        S, keep = _Interner(), []
        internal, ip, ns, lcnt, lk, lv, ncnt, nk, nv = ([] for _ in range(9))
        port, pname, proto = [], [], []
        for t in traffics:
            for end in (_field(t, "Source", {}, True) or {}, _field(t, "Destination", {}, True) or {}):
                inner = _field(end, "Internal", None, True)
                internal.append(0 if inner is None else 1)
                ip.append(S(_field(end, "IP")))
                inner = inner or {}
                ns.append(S(_field(inner, "Namespace")))
                labels = _field(inner, "PodLabels", None, True) or {}
                nsl = _field(inner, "NamespaceLabels", None, True) or {}
                lcnt.append(len(labels))
                lk += [S(k) for k in labels]
                lv += [S(v) for v in labels.values()]
                ncnt.append(len(nsl))
                nk += [S(k) for k in nsl]
                nv += [S(v) for v in nsl.values()]
            port.append(_go_int32(_field(t, "ResolvedPort", 0)))
            pname.append(S(_field(t, "ResolvedPortName")))
            proto.append(S(_field(t, "Protocol")))
        c = TrafficTablesC()
        c.str = S.table(keep)
        c.n = len(port)
        c.internal = _arr(keep, internal, np.uint8, u8p)
        c.ip = _arr(keep, ip, np.int32, i32p)
        c.ns = _arr(keep, ns, np.int32, i32p)
        c.label_off = _arr(keep, _offsets(lcnt), np.int64, i64p)
        c.label_key = _arr(keep, lk, np.int32, i32p)
        c.label_val = _arr(keep, lv, np.int32, i32p)
        c.ns_label_off = _arr(keep, _offsets(ncnt), np.int64, i64p)
        c.ns_label_key = _arr(keep, nk, np.int32, i32p)
        c.ns_label_val = _arr(keep, nv, np.int32, i32p)
        c.port = _arr(keep, port, np.int32, i32p)
        c.port_name = _arr(keep, pname, np.int32, i32p)
        c.protocol = _arr(keep, proto, np.int32, i32p)
        self.c, self.n, self._keep = c, len(port), keep


class ProbeConfigs:
    """cyc_probe_config[] of generator.ProbeConfig values: {"AllAvailable": true} or {"Port": int | str,
    "Protocol": str} (also {"PortProtocol": {...}})."""

    def __init__(self, probes):
        if isinstance(probes, dict):
            probes = [probes]
        self.n = len(probes)
        self.c = (ProbeConfigC * max(self.n, 1))()
        self._keep = []
        for i, p in enumerate(probes):
            if p.get("AllAvailable"):
                self.c[i].all_available = 1
                continue
            pp = p.get("PortProtocol") or p
            port, proto = pp.get("Port"), (pp.get("Protocol") or "").encode()
            self._keep.append(proto)
            self.c[i].protocol_ptr, self.c[i].protocol_len = proto, len(proto)
            if isinstance(port, str):
                b = port.encode()
                self._keep.append(b)
                self.c[i].port_is_name, self.c[i].port_name_ptr, self.c[i].port_name_len = 1, b, len(b)
            else:
                self.c[i].port = int(port or 0)


class PolicyTables:
    """cyc_policy_tables of an already-built *matcher.Policy, given as json.Marshal renders it
    ({"Ingress": {pk: Target}, "Egress": {...}}; Engine.policy_ir())."""

    def __init__(self, ir: dict):
        S, keep = _Interner(), []
        sel_ids = {}
        sl_cnt, sl_k, sl_v, se_cnt, e_k, e_op, ev_cnt, e_v = ([] for _ in range(8))

        def selector(sel) -> int:
            sel = sel or {}
            ml, me = sel.get("matchLabels") or {}, sel.get("matchExpressions") or []
            key = repr((sorted(ml.items()), [(e.get("key"), e.get("operator"), e.get("values")) for e in me]))
            if key in sel_ids:
                return sel_ids[key]
            sel_ids[key] = len(sl_cnt)
            sl_cnt.append(len(ml))
            sl_k.extend(S(k) for k in ml)
            sl_v.extend(S(v) for v in ml.values())
            se_cnt.append(len(me))
            for e in me:
                e_k.append(S(e.get("key")))
                e_op.append(S(e.get("operator")))
                vs = e.get("values") or []
                ev_cnt.append(len(vs))
                e_v.extend(S(v) for v in vs)
            return sel_ids[key]

        pm_all, pm_pnil, pm_rnil, pm_pc, pk_, pv, pp, pm_rc, rf, rt, rp = ([] for _ in range(11))

        def port_matcher(pm) -> int:
            idx = len(pm_all)
            if not pm or pm.get("Type") == "all ports":
                pm_all.append(1), pm_pnil.append(1), pm_rnil.append(1), pm_pc.append(0), pm_rc.append(0)
                return idx
            ports, ranges = pm.get("Ports"), pm.get("PortRanges")
            pm_all.append(0)
            pm_pnil.append(1 if ports is None else 0)
            pm_rnil.append(1 if ranges is None else 0)
            pm_pc.append(len(ports or []))
            for p in ports or []:
                port = p.get("Port")
                pk_.append(0 if port is None else 2 if isinstance(port, str) else 1)
                pv.append(0 if port is None else S(port) if isinstance(port, str) else int(port))
                pp.append(S(p.get("Protocol")))
            pm_rc.append(len(ranges or []))
            for r in ranges or []:
                rf.append(int(r.get("From") or 0))
                rt.append(int(r.get("To") or 0))
                rp.append(S(r.get("Protocol")))
            return idx

        n_t = [0, 0]
        t_ns, t_sel, t_pnil, t_pc, t_rc, rules = ([] for _ in range(6))
        kind, pport, nsk, nsv, psel, cidr, ex_cnt, ex_nil, exc = ([] for _ in range(9))
        for d, name in enumerate(("Ingress", "Egress")):
            for tg in (ir.get(name) or {}).values():
                n_t[d] += 1
                t_ns.append(S(tg.get("Namespace")))
                t_sel.append(selector(tg.get("PodSelector")))
                peers = tg.get("Peers")
                t_pnil.append(1 if peers is None else 0)
                t_pc.append(len(peers or []))
                srs = tg.get("SourceRules") or []
                t_rc.append(len(srs))
                rules.extend(S(((r or {}).get("metadata") or {}).get("name")) for r in srs)
                for p in peers or []:
                    ty = p.get("Type")
                    nsk_, nsv_, psel_, cidr_, exs, exnil = 0, 0, -1, 0, [], 1
                    if ty == "all peers":
                        k, port = _lib.PEER_ALL, -1
                    elif ty == "all peers for port":
                        k, port = _lib.PEER_PORTS, port_matcher(p.get("Port"))
                    elif ty == "IPBlock":
                        k, port = _lib.PEER_IP, port_matcher(p.get("Port"))
                        cidr_ = S(p.get("CIDR"))
                        exs = p.get("Except")
                        exnil = 1 if exs is None else 0
                        exs = [S(e) for e in exs or []]
                    else:
                        k, port = _lib.PEER_POD, port_matcher(p.get("Port"))
                        ns = p.get("Namespace") or {"Type": "all namespaces"}
                        if ns.get("Type") == "specific namespace":
                            nsk_, nsv_ = _lib.NS_EXACT, S(ns.get("Namespace"))
                        elif ns.get("Type") == "matching namespace by label":
                            nsk_, nsv_ = _lib.NS_LABEL, selector(ns.get("Selector"))
                        else:
                            nsk_ = _lib.NS_ALL
                        pod = p.get("Pod") or {}
                        if pod.get("Type") == "matching pods by label":
                            psel_ = selector(pod.get("Selector"))
                    kind.append(k), pport.append(port), nsk.append(nsk_), nsv.append(nsv_), psel.append(psel_)
                    cidr.append(cidr_), ex_cnt.append(len(exs)), ex_nil.append(exnil)
                    exc.extend(exs)
        t = PolicyTablesC()
        t.str = S.table(keep)
        t.n_selectors = len(sl_cnt)
        t.sel_label_off, t.sel_label_key, t.sel_label_val = (_arr(keep, _offsets(sl_cnt), np.int64, i64p),
                                                             _arr(keep, sl_k, np.int32, i32p), _arr(keep, sl_v, np.int32, i32p))
        t.sel_expr_off, t.expr_key, t.expr_op = (_arr(keep, _offsets(se_cnt), np.int64, i64p), _arr(keep, e_k, np.int32, i32p),
                                                 _arr(keep, e_op, np.int32, i32p))
        t.expr_value_off, t.expr_value = _arr(keep, _offsets(ev_cnt), np.int64, i64p), _arr(keep, e_v, np.int32, i32p)
        t.n_port_matchers = len(pm_all)
        t.pm_all, t.pm_ports_nil, t.pm_ranges_nil = (_arr(keep, pm_all, np.uint8, u8p), _arr(keep, pm_pnil, np.uint8, u8p),
                                                     _arr(keep, pm_rnil, np.uint8, u8p))
        t.pm_port_off, t.port_kind, t.port_value, t.port_proto = (_arr(keep, _offsets(pm_pc), np.int64, i64p),
                                                                  _arr(keep, pk_, np.uint8, u8p), _arr(keep, pv, np.int32, i32p),
                                                                  _arr(keep, pp, np.int32, i32p))
        t.pm_range_off, t.range_from, t.range_to, t.range_proto = (_arr(keep, _offsets(pm_rc), np.int64, i64p),
                                                                   _arr(keep, rf, np.int32, i32p), _arr(keep, rt, np.int32, i32p),
                                                                   _arr(keep, rp, np.int32, i32p))
        t.n_targets[0], t.n_targets[1] = n_t
        t.target_ns, t.target_sel, t.target_peers_nil = (_arr(keep, t_ns, np.int32, i32p), _arr(keep, t_sel, np.int32, i32p),
                                                         _arr(keep, t_pnil, np.uint8, u8p))
        t.target_peer_off, t.target_rule_off, t.rule_name = (_arr(keep, _offsets(t_pc), np.int64, i64p),
                                                             _arr(keep, _offsets(t_rc), np.int64, i64p),
                                                             _arr(keep, rules, np.int32, i32p))
        t.peer_kind, t.peer_port, t.peer_ns_kind, t.peer_ns = (_arr(keep, kind, np.uint8, u8p), _arr(keep, pport, np.int32, i32p),
                                                               _arr(keep, nsk, np.uint8, u8p), _arr(keep, nsv, np.int32, i32p))
        t.peer_pod_sel, t.peer_cidr = _arr(keep, psel, np.int32, i32p), _arr(keep, cidr, np.int32, i32p)
        t.peer_except_off, t.peer_except_nil, t.except_cidr = (_arr(keep, _offsets(ex_cnt), np.int64, i64p),
                                                               _arr(keep, ex_nil, np.uint8, u8p), _arr(keep, exc, np.int32, i32p))
        self.c, self._keep = t, keep


def _dump_struct(t, keep, f, prefix=""):
    """Write a tables struct field by field: a "name kind count" line, then the raw bytes (kind i64 /
    i32 / u8; count -1 = NULL).  tests/native/capi_driver.cpp --flat reads this back into the C struct."""
    kinds = {ctypes.c_int64: "i64", ctypes.c_int32: "i32", ctypes.c_uint8: "u8"}
    by_addr = {a.ctypes.data: a for a in keep if isinstance(a, np.ndarray)}
    for name, ty in t._fields_:
        v = getattr(t, name)
        if isinstance(v, Strings):
            blob = next(b for b in keep if isinstance(b, ctypes.Array) and ctypes.addressof(b) == v.bytes)
            n_bytes = int(by_addr[ctypes.cast(v.off, ctypes.c_void_p).value][-1])
            f.write(f"{prefix}{name}.n i64 1\n".encode() + np.int64(v.n).tobytes())
            f.write(f"{prefix}{name}.bytes u8 {n_bytes}\n".encode() + bytes(blob)[:n_bytes])
            off = by_addr[ctypes.cast(v.off, ctypes.c_void_p).value]
            f.write(f"{prefix}{name}.off i64 {off.size}\n".encode() + off.tobytes())
        elif ty is ctypes.c_int64:
            f.write(f"{prefix}{name} i64 1\n".encode() + np.int64(v).tobytes())
        elif isinstance(v, ctypes.Array):  # int64[2]
            f.write(f"{prefix}{name} i64 {len(v)}\n".encode() + np.array(list(v), np.int64).tobytes())
        else:
            addr = ctypes.cast(v, ctypes.c_void_p).value
            kind = kinds[ty._type_]
            if addr is None:
                f.write(f"{prefix}{name} {kind} -1\n".encode())
                continue
            a = by_addr[addr]
            f.write(f"{prefix}{name} {kind} {a.size}\n".encode() + a.tobytes())


def dump_tables(tables, path):
    """ResourceTables / PolicyTables -> the field dump capi_driver --flat reads."""
    with open(path, "wb") as f:
        _dump_struct(tables.c, tables._keep, f)


def dump_probe_configs(probes, path):
    """generator.ProbeConfig values as capi_driver --flat lines: "all", "int PORT PROTO", "name NAME PROTO"."""
    pc = ProbeConfigs(probes)
    with open(path, "w") as f:
        for i in range(pc.n):
            c = pc.c[i]
            proto = (c.protocol_ptr or b"").decode()
            if c.all_available:
                f.write("all\n")
            elif c.port_is_name:
                f.write(f"name {c.port_name_ptr.decode()} {proto}\n")
            else:
                f.write(f"int {c.port} {proto}\n")


def prepare_flat(eng, policies, resources, probes) -> dict:
    """The drop-in's host path as bench.py times it (analyze --mode probe, pkg/cli/analyze.go:121,
    232-243): BuildNetworkPolicies + Simplify from the NetworkPolicy JSON (cyc_policy_build_json),
    the probe model through the flat tables a cgo binding passes (cyc_resources_load, no JSON) and
    cyc_probe_prepare_configs.  Returns the probe shape plus a "prepare_s" dict of the phase times
    (tables_marshal_s = building the flat tables in Python from the dicts, which a Go binding does from
    its structs; not in total_s)."""
    import json
    import time

    pols_json = json.dumps(policies)
    t_m = time.perf_counter()
    res_tables = ResourceTables(resources)
    cfgs = ProbeConfigs(probes)
    marshal_s = time.perf_counter() - t_m
    t0 = time.perf_counter()
    eng.build_policies(pols_json)
    t_built = time.perf_counter()
    eng.load_resources_tables(res_tables)
    t_loaded = time.perf_counter()
    shape = eng.prepare_configs(cfgs)
    t_prepared = time.perf_counter()
    shape = dict(shape)
    shape["prepare_s"] = {"policy_build_s": t_built - t0, "resources_load_s": t_loaded - t_built,
                          "probe_prepare_s": t_prepared - t_loaded, "total_s": t_prepared - t0,
                          "path": "cyc_policy_build_json + cyc_resources_load (flat tables) + cyc_probe_prepare_configs",
                          "tables_marshal_s": marshal_s,
                          "note": "tables_marshal_s = building the flat tables in Python from the synthetic dicts (a Go "
                                  "binding fills them from its structs); not in total_s"}
    return shape
