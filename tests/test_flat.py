"""Flat-table ingestion on the CPU (include/cyclonus_hip.h cyc_resources_load / cyc_policy_load /
cyc_probe_prepare_configs): the tables a cgo binding passes without JSON load the same probe model and
the same compiled policy as the JSON entry points, and malformed tables are refused with CYC_ERR_ARG."""
import ctypes
import json
import os

import numpy as np
import pytest

from cyclonus_amd import _lib, flat
from cyclonus_amd.engine import Engine
from randgen import random_problem

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _both(res):
    a = Engine(0).load_resources(res).resources_json()
    b = Engine(0).load_resources_tables(res).resources_json()
    return a, b


def test_resources_tables_equal_json_random():
    for seed in range(60):
        _, res, _ = random_problem(7000 + seed, dups=seed % 2 == 0)
        a, b = _both(res)
        assert a == b, seed


def test_resources_tables_equal_json_config1_and_edges():
    res = json.load(open(os.path.join(ROOT, "tests", "golden", "config1.json")))["resources"]
    a, b = _both(res)
    assert a == b
    edge = {"Namespaces": {"x": None, "y": {}, "z": {"k": ""}},
            "Pods": [{"Namespace": "x", "Name": "a", "Labels": None, "IP": "", "Containers": None},
                     {"Namespace": "x/y", "Name": "é\u0000b", "Labels": {"": ""}, "IP": "::1",
                      "Containers": [{"Name": "c", "Port": -5, "Protocol": "tcp", "PortName": ""}]}]}
    a, b = _both(edge)
    assert a == b
    assert a["Namespaces"]["x"] is None and a["Pods"][1]["Name"] == "é\u0000b"
    # nil label maps and container slices marshal as null (json.Marshal), empty ones as {} / []
    assert a["Pods"][0]["Labels"] is None and a["Pods"][0]["Containers"] is None
    edge["Pods"][0].update(Labels={}, Containers=[])
    del edge["Pods"][1]["Labels"]
    a, b = _both(edge)
    assert a == b and a["Pods"][0]["Labels"] == {} and a["Pods"][0]["Containers"] == []
    assert a["Pods"][1]["Labels"] is None  # an absent field decodes as nil


def test_json_dumps_report_errors():
    """cyc_resources_json / cyc_policy_ir_json: -(cyc_status) with a message when nothing is loaded; a
    buffer smaller than the text gets nothing written (run under ASan by test_sanitized)."""
    e = Engine(0)
    with pytest.raises(_lib.CyclonusError, match="no resources loaded"):
        e.resources_json()
    with pytest.raises(_lib.CyclonusError, match="no policy loaded"):
        e.policy_ir()
    assert _lib.lib().cyc_resources_json(e._ctx, None, 0) == -_lib.ERR_ARG
    e.load_resources(json.load(open(os.path.join(ROOT, "tests", "golden", "config1.json")))["resources"])
    need = _lib.lib().cyc_resources_json(e._ctx, None, 0)
    assert need > 1
    small = ctypes.create_string_buffer(b"\x7f" * 16, 16)
    assert _lib.lib().cyc_resources_json(e._ctx, small, 16) == need
    assert small.raw == b"\x7f" * 16
    full = ctypes.create_string_buffer(int(need))
    assert _lib.lib().cyc_resources_json(e._ctx, full, int(need)) == need and full.raw[need - 1] == 0


def test_policy_tables_roundtrip():
    """json.Marshal(*Policy) -> flat tables -> cyc_policy_load -> the same IR (targets, ordered peers,
    shared and range port matchers, selectors with expressions, IPBlocks with nil / empty excepts)."""
    for seed in range(80):
        pols, _, _ = random_problem(8000 + seed)
        e = Engine(0).build_policies(pols)
        ir = e.policy_ir()
        got = Engine(0).load_policy_tables(ir).policy_ir()
        assert got == ir, seed


def test_probe_configs():
    pc = flat.ProbeConfigs([{"Port": 80, "Protocol": "TCP"}, {"Port": "serve-81-udp", "Protocol": "UDP"},
                            {"AllAvailable": True}, {"PortProtocol": {"Port": 53, "Protocol": "sctp"}}])
    assert pc.n == 4
    assert (pc.c[0].port, pc.c[0].port_is_name, pc.c[0].protocol_ptr, pc.c[0].protocol_len) == (80, 0, b"TCP", 3)
    assert (pc.c[1].port_is_name, pc.c[1].port_name_ptr, pc.c[1].port_name_len) == (1, b"serve-81-udp", 12)
    assert pc.c[2].all_available == 1
    assert (pc.c[3].port, pc.c[3].protocol_ptr) == (53, b"sctp")
    # Go strings may hold NUL bytes: they travel as pointer + length, not as C strings
    pc = flat.ProbeConfigs([{"Port": "a\u0000b", "Protocol": "T\u0000CP"}])
    assert pc.c[0].port_name_len == 3 and pc.c[0].protocol_len == 4
    addr = ctypes.c_void_p.from_buffer(pc.c[0], flat.ProbeConfigC.protocol_ptr.offset).value
    assert ctypes.string_at(addr, 4) == b"T\x00CP"


def test_traffic_tables():
    """cyc_traffic_tables (the flat matcher.Traffic a Go JobRunner passes): endpoints, labels, ports as
    indices; malformed tables are refused with the offending index before any device work."""
    tr = [{"Source": {"Internal": {"PodLabels": {"a": "b"}, "NamespaceLabels": None, "Namespace": "x"}, "IP": "10.0.0.1"},
           "Destination": {"Internal": None, "IP": "1.2.3.4"}, "ResolvedPort": 80, "ResolvedPortName": "", "Protocol": "TCP"}]
    t = flat.TrafficTables(tr)
    assert t.n == 1 and list(np.ctypeslib.as_array(t.c.internal, (2,))) == [1, 0]
    e = Engine(0).build_policies(random_problem(8100)[0])
    bad = np.array([99, 0], np.int32)
    t.c.ip = bad.ctypes.data_as(flat.i32p)
    out = (ctypes.c_uint8 * 1)()
    rc = _lib.lib().cyc_query_traffic_tables(e._ctx, ctypes.byref(t.c), out, 1)
    assert rc == _lib.ERR_ARG and "ip[0] = 99 out of range" in _lib.lib().cyc_last_error(e._ctx).decode()
    t = flat.TrafficTables(tr)
    rc = _lib.lib().cyc_query_traffic_tables(e._ctx, ctypes.byref(t.c), out, 0)  # output smaller than the list
    assert rc == _lib.ERR_ARG and "smaller" in _lib.lib().cyc_last_error(e._ctx).decode()
    bare = Engine(0)
    rc = _lib.lib().cyc_query_traffic_tables(bare._ctx, ctypes.byref(t.c), out, 1)
    assert rc == _lib.ERR_ARG  # no policy loaded


def test_malformed_tables_refused():
    res = {"Namespaces": {"x": {"a": "b"}}, "Pods": [{"Namespace": "x", "Name": "p", "IP": "10.0.0.1",
                                                      "Labels": {"a": "b"}, "Containers": []}]}
    e = Engine(0)

    def load(mutate):
        t = flat.ResourceTables(res)
        mutate(t.c)
        return _lib.lib().cyc_resources_load(e._ctx, ctypes.byref(t.c)), _lib.lib().cyc_last_error(e._ctx).decode()

    bad = np.array([99], np.int32)
    rc, msg = load(lambda c: setattr(c, "pod_ns", bad.ctypes.data_as(flat.i32p)))
    assert rc == _lib.ERR_ARG and "pod_ns[0]" in msg and "out of range" in msg
    dec = np.array([0, 2, 1], np.int64)
    rc, msg = load(lambda c: (setattr(c, "n_pods", 2), setattr(c, "pod_label_off", dec.ctypes.data_as(flat.i64p))))
    assert rc == _lib.ERR_ARG and "decreases" in msg
    rc, msg = load(lambda c: setattr(c, "pod_ns", None))
    assert rc == _lib.ERR_ARG and "null pod_ns" in msg
    # counts kept as 32-bit values are refused at 2^32, not truncated
    rc, msg = load(lambda c: setattr(c, "n_pods", 1 << 32))
    assert rc == _lib.ERR_ARG and "n_pods" in msg and "2^32" in msg
    rc, msg = load(lambda c: setattr(c, "n_namespaces", 1 << 32))
    assert rc == _lib.ERR_ARG and "n_namespaces" in msg
    rc, msg = load(lambda c: setattr(c.str, "n", 1 << 32))
    assert rc == _lib.ERR_ARG and "str.n" in msg
    big = np.array([0, 1 << 32], np.int64)
    rc, msg = load(lambda c: setattr(c, "ns_label_off", big.ctypes.data_as(flat.i64p)))
    assert rc == _lib.ERR_ARG and "namespace labels" in msg
    # a nil map or slice holds nothing
    nil = np.array([1], np.uint8)
    rc, msg = load(lambda c: setattr(c, "pod_nil", nil.ctypes.data_as(flat.u8p)))
    assert rc == _lib.ERR_ARG and "nil Labels" in msg
    # a refused load leaves the earlier model in place
    e.load_resources(res)
    rc, _ = load(lambda c: setattr(c, "pod_ip", bad.ctypes.data_as(flat.i32p)))
    assert rc == _lib.ERR_ARG and e.resources_json()["Pods"][0]["IP"] == "10.0.0.1"
    # policy tables: a peer's port matcher out of range, duplicate primary keys
    ir = Engine(0).build_policies(random_problem(8100)[0]).policy_ir()
    t = flat.PolicyTables(ir)
    t.c.n_port_matchers = 0
    assert _lib.lib().cyc_policy_load(e._ctx, ctypes.byref(t.c)) == _lib.ERR_ARG
    one = {"Ingress": {"a": {"Namespace": "x", "PodSelector": {}, "Peers": None, "SourceRules": []},
                       "b": {"Namespace": "x", "PodSelector": {}, "Peers": None, "SourceRules": []}}, "Egress": {}}
    with pytest.raises(_lib.CyclonusError, match="primary key"):
        Engine(0).load_policy_tables(one)


def test_traffic_tables_follow_encoding_json():
    """The flat traffic tables read a matcher.Traffic dict as encoding/json (and the JSON entry point)
    would: field names case-insensitively with the last key winning, null pointers / maps as nil, and
    ResolvedPort stored as int32 (two's-complement wrap) like the JSON path."""
    a = [{"Source": {"Internal": {"PodLabels": {"a": "b"}, "Namespace": "x"}, "IP": "10.0.0.1"},
          "Destination": {"Internal": None, "IP": "1.2.3.4"}, "ResolvedPort": 80, "Protocol": "TCP"}]
    b = [{"source": {"internal": {"podlabels": {"a": "b"}, "NAMESPACE": "x"}, "ip": "10.0.0.1"},
          "DESTINATION": {"internal": {"Namespace": "y"}, "Internal": None, "Ip": "1.2.3.4"},
          "resolvedport": 80, "Protocol": "UDP", "protocol": "TCP"}]
    ta, tb = flat.TrafficTables(a), flat.TrafficTables(b)

    def rows(t):
        strs = np.ctypeslib.as_array(t.c.str.off, (t.c.str.n + 1,))
        blob = ctypes.string_at(t.c.str.bytes, int(strs[-1]))
        s = [blob[strs[i]:strs[i + 1]].decode() for i in range(t.c.str.n)]
        g = lambda p, n: list(np.ctypeslib.as_array(p, (n,)))  # noqa: E731
        return (g(t.c.internal, 2), [s[i] for i in g(t.c.ip, 2)], [s[i] for i in g(t.c.ns, 2)], g(t.c.label_off, 3),
                g(t.c.port, 1), [s[i] for i in g(t.c.protocol, 1)])

    assert rows(ta) == rows(tb)
    assert flat._go_int32(1 << 31) == -(1 << 31) and flat._go_int32(70000) == 70000 and flat._go_int32((1 << 32) + 80) == 80
