"""The C ABI library loads on a GPU-less host and exports every symbol include/cyclonus_hip.h declares."""
import ctypes
import os
import re

from cyclonus_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "cyclonus_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cyc_[a-z_]+)\s*\(", src)))


def test_exports_match_header():
    L = ctypes.CDLL(_lib.SO_PATH)
    syms = header_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(_lib.EXPORTS) == syms


def test_no_gpu_paths_fail_cleanly():
    from cyclonus_amd.engine import Engine

    e = Engine(0)
    assert _lib.lib().cyc_version().startswith(b"cyclonus_hip")
    e.build_policies([]).load_resources({"Namespaces": {}, "Pods": []})
    # without a loaded probe the run must refuse, not crash
    rc = _lib.lib().cyc_probe_run(e._ctx, None, None, None, None, 0, 0)
    assert rc == _lib.ERR_ARG
    assert b"prepare" in _lib.lib().cyc_last_error(e._ctx)


def test_json_depth_limit_and_last_key_wins():
    """encoding/json semantics at the boundary: documents nested deeper than 10000 are refused
    (not a stack overflow), and among keys that name one struct field the last one wins."""
    from cyclonus_amd.engine import Engine

    e = Engine(0)
    deep = b"[" * 20000 + b"]" * 20000
    rc = _lib.lib().cyc_policy_build_json(e._ctx, 1, deep, len(deep))
    assert rc == _lib.ERR_JSON and b"max depth" in _lib.lib().cyc_last_error(e._ctx)
    ok = b"[" * 9000 + b"]" * 9000  # within the limit: parses (an empty policy list nested)
    assert _lib.lib().cyc_resources_load_json(e._ctx, ok, len(ok)) in (_lib.OK, _lib.ERR_JSON)
    pol = [{"metadata": {"name": "p", "namespace": "a", "Namespace": "b"},
            "spec": {"podSelector": {}, "policyTypes": ["Ingress"]}}]
    ir = e.build_policies(pol).policy_ir()
    ns = [t["Namespace"] for t in ir["Ingress"].values()]
    assert ns == ["b"], ir
    # a JSON null leaves a scalar (or struct-valued) field unchanged: the last non-null key decides
    # ({"namespace":"a","Namespace":null} is "a"); into a pointer / slice field null means nil
    pol = [{"metadata": {"name": "p", "namespace": "a", "Namespace": None},
            "spec": {"podSelector": {"matchLabels": {"x": "1"}}, "policyTypes": ["Ingress"], "PodSelector": None,
                     "ingress": [{"from": [{"ipBlock": {"cidr": "10.0.0.0/8", "CIDR": None}}]}]}}]
    ir = e.build_policies(pol).policy_ir()
    (t,) = ir["Ingress"].values()
    assert t["Namespace"] == "a" and t["PodSelector"]["matchLabels"] == {"x": "1"}, ir
    assert t["Peers"][0]["CIDR"] == "10.0.0.0/8", ir
    pol[0]["spec"]["ingress"][0]["From"] = None  # []NetworkPolicyPeer: null = nil, i.e. all peers
    t2 = list(e.build_policies(pol).policy_ir()["Ingress"].values())[0]
    assert t2["Peers"] != t["Peers"], (t, t2)


def test_malformed_inputs_fail_cleanly():
    """Random truncations / byte flips of valid documents: every entry point returns a status (the
    sanitizer run of this file, tests/test_sanitized.py, checks there is no memory error either)."""
    import json
    import random

    from cyclonus_amd.engine import Engine

    c = json.load(open(os.path.join(ROOT, "tests", "golden", "config1.json")))
    docs = [json.dumps(c["policies"]).encode(), json.dumps(c["resources"]).encode()]
    e = Engine(0)
    L = _lib.lib()
    rng = random.Random(5)
    for i in range(400):
        d = bytearray(docs[i % 2])
        op = rng.randrange(3)
        if op == 0:
            d = d[: rng.randrange(len(d))]
        elif op == 1:
            for _ in range(rng.randrange(1, 6)):
                d[rng.randrange(len(d))] = rng.choice(b'{}[]",:\\0aZ-9 \x00\xff')
        else:
            x = rng.randrange(len(d))
            d = d[:x] + d[x: x + rng.randrange(1, 40)] * rng.randrange(2, 5) + d[x:]
        b = bytes(d)
        for fn in (L.cyc_policy_build_json, L.cyc_policy_load_ir_json, L.cyc_resources_load_json):
            rc = fn(e._ctx, 1, b, len(b)) if fn is L.cyc_policy_build_json else fn(e._ctx, b, len(b))
            assert rc in (_lib.OK, _lib.ERR_JSON, _lib.ERR_INVALID_POLICY, _lib.ERR_ARG), (i, rc)


def _driver_inputs(tmp_path, pols, res, probes):
    import json

    paths = []
    for name, doc in (("pols", pols), ("res", res), ("probes", probes)):
        p = tmp_path / f"{name}.json"
        p.write_text(json.dumps(doc))
        paths.append(str(p))
    return paths


def test_cpp_driver_compile_path(tmp_path):
    """The C++ client of the C ABI (stand-in for the cgo binding) compiles a policy and exports the
    same json.Marshal(*Policy) as the Python binding; a panicking build reports the Go panic text."""
    import json
    import subprocess

    from cyclonus_amd import build
    from cyclonus_amd.engine import Engine

    drv = build.build_driver()
    c = json.load(open(os.path.join(ROOT, "tests", "golden", "config1.json")))
    args = _driver_inputs(tmp_path, c["policies"], c["resources"], c["probes"])
    r = subprocess.run([drv, *args, "--no-gpu"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    ir = json.loads(r.stdout.split("ir ", 1)[1])
    assert ir == Engine(0).build_policies(c["policies"]).policy_ir()
    bad = [{"metadata": {"name": "p", "namespace": "x"},
            "spec": {"podSelector": {}, "policyTypes": ["Ingress"], "ingress": [{"ports": [{"port": "x", "endPort": 9}]}]}}]
    args = _driver_inputs(tmp_path, bad, c["resources"], c["probes"])
    r = subprocess.run([drv, *args, "--no-gpu"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 3 and r.stdout.startswith("error cyc_policy_build_json rc=3"), r.stdout


def _flat_inputs(tmp_path, tag, pols, res, probes):
    from cyclonus_amd import flat
    from cyclonus_amd.engine import Engine

    ir = Engine(0).build_policies(pols).policy_ir()
    paths = [str(tmp_path / f"{tag}.{x}") for x in ("pol.tab", "res.tab", "probes.txt")]
    flat.dump_tables(flat.PolicyTables(ir), paths[0])
    flat.dump_tables(flat.ResourceTables(res), paths[1])
    flat.dump_probe_configs(probes, paths[2])
    return ir, paths


def test_cpp_driver_flat_tables(tmp_path):
    """The C++ client through the flat-table entry points (cyc_policy_load, cyc_resources_load — what a
    cgo binding passes from its Go values): the loaded policy and probe model export the same
    json.Marshal forms as the JSON path; a table with an out-of-range index is refused with the
    reference-free CYC_ERR_ARG message, not a crash."""
    import json
    import subprocess

    from cyclonus_amd import build, flat
    from cyclonus_amd.engine import Engine
    from tests.randgen import random_problem

    drv = build.build_driver()
    cases = [json.load(open(os.path.join(ROOT, "tests", "golden", "config1.json")))]
    cases = [(c["policies"], c["resources"], c["probes"]) for c in cases] + [random_problem(s) for s in (11, 12, 13)]
    for n, (pols, res, probes) in enumerate(cases):
        ir, paths = _flat_inputs(tmp_path, str(n), pols, res, probes)
        r = subprocess.run([drv, "--flat", *paths, "--no-gpu"], capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        lines = dict(line.split(" ", 1) for line in r.stdout.splitlines())
        assert json.loads(lines["ir"]) == ir, n
        assert json.loads(lines["resources"]) == Engine(0).load_resources(res).resources_json(), n
    # a pod whose namespace index is past the string table
    rt = flat.ResourceTables(cases[0][1])
    rt.c.pod_ns[0] = 99
    flat.dump_tables(rt, paths[1])
    r = subprocess.run([drv, "--flat", *paths, "--no-gpu"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 3 and r.stdout.startswith("error cyc_resources_load rc=%d" % _lib.ERR_ARG), r.stdout
    assert "pod_ns[0] = 99 out of range" in r.stdout, r.stdout


def test_comm_entry_points_validate_arguments():
    """The RCCL assembly entry points refuse bad arguments and calls out of order without touching a
    GPU (the collectives themselves run in tests/test_gpu_assemble.py)."""
    import ctypes

    from cyclonus_amd.engine import Engine

    L = _lib.lib()
    e = Engine(0)
    uid = (ctypes.c_uint8 * 128)()
    assert L.cyc_comm_unique_id(None) == _lib.ERR_ARG
    assert L.cyc_comm_init(None, 1, 0, uid) == _lib.ERR_ARG
    assert L.cyc_comm_init(e._ctx, 1, 0, None) == _lib.ERR_ARG
    assert L.cyc_comm_init(e._ctx, 0, 0, uid) == _lib.ERR_ARG
    assert L.cyc_comm_init(e._ctx, 65, 0, uid) == _lib.ERR_ARG
    assert L.cyc_comm_init(e._ctx, 2, 2, uid) == _lib.ERR_ARG
    assert L.cyc_comm_init(e._ctx, 2, -1, uid) == _lib.ERR_ARG
    lo, hi = ctypes.c_int64(), ctypes.c_int64()
    assert L.cyc_rows_shard(e._ctx, 1, 2, 0, ctypes.byref(lo), ctypes.byref(hi)) == _lib.ERR_ARG
    assert b"prepare" in L.cyc_last_error(e._ctx)
    p = ctypes.c_void_p(16)
    rc = L.cyc_planes_allgather(e._ctx, None, 1, p, p, p, p)
    assert rc == _lib.ERR_ARG and b"cyc_comm_init first" in L.cyc_last_error(e._ctx)
    out = ctypes.c_void_p()
    assert L.cyc_table_allgather(e._ctx, None, ctypes.byref(out)) == _lib.ERR_ARG
    assert L.cyc_rows_merge_sources(e._ctx, None, 2, None, p) == _lib.ERR_ARG
    assert L.cyc_comm_destroy(e._ctx) == _lib.OK  # no communicator: nothing to do
    assert L.cyc_abi_version() == _lib.ABI_VERSION
