"""ctypes wrapper for the CPU oracle (oracle/oracle.cpp) — TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may import this
module, and only as the checker / the timed CPU baseline.  The product package
(``cyclonus_amd``) never imports it.

The oracle is a per-cell restatement of the reference's ``Policy.IsTrafficAllowed`` walk
(pkg/matcher/policy.go:131-174) plus ``BuildNetworkPolicies`` (builder.go:11-26) and the probe
job expansion (pkg/connectivity/probe/resources.go:274-364).  Parity pins: see oracle.cpp header.
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

ST_NONE, ST_VALID, ST_BAD_NAMED_PORT, ST_BAD_PORT_PROTOCOL = 0, 1, 2, 3


def build() -> str:
    """Compile the oracle with its Makefile (g++ only; no reference sources involved)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO) or os.path.getmtime(_SO) < max(
            os.path.getmtime(os.path.join(_HERE, f)) for f in ("oracle.cpp", "ojson.hpp", "gonet.hpp", "goslice.hpp")
        ):
            build()
        L = ctypes.CDLL(_SO)
        c, vp, i, sz = ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        L.orc_new.restype = vp
        L.orc_new.argtypes = [c, i, c, c, sz]
        L.orc_free.argtypes = [vp]
        L.orc_policy_json.restype = i
        L.orc_policy_json.argtypes = [vp, c, sz]
        L.orc_probe_shape.argtypes = [vp, c, ctypes.POINTER(i), ctypes.POINTER(i), c, sz]
        L.orc_probe_run.argtypes = [vp, c, vp, vp, vp, ctypes.POINTER(ctypes.c_longlong), c, sz]
        L.orc_probe_cells.argtypes = [vp, c, vp, vp, vp, i, vp, c, sz]
        L.orc_probe_cells_mt.argtypes = [vp, c, vp, vp, vp, i, vp, i, c, sz]
        L.orc_probe_row.argtypes = [vp, c, i, i, i, vp, i, c, sz]
        L.orc_query_traffic.argtypes = [vp, c, vp, i, c, sz]
        L.orc_query_traffic_targets.argtypes = [vp, c, c, sz, c, sz]
        L.orc_query_targets.argtypes = [vp, c, c, sz, c, sz]
        L.orc_ip_in_cidr.argtypes = [c, c]
        L.orc_ipblock_match.argtypes = [c, c, ctypes.POINTER(c), i]
        L.orc_selector_match.argtypes = [c, c]
        L.orc_make_ipv4_cidr.argtypes = [c, i, c, sz]
        _lib = L
    return _lib


class OraclePanic(RuntimeError):
    """The reference would panic (Go ``panic``) on this input."""

    def __init__(self, msg, cell=None):
        super().__init__(msg)
        self.cell = cell


def _j(x) -> bytes:
    return (x if isinstance(x, str) else json.dumps(x)).encode()


class Oracle:
    """Per-cell CPU restatement handle: policies (k8s NetworkPolicy JSON list) + Resources."""

    def __init__(self, policies, resources=None, simplify: bool = True):
        L = lib()
        err = ctypes.create_string_buffer(4096)
        self._h = L.orc_new(_j(policies), int(simplify), _j(resources) if resources is not None else b"", err, 4096)
        if not self._h:
            raise OraclePanic(err.value.decode())

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_free(self._h)
            self._h = None

    def policy_json(self) -> dict:
        L = lib()
        n = L.orc_policy_json(self._h, None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        L.orc_policy_json(self._h, buf, n + 1)
        return json.loads(buf.value.decode())

    def shape(self, probes):
        P, K = ctypes.c_int(), ctypes.c_int()
        err = ctypes.create_string_buffer(4096)
        if lib().orc_probe_shape(self._h, _j(probes), ctypes.byref(P), ctypes.byref(K), err, 4096) != 0:
            raise ValueError(err.value.decode())
        return P.value, K.value

    def probe(self, probes):
        """Full truth table: (status[P,K] u8, in_plane[P,K,W] u64, eg_plane[P,K,W] u64)."""
        P, K = self.shape(probes)
        W = (P + 63) // 64
        status = np.zeros((P, K), np.uint8)
        inp = np.zeros((P, K, W), np.uint64)
        egp = np.zeros((P, K, W), np.uint64)
        cell = ctypes.c_longlong(-1)
        err = ctypes.create_string_buffer(4096)
        rc = lib().orc_probe_run(
            self._h, _j(probes), status.ctypes.data, inp.ctypes.data, egp.ctypes.data, ctypes.byref(cell), err, 4096
        )
        if rc == 1:
            raise OraclePanic(err.value.decode(), cell.value)
        if rc != 0:
            raise ValueError(err.value.decode())
        return status, inp, egp

    def cells(self, probes, s, d, k, threads=1):
        """Sampled cells -> u8 array: status | ingress<<4 | egress<<5 | panic<<6.
        threads > 1 splits the cells over std::threads (read-only walk over the shared policy)."""
        s = np.ascontiguousarray(s, np.int32)
        d = np.ascontiguousarray(d, np.int32)
        k = np.ascontiguousarray(k, np.int32)
        out = np.zeros(len(s), np.uint8)
        err = ctypes.create_string_buffer(4096)
        rc = lib().orc_probe_cells_mt(self._h, _j(probes), s.ctypes.data, d.ctypes.data, k.ctypes.data, len(s),
                                      out.ctypes.data, int(threads), err, 4096)
        if rc != 0:
            raise ValueError(err.value.decode())
        return out

    def row(self, probes, direction: str, pod: int, k: int, threads: int = 1):
        """One plane row as u64[W]: "ingress" = row of destination `pod` (bits over sources),
        "egress" = row of source `pod` (bits over destinations), job slot k."""
        P, _ = self.shape(probes)
        out = np.zeros((P + 63) // 64, np.uint64)
        err = ctypes.create_string_buffer(4096)
        rc = lib().orc_probe_row(self._h, _j(probes), 0 if direction == "ingress" else 1, int(pod), int(k),
                                 out.ctypes.data, int(threads), err, 4096)
        if rc == 1:
            raise OraclePanic(err.value.decode())
        if rc != 0:
            raise ValueError(err.value.decode())
        return out

    def _json_call(self, fn, doc):
        err = ctypes.create_string_buffer(4096)
        cap = 1 << 16
        while True:
            buf = ctypes.create_string_buffer(cap)
            rc = fn(self._h, _j(doc), buf, cap, err, 4096)
            if rc == 1:
                raise OraclePanic(err.value.decode())
            if rc < 0 and err.value.startswith(b"buffer too small"):
                cap = int(err.value.split()[-1])
                continue
            if rc < 0:
                raise ValueError(err.value.decode())
            return json.loads(buf.value.decode())

    def query_traffic_targets(self, traffics):
        """AllowedResult with target lists per traffic (pk order); raises OraclePanic."""
        return self._json_call(lib().orc_query_traffic_targets, traffics)

    def query_targets(self, pods):
        """TargetsApplyingToPod per direction for QueryTargetPod dicts; raises OraclePanic."""
        return self._json_call(lib().orc_query_targets, pods)

    def query_traffic(self, traffics):
        """List of matcher.Traffic JSON objects -> list of (ingress, egress) or OraclePanic."""
        out = np.zeros(len(traffics), np.uint8)
        err = ctypes.create_string_buffer(4096)
        n = lib().orc_query_traffic(self._h, _j(traffics), out.ctypes.data, len(traffics), err, 4096)
        if n < 0:
            raise ValueError(err.value.decode())
        res = []
        for o in out[:n]:
            if o & 4:
                res.append(OraclePanic(err.value.decode()))
            else:
                res.append((bool(o & 1), bool(o & 2)))
        return res


def ip_in_cidr(ip: str, cidr: str):
    r = lib().orc_ip_in_cidr(ip.encode(), cidr.encode())
    return None if r < 0 else bool(r)


def ipblock_match(ip: str, cidr: str, excepts=()):
    arr = (ctypes.c_char_p * max(1, len(excepts)))(*[e.encode() for e in excepts])
    r = lib().orc_ipblock_match(ip.encode(), cidr.encode(), arr, len(excepts))
    return None if r < 0 else bool(r)


def selector_match(labels, selector):
    r = lib().orc_selector_match(_j(labels), _j(selector))
    if r == -1:
        raise OraclePanic("invalid operator")
    if r < 0:
        raise ValueError("bad json")
    return bool(r)


def make_ipv4_cidr(ip: str, bits: int) -> str:
    buf = ctypes.create_string_buffer(64)
    lib().orc_make_ipv4_cidr(ip.encode(), bits, buf, 64)
    return buf.value.decode()


def combined_table(status, inp, egp):
    """Dense [s, d, k] array of Connectivity short strings from packed planes (oracle helper)."""
    P, K, W = inp.shape
    inb = np.unpackbits(inp.view(np.uint8).reshape(P, K, W * 8), axis=2, bitorder="little")[:, :, :P]  # [d,k,s]
    egb = np.unpackbits(egp.view(np.uint8).reshape(P, K, W * 8), axis=2, bitorder="little")[:, :, :P]  # [s,k,d]
    ing = inb.transpose(2, 0, 1)  # [s,d,k]
    eg = egb.transpose(0, 2, 1)  # [s,d,k]
    return ing, eg
