"""Engine: one libcyclonus_hip context on one GPU (thin wrapper over include/cyclonus_hip.h)."""
from __future__ import annotations

import ctypes
import json
from typing import Any, Optional

import numpy as np

from . import _lib
from ._lib import check, lib


def _bytes(doc: Any) -> bytes:
    if isinstance(doc, bytes):
        return doc
    if isinstance(doc, str):
        return doc.encode()
    return json.dumps(doc, separators=(",", ":")).encode()


class Engine:
    """A verdict-engine context bound to `device` (HIP device ordinal)."""

    def __init__(self, device: int = 0):
        self._ctx = ctypes.c_void_p()
        rc = lib().cyc_ctx_create(int(device), ctypes.byref(self._ctx))
        if rc != _lib.OK:
            raise _lib.CyclonusError(rc, f"cyc_ctx_create(device={device}) failed")
        self.device = device
        self.shape: Optional[dict] = None

    def close(self):
        if self._ctx:
            lib().cyc_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- inputs
    def build_policies(self, netpols, simplify: bool = True) -> "Engine":
        b = _bytes(netpols)
        check(self._ctx, lib().cyc_policy_build_json(self._ctx, int(bool(simplify)), b, len(b)))
        return self

    def load_policy_ir(self, policy_ir) -> "Engine":
        b = _bytes(policy_ir)
        check(self._ctx, lib().cyc_policy_load_ir_json(self._ctx, b, len(b)))
        return self

    def _dump(self, fn) -> dict:
        """A JSON dump entry point (bytes needed, or -(cyc_status) with cyc_last_error set)."""
        n = fn(self._ctx, None, 0)
        if n < 0:
            check(self._ctx, int(-n))
        buf = ctypes.create_string_buffer(int(n))
        m = fn(self._ctx, buf, int(n))
        if m < 0:
            check(self._ctx, int(-m))
        return json.loads(buf.value.decode())

    def policy_ir(self) -> dict:
        return self._dump(lib().cyc_policy_ir_json)

    def load_resources(self, resources) -> "Engine":
        b = _bytes(resources)
        check(self._ctx, lib().cyc_resources_load_json(self._ctx, b, len(b)))
        return self

    # ---------------------------------------------------------------- flat tables (no JSON)
    def load_resources_tables(self, tables) -> "Engine":
        """cyc_resources_load: a flat.ResourceTables (or a probe.Resources dict, flattened here)."""
        from . import flat

        t = tables if isinstance(tables, flat.ResourceTables) else flat.ResourceTables(tables)
        check(self._ctx, lib().cyc_resources_load(self._ctx, ctypes.byref(t.c)))
        return self

    def load_policy_tables(self, tables) -> "Engine":
        """cyc_policy_load: a flat.PolicyTables (or a json.Marshal(*matcher.Policy) dict, flattened here)."""
        from . import flat

        t = tables if isinstance(tables, flat.PolicyTables) else flat.PolicyTables(tables)
        check(self._ctx, lib().cyc_policy_load(self._ctx, ctypes.byref(t.c)))
        return self

    def prepare_configs(self, probes) -> dict:
        """cyc_probe_prepare_configs: the probe configs as cyc_probe_config structs."""
        from . import flat

        cfg = probes if isinstance(probes, flat.ProbeConfigs) else flat.ProbeConfigs(probes)
        sh = _lib.ProbeShape()
        check(self._ctx, lib().cyc_probe_prepare_configs(self._ctx, cfg.c, cfg.n, ctypes.byref(sh)))
        self.shape = sh.as_dict()
        return self.shape

    def resources_json(self) -> dict:
        """The loaded probe model (cyc_resources_json: json.Marshal(*probe.Resources) of the kept fields)."""
        return self._dump(lib().cyc_resources_json)

    def prepare(self, probes) -> dict:
        b = _bytes(probes)
        sh = _lib.ProbeShape()
        check(self._ctx, lib().cyc_probe_prepare(self._ctx, b, len(b), ctypes.byref(sh)))
        self.shape = sh.as_dict()
        return self.shape

    # ---------------------------------------------------------------- runs
    # partition: "target" (rows are the pods both planes are keyed by) or "source" (rows are source
    # pods: every cell (s in rows, d, k); include/cyclonus_hip.h, cyc_rows)
    def layout(self, row_lo: int = 0, row_hi: Optional[int] = None, partition: str = "target"):
        """(ingress rows, ingress words per slot, egress rows, egress words per slot, window start word)."""
        hi = self.shape["pods"] if row_hi is None else row_hi
        v = (ctypes.c_int64 * 5)()
        check(self._ctx, lib().cyc_rows_layout(self._ctx, _lib.PARTITIONS[partition], int(row_lo), int(hi), v, 5))
        return tuple(int(x) for x in v)

    def run_host(self, row_lo: int = 0, row_hi: Optional[int] = None, partition: str = "target"):
        """Run on the GPU and copy back: (status[P,K] u8, ingress[rows_in,K,Wi] u64, egress[rows_eg,K,W] u64).
        Target rows: both planes are [row_hi - row_lo, K, W].  Source rows: ingress is [P, K, Wi], the
        words [row_lo/64, row_lo/64 + Wi) of every destination's row."""
        P, K = self.shape["pods"], self.shape["slots"]
        hi = P if row_hi is None else row_hi
        ri, wi, re_, we, _ = self.layout(row_lo, hi, partition)
        ing = np.zeros((ri, K, wi), np.uint64)
        eg = np.zeros((re_, K, we), np.uint64)
        st = np.zeros((P, K), np.uint8)
        check(
            self._ctx,
            lib().cyc_probe_run_host_rows(self._ctx, ing.ctypes.data, eg.ctypes.data, st.ctypes.data,
                                          _lib.PARTITIONS[partition], int(row_lo), int(hi)),
        )
        return st, ing, eg

    def run_device(self, d_ingress: int, d_egress: int, d_status: int, stream: int = 0, row_lo: int = 0, row_hi=None,
                   partition: str = "target"):
        """Enqueue the pipeline on `stream` writing device pointers (e.g. torch .data_ptr())."""
        P = self.shape["pods"]
        hi = P if row_hi is None else row_hi
        check(
            self._ctx,
            lib().cyc_probe_run_rows(
                self._ctx, ctypes.c_void_p(stream or None), ctypes.c_void_p(d_ingress), ctypes.c_void_p(d_egress),
                ctypes.c_void_p(d_status or None), _lib.PARTITIONS[partition], int(row_lo), int(hi),
            ),
        )

    def table(self, row_lo: int = 0, row_hi: Optional[int] = None, partition: str = "target") -> "DeviceTable":
        """Run the probe into a device-resident table (cyc_table_run_rows) for rows [row_lo, row_hi)."""
        hi = self.shape["pods"] if row_hi is None else row_hi
        t = ctypes.c_void_p()
        check(self._ctx, lib().cyc_table_run_rows(self._ctx, _lib.PARTITIONS[partition], int(row_lo), int(hi), ctypes.byref(t)))
        return DeviceTable(t)

    def wrap_table(self, d_ingress: int, d_egress: int, d_status: int, row_lo: int = 0, row_hi=None,
                   partition: str = "target") -> "DeviceTable":
        """A table over planes produced by run_device (cyc_table_wrap_rows; the caller keeps them alive)."""
        hi = self.shape["pods"] if row_hi is None else row_hi
        t = ctypes.c_void_p()
        check(self._ctx, lib().cyc_table_wrap_rows(self._ctx, ctypes.c_void_p(d_ingress), ctypes.c_void_p(d_egress),
                                                   ctypes.c_void_p(d_status), _lib.PARTITIONS[partition], int(row_lo), int(hi),
                                                   ctypes.byref(t)))
        return DeviceTable(t)

    # ---------------------------------------------------------------- multi-GPU assembly (RCCL, comm.hpp)
    @staticmethod
    def comm_unique_id() -> bytes:
        """cyc_comm_unique_id: the 128-byte RCCL unique id rank 0 makes and hands to every rank."""
        buf = (ctypes.c_uint8 * 128)()
        rc = lib().cyc_comm_unique_id(buf)
        if rc != _lib.OK:
            raise _lib.CyclonusError(rc, "cyc_comm_unique_id failed")
        return bytes(buf)

    def comm_init(self, nranks: int, rank: int, uid: bytes):
        """cyc_comm_init: collective over the ranks; the context owns the communicator."""
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        check(self._ctx, lib().cyc_comm_init(self._ctx, int(nranks), int(rank), buf))
        return self

    def comm_destroy(self):
        check(self._ctx, lib().cyc_comm_destroy(self._ctx))

    def rows_shard(self, nranks: int, rank: int, partition: str = "source"):
        """cyc_rows_shard: rank's rows [lo, hi) of the library's partition of the prepared pods."""
        lo, hi = ctypes.c_int64(0), ctypes.c_int64(0)
        check(self._ctx, lib().cyc_rows_shard(self._ctx, _lib.PARTITIONS[partition], int(nranks), int(rank),
                                              ctypes.byref(lo), ctypes.byref(hi)))
        return int(lo.value), int(hi.value)

    def planes_allgather(self, d_ingress: int, d_egress: int, d_ingress_full: int, d_egress_full: int, stream: int = 0,
                         partition: str = "source"):
        """cyc_planes_allgather (collective): this rank's shard planes -> the whole [P][K][W] planes."""
        check(self._ctx, lib().cyc_planes_allgather(self._ctx, ctypes.c_void_p(stream or None), _lib.PARTITIONS[partition],
                                                    ctypes.c_void_p(d_ingress), ctypes.c_void_p(d_egress),
                                                    ctypes.c_void_p(d_ingress_full), ctypes.c_void_p(d_egress_full)))

    def table_allgather(self, shard: "DeviceTable") -> "DeviceTable":
        """cyc_table_allgather (collective): a whole device table from this rank's shard table."""
        t = ctypes.c_void_p()
        check(self._ctx, lib().cyc_table_allgather(self._ctx, shard._t, ctypes.byref(t)))
        return DeviceTable(t)

    def merge_sources(self, d_slices, d_ingress_full: int, stream: int = 0):
        """cyc_rows_merge_sources: every source shard's ingress slices (device pointers, rank order) ->
        the whole ingress plane, on one GPU."""
        arr = (ctypes.c_void_p * len(d_slices))(*[ctypes.c_void_p(p) for p in d_slices])
        check(self._ctx, lib().cyc_rows_merge_sources(self._ctx, ctypes.c_void_p(stream or None), len(d_slices), arr,
                                                      ctypes.c_void_p(d_ingress_full)))

    # ---------------------------------------------------------------- batched blocks
    def prepare_blocks(self, probes, block_end, block_config) -> dict:
        """Batched independent problems (cyc_probe_prepare_blocks): block b = pods
        [block_end[b-1], block_end[b]) answering probes[block_config[b]] over its own pods."""
        b = _bytes(probes)
        ends = np.ascontiguousarray(block_end, np.int64)
        cfgs = np.ascontiguousarray(block_config, np.int32)
        sh = _lib.ProbeShape()
        check(self._ctx, lib().cyc_probe_prepare_blocks(self._ctx, b, len(b), ends.ctypes.data, cfgs.ctypes.data, len(ends),
                                                        ctypes.byref(sh)))
        self.shape = sh.as_dict()
        self.n_blocks = len(ends)
        lay = np.zeros(2 * (self.n_blocks + 1), np.int64)
        check(self._ctx, lib().cyc_blocks_layout(self._ctx, lay.ctypes.data, len(lay)))
        self.block_layout = lay.reshape(-1, 2)  # per block (plane slab offset in words, status offset); then totals
        return self.shape

    def run_blocks_device(self, d_ingress: int, d_egress: int, d_status: int, stream: int = 0):
        """Every block's slab on the device (cyc_probe_run_blocks) -> per block (cyc_status, message)."""
        rc = np.zeros(self.n_blocks, np.int32)
        check(self._ctx, lib().cyc_probe_run_blocks(self._ctx, ctypes.c_void_p(stream or None), ctypes.c_void_p(d_ingress),
                                                    ctypes.c_void_p(d_egress), ctypes.c_void_p(d_status), rc.ctypes.data))
        return [(int(c), lib().cyc_block_error(self._ctx, b).decode(errors="replace") if c else "") for b, c in enumerate(rc)]

    def query_traffic(self, traffics):
        """Policy.IsTrafficAllowed on the GPU for a list of matcher.Traffic dicts -> [(ingress, egress)]."""
        b = _bytes(list(traffics))
        n = len(traffics)
        out = np.zeros(max(n, 1), np.uint8)
        check(self._ctx, lib().cyc_query_traffic(self._ctx, b, len(b), out.ctypes.data, n))
        return [(bool(o & 1), bool(o & 2)) for o in out[:n]]

    def query_traffic_tables(self, traffics):
        """query_traffic through the flat tables (cyc_query_traffic_tables: no JSON)."""
        from . import flat

        t = traffics if isinstance(traffics, flat.TrafficTables) else flat.TrafficTables(traffics)
        out = np.zeros(max(t.n, 1), np.uint8)
        check(self._ctx, lib().cyc_query_traffic_tables(self._ctx, ctypes.byref(t.c), out.ctypes.data, t.n))
        return [(bool(o & 1), bool(o & 2)) for o in out[:t.n]]

    def _json_out(self, fn, doc):
        b = _bytes(doc)
        need = ctypes.c_size_t(0)
        cap = 1 << 16
        while True:
            buf = ctypes.create_string_buffer(cap)
            rc = fn(self._ctx, b, len(b), buf, cap, ctypes.byref(need))
            if rc == _lib.ERR_ARG and need.value > cap:
                cap = need.value
                continue
            check(self._ctx, rc)
            return json.loads(buf.value.decode())

    def query_traffic_targets(self, traffics):
        """IsTrafficAllowed with the DirectionResult lists: per traffic
        {"Ingress": {"AllowingTargets": [pk..], "DenyingTargets": [pk..], "IsAllowed": b}, "Egress": .., "IsAllowed": b}."""
        return self._json_out(lib().cyc_query_traffic_targets, list(traffics))

    def query_targets(self, pods):
        """TargetsApplyingToPod per direction for QueryTargetPod dicts {Namespace, Labels}."""
        return self._json_out(lib().cyc_query_targets, list(pods))

    def classes(self):
        """(ingress, egress) number of distinct classes of the last run."""
        out = (ctypes.c_int64 * 2)()
        check(self._ctx, lib().cyc_last_classes(self._ctx, out, 2))
        return int(out[0]), int(out[1])

    def last_emit(self):
        """(kernel name(s), launch count) of the last run's emit, as the library launched it."""
        buf = ctypes.create_string_buffer(256)
        n = ctypes.c_int64(0)
        check(self._ctx, lib().cyc_last_emit(self._ctx, buf, 256, ctypes.byref(n)))
        return buf.value.decode(), int(n.value)

    def set_option(self, name: str, value: int):
        check(self._ctx, lib().cyc_set_option(self._ctx, name.encode(), int(value)))

    def get_option(self, name: str) -> int:
        v = ctypes.c_int64(0)
        check(self._ctx, lib().cyc_get_option(self._ctx, name.encode(), ctypes.byref(v)))
        return int(v.value)

    def timings(self):
        """(pipeline_ms, emit_ms, class_rows_ms) of the last run, from HIP events on its stream."""
        ms = (ctypes.c_double * 3)()
        check(self._ctx, lib().cyc_last_timings(self._ctx, ms, 3))
        return tuple(ms)


class DeviceTable:
    """A cyc_table: verdict planes resident on the GPU; cells() returns probe.Connectivity codes."""

    def __init__(self, handle: ctypes.c_void_p):
        self._t = handle
        v = (ctypes.c_int64 * 8)()
        lib().cyc_table_shape(self._t, v, 8)
        self.pods, self.slots, self.words, self.row_lo, self.row_hi = (int(x) for x in v[:5])
        self.partition = "source" if v[5] == _lib.ROWS_SOURCE else "target"
        self.window = (int(v[6]), int(v[7]))  # ingress words [first, first + count) of a source-row table

    def close(self):
        if self._t:
            lib().cyc_table_destroy(self._t)
            self._t = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def cells(self, s_lo, s_hi, d_lo, d_hi, k_lo=0, k_hi=None, want=("ingress", "egress", "combined")):
        """{name: u8 array [s, d, k]} of cyc_connectivity codes for the requested block."""
        k_hi = self.slots if k_hi is None else k_hi
        shp = (max(s_hi - s_lo, 0), max(d_hi - d_lo, 0), max(k_hi - k_lo, 0))
        out = {n: np.zeros(shp, np.uint8) for n in want}
        ptr = [out[n].ctypes.data if n in out else None for n in ("ingress", "egress", "combined")]
        rc = lib().cyc_table_cells(self._t, int(s_lo), int(s_hi), int(d_lo), int(d_hi), int(k_lo), int(k_hi), *ptr)
        if rc != _lib.OK:
            raise _lib.CyclonusError(rc, lib().cyc_table_error(self._t).decode(errors="replace"))
        return out
