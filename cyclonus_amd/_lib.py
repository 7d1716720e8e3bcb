"""ctypes binding of libcyclonus_hip.so (include/cyclonus_hip.h).

The product path is the HIP library; there is no CPU fallback.  If the shared library is
missing or fails to load, every entry point raises instead of silently computing on the host.
"""
from __future__ import annotations

import ctypes
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
# CYC_HIP_LIB: another build of the same library (A/B timing of two builds in one GPU session)
SO_PATH = os.environ.get("CYC_HIP_LIB") or os.path.join(_PKG, "libcyclonus_hip.so")

# CYC_ABI_VERSION of the header these ctypes declarations mirror (include/cyclonus_hip.h)
ABI_VERSION = 2

# cyc_status
OK, ERR_ARG, ERR_JSON, ERR_INVALID_POLICY, ERR_PANIC_IP, ERR_PANIC_CIDR, ERR_PANIC_SELECTOR = 0, 1, 2, 3, 4, 5, 6
ERR_DUPLICATE_KEY, ERR_HIP, ERR_OOM, ERR_RCCL, ERR_PANIC_RUNTIME = 7, 8, 9, 10, 11
PANIC_CODES = (ERR_INVALID_POLICY, ERR_PANIC_IP, ERR_PANIC_CIDR, ERR_PANIC_SELECTOR, ERR_PANIC_RUNTIME)

# cyc_job_status
JOB_NONE, JOB_VALID, JOB_BAD_NAMED_PORT, JOB_BAD_PORT_PROTOCOL = 0, 1, 2, 3

# cyc_connectivity (probe.Connectivity in AllConnectivity order, connectivity.go:16-23)
CONN_UNKNOWN, CONN_CHECK_FAILED, CONN_INVALID_NAMED_PORT, CONN_INVALID_PORT_PROTOCOL, CONN_BLOCKED, CONN_ALLOWED = range(6)
CONN_NO_JOB = 255
CONNECTIVITY = ("unknown", "checkfailed", "invalidnamedport", "invalidportprotocol", "blocked", "allowed")

EXPORTS = [
    "cyc_ctx_create",
    "cyc_ctx_destroy",
    "cyc_last_error",
    "cyc_version",
    "cyc_abi_version",
    "cyc_policy_build_json",
    "cyc_policy_load_ir_json",
    "cyc_policy_ir_json",
    "cyc_resources_load_json",
    "cyc_probe_prepare",
    "cyc_probe_run",
    "cyc_probe_run_host",
    "cyc_last_timings",
    "cyc_last_classes",
    "cyc_last_emit",
    "cyc_set_option",
    "cyc_get_option",
    "cyc_query_traffic",
    "cyc_query_traffic_tables",
    "cyc_query_traffic_targets",
    "cyc_query_targets",
    "cyc_table_run",
    "cyc_table_wrap",
    "cyc_table_cells",
    "cyc_table_shape",
    "cyc_table_error",
    "cyc_table_destroy",
    "cyc_rows_layout",
    "cyc_probe_run_rows",
    "cyc_probe_run_host_rows",
    "cyc_table_run_rows",
    "cyc_table_wrap_rows",
    "cyc_comm_unique_id",
    "cyc_comm_init",
    "cyc_comm_destroy",
    "cyc_rows_shard",
    "cyc_planes_allgather",
    "cyc_table_allgather",
    "cyc_rows_merge_sources",
    "cyc_probe_prepare_blocks",
    "cyc_blocks_layout",
    "cyc_probe_run_blocks",
    "cyc_block_error",
    "cyc_resources_load",
    "cyc_policy_load",
    "cyc_probe_prepare_configs",
    "cyc_resources_json",
]

# flat tables (cyc_policy_tables): cyc_peer_kind, cyc_ns_kind, cyc_port_kind
PEER_ALL, PEER_PORTS, PEER_POD, PEER_IP = 0, 1, 2, 3
NS_EXACT, NS_ALL, NS_LABEL = 0, 1, 2
PORT_ANY, PORT_NUMBER, PORT_NAME = 0, 1, 2

# cyc_rows (row partitions for one-process-per-GPU runs)
ROWS_TARGET, ROWS_SOURCE = 0, 1
PARTITIONS = {"target": ROWS_TARGET, "source": ROWS_SOURCE}


class CyclonusError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[cyc_status {code}] {msg}")
        self.code = code
        self.msg = msg


class CyclonusPanic(CyclonusError):
    """The Go reference would panic (or log.Fatalf) on this input; msg is the panic text."""


class ProbeShape(ctypes.Structure):
    _fields_ = [
        (n, ctypes.c_int64)
        for n in ("pods", "slots", "words", "configs", "targets_in", "targets_eg", "peers", "classes_in", "classes_eg", "may_panic",
                  "selectors", "label_sets", "pod_peers", "ip_peers", "descriptors", "max_word_runs")
    ]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


_lib = None


def lib():
    """Load libcyclonus_hip.so (raises if it is missing: no fallback path exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(SO_PATH):
            raise ImportError(f"{SO_PATH} is missing: run `python -m cyclonus_amd.build` (hipcc, gfx950)")
        L = ctypes.CDLL(SO_PATH)
        vp, cp, sz, i, i64 = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int64
        L.cyc_ctx_create.argtypes = [i, ctypes.POINTER(vp)]
        L.cyc_ctx_destroy.argtypes = [vp]
        L.cyc_ctx_destroy.restype = None
        L.cyc_last_error.argtypes = [vp]
        L.cyc_last_error.restype = cp
        L.cyc_version.restype = cp
        L.cyc_abi_version.restype = i
        if L.cyc_abi_version() != ABI_VERSION:
            raise ImportError(f"{SO_PATH}: ABI {L.cyc_abi_version()}, these bindings expect ABI {ABI_VERSION} (rebuild)")
        L.cyc_policy_build_json.argtypes = [vp, i, cp, sz]
        L.cyc_policy_load_ir_json.argtypes = [vp, cp, sz]
        L.cyc_policy_ir_json.argtypes = [vp, cp, sz]
        L.cyc_policy_ir_json.restype = i64
        L.cyc_resources_load_json.argtypes = [vp, cp, sz]
        L.cyc_probe_prepare.argtypes = [vp, cp, sz, ctypes.POINTER(ProbeShape)]
        L.cyc_probe_run.argtypes = [vp, vp, vp, vp, vp, i64, i64]
        L.cyc_probe_run_host.argtypes = [vp, vp, vp, vp, i64, i64]
        L.cyc_last_timings.argtypes = [vp, ctypes.POINTER(ctypes.c_double), i]
        L.cyc_last_classes.argtypes = [vp, ctypes.POINTER(ctypes.c_int64), i]
        L.cyc_last_emit.argtypes = [vp, cp, sz, ctypes.POINTER(i64)]
        L.cyc_set_option.argtypes = [vp, cp, i64]
        L.cyc_get_option.argtypes = [vp, cp, ctypes.POINTER(i64)]
        L.cyc_query_traffic.argtypes = [vp, cp, sz, vp, i64]
        L.cyc_query_traffic_tables.argtypes = [vp, vp, vp, i64]
        L.cyc_query_traffic_targets.argtypes = [vp, cp, sz, vp, sz, ctypes.POINTER(sz)]
        L.cyc_query_targets.argtypes = [vp, cp, sz, vp, sz, ctypes.POINTER(sz)]
        L.cyc_table_run.argtypes = [vp, i64, i64, ctypes.POINTER(vp)]
        L.cyc_table_wrap.argtypes = [vp, vp, vp, vp, i64, i64, ctypes.POINTER(vp)]
        L.cyc_table_cells.argtypes = [vp, i64, i64, i64, i64, i64, i64, vp, vp, vp]
        L.cyc_table_shape.argtypes = [vp, ctypes.POINTER(i64), i]
        L.cyc_table_error.argtypes = [vp]
        L.cyc_table_error.restype = cp
        L.cyc_table_destroy.argtypes = [vp]
        L.cyc_table_destroy.restype = None
        L.cyc_rows_layout.argtypes = [vp, i, i64, i64, ctypes.POINTER(i64), i]
        L.cyc_probe_run_rows.argtypes = [vp, vp, vp, vp, vp, i, i64, i64]
        L.cyc_probe_run_host_rows.argtypes = [vp, vp, vp, vp, i, i64, i64]
        L.cyc_table_run_rows.argtypes = [vp, i, i64, i64, ctypes.POINTER(vp)]
        L.cyc_table_wrap_rows.argtypes = [vp, vp, vp, vp, i, i64, i64, ctypes.POINTER(vp)]
        L.cyc_comm_unique_id.argtypes = [vp]
        L.cyc_comm_init.argtypes = [vp, i, i, vp]
        L.cyc_comm_destroy.argtypes = [vp]
        L.cyc_rows_shard.argtypes = [vp, i, i, i, ctypes.POINTER(i64), ctypes.POINTER(i64)]
        L.cyc_planes_allgather.argtypes = [vp, vp, i, vp, vp, vp, vp]
        L.cyc_table_allgather.argtypes = [vp, vp, ctypes.POINTER(vp)]
        L.cyc_rows_merge_sources.argtypes = [vp, vp, i, vp, vp]
        L.cyc_probe_prepare_blocks.argtypes = [vp, cp, sz, vp, vp, i64, ctypes.POINTER(ProbeShape)]
        L.cyc_blocks_layout.argtypes = [vp, vp, i64]
        L.cyc_probe_run_blocks.argtypes = [vp, vp, vp, vp, vp, vp]
        L.cyc_block_error.argtypes = [vp, i64]
        L.cyc_block_error.restype = cp
        L.cyc_resources_load.argtypes = [vp, vp]
        L.cyc_policy_load.argtypes = [vp, vp]
        L.cyc_probe_prepare_configs.argtypes = [vp, vp, i64, ctypes.POINTER(ProbeShape)]
        L.cyc_resources_json.argtypes = [vp, cp, sz]
        L.cyc_resources_json.restype = i64
        _lib = L
    return _lib


def check(ctx, rc: int):
    if rc == OK:
        return
    msg = lib().cyc_last_error(ctx).decode(errors="replace")
    if rc in PANIC_CODES or rc == ERR_DUPLICATE_KEY:
        raise CyclonusPanic(rc, msg)
    raise CyclonusError(rc, msg)
