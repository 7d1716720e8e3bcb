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
