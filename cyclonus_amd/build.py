"""Build recipe for libcyclonus_hip.so (gfx950 only), in-tree so it travels to the GPU box.

    python -m cyclonus_amd.build        # or __graft_entry__.build()

host.cpp (policy compiler, probe model, table flattening) is compiled with g++; engine.hip
(kernels + C ABI) with hipcc --offload-arch=gfx950; both are linked by hipcc into one shared
library with plain C entry points declared in include/cyclonus_hip.h.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
OUT = os.path.join(PKG, "libcyclonus_hip.so")
BUILD = os.path.join(PKG, "_build")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

SOURCES_CPP = ["host.cpp"]
SOURCES_HIP = ["engine.hip"]
HEADERS = ["cjson.hpp", "host.hpp", "tables.h"]


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def build(verbose: bool = True, force: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(INCLUDE, "cyclonus_hip.h")]
    objs = []
    common = ["-O3", "-std=c++17", "-fPIC", "-I", CSRC, "-I", INCLUDE, "-Wall", "-Wno-unused-parameter"]
    for s in SOURCES_CPP:
        src = os.path.join(CSRC, s)
        obj = os.path.join(BUILD, s + ".o")
        if force or _newer(obj, [src] + hdrs):
            _run(["g++", *common, "-c", src, "-o", obj])
        objs.append(obj)
    for s in SOURCES_HIP:
        src = os.path.join(CSRC, s)
        obj = os.path.join(BUILD, s + ".o")
        if force or _newer(obj, [src] + hdrs):
            _run([HIPCC, f"--offload-arch={ARCH}", *common, "-munsafe-fp-atomics", "-c", src, "-o", obj])
        objs.append(obj)
    if force or _newer(OUT, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT, *objs])
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
