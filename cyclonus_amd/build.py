"""Build recipe for libcyclonus_hip.so (gfx950 only), in-tree so it travels to the GPU box.

    python -m cyclonus_amd.build        # or __graft_entry__.build()

host.cpp (policy compiler, probe model, table flattening) is compiled with g++; engine.hip
(kernels + C ABI, with its stage headers dev_*.hpp / ctx / plan / enqueue.hpp as one translation
unit) with hipcc --offload-arch=gfx950; both are linked by hipcc into one shared
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
# engine.hip's stage headers (one translation unit) and the host headers
HEADERS = ["cjson.hpp", "host.hpp", "tables.h", "dev_select.hpp", "dev_peer_rows.hpp", "dev_slots.hpp", "dev_member.hpp",
           "dev_class_rows.hpp", "dev_front.hpp", "dev_emit.hpp", "dev_query.hpp", "dev_gather.hpp", "ctx.hpp", "plan.hpp",
           "enqueue.hpp", "comm.hpp"]
LIBS = ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]  # RCCL: the table assembly's all-gathers (comm.hpp)


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


DRIVER_SRC = os.path.join(ROOT, "tests", "native", "capi_driver.cpp")
DRIVER = os.path.join(ROOT, "tests", "native", "capi_driver")
ASAN_DIR = os.path.join(BUILD, "asan")
ASAN_LIB = os.path.join(ASAN_DIR, "libcyclonus_hip.so")
SAN = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"]


def build_driver(force: bool = False) -> str:
    """The C++ C-ABI driver (tests/native/capi_driver.cpp), linked against the in-tree library."""
    if force or _newer(DRIVER, [DRIVER_SRC, OUT, os.path.join(INCLUDE, "cyclonus_hip.h")]):
        _run(["g++", "-O2", "-std=c++17", "-I", INCLUDE, DRIVER_SRC, "-o", DRIVER, "-L", PKG, "-lcyclonus_hip",
              f"-Wl,-rpath,{PKG}"])
    return DRIVER


def asan_runtime() -> str:
    """clang's ASan runtime (LD_PRELOAD it to load the sanitized library into an unsanitized python)."""
    import glob

    hits = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    if not hits:
        raise FileNotFoundError("libclang_rt.asan-x86_64.so not found under /opt/rocm/lib/llvm")
    return hits[-1]


def build_asan(force: bool = False) -> str:
    """ASan + UBSan build of the host side (host.cpp, cjson.hpp, the C ABI in engine.hip) for CPU
    tests in this container: CYC_HIP_LIB=<this> LD_PRELOAD=asan_runtime() python -m pytest ...
    The sanitizers apply to host code only (-Xarch_host); device code is compiled as usual."""
    os.makedirs(ASAN_DIR, exist_ok=True)
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(INCLUDE, "cyclonus_hip.h")]
    common = ["-O1", "-g", "-std=c++17", "-fPIC", "-I", CSRC, "-I", INCLUDE]
    host_san = [f for x in SAN for f in ("-Xarch_host", x)]
    objs = []
    for s in SOURCES_CPP:
        src, obj = os.path.join(CSRC, s), os.path.join(ASAN_DIR, s + ".o")
        if force or _newer(obj, [src] + hdrs):
            _run([HIPCC, "-x", "c++", *common, *SAN, "-c", src, "-o", obj])
        objs.append(obj)
    for s in SOURCES_HIP:
        src, obj = os.path.join(CSRC, s), os.path.join(ASAN_DIR, s + ".o")
        if force or _newer(obj, [src] + hdrs):
            _run([HIPCC, f"--offload-arch={ARCH}", *common, *host_san, "-munsafe-fp-atomics", "-c", src, "-o", obj])
        objs.append(obj)
    if force or _newer(ASAN_LIB, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *host_san, "-shared-libsan", "-o", ASAN_LIB, *objs, *LIBS])
    return ASAN_LIB


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
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT, *objs, *LIBS])
    write_build_info()
    build_driver(force)
    return OUT


BUILD_INFO = os.path.join(BUILD, "build_info.json")


def lib_sha256(path: str = OUT) -> str:
    import hashlib

    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def write_build_info():
    """Provenance of the built library (travels to the GPU box with it): the git head it was built
    from (and whether the tree differed from it) and the library's sha256.  Profiles record it, and
    bench.py quotes a profile's counters only for the same library."""
    import json

    info = {"lib_sha256": lib_sha256(OUT)}
    try:
        info["git_head"] = subprocess.run(["git", "-C", ROOT, "rev-parse", "HEAD"], capture_output=True, text=True,
                                          check=True).stdout.strip()
        info["git_dirty"] = bool(subprocess.run(["git", "-C", ROOT, "status", "--porcelain", "--untracked-files=no"],
                                                capture_output=True, text=True, check=True).stdout.strip())
    except Exception:  # no git (e.g. on the GPU box): keep what the build host wrote
        if os.path.exists(BUILD_INFO):
            old = json.load(open(BUILD_INFO))
            if old.get("lib_sha256") == info["lib_sha256"]:
                return
    with open(BUILD_INFO, "w") as f:
        json.dump(info, f)


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    if "--asan" in sys.argv:
        build_asan(force="--force" in sys.argv)
