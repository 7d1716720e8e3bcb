"""Build an A/B variant of libcyclonus_hip.so with extra -D flags (dev helper):
    python scripts/build_variant.py NAME -DMACRO=1          -> cyclonus_amd/_build/var_NAME/libcyclonus_hip.so
    python scripts/build_variant.py NAME --rev HEAD           -> engine.hip (and its headers) of a git revision
    python scripts/build_variant.py NAME --src FILE           -> a patched copy of engine.hip (diagnostics)
Run it with CYC_HIP_LIB=<that path> (cyclonus_amd/_lib.py)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cyclonus_amd import build as b  # noqa: E402

name, defs = sys.argv[1], sys.argv[2:]
out = os.path.join(b.BUILD, f"var_{name}")
os.makedirs(out, exist_ok=True)
src = os.path.join(b.CSRC, "engine.hip")
if "--rev" in defs:
    rev = defs[defs.index("--rev") + 1]
    defs = [d for d in defs if d not in ("--rev", rev)]
    # the revision's whole csrc/ (engine.hip includes its stage headers from its own directory)
    rdir = os.path.join(out, "csrc_rev")
    os.makedirs(rdir, exist_ok=True)
    tar = subprocess.run(["git", "-C", ROOT, "archive", rev, "cyclonus_amd/csrc"], check=True, capture_output=True).stdout
    subprocess.run(["tar", "-x", "-C", rdir, "--strip-components=2"], input=tar, check=True)
    src = os.path.join(rdir, "engine.hip")
if "--src" in defs:
    src = os.path.abspath(defs[defs.index("--src") + 1])
    defs = [d for d in defs if d not in ("--src", src) and os.path.abspath(d) != src]
common = ["-O3", "-std=c++17", "-fPIC", "-I", b.CSRC, "-I", b.INCLUDE, *defs]
host = os.path.join(b.BUILD, "host.cpp.o")
eng = os.path.join(out, "engine.hip.o")
subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", *common, "-munsafe-fp-atomics", "-c", src, "-o", eng], check=True)
subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", os.path.join(out, "libcyclonus_hip.so"), host, eng, *b.LIBS], check=True)
print(os.path.join(out, "libcyclonus_hip.so"))
