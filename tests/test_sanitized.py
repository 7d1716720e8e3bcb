"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only): the policy compiler,
JSON reader, flat-table loaders and C ABI entry points of libcyclonus_hip (cyclonus_amd.build.build_asan) run the
compiler / C-ABI test files in a child process with the sanitized library preloaded."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_compiler_and_capi_under_asan_ubsan():
    sys.path.insert(0, ROOT)
    from cyclonus_amd import build

    lib = build.build_asan()
    env = dict(os.environ, CYC_HIP_LIB=lib, LD_PRELOAD=build.asan_runtime(),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               CYC_SANITIZED_CHILD="1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        "tests/test_compiler.py", "tests/test_capi.py", "tests/test_flat.py",
                        "tests/test_sanitized.py::test_child_loaded_sanitized_lib"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "passed" in r.stdout and "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr


def test_child_loaded_sanitized_lib():
    if os.environ.get("CYC_SANITIZED_CHILD") != "1":
        return  # only meaningful inside the sanitized child
    from cyclonus_amd import _lib

    _lib.lib()
    maps = open("/proc/self/maps").read()
    assert "_build/asan/libcyclonus_hip.so" in maps and "libclang_rt.asan" in maps
