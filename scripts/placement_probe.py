"""Does the emit's speed depend on WHERE the planes are (VERDICT r4 ask 7)?  One process, config #3
prepared through bench.py's flat path, N pairs of output planes allocated side by side (torch's
caching allocator: one hipMalloc each), then whole-table steps timed round-robin over the pairs, and a
torch fill_ of each pair — same library, same process, same front: only the planes' placement differs.

    python scripts/placement_probe.py [pairs=4] [steps=20] [reps=3] [NAME=VALUE ...]   (cyc_set_option)
    python scripts/placement_probe.py pairs=4 "alt=class_inplace:0;emit_interleave:0"   (each pair also
                                                                   with each option set)
    python scripts/placement_probe.py pairs=2 hip=2 contig=2     (+ pairs from hipExtMallocWithFlags: flags 0 /
                                                                   hipDeviceMallocContiguous)
The fill of each pair is hipMemsetD32Async over both planes (one kernel for every allocation kind).
"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from cyclonus_amd import synth
from cyclonus_amd.engine import Engine
from cyclonus_amd.flat import prepare_flat

kw = dict(a.split("=") for a in sys.argv[1:])
pairs, steps, reps = int(kw.pop("pairs", 4)), int(kw.pop("steps", 20)), int(kw.pop("reps", 3))
# alt=name:v,name:v[;name:v...]: option sets run on every pair besides the defaults
alts = [dict(x.split(":") for x in grp.split(",") if x) for grp in kw.pop("alt", "").split(";") if grp]
n_hip, n_contig = int(kw.pop("hip", 0)), int(kw.pop("contig", 0))
name = kw.pop("config", "config3")
data = synth.CONFIGS[name]()
eng = Engine(0)
sh = prepare_flat(eng, data["policies"], data["resources"], data["probes"])
for k, v in kw.items():
    eng.set_option(k, int(v))
P, K, W = sh["pods"], sh["slots"], sh["words"]
n = P * K * W
st = torch.cuda.current_stream().cuda_stream
d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
hip = ctypes.CDLL("libamdhip64.so")


class Raw:  # a device allocation of hipExtMallocWithFlags (data_ptr like a tensor's)
    def __init__(self, flags):
        p = ctypes.c_void_p()
        rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(n * 8), ctypes.c_uint(flags))
        if rc != 0:
            raise RuntimeError(f"hipExtMallocWithFlags(flags={flags}) failed: {rc}")
        self.p = p.value

    def data_ptr(self):
        return self.p


planes = [(torch.empty((n,), dtype=torch.int64, device="cuda"), torch.empty((n,), dtype=torch.int64, device="cuda"))
          for _ in range(pairs)]
kinds = ["torch"] * pairs
for flags, cnt, kind in ((0, n_hip, "hipMalloc"), (4, n_contig, "contiguous")):
    for _ in range(cnt):
        planes.append((Raw(flags), Raw(flags)))
        kinds.append(kind)
pairs = len(planes)
print(f"{name}: {pairs} plane pairs of 2 x {n * 8 / 1e9:.2f} GB, options {kw}", flush=True)
for i, (a, b) in enumerate(planes):
    print(f"pair {i} ({kinds[i]}): ingress {a.data_ptr():#x} egress {b.data_ptr():#x} "
          f"(mod 1 GiB {a.data_ptr() % (1 << 30):#x} / {b.data_ptr() % (1 << 30):#x})", flush=True)


def step_ms(a, b):
    for _ in range(3):
        eng.run_device(a.data_ptr(), b.data_ptr(), d_st.data_ptr(), st)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.run_device(a.data_ptr(), b.data_ptr(), d_st.data_ptr(), st)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def emit_ms(a, b):
    eng.set_option("graphs", 0)
    out = []
    for _ in range(5):
        eng.run_device(a.data_ptr(), b.data_ptr(), d_st.data_ptr(), st)
        out.append(eng.timings()[1])
    eng.set_option("graphs", -1)
    return sorted(out)[2]


def fill_ms(a, b):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record()
        for x in (a, b):
            hip.hipMemsetD32Async(ctypes.c_void_p(x.data_ptr()), ctypes.c_int(0), ctypes.c_size_t(2 * n), ctypes.c_void_p(st))
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


base = {k: eng.get_option(k) for alt in alts for k in alt}
sets = [("default", base)] + [(",".join(f"{k}={v}" for k, v in alt.items()), {**base, **{k: int(v) for k, v in alt.items()}})
                              for alt in alts]


def use(opts):
    for k, v in opts.items():
        eng.set_option(k, v)


res = {(i, nm): [] for i in range(pairs) for nm, _ in sets}
for r in range(reps):
    for nm, opts in sets:
        use(opts)
        for i, (a, b) in enumerate(planes):
            res[(i, nm)].append(step_ms(a, b))
        print(f"rep {r} {nm}: " + ", ".join(f"pair {i} {res[(i, nm)][-1]:.3f}" for i in range(pairs)), flush=True)
for nm, opts in sets:
    use(opts)
    for i, (a, b) in enumerate(planes):
        em, fm = emit_ms(a, b), fill_ms(a, b)
        print(f"{nm}: pair {i} ({kinds[i]}): {min(res[(i, nm)]):.3f} ms/step, emit {em:.3f} ms ({2 * n * 8 / em / 1e6:.0f} GB/s), "
              f"fill {fm:.3f} ms ({2 * n * 8 / fm / 1e6:.0f} GB/s), emit / fill {em / fm:.3f}", flush=True)
