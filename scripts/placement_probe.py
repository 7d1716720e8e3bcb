"""Does the emit's speed depend on WHERE the planes are (VERDICT r4 ask 7)?  One process, config #3
prepared through bench.py's flat path, N pairs of output planes allocated side by side (torch's
caching allocator: one hipMalloc each), then whole-table steps timed round-robin over the pairs, and a
torch fill_ of each pair — same library, same process, same front: only the planes' placement differs.

    python scripts/placement_probe.py [pairs=4] [steps=20] [reps=3] [NAME=VALUE ...]   (cyc_set_option)
"""
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
data = synth.CONFIGS["config3"]()
eng = Engine(0)
sh = prepare_flat(eng, data["policies"], data["resources"], data["probes"])
for k, v in kw.items():
    eng.set_option(k, int(v))
P, K, W = sh["pods"], sh["slots"], sh["words"]
n = P * K * W
st = torch.cuda.current_stream().cuda_stream
d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
planes = [(torch.empty((n,), dtype=torch.int64, device="cuda"), torch.empty((n,), dtype=torch.int64, device="cuda"))
          for _ in range(pairs)]
print(f"config3: {pairs} plane pairs of 2 x {n * 8 / 1e9:.2f} GB, options {kw}", flush=True)
for i, (a, b) in enumerate(planes):
    print(f"pair {i}: ingress {a.data_ptr():#x} egress {b.data_ptr():#x} "
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
        a.fill_(0)
        b.fill_(0)
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


res = [[] for _ in planes]
for r in range(reps):
    for i, (a, b) in enumerate(planes):
        res[i].append(step_ms(a, b))
    print(f"rep {r}: " + ", ".join(f"pair {i} {res[i][-1]:.3f}" for i in range(pairs)), flush=True)
for i, (a, b) in enumerate(planes):
    em, fm = emit_ms(a, b), fill_ms(a, b)
    print(f"pair {i}: {min(res[i]):.3f} ms/step, emit {em:.3f} ms ({2 * n * 8 / em / 1e6:.0f} GB/s), "
          f"fill {fm:.3f} ms ({2 * n * 8 / fm / 1e6:.0f} GB/s), emit / fill {em / fm:.3f}", flush=True)
