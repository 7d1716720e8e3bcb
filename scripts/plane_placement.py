"""Step time against the placement of the two output planes (dev probe): does where the ingress and
egress planes sit in device memory (their base alignment, their distance) change the emit's rate?

    python scripts/plane_placement.py config4 [pairs=8] [steps=20]
Part 1: `pairs` pairs of separate torch allocations (as bench.py makes them), kept alive so each
pair lands elsewhere; part 2: both planes in ONE allocation, the egress plane at the ingress
plane's end + delta for a list of deltas.  Prints ms / step with the planes' addresses.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from cyclonus_amd import synth
from cyclonus_amd.engine import Engine

name = sys.argv[1] if len(sys.argv) > 1 else "config4"
kw = dict(a.split("=") for a in sys.argv[2:])
pairs, steps = int(kw.get("pairs", 8)), int(kw.get("steps", 20))
data = synth.CONFIGS[name]()
eng = Engine(0).build_policies(json.dumps(data["policies"])).load_resources(json.dumps(data["resources"]))
sh = eng.prepare(data["probes"])
P, K, W = sh["pods"], sh["slots"], sh["words"]
n = P * K * W
plane = n * 8
d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
print(f"{name}: P={P} K={K} W={W} plane {plane / 1e9:.3f} GB, row {K * W * 8} B", flush=True)


def step_ms(a_in, a_eg):
    for _ in range(3):
        eng.run_device(a_in, a_eg, d_st.data_ptr(), st)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(steps):
        eng.run_device(a_in, a_eg, d_st.data_ptr(), st)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def show(tag, a_in, a_eg):
    t = min(step_ms(a_in, a_eg) for _ in range(2))
    d = a_eg - a_in
    print(f"{tag}: {t:.4f} ms  in {a_in:#x} eg {a_eg:#x}  in%2M {a_in % (2 << 20):#x}  eg-in {d:#x} "
          f"(eg-in-plane)%2M {(d - plane) % (2 << 20):#x} %64M {(d - plane) % (64 << 20):#x}", flush=True)


keep = []
for i in range(pairs):
    a = torch.empty((n,), dtype=torch.int64, device="cuda")
    b = torch.empty((n,), dtype=torch.int64, device="cuda")
    keep.append((a, b))
    show(f"separate {i}", a.data_ptr(), b.data_ptr())
del keep
torch.cuda.empty_cache()
MB = 1 << 20
deltas = [0, 4096, 64 * 1024, 256 * 1024, MB, 2 * MB, 3 * MB, 4 * MB, 8 * MB, 32 * MB, 64 * MB, 96 * MB, 128 * MB]
big = torch.empty((2 * plane + max(deltas) + 4 * MB) // 8, dtype=torch.int64, device="cuda")
base = (big.data_ptr() + 2 * MB - 1) // (2 * MB) * (2 * MB)
for dl in deltas:
    show(f"one buffer, delta {dl // 1024:6d} KB", base, base + plane + dl)
for off in (4096, MB):
    show(f"one buffer, in +{off // 1024} KB, delta 0", base + off, base + off + plane)
