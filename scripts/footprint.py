"""Write rate vs written footprint on one GPU (is the 20 GB emit slower per byte than a 10 GB one?).

    python scripts/footprint.py [config3]

1. torch fill of a 20 GB buffer as one launch vs the same bytes as 2 / 4 / 8 sequential slice fills.
2. k_emit (eager HIP-event timings) over the whole row range vs. the same rows as sequential
   sub-ranges (each call also reruns the front; only the emit time is summed).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cyclonus_amd import synth
from cyclonus_amd.engine import Engine


def ev_time(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


GB = 20_006_400_000
buf = torch.empty(GB // 8, dtype=torch.int64, device="cuda")
for parts in (1, 2, 4, 8, 16):
    sl = [buf[i * (buf.numel() // parts):(i + 1) * (buf.numel() // parts)] for i in range(parts)]

    def f():
        for s in sl:
            s.fill_(parts)

    ms = ev_time(f)
    print(f"torch fill 20 GB as {parts:2d} sequential slices: {ms:.3f} ms ({GB / ms / 1e6:.0f} GB/s)", flush=True)
del buf
torch.cuda.empty_cache()

name = sys.argv[1] if len(sys.argv) > 1 else "config3"
data = synth.CONFIGS[name]()
eng = Engine(0).build_policies(json.dumps(data["policies"])).load_resources(json.dumps(data["resources"]))
sh = eng.prepare(data["probes"])
P, K, W = sh["pods"], sh["slots"], sh["words"]
d_in = torch.empty((P, K, W), dtype=torch.int64, device="cuda")
d_eg = torch.empty((P, K, W), dtype=torch.int64, device="cuda")
d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
eng.set_option("graphs", 0)
for parts in (1, 2, 4, 8):
    tot = []
    for rep in range(4):
        emit = 0.0
        for i in range(parts):
            lo, hi = P * i // parts, P * (i + 1) // parts
            eng.run_device(d_in[lo:].data_ptr(), d_eg[lo:].data_ptr(), d_st.data_ptr(), st, lo, hi)
            emit += eng.timings()[1]
        tot.append(emit)
    ms = float(np.mean(tot[1:]))
    print(f"k_emit {name} as {parts} sequential row ranges: emit {ms:.3f} ms ({2 * P * K * W * 8 / ms / 1e6:.0f} GB/s)", flush=True)
