"""One-GPU prediction of multi-GPU strong scaling for both row partitions: back-to-back step time
(what bench.py times) of the slowest of ranks 0, N/2 and N-1 for N = 1, 2, 4, 8, target rows and
source rows interleaved on one box.

    python scripts/partition_scaling.py config3 [steps=20] [reps=2] [parts=target,source] [NAME=VALUE ...]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cyclonus_amd import synth
from cyclonus_amd.engine import Engine
from cyclonus_amd.shard import shard_range

name = sys.argv[1] if len(sys.argv) > 1 else "config3"
kw = dict(a.split("=") for a in sys.argv[2:])
steps, reps = int(kw.pop("steps", 20)), int(kw.pop("reps", 2))
parts = kw.pop("parts", "target,source").split(",")
data = synth.CONFIGS[name]()
eng = Engine(0).build_policies(json.dumps(data["policies"])).load_resources(json.dumps(data["resources"]))
sh = eng.prepare(data["probes"])
for k, v in kw.items():  # cyc_set_option NAME=VALUE
    eng.set_option(k, int(v))
P, K, W = sh["pods"], sh["slots"], sh["words"]
d_in = torch.empty((P * K * W,), dtype=torch.int64, device="cuda")
d_eg = torch.empty((P * K * W,), dtype=torch.int64, device="cuda")
d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream


def step_ms(lo, hi, part):
    for _ in range(3):
        eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), st, lo, hi, part)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), st, lo, hi, part)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


print(f"{name}: P={P} K={K} W={W} steps={steps} reps={reps}", flush=True)
base = {}
for n in (1, 2, 4, 8):
    for part in parts:
        worst, per = 0.0, []
        for rank in sorted({0, n // 2, n - 1}):
            lo, hi = shard_range(P, n, rank, part)
            t = min(step_ms(lo, hi, part) for _ in range(reps))
            per.append(f"r{rank} {t:.3f}")
            worst = max(worst, t)
        base.setdefault(part, worst)
        print(f"N={n} {part:6s}: max over ranks {worst:.3f} ms/step ({', '.join(per)}); predicted speedup "
              f"{base[part] / worst:.2f} (efficiency {base[part] / worst / n:.0%})", flush=True)
