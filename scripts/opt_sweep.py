"""Diagnostic: A/B any cyc_set_option knobs on a synthetic config (HIP-event timings, same
process, interleaved repetitions so box drift hits every variant alike).

    python scripts/opt_sweep.py config3 class_variant_in=0,1 class_variant_eg=0,1 [reps=3]
"""
import itertools
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cyclonus_amd import synth
from cyclonus_amd.engine import Engine

name = sys.argv[1]
grid, reps = [], 3
for a in sys.argv[2:]:
    k, v = a.split("=")
    if k == "reps":
        reps = int(v)
    else:
        grid.append((k, [int(x) for x in v.split(",")]))
data = synth.CONFIGS[name]()
eng = Engine(0).build_policies(json.dumps(data["policies"])).load_resources(json.dumps(data["resources"]))
sh = eng.prepare(data["probes"])
P, K, W = sh["pods"], sh["slots"], sh["words"]
d_in = torch.empty((P, K, W), dtype=torch.int64, device="cuda")
d_eg = torch.empty((P, K, W), dtype=torch.int64, device="cuda")
d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream


def run(n, graphs):
    eng.set_option("graphs", graphs)
    eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), st)
    ts = []
    for _ in range(n):
        eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), st)
        ts.append(eng.timings())
    return np.median(np.array(ts), axis=0)


keys = [k for k, _ in grid]
combos = list(itertools.product(*[v for _, v in grid]))
res, ref = {}, None
for _ in range(reps):
    for combo in combos:
        for k, v in zip(keys, combo):
            eng.set_option(k, v)
        e = run(5, 0)
        g = run(10, 1)[0]
        res.setdefault(combo, []).append((e[0], e[1], e[2], g))
        torch.cuda.synchronize()
        out = (d_in.sum().item(), d_eg.sum().item())
        ref = ref or out
        assert out == ref, f"{combo} changed the planes"
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
fills = []
for _ in range(5):
    e0.record()
    d_in.fill_(0)
    d_eg.fill_(0)
    e1.record()
    torch.cuda.synchronize()
    fills.append(e0.elapsed_time(e1))
print(f"{name}: P={P} K={K} W={W}; torch fill of both planes {min(fills):.3f} ms "
      f"({2 * P * K * W * 8 / (min(fills) * 1e-3) / 1e9:.0f} GB/s)", flush=True)
for combo in combos:
    v = np.median(np.array(res[combo]), axis=0)
    tag = " ".join(f"{k}={x}" for k, x in zip(keys, combo))
    print(f"  {tag}: eager {v[0]:.3f} ms (emit {v[1]:.3f}, class rows {v[2]:.3f}, front {v[0]-v[1]-v[2]:.3f})  graph {v[3]:.3f} ms",
          flush=True)
