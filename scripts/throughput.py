"""Back-to-back step throughput (what bench.py times) under cyc_set_option settings, interleaved
repetitions so box drift hits every setting alike.

    python scripts/throughput.py config3 pr_group=4,8 [steps=20] [reps=3] [shards=N] [rank=R] [part=target|source] [init.<option>=v]
"""
import itertools
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cyclonus_amd import synth
from cyclonus_amd.engine import Engine

name = sys.argv[1]
grid, steps, reps, shards, rank, part = [], 20, 3, 1, 0, "target"
for a in sys.argv[2:]:
    k, v = a.split("=")
    if k == "steps":
        steps = int(v)
    elif k == "reps":
        reps = int(v)
    elif k == "shards":
        shards = int(v)
    elif k == "part":
        part = v
    elif k == "rank":  # the shard of this rank (default 0)
        rank = int(v)
    else:
        grid.append((k, [int(x) for x in v.split(",")]))
data = synth.CONFIGS[name]()
eng = Engine(0).build_policies(json.dumps(data["policies"])).load_resources(json.dumps(data["resources"]))
for a in list(grid):  # set-once options (before the first run): "name=value" with one value, prefixed "init."
    if a[0].startswith("init."):
        eng.set_option(a[0][5:], a[1][0])
        grid.remove(a)
sh = eng.prepare(data["probes"])
P, K, W = sh["pods"], sh["slots"], sh["words"]
lo, hi = 0, P
if shards > 1:
    from cyclonus_amd.shard import shard_range

    lo, hi = shard_range(P, shards, rank, part)
rows = hi - lo
d_in = torch.empty((P * K * W if part == "source" else rows * K * W,), dtype=torch.int64, device="cuda")
d_eg = torch.empty((rows * K * W,), dtype=torch.int64, device="cuda")
d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
keys = [k for k, _ in grid]
combos = list(itertools.product(*[v for _, v in grid])) or [()]
res = {}
for _ in range(reps):
    for combo in combos:
        for k, v in zip(keys, combo):
            eng.set_option(k, v)
        for _ in range(3):
            eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), st, lo, hi, part)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), st, lo, hi, part)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        res.setdefault(combo, []).append(((time.perf_counter() - t0) / steps * 1e3, (t1 - t0) / steps * 1e3))
print(f"{name}: P={P} K={K} W={W} rows [{lo},{hi}) {part} steps={steps}", flush=True)
for combo in combos:
    tag = " ".join(f"{k}={x}" for k, x in zip(keys, combo)) or "default"
    v = np.array(res[combo])[:, 0]
    h = np.array(res[combo])[:, 1]
    print(f"  {tag}: {np.median(v):.4f} ms/step (min {v.min():.4f}, max {v.max():.4f}); "
          f"{P * K * rows / (np.median(v) * 1e-3):.3e} verdicts/s; host enqueue {np.median(h):.4f} ms/step", flush=True)
