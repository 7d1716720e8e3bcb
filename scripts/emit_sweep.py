"""Diagnostic: A/B the emit-kernel variants / persistent grid sizes / graph branching on a
synthetic config (HIP-event timings, same process).

    python scripts/emit_sweep.py [config3] [quick]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cyclonus_amd import synth
from cyclonus_amd.engine import Engine

name = sys.argv[1] if len(sys.argv) > 1 else "config3"
quick = len(sys.argv) > 2
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
    return np.mean(ts, axis=0)


variants = (0, 3, 4) if quick else (0, 1, 2, 3, 4, 5)
blocks = (0, 1024, 2048) if quick else (0, 512, 1024, 2048, 4096)
rows = []
for rep in range(2 if quick else 3):
    for v in variants:
        for b in blocks:
            eng.set_option("emit_variant", v)
            eng.set_option("emit_blocks", b)
            e = run(4, 0)
            out = [v, b, e[0], e[1], e[2]]
            for br in (0, 1):
                eng.set_option("graph_branches", br)
                out.append(run(4, 1)[0])
            eng.set_option("graph_branches", 1)
            rows.append(out)
rows = np.array(rows)
print(f"{name}: P={P} K={K} W={W}; plane bytes {P*K*W*8/1e9:.2f} GB x 2")
for v in variants:
    for b in blocks:
        r = rows[(rows[:, 0] == v) & (rows[:, 1] == b)].mean(axis=0)
        print(f"variant {v} emit_blocks {b:5d}: eager pipeline {r[2]:.3f} ms  emit {r[3]:.3f} ms "
              f"({2*P*K*W*8/(r[3]*1e-3)/1e9:.0f} GB/s)  class_rows {r[4]:.3f} ms  "
              f"graph 1-branch {r[5]:.3f} ms  graph 2-branch {r[6]:.3f} ms", flush=True)
