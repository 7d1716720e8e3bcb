"""Diagnostic: A/B the emit-kernel variants on config3 (HIP-event timings, same process)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cyclonus_amd import synth
from cyclonus_amd.engine import Engine

data = synth.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "config3"]()
eng = Engine(0).build_policies(json.dumps(data["policies"])).load_resources(json.dumps(data["resources"]))
sh = eng.prepare(data["probes"])
P, K, W = sh["pods"], sh["slots"], sh["words"]
d_in = torch.empty((P, K, W), dtype=torch.int64, device="cuda")
d_eg = torch.empty((P, K, W), dtype=torch.int64, device="cuda")
d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
res = {}
for rep in range(3):
    for v in range(6):
        eng.set_option("emit_variant", v)
        eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), st)
        ts = []
        for _ in range(4):
            eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), st)
            ts.append(eng.timings())
        res.setdefault(v, []).append(np.mean(ts, axis=0).tolist())
for v, r in res.items():
    r = np.array(r)
    print(f"variant {v}: pipeline {r[:,0].mean():.3f} ms  emit {r[:,1].mean():.3f} ms ({2*P*K*W*8/(r[:,1].mean()*1e-3)/1e9:.0f} GB/s)  class_rows {r[:,2].mean():.3f} ms")
