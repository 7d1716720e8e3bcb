"""Predict multi-GPU strong scaling on one GPU: time rank 0's row shard for N = 1, 2, 4, 8."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from cyclonus_amd import synth
from cyclonus_amd.engine import Engine
from cyclonus_amd.shard import row_range
data = synth.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "config3"]()
eng = Engine(0).build_policies(json.dumps(data["policies"])).load_resources(json.dumps(data["resources"]))
sh = eng.prepare(data["probes"])
eng.set_option("step_events", 1)  # whole-step timing events (cyc_last_timings)
P, K, W = sh["pods"], sh["slots"], sh["words"]
d_in = torch.empty((P, K, W), dtype=torch.int64, device="cuda")
d_eg = torch.empty((P, K, W), dtype=torch.int64, device="cuda")
d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
base = None
for n in (1, 2, 4, 8):
    worst = 0
    for rank in (0, n - 1):
        lo, hi = row_range(P, n, rank)
        for _ in range(2):
            eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), st, lo, hi)
        ts = []
        for _ in range(5):
            eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), st, lo, hi)
            ts.append(eng.timings())
        t = np.mean(ts, axis=0)
        worst = max(worst, t[0])
        print(f"N={n} rank {rank}: pipeline {t[0]:.3f} ms emit {t[1]:.3f} class_rows {t[2]:.3f} front {t[0]-t[1]-t[2]:.3f}", flush=True)
    base = base or worst
    print(f"N={n}: predicted speedup {base / worst:.2f} (efficiency {base / worst / n:.0%})", flush=True)
