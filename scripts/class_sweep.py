"""Diagnostic: A/B the class-row kernel variants per direction (cyc_set_option class_variant_in /
class_variant_eg; bit 0 = 4 slots per thread, bit 1 = strided representative grid) on a
synthetic config, eager path, HIP-event class-rows time.

    python scripts/class_sweep.py [config3]
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
data = synth.CONFIGS[name]()
eng = Engine(0).build_policies(json.dumps(data["policies"])).load_resources(json.dumps(data["resources"]))
sh = eng.prepare(data["probes"])
P, K, W = sh["pods"], sh["slots"], sh["words"]
d_in = torch.empty((P, K, W), dtype=torch.int64, device="cuda")
d_eg = torch.empty((P, K, W), dtype=torch.int64, device="cuda")
d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
eng.set_option("graphs", 0)


def rows_ms(n=5):
    eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), st)
    ts = []
    for _ in range(n):
        eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), st)
        ts.append(eng.timings()[2])
    return float(np.median(ts))


print(f"{name}: P={P} K={K} W={W} classes={eng.classes() if False else ''}", flush=True)
for direction in ("in", "eg"):
    other = "eg" if direction == "in" else "in"
    eng.set_option(f"class_variant_{other}", 0)
    base = None
    for v in range(4):
        eng.set_option(f"class_variant_{direction}", v)
        t = rows_ms()
        print(f"class_variant_{direction}={v} (KC={'4' if v & 1 else '8'}, {'strided' if v & 2 else 'row per identity'}): "
              f"class rows both directions {t:.3f} ms", flush=True)
print("classes", eng.classes())
