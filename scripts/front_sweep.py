"""Diagnostic: A/B the front-end knobs on a synthetic config (HIP-event timings, same process):
graph_stagger (egress class rows under the ingress emit) x emit_merged (both planes in one emit launch)
x pod_words (pod-peer words from
materialised peer rows or expanded from identity outcomes in the class rows).

    python scripts/front_sweep.py [config3 ...]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cyclonus_amd import synth
from cyclonus_amd.engine import Engine

for name in sys.argv[1:] or ["config3"]:
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

    ref = None
    res = {}
    for rep in range(3):
        for pw in (0, 1):
            eng.set_option("pod_words", pw)
            e = run(5, 0)
            for sg in (0, 1):
                for pr in (0, 1):
                    eng.set_option("graph_stagger", sg)
                    eng.set_option("emit_merged", pr)
                    g = run(10, 1)[0]
                    res.setdefault((pw, sg, pr), []).append((e[0], e[1], e[2], g))
            torch.cuda.synchronize()
            out = (d_in.sum().item(), d_eg.sum().item())
            ref = ref or out
            assert out == ref, "knobs changed the planes"
    print(f"{name}: P={P} K={K} W={W} effective pod_words(1)={eng.get_option('pod_words')}", flush=True)
    for (pw, sg, pr), v in sorted(res.items()):
        v = np.median(np.array(v), axis=0)
        print(f"  pod_words {pw} stagger {sg} merged {pr}: eager pipeline {v[0]:.3f} ms (emit {v[1]:.3f}, class rows {v[2]:.3f}, "
              f"front {v[0]-v[1]-v[2]:.3f})  graph {v[3]:.3f} ms", flush=True)
