import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from cyclonus_amd import synth
from cyclonus_amd.engine import Engine
data = synth.config3()
eng = Engine(0).build_policies(json.dumps(data["policies"])).load_resources(json.dumps(data["resources"]))
sh = eng.prepare(data["probes"])
P, K, W = sh["pods"], sh["slots"], sh["words"]
outs = []
for it in range(3):
    d_in = torch.empty((P, K, W), dtype=torch.int64, device="cuda")
    d_eg = torch.empty((P, K, W), dtype=torch.int64, device="cuda")
    d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
    if it == 2:
        d_in.fill_(7); d_eg.fill_(7)
    eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    outs.append((d_in, d_eg))
for a in range(3):
    for b in range(a+1, 3):
        di = (outs[a][0] != outs[b][0]).any(dim=2)  # [P,K]
        de = (outs[a][1] != outs[b][1]).any(dim=2)
        rows = torch.nonzero(di.any(dim=1)).flatten()
        print(f"run{a} vs run{b}: ingress rows differ {rows.numel()} first {rows[:10].tolist()} slots {di.any(dim=0).tolist()}; egress rows differ {int(de.any(dim=1).sum())}")
        if rows.numel():
            r = int(rows[0]); k = int(torch.nonzero(di[r])[0])
            x = outs[a][0][r, k]; y = outs[b][0][r, k]
            w = torch.nonzero(x != y).flatten()
            print("  row", r, "slot", k, "words differ", w.numel(), "first", w[:8].tolist(), [hex(int(x[i]) & (2**64-1)) for i in w[:3]], [hex(int(y[i]) & (2**64-1)) for i in w[:3]])
