"""Timeline of the captured step graph: run N graph replays of a synthetic config (default
options) for `rocprofv3 --kernel-trace`, then print the last replay's kernels with start / end
offsets from the replay's first kernel (shows what overlaps what across the two branches).

    rocprofv3 --kernel-trace -d OUT -o run -- python scripts/graph_timeline.py run [config3] [N]
    python scripts/graph_timeline.py show OUT/run_results.db
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if sys.argv[1] == "show":
    import sqlite3

    db = sqlite3.connect(sys.argv[2])
    rows = db.execute("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s "
                      "on d.kernel_id = s.id order by d.start").fetchall()
    # last replay = kernels after the last k_selectors launch
    last = max(i for i, r in enumerate(rows) if "k_selectors" in r[0])
    rows = rows[last:]
    t0 = rows[0][1]
    for name, a, b in rows:
        short = name.split("(")[0].replace("_ZN3cyc", "")[:48]
        print(f"{(a - t0) / 1e3:9.1f} us -> {(b - t0) / 1e3:9.1f} us  ({(b - a) / 1e3:8.1f})  {short}")
    sys.exit(0)

import torch

from cyclonus_amd import synth
from cyclonus_amd.engine import Engine

name = sys.argv[2] if len(sys.argv) > 2 else "config3"
n = int(sys.argv[3]) if len(sys.argv) > 3 else 10
data = synth.CONFIGS[name]()
eng = Engine(0).build_policies(json.dumps(data["policies"])).load_resources(json.dumps(data["resources"]))
sh = eng.prepare(data["probes"])
P, K, W = sh["pods"], sh["slots"], sh["words"]
d_in = torch.empty((P, K, W), dtype=torch.int64, device="cuda")
d_eg = torch.empty((P, K, W), dtype=torch.int64, device="cuda")
d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
for opt in sys.argv[4:]:
    k, v = opt.split("=")
    eng.set_option(k, int(v))
for _ in range(n):
    eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), st)
torch.cuda.synchronize()
print(json.dumps({"config": name, "timings_last": eng.timings()}))
