"""Timeline of the captured step graph: run N graph replays of a synthetic config (default
options) for `rocprofv3 --kernel-trace`, then print the last replay's kernels with start / end
offsets from the replay's first kernel (shows what overlaps what across the two branches).

    rocprofv3 --kernel-trace -d OUT -o run -- python scripts/graph_timeline.py run [config3] [N] [opt=v ...] [shards=N]
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
    # replays end with the emit (and the graph's trailing copy, if any): the last replay = the kernels
    # after the second-to-last emit ended
    # a step's last emit launch (source shards emit each plane with its own launch; a row-phased step
    # runs phase 2's class rows between its two emits)
    mid = ("k_emit", "k_front_e", "k_class_rows", "k_front_d")
    ends = [i for i, r in enumerate(rows) if "k_emit" in r[0] and (i + 1 == len(rows) or not any(m in rows[i + 1][0] for m in mid))]
    spans = []
    for a, b in zip(ends, ends[1:]):
        seg = rows[a + 1:b + 1]
        spans.append((min(r[1] for r in seg), max(r[2] for r in seg), rows[a][2]))
    if spans:
        import statistics
        print(f"replays: first kernel -> emit end {statistics.median(s[1] - s[0] for s in spans) / 1e3:.1f} us median; "
              f"previous emit end -> first kernel {statistics.median(s[0] - s[2] for s in spans) / 1e3:.1f} us median")
    rows = rows[ends[-2] + 1:] if len(ends) > 1 else rows
    t0 = min(r[1] for r in rows)
    for name, a, b in sorted(rows, key=lambda r: r[1]):
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
eng.set_option("step_events", 1)  # whole-step timing events (cyc_last_timings)
P, K, W = sh["pods"], sh["slots"], sh["words"]
d_in = torch.empty((P, K, W), dtype=torch.int64, device="cuda")
d_eg = torch.empty((P, K, W), dtype=torch.int64, device="cuda")
d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
lo, hi = 0, P
part = "source"
for opt in sys.argv[4:]:
    k, v = opt.split("=")
    if k == "part":  # source (default) or target shards
        part = v
    elif k == "shards":  # rank 0's rows of an N-way shard (cyclonus_amd.shard.shard_range)
        from cyclonus_amd.shard import shard_range

        lo, hi = shard_range(P, int(v), 0, part)
    else:
        eng.set_option(k, int(v))
for _ in range(n):
    eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), st, lo, hi, part)
torch.cuda.synchronize()
print(json.dumps({"config": name, "timings_last": eng.timings()}))
