"""Run N eager (non-graph) pipeline steps of a synthetic config, for rocprofv3 --kernel-trace --stats
(per-kernel durations without the two-branch graph overlap).

    rocprofv3 --kernel-trace --stats -d OUT -o run -- python scripts/profile_eager.py config3 20 [NAME=VALUE ...]
(CYC_SHARD=r/N: rank r's row shard of an N-way run.)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from cyclonus_amd import synth
from cyclonus_amd.engine import Engine

name = sys.argv[1] if len(sys.argv) > 1 else "config3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
opts = [a.split("=") for a in sys.argv[3:]]  # cyc_set_option NAME=VALUE
data = synth.CONFIGS[name]()
eng = Engine(0).build_policies(json.dumps(data["policies"])).load_resources(json.dumps(data["resources"]))
sh = eng.prepare(data["probes"])
P, K, W = sh["pods"], sh["slots"], sh["words"]
# CYC_SHARD=r/N: rank r's shard of an N-way run, as bench.py --gpus N runs it; CYC_PART = source
# (default, shard.source_range) or target (shard.row_range)
lo, hi = 0, P
part = os.environ.get("CYC_PART", "source")
if os.environ.get("CYC_SHARD"):
    from cyclonus_amd.shard import shard_range

    r_, n_ = (int(x) for x in os.environ["CYC_SHARD"].split("/"))
    lo, hi = shard_range(P, n_, r_, part)
d_in = torch.empty((P * K * W,), dtype=torch.int64, device="cuda")
d_eg = torch.empty((P * K * W,), dtype=torch.int64, device="cuda")
d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
eng.set_option("graphs", 0)
for k, v in opts:
    eng.set_option(k, int(v))
for _ in range(n):
    eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), st, lo, hi, part)
torch.cuda.synchronize()
print(json.dumps({"config": name, "steps": n, "shape": sh, "timings_last": eng.timings(), "classes": eng.classes()}))
