"""Host-side phases of bench.py's preparation (flat.prepare_flat) with the library's phase clock
(CYC_TRACE_PREPARE=1 prints each phase of the policy build, Resources load, job expansion, planning
and table upload to stderr), twice in one process: a cold and a warm prepare.

    python scripts/prepare_trace.py [config3]
"""
import os
import sys

os.environ["CYC_TRACE_PREPARE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from cyclonus_amd import synth
from cyclonus_amd.engine import Engine
from cyclonus_amd.flat import prepare_flat

name = sys.argv[1] if len(sys.argv) > 1 else "config3"
data = synth.CONFIGS[name]()
torch.cuda.init()
for rep in range(2):
    eng = Engine(0)
    sh = prepare_flat(eng, data["policies"], data["resources"], data["probes"])
    print(f"{name} prepare {rep}: {sh['prepare_s']}", file=sys.stderr, flush=True)
    eng.close()
