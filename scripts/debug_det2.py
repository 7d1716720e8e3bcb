import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, torch
from cyclonus_amd import synth
from cyclonus_amd.engine import Engine
from test_gpu_parity import _device_cells
for name, kw in [("config3", {}), ("config3", {}), ("config2", {})]:
    data = synth.CONFIGS[name](**kw)
    eng = Engine(0).build_policies(json.dumps(data["policies"])).load_resources(json.dumps(data["resources"]))
    shape = eng.prepare(data["probes"])
    rng = np.random.default_rng(7)
    P, K = shape["pods"], shape["slots"]
    s, d, k = rng.integers(0, P, 6000), rng.integers(0, P, 6000), rng.integers(0, K, 6000)
    digs = []
    for it in range(4):
        got, dig = _device_cells(eng, shape, s, d, k)
        digs.append(dig)
    print(name, digs, flush=True)
