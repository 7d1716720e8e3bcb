import json, sys
sys.path.insert(0, '.')
from cyclonus_amd import synth
from cyclonus_amd.engine import Engine
for name in sys.argv[1:]:
    d = synth.CONFIGS[name]()
    e = Engine(0).build_policies(json.dumps(d["policies"])).load_resources(json.dumps(d["resources"]))
    print(name, e.prepare(d["probes"]))
