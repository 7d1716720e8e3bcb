"""Print the key figures of bench.py JSON lines in the given log files (dev helper)."""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        if line.startswith("{"):
            d = json.loads(line)
            rf = d["roofline"]
            print(f"{path}: {d['config']['workload'][:8]} ms/step {d['ms_per_step']:.4f} value {d['value']:.3e} "
                  f"emit frac {rf['frac']:.3f} step GB/s {rf['algorithmic_bytes_per_launch'] / d['ms_per_step'] / 1e6:.0f} "
                  f"pipeline {json.dumps({k: round(v, 4) for k, v in d['pipeline_ms'].items()})}")
