"""One line per bench log of a GPU call: ms/step, the emit's roofline fraction, pipeline split, emit kernel.
    python scripts/bench_lines.py gpurun_out/r06m [more dirs]"""
import glob
import json
import os
import sys


def main():
    for d in sys.argv[1:]:
        for f in sorted(glob.glob(os.path.join(d, "bench_*.log"))):
            line = None
            for raw in open(f):
                if raw.startswith("{"):
                    line = json.loads(raw)
            name = os.path.basename(f)[len("bench_"):-len(".log")]
            if line is None:
                print(f"{name:70s} (no bench line)")
                continue
            rf = line.get("roofline") or {}
            pm = line.get("pipeline_ms", {})
            print(f"{name:70s} {line['ms_per_step']:.4f} ms  frac {rf.get('frac', 0):.3f}  "
                  f"front {pm.get('front', 0) * 1e3:6.1f} rows {pm.get('class_rows', 0) * 1e3:6.1f} "
                  f"emit {pm.get('emit', 0) * 1e3:7.1f} us  {rf.get('emit_kernel', '')}")
        t = os.path.join(d, "gpu_tests.log")
        if os.path.exists(t):
            tail = [x for x in open(t) if " passed" in x or " failed" in x]
            if tail:
                print("tests:", tail[-1].strip())


if __name__ == "__main__":
    main()
