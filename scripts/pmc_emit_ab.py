"""Summarise scripts/pmc_emit_ab.sh: per variant of scripts/emit_halves_ab.py, every emit counter summed
over the emit launches of one step (each variant ran n = 3 steps, in the order given).

    python scripts/pmc_emit_ab.py gpurun_out/OUT VARIANT...

FETCH_SIZE doubled (gfx950, MI355X_MICROARCH.md §HBM), KiB -> bytes; WRITE_SIZE KiB -> bytes."""
import collections
import csv
import glob
import os
import sys

out, variants = sys.argv[1], sys.argv[2:]
N = 3
# emit launches per step: the runs a step makes x the launches a run's emit makes
PER_STEP = {"whole": 1, "whole_il0": 1, "halves": 2, "halves_il1": 2, "half_same": 2, "first": 1, "second": 1}
per = collections.defaultdict(lambda: collections.defaultdict(float))
for path in sorted(glob.glob(os.path.join(out, "pmcab_*", "**", "*counter_collection.csv"), recursive=True)):
    rows = [r for r in csv.DictReader(open(path)) if "k_emit" in r["Kernel_Name"]]
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})
    owner, at = {}, 0
    for v in variants:
        k = PER_STEP[v.split(":")[0]]
        for d in ids[at:at + N * k]:
            owner[d] = v
        at += N * k
    for r in rows:
        v = owner.get(int(r["Dispatch_Id"]))
        if v:
            per[v][r["Counter_Name"]] += float(r["Counter_Value"]) / N
cols = sorted({c for v in per.values() for c in v})
print("emit counters per step (summed over the step's emit launches; mean of %d steps)" % N)
for v in variants:
    c = per[v]
    fb, wb = 2 * c.get("FETCH_SIZE", 0) * 1024, c.get("WRITE_SIZE", 0) * 1024
    print(f"{v}: fetch {fb / 1e9:.3f} GB, write {wb / 1e9:.3f} GB, hbm {(fb + wb) / 1e9:.3f} GB")
    for k in cols:
        if k not in ("FETCH_SIZE", "WRITE_SIZE"):
            print(f"    {k:40s} {c.get(k, 0):.4g}")
