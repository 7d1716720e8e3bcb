"""Per-kernel PMC averages per launch from rocprofv3 --pmc CSV passes (dev helper).
    python scripts/pmc_table.py gpurun_out/X/sq1_config4 gpurun_out/X/sq2_config4 ...
Each argument is a pass output directory (its *_counter_collection.csv is read)."""
import collections
import csv
import glob
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(path)):
            per[(r["Kernel_Name"], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, _, c), v in per.items():
            vals[k][c].append(v)
for k in sorted(vals):
    name = k.split("(")[0][:60]
    cs = vals[k]
    line = ", ".join(f"{c} {sum(v) / len(v):.4g}" for c, v in sorted(cs.items()))
    print(f"{name}: {line}")
