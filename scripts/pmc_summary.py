"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-kernel HBM bytes per launch.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts half the bytes of a wide
coalesced streaming read -> doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores;
both are in KiB (hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024).

    python scripts/pmc_summary.py FETCH.csv WRITE.csv OUT.json [workload-name]
"""
import collections
import csv
import json
import sys


def per_kernel(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    fetch, write, out = sys.argv[1], sys.argv[2], sys.argv[3]
    name = sys.argv[4] if len(sys.argv) > 4 else "config3"
    f = per_kernel(fetch, "FETCH_SIZE")
    w = per_kernel(write, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(f) | set(w)):
        fb = 2 * f.get(k, 0.0) * 1024
        wb = w.get(k, 0.0) * 1024
        kernels[k] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb}
    emit = [v for k, v in kernels.items() if "k_emit" in k]
    doc = {"workload": name, "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
           "FETCH_SIZE doubled (gfx950), KiB -> bytes", "kernels": kernels,
           "emit_hbm_bytes_per_launch": emit[0]["hbm_bytes"] if emit else None}
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps({"emit_hbm_bytes_per_launch": doc["emit_hbm_bytes_per_launch"]}))


if __name__ == "__main__":
    main()
