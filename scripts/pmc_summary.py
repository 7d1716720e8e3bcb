"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-kernel HBM bytes per launch.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts half the bytes of a wide
coalesced streaming read -> doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores;
both are in KiB (hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024).

    python scripts/pmc_summary.py FETCH.csv WRITE.csv OUT.json [workload-name] [--mfma MFMA.csv] [--build-info INFO.json]

--build-info: the cyclonus_amd/_build/build_info.json of the profiled library (copied into the run's
output directory by the profiling script): its git head and sha256 go into OUT.json, and bench.py
quotes OUT.json's traffic only when the library it loads has that sha256.

--mfma: a pass with SQ_INSTS_VALU_MFMA_* / SQ_INSTS_MFMA / SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES
(scripts/pmc_mfma.sh) -> per step (one launch of every library kernel): MFMA instructions, MFMA
busy cycles and their share of the SQ busy cycles.
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


def mfma_summary(path):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        per[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    step = collections.defaultdict(float)  # one launch of each library kernel = one step
    for k, cs in per.items():
        if "cyc::" not in k:
            continue
        for c, v in cs.items():
            step[c] += sum(v) / len(v)
    insts = sum(v for c, v in step.items() if c.startswith("SQ_INSTS_VALU_MFMA_") and "MOPS" not in c or c == "SQ_INSTS_MFMA")
    busy = step.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    sq = step.get("SQ_BUSY_CYCLES", 0.0)
    return {"counters": sorted(step), "mfma_insts_per_step": insts, "mfma_busy_cycles_per_step": busy,
            "sq_busy_cycles_per_step": sq, "valu_insts_per_step": step.get("SQ_INSTS_VALU", 0.0),
            "util": busy / sq if sq else None,
            "util_definition": "SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES summed over one launch of every library kernel"}


def main():
    args = sys.argv[1:]
    mfma = info = None
    if "--mfma" in args:
        mfma = args[args.index("--mfma") + 1]
        args = [a for a in args if a not in ("--mfma", mfma)]
    if "--build-info" in args:
        info = args[args.index("--build-info") + 1]
        args = [a for a in args if a not in ("--build-info", info)]
    fetch, write, out = args[0], args[1], args[2]
    name = args[3] if len(args) > 3 else "config3"
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
    if mfma:
        doc["mfma"] = mfma_summary(mfma)
    if info:
        doc["build"] = json.load(open(info))
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps({"emit_hbm_bytes_per_launch": doc["emit_hbm_bytes_per_launch"], "mfma": doc.get("mfma")}))


if __name__ == "__main__":
    main()
