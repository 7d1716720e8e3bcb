"""Compare per-kernel average durations (us) across ab_kernels.sh runs: ks_compare.py DIR CFG SPEC..."""
import glob
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rocpd_stats import kernel_rows  # noqa: E402

d, cfg, specs = sys.argv[1], sys.argv[2], sys.argv[3:]
table, names = {}, []
for sp in specs:
    runs = sorted(glob.glob(os.path.join(d, f"k_{cfg}_{sp}*", "run_results.db")))
    acc = {}
    for r in runs:
        for name, n, tot, avg in kernel_rows(sqlite3.connect(r)):
            short = name.replace("_ZN3cyc", "").split("E")[0][:28] if name.startswith("_ZN3cyc") else name[:28]
            acc.setdefault(short, []).append(avg / 1e3)
            if short not in names:
                names.append(short)
    table[sp] = {k: sum(v) / len(v) for k, v in acc.items()}
print("kernel".ljust(30) + "".join(sp[:12].rjust(13) for sp in specs))
for n in names:
    if "rocclr" in n:
        continue
    print(n.ljust(30) + "".join((f"{table[sp][n]:.1f}" if n in table[sp] else "-").rjust(13) for sp in specs))
tot = {sp: sum(v for k, v in table[sp].items() if "rocclr" not in k) for sp in specs}
print("sum".ljust(30) + "".join(f"{tot[sp]:.1f}".rjust(13) for sp in specs))
