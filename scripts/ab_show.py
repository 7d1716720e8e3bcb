"""Print the top kernels (average ns) of ab_kernels.sh runs: ab_show.py OUT CFG VAR... [--top N]"""
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rocpd_stats import kernel_rows  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 4
if "--top" in sys.argv:
    args.remove(str(top))
out, cfg, variants = args[0], args[1], args[2:]
for v in variants:
    db = os.path.join("gpurun_out", out, f"k_{cfg}_{v}", "run_results.db")
    if not os.path.exists(db):
        print(f"== {cfg} {v}: missing")
        continue
    rows = kernel_rows(sqlite3.connect(db))[:top]
    print(f"== {cfg} {v}: " + "  ".join(f"{n.split('(')[0].replace('_ZN3cyc', '')[:28]} {avg / 1e3:.1f}us" for n, _, _, avg in rows))
