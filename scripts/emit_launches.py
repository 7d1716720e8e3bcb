"""Per-launch emit durations, in dispatch order, from a rocprofv3 --kernel-trace database
(scripts/emit_halves_ab.py run VARIANT... n=N under rocprofv3): which launch of a multi-launch emit is
slow, and how the launches of one variant compare with another's.

    python scripts/emit_launches.py OUT/run_results.db VARIANT:LAUNCHES_PER_STEP... [n=N]
"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
spec = [a.split(":") for a in sys.argv[2:] if not a.startswith("n=")]
n = int(next((a[2:] for a in sys.argv[2:] if a.startswith("n=")), 10))
rows = db.execute("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s "
                  "on d.kernel_id = s.id order by d.start").fetchall()
emits = [(b - a) / 1e3 for name, a, b in rows if "k_emit" in name]
at = 0
for name, per in spec:
    per = int(per)
    mine = emits[at:at + n * per]
    at += n * per
    for k in range(per):
        xs = sorted(mine[k::per])
        print(f"{name} launch {k}: median {xs[len(xs) // 2]:.1f} us, min {xs[0]:.1f} us over {len(xs)} steps")
