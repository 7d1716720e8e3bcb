"""Per-wave view of per-kernel PMC averages (dev helper): instructions per wave by kind, the share of
wave cycles waiting (s_waitcnt / barrier), stalled on issue, and active.
    python scripts/pmc_perwave.py gpurun_out/X/sq1_CFG gpurun_out/X/sq2_CFG [...]"""
import re
import subprocess
import sys

out = subprocess.run([sys.executable, __file__.replace("pmc_perwave.py", "pmc_table.py"), *sys.argv[1:]], capture_output=True,
                     text=True, check=True).stdout
for line in out.splitlines():
    name, rest = line.split(": ", 1)
    if "rocclr" in name:
        continue
    kv = {m.group(1): float(m.group(2)) for m in re.finditer(r"(\w+) ([0-9.e+-]+)", rest)}
    w = kv.get("SQ_WAVES", 1) or 1
    cyc = kv.get("SQ_WAVE_CYCLES", 1) or 1
    print(f"{name.replace('cyc::', '')[:34]:34s} waves {w:7.0f} | per wave: VALU {kv.get('SQ_INSTS_VALU', 0) / w:6.0f} "
          f"SALU {kv.get('SQ_INSTS_SALU', 0) / w:5.0f} VMEM rd {kv.get('SQ_INSTS_VMEM_RD', 0) / w:5.1f} "
          f"wr {kv.get('SQ_INSTS_VMEM_WR', 0) / w:5.1f} LDS {kv.get('SQ_INSTS_LDS', 0) / w:5.1f} cycles {cyc / w:6.0f} | "
          f"wait {kv.get('SQ_WAIT_ANY', 0) / cyc:.2f} issue-stall {kv.get('SQ_WAIT_INST_ANY', 0) / cyc:.2f} "
          f"active {kv.get('SQ_ACTIVE_INST_ANY', 0) / cyc:.2f} | VALU total {kv.get('SQ_INSTS_VALU', 0):.3g}")
