"""Config #3's whole-table emit against its halves, on one box in one process (VERDICT r4 ask 3).

    python scripts/emit_halves_ab.py time [steps=20] [reps=3]     # the A/B table
    python scripts/emit_halves_ab.py run VARIANT... [n=10]         # n steps of each variant (rocprofv3 --pmc)

The engine is prepared through bench.py's flat path (flat.prepare_flat).  Variants:
  whole      one cyc_probe_run over all target rows (the bench step; emit_interleave auto = 1)
  whole_il0  the same with the row list [ingress rows][egress rows] (emit_interleave = 0)
  halves     two cyc_probe_run calls, target rows [0, P/2) then [P/2, P), into the two halves of the
             same 2 x 10 GB planes (the whole pass's footprint)
  halves_il1 halves with the planes' rows alternating (emit_interleave = 1)
  half_same  the first half twice into the first half of the planes (10 GB footprint: what
             scripts/partition_scaling.py times for N = 2)
  first / second  one half run alone into its own half of the planes
Reported per variant: back-to-back ms per step (the bench clock; min over reps) and the emit's
HIP-event time per step from eager runs (graphs = 0: the emit launches of the step summed).
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cyclonus_amd import synth
from cyclonus_amd.engine import Engine
from cyclonus_amd.flat import prepare_flat

mode = sys.argv[1] if len(sys.argv) > 1 else "time"
pos = [a for a in sys.argv[2:] if "=" not in a or ":" in a]
kw = dict(a.split("=") for a in sys.argv[2:] if "=" in a and ":" not in a)
steps, reps, n_run = int(kw.get("steps", 20)), int(kw.get("reps", 3)), int(kw.get("n", 10))

data = synth.CONFIGS["config3"]()
eng = Engine(0)
sh = prepare_flat(eng, data["policies"], data["resources"], data["probes"])
P, K, W = sh["pods"], sh["slots"], sh["words"]
row = K * W
d_in = torch.empty((P * row,), dtype=torch.int64, device="cuda")
d_eg = torch.empty((P * row,), dtype=torch.int64, device="cuda")
d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
H = P // 2
B_IN, B_EG = d_in.data_ptr(), d_eg.data_ptr()

VARIANTS = {
    "whole": ({}, [(0, P, 0)]),
    "whole_il0": ({"emit_interleave": 0}, [(0, P, 0)]),
    "halves": ({}, [(0, H, 0), (H, P, H)]),
    "halves_il1": ({"emit_interleave": 1}, [(0, H, 0), (H, P, H)]),
    "half_same": ({}, [(0, H, 0), (0, H, 0)]),
    # each half run alone into its own half of the same planes (VERDICT r5 ask 2; round 6 also timed the
    # emit as launches over the address halves — option emit_footprint, removed: profiles/r06_emit_footprint_ab.txt)
    "first": ({}, [(0, H, 0)]),
    "second": ({}, [(H, P, H)]),
}


def spec(name):
    """A variant, optionally with options: "whole:emit_interleave=0,class_inplace=0"."""
    base, _, extra = name.partition(":")
    opts = dict(VARIANTS[base][0])
    for kv in filter(None, extra.split(",")):
        k, v = kv.split("=")
        opts[k] = int(v)
    return opts, VARIANTS[base][1]


def setv(name):
    for k, v in (("emit_interleave", -1), ("class_inplace", -1)):
        eng.set_option(k, v)
    for k, v in spec(name)[0].items():
        eng.set_option(k, v)


def step(name):
    for lo, hi, at in spec(name)[1]:
        # a target-row run writes its rows from the given pointers' row 0: place them at row `at`
        eng.run_device(B_IN + at * row * 8, B_EG + at * row * 8, d_st.data_ptr(), st, lo, hi)


if mode == "run":  # for rocprofv3 --pmc passes: n eager steps (graphs = 0) of each variant named, in order
    eng.set_option("graphs", 0)
    for name in pos:
        setv(name)
        for _ in range(n_run):
            step(name)
        torch.cuda.synchronize()
        print(f"{name}: {n_run} steps, emit {eng.last_emit()} per run, {len(spec(name)[1])} runs a step", flush=True)
    sys.exit(0)


def timed(name):
    setv(name)
    for _ in range(3):
        step(name)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(name)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def emit_events(name, n=5):
    setv(name)
    eng.set_option("graphs", 0)
    out = []
    for _ in range(n):
        tot = 0.0
        for lo, hi, at in spec(name)[1]:
            eng.run_device(B_IN + at * row * 8, B_EG + at * row * 8, d_st.data_ptr(), st, lo, hi)
            tot += eng.timings()[1]
        out.append(tot)
    eng.set_option("graphs", -1)
    return float(np.median(out)), eng.last_emit()


def fill_ms():
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record()
        d_in.fill_(0)
        d_eg.fill_(0)
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


names = pos or list(VARIANTS)
print(f"config3 flat-prepared: P={P} K={K} W={W}, plane row {row * 8} B; steps={steps} reps={reps}; planes at "
      f"{B_IN:#x} / {B_EG:#x} (mod 1 GiB {B_IN % (1 << 30):#x} / {B_EG % (1 << 30):#x})", flush=True)
res = {n: [] for n in names}
for r in range(reps):
    for n in names:
        res[n].append(timed(n))
    print(f"rep {r}: " + ", ".join(f"{n} {res[n][-1]:.3f}" for n in names), flush=True)
fill = fill_ms()
alg = 2.0 * P * row * 8
print(f"torch fill_ of both planes: {fill:.3f} ms = {alg / fill / 1e6:.0f} GB/s", flush=True)
base = min(res["whole"]) if "whole" in res else None
for n in names:
    ev, (kern, launches) = emit_events(n)
    t = min(res[n])
    rel = f" ({(t / base - 1) * 100:+.1f} % vs whole)" if base else ""
    print(f"{n:24s}: {t:.3f} ms/step{rel}; emit events {ev:.3f} ms/step = {alg / ev / 1e6:.0f} GB/s "
          f"({launches} x {kern})", flush=True)
print(json.dumps({"ms_per_step": {n: min(v) for n, v in res.items()}, "fill_ms": fill}), flush=True)
