"""Wide random parity sweep on the GPU (beyond the test suite's 400 seeds): random problems
through the default launch (fused front where it applies) and, every third seed, a second run on
the same context, each compared with the oracle.  Stops at the first difference.

    python tests/stress_parity.py FIRST_SEED N [seconds] [ido]   (test infrastructure: not collected by pytest)

"ido": deployment-style problems (contiguous runs of identical pods), the identity-set path.
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from cyclonus_amd.engine import Engine  # noqa: E402
from randgen import random_problem  # noqa: E402
from test_gpu_parity import _deployment_problem, assert_same, run_both  # noqa: E402

first, n = int(sys.argv[1]), int(sys.argv[2])
budget = float(sys.argv[3]) if len(sys.argv) > 3 else 90.0
ido = len(sys.argv) > 4 and sys.argv[4] == "ido"
eng = Engine(0)
t0, done, fused = time.time(), 0, 0
for seed in range(first, first + n):
    if time.time() - t0 > budget:
        break
    if ido:
        pols, res, probes = _deployment_problem(seed, min_run=16 + seed % 16)
    else:
        pols, res, probes = random_problem(seed, n_pods=20 + seed % 180, bad=(seed % 7 == 0))
    o, g = run_both(pols, res, probes, simplify=(seed % 5 != 0), engine=eng)
    assert_same(o, g, f"seed {seed}")
    if not hasattr(g, "msg"):
        fused += eng.get_option("front_fused_active")
        if seed % 3 == 0:
            assert_same(o, eng.run_host(), f"seed {seed} second run")
    done += 1
    if done % 200 == 0:
        print(f"{done} problems ok ({fused} on the fused front), {time.time() - t0:.0f} s", flush=True)
print(f"stress parity: {done} problems from seed {first} bit-exact with the oracle ({fused} on the fused front)")
