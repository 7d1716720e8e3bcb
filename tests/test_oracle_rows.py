"""The oracle's row entry (orc_probe_row: one plane row with the fixed target pod's matching
targets computed once) equals the same rows of its full per-cell table (CPU only)."""
import numpy as np

from oracle.oracle import Oracle, OraclePanic
from randgen import random_problem


def test_rows_equal_full_table():
    n = 0
    for seed in range(40):
        pols, res, probes = random_problem(seed)
        try:
            o = Oracle(pols, res)
            st, ing, eg = o.probe(probes)
        except OraclePanic:
            continue
        P, K = st.shape
        for pod in range(0, P, max(1, P // 4)):
            for k in range(K):
                assert np.array_equal(o.row(probes, "ingress", pod, k, threads=3), ing[pod, k]), (seed, pod, k)
                assert np.array_equal(o.row(probes, "egress", pod, k, threads=2), eg[pod, k]), (seed, pod, k)
                n += 1
    assert n > 200
