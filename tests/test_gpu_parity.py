"""GPU parity: libcyclonus_hip (through the C ABI) vs the per-cell CPU oracle, bit-exact.

Every comparison is on the full truth table: status[d,k], ingress plane[d,k,s] and egress
plane[s,k,d]; Go panics must be reported with the reference's message for the first
panicking job in the reference's job order.
"""
import json
import os

import numpy as np
import pytest

from cyclonus_amd._lib import CyclonusError, CyclonusPanic
from cyclonus_amd.engine import Engine
from oracle.oracle import Oracle, OraclePanic, combined_table
from randgen import random_problem

GOLD = os.path.join(os.path.dirname(__file__), "golden")
pytestmark = pytest.mark.gpu


class Panicked:
    def __init__(self, msg):
        self.msg = msg

    def __repr__(self):
        return f"Panicked({self.msg!r})"


def run_both(pols, res, probes, simplify=True, engine=None):
    try:
        o = Oracle(pols, res, simplify).probe(probes)
    except OraclePanic as e:
        o = Panicked(str(e))
    eng = engine or Engine(0)
    try:
        eng.build_policies(pols, simplify).load_resources(res)
        eng.prepare(probes)
        g = eng.run_host()
    except CyclonusPanic as e:
        g = Panicked(e.msg)
    return o, g


def run_gpu(eng, pols, res, probes, simplify=True):
    """run_both's GPU side alone (the caller holds the oracle's table)."""
    try:
        eng.build_policies(pols, simplify).load_resources(res)
        eng.prepare(probes)
        return eng.run_host()
    except CyclonusPanic as e:
        return Panicked(e.msg)


def assert_same(o, g, ctx=""):
    if isinstance(o, Panicked) or isinstance(g, Panicked):
        assert isinstance(o, Panicked) and isinstance(g, Panicked), f"{ctx}: oracle={o!r:.300} gpu={g!r:.300}"
        assert o.msg == g.msg, f"{ctx}: panic message differs: oracle={o.msg!r} gpu={g.msg!r}"
        return
    for name, a, b in zip(("status", "ingress", "egress"), o, g):
        assert a.shape == b.shape, f"{ctx}: {name} shape {a.shape} vs {b.shape}"
        if not np.array_equal(a, b):
            idx = np.argwhere(a != b)[:5]
            pytest.fail(f"{ctx}: {name} differs at {idx.tolist()} ({int((a != b).sum())} words)")


def test_config1_readme(gpu):
    c = json.load(open(os.path.join(GOLD, "config1.json")))
    o, g = run_both(c["policies"], c["resources"], c["probes"])
    assert_same(o, g, "config1")
    status, inp, egp = g
    ing, eg = combined_table(status, inp, egp)
    names = [p["Namespace"] + "/" + p["Name"] for p in c["resources"]["Pods"]]
    exp = c["readme_combined_tcp80"]["rows"]
    for s, fr in enumerate(names):
        for d, to in enumerate(names):
            got = "." if (ing[s, d, 0] and eg[s, d, 0]) else "X"
            assert got == exp[fr][to.upper()], (fr, to)


@pytest.mark.parametrize("block", range(8))
def test_random_parity(gpu, block):
    eng = Engine(0)
    for seed in range(block * 50, block * 50 + 50):
        pols, res, probes = random_problem(seed)
        o, g = run_both(pols, res, probes, simplify=(seed % 5 != 0), engine=eng)
        assert_same(o, g, f"seed {seed}")


@pytest.mark.parametrize("block", range(3))
def test_random_panics(gpu, block):
    eng = Engine(0)
    n_panics = 0
    for seed in range(10_000 + block * 60, 10_000 + block * 60 + 60):
        pols, res, probes = random_problem(seed, bad=True)
        o, g = run_both(pols, res, probes, engine=eng)
        n_panics += isinstance(o, Panicked)
        assert_same(o, g, f"bad seed {seed}")
    assert n_panics > 0


def test_larger_random(gpu):
    eng = Engine(0)
    for seed in range(5):
        pols, res, probes = random_problem(50_000 + seed, n_pods=300, n_pols=60)
        o, g = run_both(pols, res, probes, engine=eng)
        assert_same(o, g, f"large seed {seed}")


def test_row_ranges_and_device_path(gpu):
    import torch

    pols, res, probes = random_problem(777, n_pods=200, n_pols=30)
    eng = Engine(0).build_policies(pols).load_resources(res)
    sh = eng.prepare(probes)
    st, ing, eg = eng.run_host()
    P, K, W = sh["pods"], sh["slots"], sh["words"]
    for lo, hi in [(0, 1), (3, 77), (100, 200), (199, 200), (50, 50)]:
        st2, ing2, eg2 = eng.run_host(lo, hi)
        assert np.array_equal(st, st2)
        assert np.array_equal(ing[lo:hi], ing2) and np.array_equal(eg[lo:hi], eg2)
    d_in = torch.zeros((P, K, W), dtype=torch.int64, device="cuda")
    d_eg = torch.zeros((P, K, W), dtype=torch.int64, device="cuda")
    d_st = torch.zeros((P, K), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(d_in.cpu().numpy().view(np.uint64), ing)
    assert np.array_equal(d_eg.cpu().numpy().view(np.uint64), eg)
    assert np.array_equal(d_st.cpu().numpy(), st)


def test_reference_policy_fixtures(gpu):
    c = json.load(open(os.path.join(GOLD, "config1.json")))
    fx = json.load(open(os.path.join(GOLD, "policy_fixtures.json")))
    probes = [{"AllAvailable": True}, {"Port": 80, "Protocol": "TCP"}, {"Port": 53, "Protocol": "UDP"},
              {"Port": "serve-81-tcp", "Protocol": "TCP"}]
    for name, pols in fx.items():
        o, g = run_both(pols, c["resources"], probes)
        assert_same(o, g, name)


def _device_cells(eng, shape, s, d, k):
    """Run the full table on the device and read back only the sampled (s, d, k) cells."""
    import torch

    P, K, W = shape["pods"], shape["slots"], shape["words"]
    d_in = torch.empty((P, K, W), dtype=torch.int64, device="cuda")
    d_eg = torch.empty((P, K, W), dtype=torch.int64, device="cuda")
    d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")
    eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), torch.cuda.current_stream().cuda_stream)
    S, D, KK = (torch.as_tensor(x, dtype=torch.int64, device="cuda") for x in (s, d, k))
    iw = d_in[D, KK, S // 64]
    ew = d_eg[S, KK, D // 64]
    ing = (iw >> (S % 64)) & 1
    eg = (ew >> (D % 64)) & 1
    st = d_st[D, KK].to(torch.int64)
    digest = (int(d_in.sum().item()), int(d_eg.sum().item()))
    out = (st | (ing << 4) | (eg << 5)).to(torch.uint8).cpu().numpy()
    del d_in, d_eg
    torch.cuda.empty_cache()
    return out, digest


@pytest.mark.parametrize("name,kw,n", [
    ("config2", {}, 20000),
    ("config3", {"n_ns": 100}, 20000),
    ("config3", {}, 6000),
    ("config4", {"n_pods": 10000, "n_policies": 1000, "n_ns": 100}, 20000),
    ("config4", {}, 6000),
])
def test_synthetic_sampled_parity(gpu, name, kw, n):
    """Full-size tables vs the oracle on random cells, plus run-to-run determinism."""
    from cyclonus_amd import synth

    data = synth.CONFIGS[name](**kw)
    eng = Engine(0).build_policies(json.dumps(data["policies"])).load_resources(json.dumps(data["resources"]))
    shape = eng.prepare(data["probes"])
    rng = np.random.default_rng(7)
    P, K = shape["pods"], shape["slots"]
    s, d, k = rng.integers(0, P, n), rng.integers(0, P, n), rng.integers(0, K, n)
    got, dig1 = _device_cells(eng, shape, s, d, k)
    _, dig2 = _device_cells(eng, shape, s, d, k)
    assert dig1 == dig2, "two runs of the same inputs differ"
    want = Oracle(data["policies"], data["resources"]).cells(data["probes"], s, d, k)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} cells differ, first {[(int(s[i]), int(d[i]), int(k[i]), int(got[i]), int(want[i])) for i in bad[:5]]}"


def test_partial_ranges_match_full_on_synthetic(gpu):
    """Range plans (active identities / peers per row shard) give the same rows as the full run."""
    from cyclonus_amd import synth
    from cyclonus_amd.shard import row_range

    data = synth.config3(n_ns=40)
    eng = Engine(0).build_policies(json.dumps(data["policies"])).load_resources(json.dumps(data["resources"]))
    eng.prepare(data["probes"])
    st, ing, eg = eng.run_host()
    P = st.shape[0]
    for world in (2, 3, 8):
        for rank in range(world):
            lo, hi = row_range(P, world, rank)
            st2, ing2, eg2 = eng.run_host(lo, hi)
            assert np.array_equal(ing[lo:hi], ing2) and np.array_equal(eg[lo:hi], eg2), (world, rank)


def _check_batch(problems, reps=1, ctx="batch"):
    """Batch.run of the problems (each repeated `reps` times) equals each problem's own oracle run:
    its table, or its panic / table-build fatal with the same message."""
    from cyclonus_amd.batch import Batch

    blocks = [p for p in problems for _ in range(reps)]
    bt = Batch(blocks)
    got = bt.run(Engine(0))
    want = []
    for p in problems:
        try:
            want.append(Oracle(p["policies"], p["resources"]).probe([p["probe"]]))
        except OraclePanic as e:
            want.append(Panicked(str(e)))
    for b, g in enumerate(got):
        w = want[b // reps]
        g = Panicked(g.msg) if isinstance(g, CyclonusPanic) else g
        assert_same(w, g, f"{ctx} block {b} ({blocks[b].get('description', '')})")
    return bt


def test_config5_generate_sweep_batched(gpu):
    """All 242 probe steps of `cyclonus generate --mock --exclude ''` in one batched GPU pass (a block
    per step: only its own cells computed), each block bit-exact vs the oracle run on that step alone."""
    from cyclonus_amd.generator import sweep

    steps = sweep()
    assert len(steps) == 242
    _check_batch(steps, ctx="sweep")


def test_config5_sweep_replicated(gpu):
    """The sweep replicated 10x: 2,420 blocks in one pass, every block bit-exact vs its step's oracle
    table; the slabs hold exactly the answered cells (2 bits per cell, 64-pod words per block row)."""
    from cyclonus_amd.generator import sweep

    steps = sweep()
    bt = _check_batch(steps, reps=10, ctx="sweep x10")
    assert len(bt.problems) == 2420
    words = int(bt.layout[-1][0])
    assert words == sum(n * k * w for n, k, w in (bt.slab_dims(b) for b in range(2420)))


def test_batch_random_blocks(gpu):
    """Random problems (panicking ones, duplicate job keys, every matcher feature) batched: each block
    reports exactly its stand-alone outcome, whatever its neighbours do."""
    probs = []
    for seed in range(300_000, 300_160):
        pols, res, probes = random_problem(seed, bad=seed % 3 == 0, dups=seed % 5 == 0)
        for pr in probes:
            probs.append({"policies": pols, "resources": res, "probe": pr})
    _check_batch(probs, ctx="random blocks")


def test_graph_and_eager_paths_agree(gpu):
    """Every launch path gives the same table: graph replay / re-capture, the DAG enqueued eagerly,
    eager with phase events, the fused front or the DAG, membership by wave or thread, pod-peer
    rows per pod or through word runs, IP rows with 1..64 peers per block."""
    import torch

    eng = Engine(0)
    for seed in range(30):
        pols, res, probes = random_problem(30_000 + seed, n_pods=50)
        eng.build_policies(pols).load_resources(res)
        sh = eng.prepare(probes)
        P, K, W = sh["pods"], sh["slots"], sh["words"]
        outs = []
        for graphs, fused, mw, pod_rows in ((0, 1, -1, -1), (1, 1, -1, -1), (1, 1, -1, -1), (2, 1, 1, 1), (1, 0, 0, 0),
                                            (2, 0, -1, 1), (0, 0, 1, 0), (-1, 1, 0, -1), (-1, 0, 1, 1)):
            eng.set_option("graphs", graphs)
            eng.set_option("front_fused", fused)
            eng.set_option("member_wave", mw)
            eng.set_option("pod_rows", pod_rows)
            eng.set_option("class_inplace", int(graphs != 2))  # class rows in the planes or in their own buffer
            d_in = torch.full((P, K, W), 7, dtype=torch.int64, device="cuda")
            d_eg = torch.full((P, K, W), 7, dtype=torch.int64, device="cuda")
            d_st = torch.zeros((P, K), dtype=torch.uint8, device="cuda")
            eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            outs.append((d_in.cpu(), d_eg.cpu(), d_st.cpu()))
        for o in outs[1:]:
            assert all(torch.equal(a, b) for a, b in zip(outs[0], o)), seed


def _ip_interval_problem(seed, n_pods=700):
    """Pods with address-ordered IPv4 / IPv6 / v4-mapped addresses in runs (so most 64-pod words
    are one interval, some straddle), and IPBlock peers whose CIDRs and excepts start and end on,
    inside and across word boundaries — exercises every branch of the per-word interval test."""
    import ipaddress

    rng = np.random.default_rng(seed)
    pods, fams = [], []
    for n in range(n_pods):
        run = (n // 96) % 3  # family runs that do not align with 64-pod words
        if rng.random() < 0.03:
            run = int(rng.integers(0, 3))  # a few stray addresses of another family
        fams.append(run)
        if run == 0:
            ip = str(ipaddress.IPv4Address((10 << 24) + 4 * n))
        elif run == 1:
            ip = str(ipaddress.IPv6Address((0xFD00 << 112) + 4 * n))
        else:
            ip = "::ffff:" + str(ipaddress.IPv4Address((10 << 24) + (1 << 16) + 4 * n))
        pods.append({"Namespace": "x", "Name": f"p{n}", "Labels": {"i": str(n % 7)}, "IP": ip,
                     "Containers": [{"Name": "c", "Port": 80, "Protocol": "TCP", "PortName": "serve-80-tcp"}]})
    res = {"Namespaces": {"x": {"ns": "x"}}, "Pods": pods}

    def cidr(fam, lo_pod, plen):
        if fam == 1:
            base = (0xFD00 << 112) + 4 * lo_pod
            net = ipaddress.IPv6Network((base >> (128 - plen) << (128 - plen), plen))
            return str(net)
        off = (1 << 16) if fam == 2 else 0
        base = (10 << 24) + off + 4 * lo_pod
        net = ipaddress.IPv4Network((base >> (32 - plen) << (32 - plen), plen))
        return str(net)

    pols = []
    for i in range(12):
        peers = []
        for _ in range(int(rng.integers(1, 4))):
            fam = int(rng.integers(0, 3))
            lo = int(rng.integers(0, n_pods))
            plen = int(rng.integers(20, 28)) if fam != 1 else int(rng.integers(116, 124))
            ib = {"cidr": cidr(fam, lo, plen)}
            ex = []
            for _ in range(int(rng.integers(0, 3))):
                eplen = min(plen + int(rng.integers(1, 6)), 32 if fam != 1 else 128)
                ex.append(cidr(fam, lo + int(rng.integers(0, 64)), eplen))
            if ex:
                ib["except"] = ex
            peers.append({"ipBlock": ib})
        spec = {"podSelector": {"matchLabels": {"i": str(i % 7)}}, "policyTypes": ["Ingress", "Egress"],
                "ingress": [{"from": peers}], "egress": [{"to": peers[::-1]}]}
        pols.append({"metadata": {"name": f"ipb{i}", "namespace": "x"}, "spec": spec})
    return pols, res, [{"AllAvailable": True}]


def _ip_stride_problem(seed, n_ns=6, per_ns=90):
    """Pod addresses that step by 256 inside a namespace (10.ns.j.1, config #2's shape: no word holds
    consecutive addresses) and IPBlocks from /16 with /24 excepts down to single pods, v4-mapped and
    IPv6 pods mixed in: IP rows built from the address index (ip_rows_range_blk) and by a test per
    word with straddling words tested a pod per lane."""
    rng = np.random.default_rng(seed)
    pods, nss = [], {}
    for i in range(n_ns):
        nss[f"n{i}"] = {"ns": f"n{i}"}
        for j in range(per_ns):
            u = rng.random()
            ip = f"10.{i}.{j}.1" if u < 0.8 else (f"::ffff:10.{i}.{j}.2" if u < 0.9 else f"fd00::{i:x}:{j:x}")
            pods.append({"Namespace": f"n{i}", "Name": f"p{j}", "Labels": {"i": str(j % 5)}, "IP": ip,
                         "Containers": [{"Name": "c", "Port": 80, "Protocol": "TCP", "PortName": "serve-80-tcp"}]})
    res = {"Namespaces": nss, "Pods": pods}
    pols = []
    for k in range(14):
        peers = []
        for _ in range(int(rng.integers(1, 4))):
            t, a, b = int(rng.integers(0, 4)), int(rng.integers(0, n_ns)), int(rng.integers(0, per_ns))
            if t == 0:
                ib = {"cidr": f"10.{a}.0.0/16", "except": [f"10.{a}.{b}.0/24", f"10.{a}.{(b + 7) % per_ns}.0/24"]}
            elif t == 1:
                ib = {"cidr": f"10.{a}.{b & ~15}.0/20"}
            elif t == 2:
                ib = {"cidr": f"10.{a}.{b}.1/32"}
            else:
                ib = {"cidr": "fd00::/64", "except": [f"fd00::{a:x}:0/112"]}
            peers.append({"ipBlock": ib})
        spec = {"podSelector": {"matchLabels": {"i": str(k % 5)}}, "policyTypes": ["Ingress", "Egress"],
                "ingress": [{"from": peers}], "egress": [{"to": peers[::-1]}]}
        pols.append({"metadata": {"name": f"s{k}", "namespace": f"n{k % n_ns}"}, "spec": spec})
    return pols, res, [{"AllAvailable": True}]


@pytest.mark.parametrize("seed", range(2))
def test_ip_interval_words(gpu, seed):
    """IP rows by a test per word (ip_range = 0), from the address index wherever an IPBlock matches
    few close pods (1), and by the auto rule (index only over non-affine words), on affine addresses
    and on addresses stepping by 256, with the fused front's IP rows as per-chunk work items (ip_items
    auto) or as groups of rows per wave (0), against the oracle."""
    for pols, res, probes in (_ip_interval_problem(seed), _ip_stride_problem(seed)):
        o = None  # the oracle's table, once per problem (every path below must give it)
        # (ip_items 0: a group of rows per wave; ip_iv 0: no pod-interval rows — the other paths run)
        for ipr, items, iv in ((-1, -1, -1), (-1, -1, 0), (0, -1, 0), (1, -1, 0), (0, 0, 0), (-1, 0, 0)):
            eng = Engine(0)
            eng.set_option("ip_range", ipr)
            eng.set_option("ip_items", items)
            eng.set_option("ip_iv", iv)
            assert eng.get_option("ip_range") == ipr
            if o is None:
                o, g = run_both(pols, res, probes, engine=eng)
            else:
                g = run_gpu(eng, pols, res, probes)
            assert_same(o, g, f"ip intervals seed {seed} ip_range {ipr} ip_items {items} ip_iv {iv}")
            for opts in ({"front_fused": 0}, {"graphs": 0}):
                for k, v in opts.items():
                    eng.set_option(k, v)
                assert_same(o, run_gpu(eng, pols, res, probes), f"ip intervals seed {seed} ip_range {ipr} {opts}")


def _ip_mono_problem(seed, n_pods=9000, wide=False):
    """Addresses handed out in pod order per family (IPv4, v4-mapped sharing the IPv4 counter, IPv6),
    families interleaved pod by pod, with gaps and repeated addresses; 141 words over 3 chunks.
    IPBlocks of every prefix length around random pods, with 0-20 nested excepts (more than IPV_MAX
    intervals falls back to the other IP-row paths), edge networks (0.0.0.0/0, ::/0, ::ffff:0:0/96)."""
    import ipaddress

    rng = np.random.default_rng(seed)
    a4, a6 = 0, 0
    pods, at4, at6 = [], [], []
    for n in range(n_pods):
        u = rng.random()
        step = int(rng.choice([0, 1, 1, 1, 2, 7]))  # 0: the previous pod's address again
        if u < 0.45 or u >= 0.9:
            a4 += step
            v4 = ipaddress.IPv4Address((10 << 24) + a4)
            ip = str(v4) if u < 0.45 else "::ffff:" + str(v4)
            at4.append(a4)
        else:
            a6 += step
            ip = str(ipaddress.IPv6Address((0xFD00 << 112) + a6))
            at6.append(a6)
        pods.append({"Namespace": "x", "Name": f"p{n}", "Labels": {"i": str(n % 7)}, "IP": ip,
                     "Containers": [{"Name": "c", "Port": 80, "Protocol": "TCP", "PortName": "serve-80-tcp"}]})
    res = {"Namespaces": {"x": {"ns": "x"}}, "Pods": pods}

    def net(v6, center, plen):
        if v6:
            base = (0xFD00 << 112) + center
            return str(ipaddress.IPv6Network((base >> (128 - plen) << (128 - plen), plen)))
        base = (10 << 24) + center
        return str(ipaddress.IPv4Network((base >> (32 - plen) << (32 - plen), plen)))

    pols = []
    for k in range(24):
        peers = []
        for _ in range(int(rng.integers(1, 4))):
            v6 = rng.random() < 0.4
            addrs = at6 if v6 else at4
            center = int(addrs[int(rng.integers(0, len(addrs)))])
            bits = 128 if v6 else 32
            plen = bits - int(rng.integers(0, 15))
            cidr = net(v6, center, plen)
            ex = []
            for _ in range(int(rng.choice([0, 1, 2, 3, 20]))):
                ec = center + int(rng.integers(-(1 << max(bits - plen - 1, 0)), 1 << max(bits - plen - 1, 0)))
                ex.append(net(v6, max(ec, 0), min(bits, plen + int(rng.integers(1, 8)))))
            if rng.random() < 0.1:
                cidr, ex = str(rng.choice(["0.0.0.0/0", "::/0", "::ffff:0:0/96"])), ex[:2]
            peers.append({"ipBlock": {"cidr": cidr, "except": ex} if ex else {"cidr": cidr}})
        spec = {"podSelector": {"matchLabels": {"i": str(k % 7)}}, "policyTypes": ["Ingress", "Egress"],
                "ingress": [{"from": peers}], "egress": [{"to": peers[::-1]}]}
        pols.append({"metadata": {"name": f"m{k}", "namespace": "x"}, "spec": spec})
    if wide:  # one policy of every pod with 48 IPBlocks of 10-15 excepts (rows of many intervals)
        peers = []
        for _ in range(48):
            v6 = rng.random() < 0.4
            addrs = at6 if v6 else at4
            center, bits = int(addrs[int(rng.integers(0, len(addrs)))]), 128 if v6 else 32
            plen = bits - 12
            ex = [net(v6, max(center + int(rng.integers(-2048, 2048)), 0), plen + int(rng.integers(4, 10)))
                  for _ in range(int(rng.integers(10, 16)))]
            peers.append({"ipBlock": {"cidr": net(v6, center, plen), "except": ex}})
        spec = {"podSelector": {}, "policyTypes": ["Ingress", "Egress"], "ingress": [{"from": peers}],
                "egress": [{"to": peers}]}
        pols.append({"metadata": {"name": "wide", "namespace": "x"}, "spec": spec})
    return pols, res, [{"AllAvailable": True}]


@pytest.mark.parametrize("seed,wide", [(0, False), (1, False), (2, True)])
def test_ip_pod_interval_rows(gpu, seed, wide):
    """IP rows as pod intervals (ip_iv, address-monotone families): whole planes equal the other IP-row
    paths' (ip_iv 0, pinned to the oracle by the tests above) through the fused front, the DAG and the
    eager launches, on the whole table and on source and target shards; sampled rows against the
    oracle.  wide: rows of 10-16 intervals in every class (an all-pods policy with 48 IPBlocks)."""
    pols, res, probes = _ip_mono_problem(seed, wide=wide)
    eng = Engine(0).build_policies(pols).load_resources(res)
    sh = eng.prepare(probes)
    P, K = sh["pods"], sh["slots"]
    ref = Engine(0).build_policies(pols).load_resources(res)
    ref.prepare(probes)
    ref.set_option("ip_iv", 0)
    orc = Oracle(pols, res)
    for part, lo, hi in (("target", 0, P), ("source", 0, 4096), ("source", 4096, P), ("target", 1000, 5000)):
        want = ref.run_host(lo, hi, part)
        for opts in ({}, {"front_fused": 0}, {"graphs": 0}, {"graphs": 1}):
            for k, v in {"front_fused": 1, "graphs": -1, **opts}.items():
                eng.set_option(k, v)
            got = eng.run_host(lo, hi, part)
            assert eng.get_option("ip_iv_rows") > 0
            for name, a, b in zip(("status", "ingress", "egress"), want, got):
                assert np.array_equal(a, b), f"seed {seed} {part} [{lo}, {hi}) {opts}: {name} plane differs"
        if part == "target" and lo == 0:
            for pod in (0, 63, 64, 4095, 4096, P // 2, P - 1):
                for k in range(K):
                    assert np.array_equal(got[1][pod, k], orc.row(probes, "ingress", pod, k)), (seed, pod, k)
                    assert np.array_equal(got[2][pod, k], orc.row(probes, "egress", pod, k)), (seed, pod, k)


@pytest.mark.parametrize("seed", range(4))
def test_row_phases(gpu, seed):
    """A whole table whose class rows and emit run in two row phases (the classes rows [0, P/2) use, the
    emit of those rows, then the other classes and the emit of rows [P/2, P)) equals the single pass,
    through every launch mode (graph replays included: the election re-lists each replay's phases), on
    target and whole-range source runs, for identity-set and materialised-row (PM) builds."""
    pols, res, probes = random_problem(91_000 + seed, n_pods=300 + 97 * seed, n_pols=10 + 3 * seed)
    eng = Engine(0).build_policies(pols).load_resources(res)
    eng.prepare(probes)
    if eng.shape["may_panic"]:
        pytest.skip("a build that may panic never splits")
    want = eng.run_host()
    want_classes = eng.classes()
    assert eng.get_option("row_phases_active") == 0  # (auto: only from 8 GB planes up)
    eng.set_option("row_phases", 2)
    for pod_words in (-1, 0):
        eng.set_option("pod_words", pod_words)
        for graphs in (-1, 1, 0):
            eng.set_option("graphs", graphs)
            for rep in range(2):
                for part in ("target", "source"):
                    got = eng.run_host(0, None, part)
                    if eng.get_option("front_fused_active"):
                        assert eng.get_option("row_phases_active") == 2
                        assert eng.last_emit()[1] == 2, eng.last_emit()
                        # both phases' representative lists (head and tail) hold every class once
                        assert eng.classes() == want_classes, (eng.classes(), want_classes)
                    for name, a, b in zip(("status", "ingress", "egress"), want, got):
                        assert np.array_equal(a, b), (f"seed {seed} pod_words {pod_words} graphs {graphs} {part} rep {rep}: "
                                                      f"{name} differs")
    eng.set_option("graphs", 0)
    eng.run_host()
    t = eng.timings()
    assert t[0] > 0 and t[1] > 0 and t[2] >= 0, t
    eng.run_host(0, 100)  # a row range never splits
    assert eng.get_option("row_phases_active") == 0
    for v in (0, 3):
        with pytest.raises(Exception):
            eng.set_option("row_phases", v)


def _shared_ipblock_problem(seed, bad=False):
    """Policies whose peers reuse a small pool of IPBlocks (equal cidr / except strings) on different
    ports and in both directions: the run plan builds ONE IP row per IPBlock and direction, and every
    peer (class rows, identity-set lists, the panic describer) reads it through peer_row.  bad: the
    pool also holds an unparsable CIDR (ipaddress.go panics when a cell reaches it)."""
    pols, res, probes = _ip_interval_problem(seed)
    rng = np.random.default_rng(seed + 100)
    pool = [p["ipBlock"] for pol in pols for p in pol["spec"]["ingress"][0]["from"]][:5]
    pool.append({"cidr": "0.0.0.0/0"})
    if bad:
        pool.append({"cidr": "10.0.0.0/33"})
    ports = [[{"port": 80, "protocol": "TCP"}], [{"port": 81, "protocol": "TCP"}], [{"port": "serve-80-tcp"}], None]
    for i in range(10):
        blocks = [pool[int(x)] for x in rng.integers(0, len(pool), 3)]
        ing = {"from": [{"ipBlock": b} for b in blocks]}
        eg = {"to": [{"ipBlock": b} for b in blocks[::-1]]}
        pp = ports[i % len(ports)]
        if pp:
            ing["ports"] = pp
            eg["ports"] = pp
        spec = {"podSelector": {"matchLabels": {"i": str(i % 7)}}, "policyTypes": ["Ingress", "Egress"],
                "ingress": [ing], "egress": [eg]}
        pols.append({"metadata": {"name": f"shared{i}", "namespace": "x"}, "spec": spec})
    return pols, res, probes


@pytest.mark.parametrize("seed", range(3))
def test_shared_ipblock_rows(gpu, seed):
    for bad in (False, True):
        pols, res, probes = _shared_ipblock_problem(seed, bad)
        o, g = run_both(pols, res, probes)
        assert_same(o, g, f"shared IPBlocks seed {seed} bad {bad}")
        for opts in ({"front_fused": 0}, {"pod_words": 0}, {"pl_wave": 0}, {"graphs": 0}):
            eng = Engine(0)
            for k, v in opts.items():
                eng.set_option(k, v)
            o2, g2 = run_both(pols, res, probes, engine=eng)
            assert_same(o2, g2, f"shared IPBlocks seed {seed} bad {bad} {opts}")


def test_pm_class_rows_wave_and_items(gpu):
    """PM-build class rows (pod_words = 0) a wave per 64-word chunk (pl_wave = 1: <= 4 slots and
    descriptors) and a thread per item (pl_wave = 0), over sparse pod-peer rows built by either block
    shape with lazy or dense selectors, against the oracle: IP-interval problems (IP
    rows with skipped and straddling chunks) and random problems, which include classes with more
    list entries than the LDS part holds only at sizes the oracle cannot check — those run through
    tests/test_gpu_fullrows.py."""
    eng = Engine(0)
    seen_wave = 0
    seen_plvt = [0, 0]  # runs without / with the per-pod label table
    problems = [_ip_interval_problem(s, n_pods=300 + 97 * s) for s in range(3)]
    problems += [random_problem(95_000 + s, n_pods=120) for s in range(40)]
    for n, (pols, res, probes) in enumerate(problems):
        want = Oracle(pols, res).probe(probes)
        try:
            eng.build_policies(pols).load_resources(res)
            eng.prepare(probes)
        except CyclonusPanic:
            continue
        eng.set_option("pod_words", 0)
        for wave in (1, 0):
            eng.set_option("pl_wave", wave)
            assert_same(want, eng.run_host(), f"problem {n} pl_wave={wave}")
        eng.set_option("pl_wave", 1)
        # sparse pod-peer rows a block per peer or a wave per chunk over peer groups, selectors
        # evaluated where used or as the dense table first
        # (per-pod label table PLVT, or pod -> label set -> LVT gathers when it is not built)
        for grp, lazy, wave, plvt in ((1, 1, 1, 1024), (8, 0, 1, 0), (3, 1, 0, 0), (64, -1, 1, 1024), (2, 0, 0, 0),
                                      (1, 1, 0, 0)):
            eng.set_option("pr_group", grp)
            eng.set_option("sel_lazy", lazy)
            eng.set_option("pl_wave", wave)  # sparse rows read per word (spans + chunk flags) or per chunk
            eng.set_option("plvt_max_mb", plvt)
            assert_same(want, eng.run_host(), f"problem {n} pr_group={grp} sel_lazy={lazy} pl_wave={wave} plvt={plvt}")
            seen_plvt[eng.get_option("plvt_active")] += plvt == 0 or eng.get_option("plvt_active") == 1
        eng.set_option("plvt_max_mb", 1024)
        eng.set_option("pr_group", -1)
        eng.set_option("sel_lazy", -1)
        eng.set_option("pl_wave", 1)
        seen_wave += eng.get_option("pl_wave_active")
    assert seen_wave >= 10
    assert min(seen_plvt) >= 10, seen_plvt


def _deployment_problem(seed, min_run=22):
    """Random policies over deployment-style pods: each random pod template is replicated into a
    contiguous run of >= min_run pods (same namespace, labels and containers; own name and IP),
    so every 64-pod word holds at most 4 identity runs and the class rows can expand pod-peer
    words from per-identity outcomes (cyc_set_option pod_words = 1)."""
    import random

    r = random.Random(seed)
    pols, res, probes = random_problem(40_000 + seed, n_pods=int(r.randint(3, 12)))
    pods = []
    for t, tpl in enumerate(res["Pods"]):
        for j in range(r.randint(min_run, min_run + 40)):
            q = dict(tpl)
            q["Name"] = f"{tpl['Name']}-{j}"
            q["IP"] = f"10.1.{len(pods) // 250}.{len(pods) % 250}" if r.random() < 0.9 else tpl["IP"]
            pods.append(q)
    res = dict(res, Pods=pods)
    return pols, res, probes


@pytest.mark.parametrize("seed", range(24))
def test_pod_words_from_identity_runs(gpu, seed):
    """Class rows with pod-peer words expanded from identity outcomes (IDO) and from
    materialised peer rows (PM) both equal the oracle, on the graph and the eager path."""
    pols, res, probes = _deployment_problem(seed)
    want = Oracle(pols, res).probe(probes)
    eng = Engine(0).build_policies(pols).load_resources(res)
    eng.prepare(probes)
    # (pod_words, graphs, front_fused, member_wave, class_rpb): graph and eager paths, the fused
    # single-stream front and the two-branch DAG (replayed and enqueued eagerly), membership by wave
    # or thread, several class representatives per class-row block, and the PM path
    for mode, graphs, fused, mw, rpb in ((1, 1, 1, -1, 1), (1, 1, 1, 1, 3), (1, 1, 1, 0, 4), (1, 1, 0, -1, 2),
                                         (1, 2, 1, 0, 1), (1, 2, 0, 1, 5), (1, 0, 1, -1, 2), (1, 0, 0, -1, 3),
                                         (1, -1, 1, -1, 16), (1, 2, 1, -1, 0), (0, 1, 1, -1, 1), (0, 0, 1, -1, 1), (0, 2, 0, 1, 1)):
        eng.set_option("pod_words", mode)
        eng.set_option("graphs", graphs)
        eng.set_option("front_fused", fused)
        eng.set_option("member_wave", mw)
        eng.set_option("class_rpb", rpb)
        assert eng.get_option("pod_words") == mode, "deployment-style words must allow the IDO path"
        for rep in range(2):  # the second run finds the hash tables the first one emptied
            assert_same(want, eng.run_host(), f"seed {seed} pod_words {mode} graphs {graphs} "
                                              f"fused {fused} member_wave {mw} rpb {rpb} run {rep}")


def _many_ip_peers(seed):
    """Deployment-style pods plus policies whose rules list 17-40 IPBlock peers each (more than the
    IDO class rows stage per representative, IDO_IPL = 16), with mixed numbered / named / no ports,
    over both directions: the staged and the global IP-peer walks both run."""
    import random

    r = random.Random(1000 + seed)
    pols, res, probes = _deployment_problem(seed)
    nss = sorted({p["Namespace"] for p in res["Pods"]})
    ports = [None, [{"port": 80, "protocol": "TCP"}], [{"port": "serve-53-udp", "protocol": "UDP"}],
             [{"port": 81, "protocol": "SCTP"}, {"port": 53, "protocol": "UDP"}]]
    for i in range(6):
        def peers():
            out = []
            for _ in range(r.randint(17, 40)):
                plen = r.choice([16, 20, 24, 26, 28, 30, 32])
                blk = {"cidr": f"10.1.{r.randint(0, 4)}.{r.randint(0, 249)}/{plen}"}
                if plen <= 28 and r.random() < 0.3:
                    blk["except"] = [f"10.1.{r.randint(0, 4)}.{r.randint(0, 249)}/32"]
                out.append({"ipBlock": blk})
            return out

        ing, eg = {"from": peers()}, {"to": peers()}
        pp = r.choice(ports)
        if pp:
            ing["ports"], eg["ports"] = pp, pp
        pols.append({"apiVersion": "networking.k8s.io/v1", "kind": "NetworkPolicy",
                     "metadata": {"name": f"many-ip-{i}", "namespace": r.choice(nss)},
                     "spec": {"podSelector": {}, "policyTypes": ["Ingress", "Egress"], "ingress": [ing], "egress": [eg]}})
    return pols, res, probes


@pytest.mark.parametrize("seed", range(6))
def test_ido_many_ip_peers(gpu, seed):
    """IDO class rows with more IP peers per class than are staged in LDS: equal to the oracle for
    one and several representatives per block, fused and DAG fronts."""
    pols, res, probes = _many_ip_peers(seed)
    want = Oracle(pols, res).probe(probes)
    eng = Engine(0).build_policies(pols).load_resources(res)
    eng.prepare(probes)
    for fused, rpb in ((1, 4), (1, 1), (0, 3)):
        eng.set_option("pod_words", 1)
        eng.set_option("front_fused", fused)
        eng.set_option("class_rpb", rpb)
        assert eng.get_option("pod_words") == 1
        assert_same(want, eng.run_host(), f"seed {seed} fused {fused} rpb {rpb}")


def _wide_ports_problem(seed, n_pods=150):
    """Pods with many containers (AllAvailable: > 32 job slots per pod) over > 32 distinct job
    descriptors, so the descriptor bit rows (<= 32) and the slot-bit list entries (<= 32) do not
    apply: the class rows take their byte-table port checks.  Policies mix numbered, named and
    ranged ports with pod and IPBlock peers."""
    import random

    r = random.Random(seed)
    pols, res, _ = random_problem(60_000 + seed, n_pods=n_pods, n_pols=14)
    protos = ["TCP", "UDP", "SCTP"]
    for i, p in enumerate(res["Pods"]):
        conts = []
        for j, (port, proto) in enumerate(r.sample([(7000 + x, pr) for x in range(25) for pr in protos], r.randint(33, 44))):
            # distinct (protocol, port) per pod: AllAvailable job keys must not collide (table.go)
            conts.append({"Name": f"c{j}", "Port": port, "Protocol": proto, "PortName": f"p{port}-{proto.lower()}"})
        p["Containers"] = conts
    for k, pol in enumerate(pols):
        spec = pol.get("spec") or {}
        for key, peer_key in (("ingress", "from"), ("egress", "to")):
            for rule in spec.get(key) or []:
                if rule is None or r.random() < 0.3:
                    continue
                rule["ports"] = [{"port": 7000 + r.randint(0, 24), "protocol": protos[r.randint(0, 2)]},
                                 {"port": f"p{7000 + r.randint(0, 24)}-tcp"},
                                 {"port": 7010, "endPort": 7010 + r.randint(0, 8), "protocol": "UDP"}][: r.randint(1, 3)]
    return pols, res, [{"AllAvailable": True}, {"Port": 7003, "Protocol": "TCP"}]


@pytest.mark.parametrize("seed", range(4))
def test_wide_ports(gpu, seed):
    """> 32 job slots and > 32 job descriptors through every class-row path (identity sets, PM
    rows by item walk; the wave-per-chunk rows do not apply) against the oracle."""
    pols, res, probes = _wide_ports_problem(seed)
    want = Oracle(pols, res).probe(probes)
    eng = Engine(0).build_policies(pols).load_resources(res)
    sh = eng.prepare(probes)
    assert sh["slots"] > 32 and sh["descriptors"] > 32, sh
    for pod_words, fused in ((0, 1), (0, 0), (1, 1), (-1, 1)):
        eng.set_option("pod_words", pod_words)
        eng.set_option("front_fused", fused)
        assert eng.get_option("pl_wave_active") == 0
        assert_same(want, eng.run_host(), f"seed {seed} pod_words {pod_words} fused {fused}")


@pytest.mark.parametrize("seed", range(6))
def test_edge_shapes(gpu, seed):
    """Empty and ragged inputs, as the reference's tables allow them: no pods, one pod, pod counts
    on and around 64-pod word boundaries, no policies, no probes, and pods without containers
    (AllAvailable yields no job for them, resources.go:336-364)."""
    pols, res, probes = random_problem(60_000 + seed, n_pods=200)
    eng = Engine(0)
    for n in (0, 1, 2, 63, 64, 65, 127, 128, 129, 200):
        r = dict(res, Pods=res["Pods"][:n])
        assert_same(*run_both(pols, r, probes, engine=eng), f"seed {seed} pods {n}")
    assert_same(*run_both([], res, probes, engine=eng), f"seed {seed} no policies")
    assert_same(*run_both(pols, res, [], engine=eng), f"seed {seed} no probes")
    bare = [dict(p, Containers=[]) if i % 3 == 0 else p for i, p in enumerate(res["Pods"][:70])]
    assert_same(*run_both(pols, dict(res, Pods=bare), probes + [{"AllAvailable": True}], engine=eng),
                f"seed {seed} pods without containers")


@pytest.mark.parametrize("bad", [False, True])
def test_direct_pod_rows_and_membership(gpu, bad):
    """Pod-peer rows computed per pod (pod_rows = 1) and through identity runs (0), membership by
    wave or by thread, on growing problems (the emit picks its kernel by row length: 8-byte copies
    for odd word counts, the flat multi-row sweep, single-pass blocks): all equal the oracle,
    panics too."""
    eng = Engine(0)
    for seed in range(40):
        pols, res, probes = random_problem(70_000 + seed, n_pods=30 + 7 * seed, bad=bad)
        try:
            want = Oracle(pols, res).probe(probes)
        except OraclePanic as e:
            want = Panicked(str(e))
        eng.build_policies(pols).load_resources(res)
        for pod_rows, mw in ((1, 1), (0, 0), (1, 0), (0, 1)):
            eng.set_option("pod_rows", pod_rows)
            eng.set_option("member_wave", mw)  # membership: a wave (1) or a thread (0) per identity
            try:
                eng.prepare(probes)
                got = eng.run_host()
            except CyclonusPanic as e:
                got = Panicked(e.msg)
            assert_same(want, got, f"seed {seed} pod_rows {pod_rows} member_wave {mw}")


def test_emit_row_lengths(gpu):
    """The emit kernels by plane-row length (K x W words): odd word counts (8-byte copies), short
    rows (flat multi-row sweep), 16-64 KB rows (256-thread single pass) and >= 64 KB rows
    (512-thread single pass), each bit-exact vs the oracle on sampled cells and whole rows."""
    from cyclonus_amd import synth

    for n_ns, probes in ((3, [{"Port": 80, "Protocol": "TCP"}]), (10, [{"AllAvailable": True}]),
                         (20, [{"AllAvailable": True}] * 1), (50, [{"AllAvailable": True}])):
        data = synth.config3(n_ns=n_ns)
        data["probes"] = probes
        pols, res = data["policies"], data["resources"]
        eng = Engine(0).build_policies(json.dumps(pols)).load_resources(json.dumps(res))
        sh = eng.prepare(probes)
        st, ing, eg = eng.run_host()
        orc = Oracle(pols, res)
        P, K = sh["pods"], sh["slots"]
        rng = np.random.default_rng(n_ns)
        for pod in [0, P - 1] + [int(x) for x in rng.integers(0, P, 6)]:
            for k in range(K):
                assert np.array_equal(ing[pod, k], orc.row(probes, "ingress", pod, k, threads=8)), (n_ns, pod, k)
                assert np.array_equal(eg[pod, k], orc.row(probes, "egress", pod, k, threads=8)), (n_ns, pod, k)


def test_graph_joins_without_status_or_rows(gpu):
    """Captured graphs for steps without a status plane (null pointer) or without rows (an empty
    row range), on the fused front and the DAG, replayed and re-captured: results unchanged."""
    import torch

    pols, res, probes = random_problem(90_001, n_pods=120)
    want = Oracle(pols, res).probe(probes)
    eng = Engine(0).build_policies(pols).load_resources(res)
    sh = eng.prepare(probes)
    P, K, W = sh["pods"], sh["slots"], sh["words"]
    st = torch.cuda.current_stream().cuda_stream
    eng.set_option("graphs", 1)
    for merged in (1, 0):  # fused front / DAG
        eng.set_option("front_fused", merged)
        for _ in range(3):  # replays of the same graph
            d_in = torch.zeros((P, K, W), dtype=torch.int64, device="cuda")
            d_eg = torch.zeros((P, K, W), dtype=torch.int64, device="cuda")
            eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), 0, st)
            eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), 0, st, 7, 7)
            torch.cuda.synchronize()
            assert np.array_equal(d_in.cpu().numpy().view(np.uint64), want[1]), f"merged {merged}"
            assert np.array_equal(d_eg.cpu().numpy().view(np.uint64), want[2]), f"merged {merged}"


def test_launch_modes_and_knobs(gpu):
    """The default launch is the fused front enqueued eagerly (graphs auto = 2) when no panic is
    possible and the graph of the two-branch DAG otherwise; tuning knobs round-trip and reject
    out-of-range values; the fused front's results equal the oracle's, run after run, also when
    switched off and on between runs (hash tables and IP spans are left clean for the next run)."""
    pols, res, probes = random_problem(91_000, n_pods=150)
    want = Oracle(pols, res).probe(probes)
    eng = Engine(0).build_policies(pols).load_resources(res)
    eng.prepare(probes)
    assert eng.get_option("graphs") == -1
    fused = not eng.shape["may_panic"]  # no-panic build: the fused front applies
    assert eng.get_option("front_fused_active") == int(fused)
    assert eng.get_option("launch") == (2 if fused else 1)
    for name, v in (("front_fused", 0), ("front_fused", 1), ("class_rpb", 7), ("class_rpb", 16), ("class_rpb", 0), ("graphs", 1), ("graphs", -1),
                    ("step_events", 1), ("step_events", 0), ("pr_group", 5), ("pr_group", -1), ("sel_lazy", 1),
                    ("sel_lazy", -1), ("class_inplace", 0), ("class_inplace", 1), ("class_inplace", -1),
                    ("emit_interleave", 1), ("emit_interleave", 0), ("emit_interleave", -1),
                    ("ip_items", 0), ("ip_items", 1), ("ip_items", -1), ("ip_iv", 0), ("ip_iv", -1)):
        eng.set_option(name, v)
        assert eng.get_option(name) == v
        assert_same(want, eng.run_host(), f"{name}={v}")
        assert eng.last_emit()[1] == 1, eng.last_emit()  # cyc_last_emit: one emit launch a run
    # whole-step timing events: off by default for graph / fused-eager runs, always for eager runs
    with pytest.raises(Exception):
        eng.timings()
    eng.set_option("step_events", 1)
    eng.run_host()
    assert eng.timings()[0] > 0
    eng.set_option("step_events", 0)
    eng.set_option("graphs", 0)
    eng.run_host()
    assert all(t >= 0 for t in eng.timings())
    eng.set_option("graphs", -1)
    eng.set_option("front_fused", 0)
    assert eng.get_option("front_fused_active") == 0 and eng.get_option("launch") == 1
    assert_same(want, eng.run_host(), "DAG graph")
    eng.set_option("front_fused", 1)
    assert_same(want, eng.run_host(), "fused again")
    for name, v in (("class_rpb", -1), ("class_rpb", 65), ("ip_range", 2), ("ip_group", 8), ("graphs", 3), ("pr_group", 65), ("sel_lazy", 2), ("emit_variant", 1),
                    ("emit_split", 2), ("emit_interleave", 2), ("emit_prefetch", 1), ("emit_sweep", 16), ("ip_items", 2), ("emit_buf", 1),
                    ("ip_iv", 2), ("emit_footprint", 2), ("emit_rows", 1),
                    ("nope", 0)):
        with pytest.raises(Exception):
            eng.set_option(name, v)
    # a build that may panic keeps the graph path (the panic walk needs the ordered peer rows)
    pols_b, res_b, probes_b = random_problem(81_003, n_pods=60, bad=True)
    eng_b = Engine(0).build_policies(pols_b).load_resources(res_b)
    try:
        eng_b.prepare(probes_b)
    except CyclonusPanic:
        return
    if eng_b.shape.get("may_panic"):
        assert eng_b.get_option("front_fused_active") == 0


def test_batch_cross_block_panic_isolated(gpu):
    """Block B holds a pod with an unparsable IP and no IPBlock rule; block A has an IPBlock peer.
    Neither panics alone (cross-block cells are never computed); a block that panics alone (C)
    reports its own panic, and its neighbours their own tables."""
    from cyclonus_amd.batch import Batch

    def pod(ns, name, ip):
        return {"Namespace": ns, "Name": name, "Labels": {"app": name}, "IP": ip,
                "Containers": [{"Name": "c", "Port": 80, "Protocol": "TCP", "PortName": "serve-80-tcp"}]}

    a = {"policies": [{"metadata": {"name": "ipb", "namespace": "x"},
                       "spec": {"podSelector": {}, "policyTypes": ["Ingress"],
                                "ingress": [{"from": [{"ipBlock": {"cidr": "10.0.0.0/8"}}]}]}}],
         "resources": {"Namespaces": {"x": {"ns": "x"}}, "Pods": [pod("x", "a", "10.0.0.1"), pod("x", "b", "10.0.0.2")]},
         "probe": {"Port": 80, "Protocol": "TCP"}}
    b = {"policies": [{"metadata": {"name": "deny", "namespace": "y"},
                       "spec": {"podSelector": {"matchLabels": {"app": "c"}}, "policyTypes": ["Ingress"]}}],
         "resources": {"Namespaces": {"y": {"ns": "y"}}, "Pods": [pod("y", "c", "not-an-ip"), pod("y", "d", "10.1.0.1")]},
         "probe": {"Port": 80, "Protocol": "TCP"}}
    c = {"policies": a["policies"], "resources": {"Namespaces": {"x": {}}, "Pods": [pod("x", "e", "bad"), pod("x", "f", "10.0.0.9")]},
         "probe": {"AllAvailable": True}}
    eng = Engine(0)
    got = Batch([a, b, c, a]).run(eng)
    for blk, g in zip((a, b, c, a), got):
        try:
            want = Oracle(blk["policies"], blk["resources"]).probe([blk["probe"]])
        except OraclePanic as e:
            want = Panicked(str(e))
        assert_same(want, Panicked(g.msg) if isinstance(g, CyclonusPanic) else g, blk["resources"]["Pods"][0]["Name"])
    assert isinstance(got[2], CyclonusPanic) and not isinstance(got[0], CyclonusPanic) and not isinstance(got[3], CyclonusPanic)


def test_row_entry_points_refuse_block_contexts(gpu):
    """A context prepared for batched blocks holds per-block slabs: the row-plane entry points
    (cyc_probe_run_rows / run_host_rows / table_run_rows / table_wrap_rows / rows_layout) refuse it
    with CYC_ERR_ARG instead of writing slabs sized by the row layout."""
    import torch

    from cyclonus_amd.batch import Batch

    steps = []
    for seed in (5, 6):
        pols, res, probes = random_problem(310_000 + seed, n_pods=40)
        steps.append({"policies": pols, "resources": res, "probe": probes[0]})
    eng = Engine(0)
    Batch(steps).prepare(eng)
    for call in (lambda: eng.run_host(0, 10), lambda: eng.layout(0, 10), lambda: eng.table(0, 10),
                 lambda: eng.run_host(0, 64, "source")):
        with pytest.raises(CyclonusError, match="blocks"):
            call()
    buf = torch.zeros(1 << 16, dtype=torch.int64, device="cuda")
    st = torch.zeros(1 << 12, dtype=torch.uint8, device="cuda")
    with pytest.raises(CyclonusError, match="blocks"):
        eng.run_device(buf.data_ptr(), buf.data_ptr(), st.data_ptr(), torch.cuda.current_stream().cuda_stream, 0, 10)
    with pytest.raises(CyclonusError, match="blocks"):
        eng.wrap_table(buf.data_ptr(), buf.data_ptr(), st.data_ptr(), 0, 10)


def _long_class_problem(seed, n_peers=300, n_pods=260):
    """One ingress target (and one egress target) whose peer list is longer than the class-row
    kernel's LDS part (> 256 entries) on a PM build with 5-32 job slots: the entries past the LDS
    part are read back from the spill list, each carrying its slot bits (they were read
    as a port matcher id).  Peers are pod selectors of one label value each (so none merge under
    Simplify), IPBlocks and ports-only rules, on numbered, named and ranged ports."""
    rng = np.random.default_rng(seed)
    ports = [(80, "TCP"), (81, "TCP"), (53, "UDP"), (443, "TCP"), (9000, "SCTP"), (8080, "TCP")]
    pods = []
    for q in range(n_pods):
        conts = [{"Name": f"c{j}", "Port": p, "Protocol": pr, "PortName": f"serve-{p}-{pr.lower()}"}
                 for j, (p, pr) in enumerate(ports)]
        pods.append({"Namespace": "x" if q % 5 else "y", "Name": f"p{q}", "Labels": {"i": str(q % n_peers), "g": str(q % 3)},
                     "IP": f"10.0.{q // 200}.{q % 200}", "Containers": conts})
    res = {"Namespaces": {"x": {"ns": "x"}, "y": {"ns": "y"}}, "Pods": pods}
    peers = []
    for n in range(n_peers):
        kind = rng.random()
        if kind < 0.8:
            peer = {"podSelector": {"matchLabels": {"i": str(n)}}}
            if rng.random() < 0.3:
                peer["namespaceSelector"] = {}
        else:
            peer = {"ipBlock": {"cidr": f"10.0.{int(rng.integers(0, 2))}.{int(rng.integers(0, 25)) * 8}/29"}}
        peers.append(peer)
    rules = []
    for x in range(0, n_peers, 20):
        p, pr = ports[int(rng.integers(0, len(ports)))]
        port = [{"port": p, "protocol": pr}, {"port": f"serve-{p}-{pr.lower()}", "protocol": pr},
                {"port": 80, "endPort": 444, "protocol": "TCP"}][int(rng.integers(0, 3))]
        rules.append({"from": peers[x:x + 20], "ports": [port]})
    pols = [{"metadata": {"name": "long", "namespace": "x"},
             "spec": {"podSelector": {"matchLabels": {"g": "1"}}, "policyTypes": ["Ingress", "Egress"],
                      "ingress": rules, "egress": [{"to": r["from"], "ports": r["ports"]} for r in rules]}}]
    return pols, res, [{"AllAvailable": True}]


@pytest.mark.parametrize("seed", range(2))
def test_long_class_lists_pm_items(gpu, seed):
    pols, res, probes = _long_class_problem(seed)
    for simplify in (True, False):
        want = Oracle(pols, res, simplify).probe(probes)
        eng = Engine(0).build_policies(pols, simplify).load_resources(res)
        sh = eng.prepare(probes)
        assert 5 <= sh["slots"] <= 32, sh
        eng.set_option("pod_words", 0)  # PM build: flattened peer lists in the class rows
        for wave in (0, 1):  # pl_wave does not apply with 6 slots: both settings take the item walk
            eng.set_option("pl_wave", wave)
            assert eng.get_option("pl_wave_active") == 0
            for fused in (1, 0):
                eng.set_option("front_fused", fused)
                assert_same(want, eng.run_host(), f"seed {seed} simplify {simplify} pl_wave {wave} fused {fused}")


def _source_shards_equal(eng, full, worlds, ctx):
    """Every source shard of every partition size equals the full table's slices: its sources'
    egress rows, and the words of its sources in every destination's ingress row."""
    from cyclonus_amd.shard import source_range

    st, ing, eg = full
    P = st.shape[0]
    for world in worlds:
        for rank in range(world):
            lo, hi = source_range(P, world, rank)
            st2, ing2, eg2 = eng.run_host(lo, hi, "source")
            w0, wa = lo // 64, ing2.shape[2]
            assert ing2.shape[0] == P and eg2.shape[0] == hi - lo, (ctx, world, rank, ing2.shape, eg2.shape)
            assert np.array_equal(st, st2), (ctx, world, rank)
            assert np.array_equal(ing[:, :, w0:w0 + wa], ing2), f"{ctx}: ingress slice of source shard {rank}/{world}"
            assert np.array_equal(eg[lo:hi], eg2), f"{ctx}: egress rows of source shard {rank}/{world}"


def test_source_rows_random(gpu):
    """Source-row runs (CYC_ROWS_SOURCE) on random problems, through the fused front, the DAG (graph
    and eager), IDO and PM builds, against the full table (itself checked against the oracle)."""
    eng = Engine(0)
    n = 0
    for seed in range(24):
        pols, res, probes = random_problem(120_000 + seed, n_pods=70 + 23 * seed, bad=seed % 4 == 3)
        try:
            want = Oracle(pols, res).probe(probes)
        except OraclePanic:
            continue
        eng.build_policies(pols).load_resources(res)
        eng.prepare(probes)
        for graphs, fused, pod_words in ((-1, 1, -1), (1, 0, -1), (0, 1, 0), (2, 0, 0)):
            eng.set_option("graphs", graphs)
            eng.set_option("front_fused", fused)
            eng.set_option("pod_words", pod_words)
            full = eng.run_host()
            assert_same(want, full, f"seed {seed}")
            _source_shards_equal(eng, full, (2, 3, 5), f"seed {seed} graphs {graphs} fused {fused} pod_words {pod_words}")
            n += 1
    assert n >= 40


def test_source_rows_deployments_and_ip(gpu):
    """Source shards on IDO builds (deployment-style identity runs) and IP-interval problems (IP rows
    computed only over the shard's chunks)."""
    eng = Engine(0)
    problems = [_deployment_problem(s) for s in range(6)] + [_ip_interval_problem(s, n_pods=900 + 131 * s) for s in range(3)]
    for n, (pols, res, probes) in enumerate(problems):
        want = Oracle(pols, res).probe(probes)
        eng.build_policies(pols).load_resources(res)
        eng.prepare(probes)
        for pod_words, wave in ((-1, 1), (0, 1), (0, 0)):
            eng.set_option("pod_words", pod_words)
            eng.set_option("pl_wave", wave)
            full = eng.run_host()
            assert_same(want, full, f"problem {n}")
            _source_shards_equal(eng, full, (2, 4, 7), f"problem {n} pod_words {pod_words} pl_wave {wave}")
        eng.set_option("pod_words", -1)
        eng.set_option("pl_wave", 1)


@pytest.mark.parametrize("name,kw", [("config3", {"n_ns": 60}), ("config4", {"n_pods": 6000, "n_policies": 600, "n_ns": 60}),
                                     ("config2", {"n_ns": 30}), ("config3u", {"n_ns": 40})])
def test_source_rows_synthetic(gpu, name, kw):
    """Source shards of the synthetic workloads (fused front, sparse pod rows, IP rows, in-place class
    rows) equal the full table's slices, on the device path with the emit's per-plane launches."""
    from cyclonus_amd import synth

    data = synth.CONFIGS[name](**kw)
    eng = Engine(0).build_policies(json.dumps(data["policies"])).load_resources(json.dumps(data["resources"]))
    eng.prepare(data["probes"])
    full = eng.run_host()
    _source_shards_equal(eng, full, (2, 8), name)


def test_source_rows_panics(gpu):
    """A panicking problem: the source shard holding the first panicking job's source reports the
    reference's panic (jobs are source-major, so the shard's first panic is the global first)."""
    from cyclonus_amd.shard import source_range

    eng = Engine(0)
    seen = 0
    for seed in range(10_000, 10_120):
        pols, res, probes = random_problem(seed, bad=True)
        try:
            Oracle(pols, res).probe(probes)
            continue
        except OraclePanic as e:
            want = e
        eng.build_policies(pols).load_resources(res)
        try:
            sh = eng.prepare(probes)
        except CyclonusPanic as e:
            assert e.msg == str(want), seed
            continue
        P, K = sh["pods"], sh["slots"]
        if want.cell is None or want.cell < 0 or not P or not K:
            continue
        s_first = want.cell // (P * K)
        for world in (2, 3):
            r = next(r for r in range(world) if source_range(P, world, r)[0] <= s_first < source_range(P, world, r)[1])
            lo, hi = source_range(P, world, r)
            with pytest.raises(CyclonusPanic) as ei:
                eng.run_host(lo, hi, "source")
            assert ei.value.msg == str(want), (seed, world)
            seen += 1
    assert seen >= 10


def test_source_rows_arguments(gpu):
    """Source rows must start on a 64-pod word (and end on one, or at P); empty shards are valid."""
    pols, res, probes = random_problem(777, n_pods=200, n_pols=30)
    eng = Engine(0).build_policies(pols).load_resources(res)
    eng.prepare(probes)
    st, ing, eg = eng.run_host()
    for lo, hi in ((1, 64), (0, 65), (64, 100)):
        with pytest.raises(Exception):
            eng.run_host(lo, hi, "source")
    st2, ing2, eg2 = eng.run_host(64, 64, "source")
    assert ing2.shape == (200, ing.shape[1], 0) and eg2.shape[0] == 0
    st2, ing2, eg2 = eng.run_host(128, 200, "source")
    assert np.array_equal(ing[:, :, 2:4], ing2) and np.array_equal(eg[128:200], eg2)
    assert eng.layout(128, 200, "source") == (200, 2, 72, 4, 2)


@pytest.mark.parametrize("block", range(2))
def test_duplicate_job_keys(gpu, block):
    """Pods sharing a ns/name and containers sharing a (protocol, port): the reference's table build
    dies on the first result whose Item already holds its key (table.go:16-22, 38-48 via
    utils.DoOrDie), in runProbe's result order (valid, BadPortProtocol, BadNamedPort jobs,
    jobrunner.go:33-58), after the config's evaluation panics and before the next config.  The GPU
    build reports CYC_ERR_DUPLICATE_KEY exactly when the oracle's literal walk does, for the same job
    and key; tables without a duplicate are unchanged."""
    eng = Engine(0)
    n_dup = n_ok = 0
    for seed in range(200_000 + block * 100, 200_000 + block * 100 + 100):
        pols, res, probes = random_problem(seed, dups=True, bad=seed % 7 == 0)
        o, g = run_both(pols, res, probes, engine=eng)
        assert_same(o, g, f"dups seed {seed}")
        if isinstance(o, Panicked) and "duplicate key" in o.msg:
            n_dup += 1
        elif not isinstance(o, Panicked):
            n_ok += 1
    assert n_dup >= 40 and n_ok >= 10, (n_dup, n_ok)


@pytest.mark.parametrize("seed", range(6))
def test_uniform_descriptors_ido(gpu, seed):
    """Every pod with the same containers (one VALID job descriptor per slot across the table, as in
    configs #3 / #4): the egress class rows take the descriptor as a scalar and skip the per-word slot
    words; equal to the oracle on IDO builds (deployment-style words) and PM builds, fused and DAG
    fronts."""
    pols, res, probes = _deployment_problem(seed)
    conts = [{"Name": "c0", "Port": 80, "Protocol": "TCP", "PortName": "serve-80-tcp"},
             {"Name": "c1", "Port": 53, "Protocol": "UDP", "PortName": "serve-53-udp"},
             {"Name": "c2", "Port": 81, "Protocol": "SCTP", "PortName": "serve-81-sctp"}]
    res = dict(res, Pods=[dict(p, Containers=conts) for p in res["Pods"]])
    probes = [{"AllAvailable": True}, {"Port": 80, "Protocol": "TCP"}, {"Port": "serve-53-udp", "Protocol": "UDP"}]
    if seed % 2 == 0:
        probes = probes[:1]  # 3 slots: the PM build's wave-per-chunk class rows apply
    want = Oracle(pols, res).probe(probes)
    eng = Engine(0).build_policies(pols).load_resources(res)
    eng.prepare(probes)
    for pod_words, fused in ((1, 1), (1, 0), (0, 1), (0, 0)):  # IDO and PM builds (wave-per-chunk rows)
        eng.set_option("pod_words", pod_words)
        eng.set_option("front_fused", fused)
        assert eng.get_option("pod_words") == pod_words
        assert_same(want, eng.run_host(), f"seed {seed} pod_words {pod_words} fused {fused}")
