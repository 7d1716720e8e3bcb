"""Batched small-problem mode (config #5): many independent probe problems in ONE GPU pass.

The reference runs each step of a generated test case as its own small table: the interpreter
calls Runner.RunProbeForConfig per step (pkg/connectivity/interpreter.go:137-148), i.e. its own
policies, Resources and probe config.  Here every problem becomes a BLOCK of one combined input
(cyc_probe_prepare_blocks, include/cyclonus_hip.h):

* its pods are a consecutive range of the combined Resources.Pods;
* its namespaces are renamed "<block>~<ns>" everywhere (pods, Resources.Namespaces keys, policy
  metadata.namespace — so the reference's default namespace becomes "<block>~default"), so a
  block's targets apply to its own pods only (TargetsApplyingToPod compares namespaces,
  policy.go:68-82) and its exact-namespace peers match its own pods only;
* it answers its own probe config only, over its own pods only: the device computes class rows over
  the block's 64-pod words and writes the block's table as a slab [pods][slots][words] with bits
  relative to its first pod — the cells computed are the cells answered;
* a Go panic or table-build fatal is reported per block, as that problem's stand-alone run would
  report it (its first panicking job in its own job order): one block's bad pod IP does not touch
  any other block.
"""
from __future__ import annotations

import copy
import json

import numpy as np


def _key(probe):
    return json.dumps(probe, sort_keys=True)


def _field(obj, name):
    """The keys of `obj` that decode into struct field `name` (encoding/json: exact or ASCII
    case-insensitive), and the value that decides it: the last non-null one (a JSON null leaves a
    string / struct field unchanged — cjson.hpp sval, the library's loader)."""
    keys = [k for k in obj if k.lower() == name.lower()]
    vals = [obj[k] for k in keys if obj[k] is not None]
    return keys, (vals[-1] if vals else None)


def _prefixed(obj, name, pre, default):
    """A copy of `obj` whose field `name` is prefix + its decoded value (or `default` when absent or
    null), held by ONE key: every case variant is dropped first, so no later variant overrides it."""
    keys, v = _field(obj, name)
    q = {k: x for k, x in obj.items() if k not in keys}
    q[name] = pre + (v or default)
    return q


class Batch:
    def __init__(self, problems):
        """problems: list of {"policies": [...], "resources": {...}, "probe": {...}}."""
        self.problems = problems
        self.probes, self.probe_index = [], {}
        for p in problems:
            k = _key(p["probe"])
            if k not in self.probe_index:
                self.probe_index[k] = len(self.probes)
                self.probes.append(p["probe"])
        pols, pods, nss = [], [], {}
        self.offsets, self.sizes, self.block_end, self.block_config = [], [], [], []
        for b, p in enumerate(problems):
            pre = f"{b}~"
            for pol in p["policies"]:
                q = copy.deepcopy(pol)
                mkeys, md = _field(q, "metadata")
                q = {k: x for k, x in q.items() if k not in mkeys}
                # the policy's namespace (builder.go: "" -> "default"), renamed into the block's
                q["metadata"] = _prefixed(md if isinstance(md, dict) else {}, "namespace", pre, "default")
                pols.append(q)
            for ns, labels in (p["resources"].get("Namespaces") or {}).items():
                nss[pre + ns] = labels
            self.offsets.append(len(pods))
            self.sizes.append(len(p["resources"].get("Pods") or []))
            for pod in p["resources"].get("Pods") or []:
                pods.append(_prefixed(pod, "Namespace", pre, ""))
            self.block_end.append(len(pods))
            self.block_config.append(self.probe_index[_key(p["probe"])])
        self.policies = pols
        self.resources = {"Namespaces": nss, "Pods": pods}
        self.maxc = max((len(p.get("Containers") or []) for p in pods), default=0)

    def prepare(self, engine):
        """Load the combined input into `engine` and prepare its blocks."""
        engine.build_policies(json.dumps(self.policies)).load_resources(json.dumps(self.resources))
        shape = engine.prepare_blocks(self.probes, self.block_end, self.block_config)
        self.layout = engine.block_layout  # per block (plane slab offset, status offset); then totals
        return shape

    def slab_dims(self, b):
        """(pods, slots, words) of block b's slab."""
        n = self.sizes[b]
        k = self.maxc if self.probes[self.block_config[b]].get("AllAvailable") else 1
        return n, k, (n + 63) // 64

    def alloc(self):
        """Device slabs (ingress, egress, status) for one run of every block."""
        import torch

        words, st = (int(x) for x in self.layout[-1])
        return (torch.empty(max(words, 2), dtype=torch.int64, device="cuda"),
                torch.empty(max(words, 2), dtype=torch.int64, device="cuda"),
                torch.empty(max(st, 16), dtype=torch.uint8, device="cuda"))

    def cells(self, status):
        """Valid intra-block cells (the verdicts the batch answers) from the host status slab."""
        n = 0
        for b in range(len(self.problems)):
            p, k, _ = self.slab_dims(b)
            so = int(self.layout[b][1])
            n += p * int((status[so : so + p * k] == 1).sum())
        return n

    def block_table(self, b, status, ingress, egress):
        """Block b's own table from host copies of the slabs: (status[P,K], in[P,K,W], eg[P,K,W])."""
        p, k, w = self.slab_dims(b)
        wo, so = (int(x) for x in self.layout[b])
        st = status[so : so + p * k].reshape(p, k)
        ing = ingress[wo : wo + p * k * w].reshape(p, k, w)
        eg = egress[wo : wo + p * k * w].reshape(p, k, w)
        if self.probes[self.block_config[b]].get("AllAvailable"):  # the stand-alone table's own max containers
            kk = max((len(q.get("Containers") or []) for q in self.problems[b]["resources"].get("Pods") or []), default=0)
            st, ing, eg = st[:, :kk], ing[:, :kk], eg[:, :kk]
        return st.copy(), ing.copy(), eg.copy()

    def run(self, engine):
        """Per block: (status, in, eg) of its own table, or the CyclonusPanic its stand-alone run raises."""
        import torch

        from ._lib import CyclonusPanic

        self.prepare(engine)
        d_in, d_eg, d_st = self.alloc()
        rcs = engine.run_blocks_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(),
                                       torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        st = d_st.cpu().numpy()
        ing = d_in.cpu().numpy().view(np.uint64)
        eg = d_eg.cpu().numpy().view(np.uint64)
        out = []
        for b, (rc, msg) in enumerate(rcs):
            # the block's own namespace names in a table-build message (pod keys ns/name, job.go)
            msg = msg.replace(f"FromKey:{b}~", "FromKey:").replace(f"ToKey:{b}~", "ToKey:")
            out.append(CyclonusPanic(rc, msg) if rc else self.block_table(b, st, ing, eg))
        return out
