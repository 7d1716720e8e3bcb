"""Batched small-problem mode (config #5): many independent probe problems in ONE GPU pass.

Each problem (policies, Resources, probe config) becomes a block of one combined problem: its
namespaces are renamed "<block>~<ns>" everywhere (pods, Resources.Namespaces keys, policy
metadata.namespace — so the reference's default namespace becomes "<block>~default").  Targets,
their primary keys and the exact-namespace peer matchers then never cross blocks, so for every
(source, destination) pair INSIDE a block the verdict is exactly the stand-alone problem's:
namespace / pod label selectors and IPBlocks can match pods of other blocks only in cross-block
cells, which are computed but never read.  The probe configs of all problems become slot ranges
of the combined problem; each block reads the slots of its own config.

Panics are the exception: the reference panics on the FIRST panicking job of a problem's own table
(ippeermatcher.go:46-48, labelselector.go:57), but a combined problem also evaluates cross-block
cells, so one block's unparsable pod IP met by another block's IPBlock peer would panic the whole
batch although neither problem panics alone.  `run` therefore answers every block from the batched
pass when that pass does not panic (then no cell panicked, intra-block cells included), and
otherwise re-runs each problem stand-alone, so each block gets its own table or its own panic.
"""
from __future__ import annotations

import copy
import json

import numpy as np


def _key(probe):
    return json.dumps(probe, sort_keys=True)


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
        self.offsets, self.sizes = [], []
        for b, p in enumerate(problems):
            pre = f"{b}~"
            for pol in p["policies"]:
                q = copy.deepcopy(pol)
                md = q.setdefault("metadata", {})
                md["namespace"] = pre + (md.get("namespace") or "default")
                pols.append(q)
            for ns, labels in (p["resources"].get("Namespaces") or {}).items():
                nss[pre + ns] = labels
            self.offsets.append(len(pods))
            self.sizes.append(len(p["resources"].get("Pods") or []))
            for pod in p["resources"].get("Pods") or []:
                q = dict(pod)
                q["Namespace"] = pre + pod.get("Namespace", "")
                pods.append(q)
        self.policies = pols
        self.resources = {"Namespaces": nss, "Pods": pods}
        maxc = max((len(p.get("Containers") or []) for p in pods), default=0)
        self.slot_lo = []
        lo = 0
        for pr in self.probes:
            self.slot_lo.append(lo)
            lo += maxc if pr.get("AllAvailable") else 1
        self.K = lo
        self.maxc = maxc

    def slots(self, b):
        c = self.probe_index[_key(self.problems[b]["probe"])]
        n = self.maxc if self.probes[c].get("AllAvailable") else 1
        return self.slot_lo[c], self.slot_lo[c] + n

    def cells(self, status):
        """Valid intra-block cells (the verdicts the batch actually answers)."""
        n = 0
        for b in range(len(self.problems)):
            o, s = self.offsets[b], self.sizes[b]
            lo, hi = self.slots(b)
            n += s * int((status[o : o + s, lo:hi] == 1).sum())
        return n

    def extract(self, b, status, ingress, egress):
        """Block b's own table in the standard layout: (status[P,K], in[P,K,W], eg[P,K,W])."""
        o, s = self.offsets[b], self.sizes[b]
        lo, hi = self.slots(b)
        W = (s + 63) // 64

        def plane(rows):
            bits = np.unpackbits(rows.view(np.uint8), axis=2, bitorder="little")[:, :, o : o + s]
            pad = np.zeros((bits.shape[0], bits.shape[1], W * 64), np.uint8)
            pad[:, :, :s] = bits
            return np.packbits(pad, axis=2, bitorder="little").view(np.uint64)

        return (status[o : o + s, lo:hi].copy(), plane(ingress[o : o + s, lo:hi]), plane(egress[o : o + s, lo:hi]))

    def run(self, engine):
        """Per block: (status, in, eg) of its own table, or the CyclonusPanic its stand-alone run raises."""
        from ._lib import CyclonusPanic

        try:
            engine.build_policies(json.dumps(self.policies)).load_resources(json.dumps(self.resources))
            engine.prepare(self.probes)
            st, ing, eg = engine.run_host()
            out = []
            for b, p in enumerate(self.problems):
                t = self.extract(b, st, ing, eg)
                if p["probe"].get("AllAvailable"):  # the stand-alone table has its own pods' max containers
                    k = max((len(q.get("Containers") or []) for q in p["resources"].get("Pods") or []), default=0)
                    t = (t[0][:, :k], t[1][:, :k], t[2][:, :k])
                out.append(t)
            return out
        except CyclonusPanic:
            pass
        out = []
        for p in self.problems:  # a cell of the combined problem panicked: each problem on its own
            try:
                engine.build_policies(json.dumps(p["policies"])).load_resources(json.dumps(p["resources"]))
                engine.prepare([p["probe"]])
                out.append(engine.run_host())
            except CyclonusPanic as e:
                out.append(e)
        return out
