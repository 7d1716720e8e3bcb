#!/usr/bin/env python3
"""Benchmark: simulated-connectivity verdict grid on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config config3]

A step is one full pass of the hot path over the synthetic workload with every input table
already resident in HBM: selector evaluation, peer rows, port tables, target membership and
class election, class rows, and the emit of both packed verdict planes (ingress keyed by
destination, egress keyed by source) for this rank's rows.  N > 1 shards the pods across ranks
(one process per GPU, torch.distributed over RCCL for the barrier / max-time reduce only; there is
no collective on the data path): --partition source (the default, north_star's partition: rank r owns
a contiguous share of the source pods, i.e. every cell Table.Get(from = s, *) of its sources, which it
can answer alone — pkg/connectivity/probe/table.go:54-56, resources.go:286-287) or target (rank r owns
the target rows of both planes; Get(from, to) then needs the ranks of both pods).  Rank 0 prints one
JSON line.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "pod-pair×port verdicts/sec (node) at 100k pods×10k policies; HBM GB/s"


def load_workload(name: str):
    from cyclonus_amd import synth

    if name != "config5":
        return synth.CONFIGS[name]()
    from cyclonus_amd.generator import sweep

    steps = sweep()
    return {"name": "config5", "steps": steps,
            "description": f"cyclonus generate sweep: {len(steps)} probe steps batched in one pass, a block per step "
                           "(only intra-step cells computed)"}


def cpu_baseline(data, seconds: float, seed: int = 1):
    """Time the per-cell CPU oracle (restated reference walk) on random cells, 1 and N threads."""
    import numpy as np

    from oracle.oracle import Oracle

    if "steps" in data:  # config #5: every cell of every step (small problems)
        t0 = time.perf_counter()
        cells = 0
        for st in data["steps"]:
            status, _, _ = Oracle(st["policies"], st["resources"]).probe([st["probe"]])
            cells += status.shape[0] * int((status == 1).sum())
        el = time.perf_counter() - t0
        return {"value": cells / el, "unit": "verdicts/s", "cores": 1, "kind": "port",
                "sample": f"all {cells} cells of the {len(data['steps'])} generate steps through the oracle "
                f"(policy build per step included), {el:.2f} s, 1 thread"}

    t0 = time.perf_counter()
    orc = Oracle(data["policies"], data["resources"], True)
    build_s = time.perf_counter() - t0
    P, K = orc.shape(data["probes"])
    rng = np.random.default_rng(seed)

    def timed(threads, budget):
        cells, elapsed, chunk = 0, 0.0, 64 * threads
        while elapsed < budget:
            s = rng.integers(0, P, chunk)
            d = rng.integers(0, P, chunk)
            k = rng.integers(0, K, chunk)
            t = time.perf_counter()
            orc.cells(data["probes"], s, d, k, threads=threads)
            elapsed += time.perf_counter() - t
            cells += chunk
            chunk = min(chunk * 2, 4096 * threads)
        return cells, elapsed

    # 1 thread and all host threads (std::thread, static split of the sampled cells);
    # the GPU box exports its CPU share as OMP_NUM_THREADS
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1), os.cpu_count() or 1, 64))
    c1, e1 = timed(1, seconds / 2)
    cn, en = timed(threads, seconds / 2) if threads > 1 else (c1, e1)
    return {
        "value": cn / en,
        "unit": "verdicts/s",
        "cores": threads,
        "kind": "port",
        "single_thread_value": c1 / e1,
        "sample": f"uniformly random (src, dst, slot) cells of {data['name']} through the oracle's per-cell "
        f"IsTrafficAllowed walk (oracle/oracle.cpp): {cn} cells in {en:.1f} s on {threads} threads (std::thread, "
        f"static split) and {c1} cells in {e1:.1f} s on 1 thread; policy build {build_s:.1f} s excluded",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=20)  # GPU clocks settle after the host-side prepare
    ap.add_argument("--config", default="config3", choices=["config2", "config3", "config4", "config5", "config3u"])
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-assemble", action="store_true", help="skip the N>1 all-gather timing")
    ap.add_argument("--partition", default="source", choices=["source", "target"],
                    help="row partition across ranks (include/cyclonus_hip.h cyc_rows; the same at N=1)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="cyc_set_option tuning knob (diagnostics; results never change)")
    args = ap.parse_args()

    import numpy as np
    import torch

    from cyclonus_amd.engine import Engine
    from cyclonus_amd.shard import shard_range

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = local % max(torch.cuda.device_count(), 1)  # ranks > GPUs only in a rehearsal
    torch.cuda.set_device(device)
    backend = os.environ.get("CYC_BENCH_BACKEND", "nccl")  # "gloo" = CPU rehearsal of the N>1 flow
    dist = None
    # CYC_BENCH_FORCE_DIST=1: the process group even for one rank (exercises the RCCL barrier /
    # max-reduce / all-gather path on a one-GPU box; two ranks cannot share one GPU under RCCL)
    if world > 1 or os.environ.get("CYC_BENCH_FORCE_DIST"):
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)

    def barrier():
        if dist is not None:
            dist.barrier()

    data = load_workload(args.config)
    bt = None
    stream = torch.cuda.current_stream().cuda_stream
    part = args.partition
    t_prep = time.perf_counter()
    eng = Engine(device)  # cyc_ctx_create: the context's HIP stream and events (once per process and GPU)
    ctx_create_s = time.perf_counter() - t_prep
    for o in args.opt:
        k, v = o.split("=")
        eng.set_option(k, int(v))
    if "steps" in data:
        # config #5: the generate sweep's probe problems as blocks of one pass (cyc_probe_prepare_blocks);
        # N > 1 gives each rank a contiguous share of the problems (independent: no exchange)
        from cyclonus_amd.batch import Batch

        steps = data["steps"]
        bt = Batch(steps[rank * len(steps) // world:(rank + 1) * len(steps) // world])
        shape = bt.prepare(eng)
        torch.cuda.synchronize()
        t_prepared = time.perf_counter()
        prepare_s = {"total_s": t_prepared - t_prep, "note": "policy build + Resources load + cyc_probe_prepare_blocks"}
        data["policies"] = bt.policies
        P, K, W = shape["pods"], shape["slots"], shape["words"]
        lo, hi, rows = 0, P, P
        d_in, d_eg, d_st = bt.alloc()

        def step():
            eng.run_blocks_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), stream)
    else:
        # the drop-in's host cost (analyze --mode probe, pkg/cli/analyze.go:121, 232-243): policy build
        # (BuildNetworkPolicies + Simplify, from the k8s NetworkPolicy JSON), the probe model through
        # the flat tables a cgo binding passes (cyc_resources_load: no JSON) and cyc_probe_prepare_configs
        # (interning, job expansion, table upload) — paid once per probe model, outside `value`
        from cyclonus_amd.flat import prepare_flat

        shape = prepare_flat(eng, data["policies"], data["resources"], data["probes"])
        torch.cuda.synchronize()
        prepare_s = shape.pop("prepare_s")
        prepare_s["context_create_s"] = ctx_create_s  # (not in total_s: once per process, not per probe model)
        P, K, W = shape["pods"], shape["slots"], shape["words"]
        lo, hi = shard_range(P, world, rank, part)
        rows = hi - lo

        # shards differ by at most one row (target) / one 64-pod word (source): every rank allocates the
        # largest, so the optional all-gather (assembled table) moves the planes as they are
        lays = [eng.layout(*shard_range(P, world, r, part), part) for r in range(world)]
        ri, wi, re_, we, w0 = lays[rank]
        max_in = max(x[0] * x[1] for x in lays)
        max_eg = max(x[2] * x[3] for x in lays)
        if os.environ.get("CYC_BENCH_ONE_BUFFER"):  # both planes carved from one allocation (layout A/B)
            n_in, n_eg = max(max_in, 1) * K, max(max_eg, 1) * K
            pad = int(os.environ.get("CYC_BENCH_PLANE_GAP", "0")) // 8
            planes = torch.empty((n_in + pad + n_eg,), dtype=torch.int64, device="cuda")
            d_in, d_eg = planes[:n_in], planes[n_in + pad:]
        else:
            d_in = torch.empty((max(max_in, 1) * K,), dtype=torch.int64, device="cuda")
            d_eg = torch.empty((max(max_eg, 1) * K,), dtype=torch.int64, device="cuda")
        d_st = torch.empty((P, K), dtype=torch.uint8, device="cuda")

        def step():
            eng.run_device(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), stream, lo, hi, part)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    # assembled table (not part of `value`): RCCL all-gather of both planes' row shards into the
    # full table on every rank, timed separately (max over ranks)
    assembled = None
    # (batched blocks: each rank holds its own problems' slabs, of rank-dependent sizes — nothing to assemble)
    if dist is not None and not args.no_assemble and bt is None:
        try:
            dev = "cuda" if backend == "nccl" else "cpu"
            out_in = torch.empty((world * d_in.numel(),), dtype=torch.int64, device=dev)
            out_eg = torch.empty((world * d_eg.numel(),), dtype=torch.int64, device=dev)
            src_in, src_eg = (d_in, d_eg) if backend == "nccl" else (d_in.cpu(), d_eg.cpu())

            def gather():  # torch's all-gather of the padded shards as they are (a raw xGMI rate, no relayout)
                for src, out in ((src_in, out_in), (src_eg, out_eg)):
                    if backend == "nccl":
                        dist.all_gather_into_tensor(out, src)
                    else:
                        dist.all_gather(list(out.chunk(world)), src)

            gather()
            torch.cuda.synchronize()
            barrier()
            ta = time.perf_counter()
            reps = 3
            for _ in range(reps):
                gather()
            torch.cuda.synchronize()
            barrier()
            ga = torch.tensor([(time.perf_counter() - ta) / reps], dtype=torch.float64,
                              device="cuda" if backend == "nccl" else "cpu")
            dist.all_reduce(ga, op=dist.ReduceOp.MAX)
            ga = float(ga.item())
            recv = (world - 1) * (d_in.numel() + d_eg.numel()) * 8
            assembled = {"all_gather_ms": ga * 1e3, "bytes_received_per_rank": recv, "xgmi_GBs_per_rank": recv / ga / 1e9}
            del out_in, out_eg
            if backend == "nccl":
                # the time to a usable whole table on every rank, through the library (cyc_comm_init +
                # cyc_planes_allgather, comm.hpp: grouped RCCL broadcasts of the row shares straight into
                # place, and for a source partition the chunked gather of the ingress slices + the HIP
                # relayout kernel); rank 0's unique id goes to the others over the process group
                uid = torch.tensor(list(Engine.comm_unique_id()) if rank == 0 else [0] * 128, dtype=torch.uint8,
                                   device="cuda")
                dist.broadcast(uid, 0)
                eng.comm_init(world, rank, bytes(uid.cpu().tolist()))
                assert eng.rows_shard(world, rank, part) == (lo, hi)
                torch.cuda.empty_cache()
                f_in = torch.empty((P * K * W,), dtype=torch.int64, device="cuda")
                f_eg = torch.empty((P * K * W,), dtype=torch.int64, device="cuda")

                def whole():
                    eng.planes_allgather(d_in.data_ptr(), d_eg.data_ptr(), f_in.data_ptr(), f_eg.data_ptr(), stream, part)

                whole()
                torch.cuda.synchronize()
                barrier()
                tw = time.perf_counter()
                for _ in range(reps):
                    whole()
                torch.cuda.synchronize()
                barrier()
                tt = torch.tensor([(time.perf_counter() - tw) / reps], dtype=torch.float64, device="cuda")
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                assembled["whole_table_ms"] = float(tt.item()) * 1e3
                assembled["whole_table_note"] = ("cyc_planes_allgather (libcyclonus_hip's own RCCL communicator): both "
                                                 "[P][K][W] planes whole on every rank, incl. the relayout of a source "
                                                 "partition's ingress slices (max over ranks)")
                eng.comm_destroy()
                del f_in, f_eg
                torch.cuda.empty_cache()
        except Exception as e:  # the assembled figure is informational; never lose the bench line
            assembled = {"error": f"{type(e).__name__}: {e}"}

    # the emit as the library launched it in the timed steps (cyc_last_emit: kernel name(s), launches)
    emit_kernel, launches = eng.last_emit()

    # per-kernel device times from HIP events on the launch stream (separate, synchronised runs)
    launch_mode, fused = eng.get_option("launch"), eng.get_option("front_fused_active")
    front = ("fused front: 4-5 block-range launches on one stream, one per dependency level, both directions' blocks in each" if fused
             else "front as a two-branch DAG (ingress / egress)")
    how = ("one captured hipGraph replay" if launch_mode == 1 else "the fused front's launches and the emit enqueued eagerly on one stream"
           if fused else "the step DAG enqueued eagerly on three streams")
    launch_desc = (f"{how} "
                   f"per step (cyc_set_option graphs={launch_mode}): {front}, then one emit launch writing both planes")
    graphs = eng.get_option("graphs")
    eng.set_option("graphs", 0)  # per-phase events need the eager launch path with events
    tm = []
    for _ in range(5):
        step()
        tm.append(eng.timings())
    eng.set_option("graphs", graphs)
    tm = np.array(tm)
    pipe_ms, emit_ms, rows_ms = (float(x) for x in tm.mean(axis=0))
    classes_in, classes_eg = eng.classes()

    # practical write ceiling for the same bytes: torch's fill kernel over both output planes
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fills = []
    for _ in range(3):
        e0.record()
        d_in.fill_(0)
        d_eg.fill_(0)
        e1.record()
        torch.cuda.synchronize()
        fills.append(e0.elapsed_time(e1))
    fill_gbs = (d_in.numel() + d_eg.numel()) * 8 / (min(fills) * 1e-3) / 1e9

    # reading the table back (not part of `value`): Table.Get(from, *) of 64 sources through the
    # device-resident table (cyc_table_cells: Ingress / Egress / Combined bytes to the host), and the
    # packed planes' device-to-host copy rate
    readback = None
    try:
        if bt is not None:
            raise RuntimeError("batched blocks: per-block slabs, no whole-table view")
        torch.cuda.synchronize()
        tab = eng.wrap_table(d_in.data_ptr(), d_eg.data_ptr(), d_st.data_ptr(), lo, hi, part)
        s_hi = min(hi, lo + 64)
        t0 = time.perf_counter()
        tab.cells(lo, s_hi, 0, P, 0, K)
        tc = time.perf_counter() - t0
        n_rb = min(d_in.numel(), 1 << 27)
        host = torch.empty(n_rb, dtype=torch.int64, pin_memory=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        host.copy_(d_in[:n_rb], non_blocking=True)
        torch.cuda.synchronize()
        tp = time.perf_counter() - t0
        readback = {"table_cells_64_sources_s": tc, "cells": (s_hi - lo) * P * K * 3,
                    "planes_d2h_GBs": n_rb * 8 / tp / 1e9}
        tab.close()
        del host
    except Exception as e:  # informational
        readback = {"error": f"{type(e).__name__}: {e}"}

    status = d_st.cpu().numpy()
    if bt is not None:  # the cells of each batched problem (the slabs hold nothing else)
        cells = bt.cells(status)
        if world > 1:
            ct = torch.tensor([cells], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
            dist.all_reduce(ct)
            cells = int(ct.item())
    else:
        valid_slots = int((status == 1).sum())  # (dst, slot) pairs with a VALID job
        cells = P * valid_slots  # every source pod x every valid (dst, slot) job
    ms_per_step = dt / args.steps * 1e3
    value = cells / (dt / args.steps)

    # the emit writes each plane (ingress, egress) of this rank's rows once, both in ONE launch:
    # rows x K x W x 8 B per plane = 2 bits per cell — less the rows that already hold their class
    # row (in-place class rows, cyc_set_option class_inplace: one row per class and plane is written
    # by the class-row kernel, the emit copies it to the class's other rows)
    # a source shard's planes differ in row length (ingress: every destination over the shard's
    # words; egress: its sources over all words) and are emitted by one launch each
    if bt is not None:  # k_emit_blocks: every block's slabs (answered cells' bits) and its status rows
        ri = re_ = P
        wi = we = W
        inplace = False
        emit_rows = 2 * P
        emit_bytes = 2 * int(bt.layout[-1][0]) * 8 + int(bt.layout[-1][1])
    else:
        inplace = eng.get_option("class_inplace_active") == 1
        emit_rows = ri + re_ - (classes_in + classes_eg if inplace else 0)
        emit_bytes = (ri - (classes_in if inplace else 0)) * K * wi * 8 + (re_ - (classes_eg if inplace else 0)) * K * we * 8
    emit_launch_ms = emit_ms / max(launches, 1)  # HIP events bracket the emit phase (all its launches)
    achieved = emit_bytes / (emit_ms * 1e-3) / 1e9

    # HBM traffic of k_emit from the committed PMC passes for this same workload (rocprofv3
    # --pmc FETCH_SIZE / WRITE_SIZE, corrected per MI355X_MICROARCH.md; scripts/pmc_summary.py)
    # (the newest round's file); MFMA use from the same file's --pmc SQ_*MFMA* pass
    # Only a profile of THIS library build is quoted: the PMC file records the sha256 of the library
    # it profiled (scripts/pmc_summary.py --build-info); another build's counters give traffic null.
    traffic, traffic_src, mfma = None, None, None
    pmcs = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]_pmc_{args.config}.json")))
    if pmcs and world == 1:
        from cyclonus_amd import _lib
        from cyclonus_amd.build import lib_sha256

        pmc = json.load(open(pmcs[-1]))
        traffic_src = os.path.relpath(pmcs[-1], ROOT)
        loaded = lib_sha256(_lib.SO_PATH)
        if (pmc.get("build") or {}).get("lib_sha256") == loaded:
            traffic = pmc.get("emit_hbm_bytes_per_launch")
        else:
            traffic_src = (f"{traffic_src} profiled library "
                           f"{(pmc.get('build') or {}).get('lib_sha256', 'unrecorded')[:12]}, loaded {loaded[:12]}: not quoted")
        if pmc.get("mfma"):
            m = pmc["mfma"]
            mfma = {"insts_per_step": m["mfma_insts_per_step"], "busy_cycles_per_step": m["mfma_busy_cycles_per_step"],
                    "util": m["util"], "source": traffic_src,
                    "note": "no GEMM-shaped step on this path (DESIGN.md section 4): measured, not assumed"}

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "verdicts/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (cyclonus_amd/generator.py restated generate sweep)" if args.config == "config5" else "synthetic (cyclonus_amd/synth.py, xoshiro256** seed 20250217)",
            "config": {
                "workload": f"{data['name']}: {data['description']}",
                "pods": P,
                "policies": len(data["policies"]),
                "slots": K,
                "cells": cells,
                "targets_in": shape["targets_in"],
                "targets_eg": shape["targets_eg"],
                "peers": shape["peers"],
                "identities_in": shape["classes_in"],
                "identities_eg": shape["classes_eg"],
                "classes_in": classes_in,
                "classes_eg": classes_eg,
                "parallelism": f"{part}-row shards x{world}",
                "partition": part,
                "rows_per_rank": rows,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": emit_kernel,
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": emit_bytes / max(launches, 1),
                "algorithmic_bytes_per_step": emit_bytes,
                "emit_rows_per_launch": emit_rows,
                "class_rows_in_place": inplace,
                "emit_ms_per_launch": emit_launch_ms,
                "launches_per_step": launches,
                "fill_ceiling_GBs": fill_gbs,
                "mfma": mfma,
            },
            "launch": launch_desc,
            "prepare_s": prepare_s,
            "readback": readback,
            "pipeline_ms": {"total": pipe_ms, "emit": emit_ms, "class_rows": rows_ms, "front": pipe_ms - emit_ms - rows_ms},
        }
        if assembled is not None:
            if "all_gather_ms" in assembled:  # whole-table-on-every-rank throughput
                assembled["value"] = cells / (dt / args.steps + assembled.get("whole_table_ms", assembled["all_gather_ms"]) * 1e-3)
            line["assembled"] = assembled
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(data, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
