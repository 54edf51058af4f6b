#!/usr/bin/env python3
"""Interleaved timing of interval-kernel ablation variants on config 3 (one process).

Variants (kacc_debug.h, bits of kacc::kVar*): 0 production, 1 skip aggregates,
2 skip processes, 3 node phases only, 4 unstaged (every node on the chunked
big-node path), 8 non-temporal stores, 32 no 64-row-group transpose, 128 late
aggregate loads, 256 / 512 / 768 big nodes without the CPU-total pass / the
segment-owner scan / both, 1024 big nodes without the item-list atomic.
Also times the namespace kernel.  Prints a JSON summary.
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from kepler_amd import accel, fleet
    from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device

    if os.environ.get("KACC_LIB"):  # A/B of another build of the engine
        accel.load(os.environ["KACC_LIB"])
    variants = [int(x) for x in os.environ.get("VARIANTS", "0,32,128,1,2,3").split(",")]
    rounds = int(os.environ.get("ROUNDS", "10"))
    cfg = int(os.environ.get("CONFIG", "3"))
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    frag = float(os.environ.get("FRAG", "0"))  # slot fragmentation (+ node_proc_span)
    if os.environ.get("PROCS"):  # config-3 shape (Z=4) with PROCS processes per node
        layout = fleet.make_layout(int(os.environ.get("NODES", "10000")), int(os.environ["PROCS"]), 4,
                                   fleet.SEED, fragment_slots=frag)
    else:
        layout = fleet.config_layout(cfg, fragment_slots=frag, fragment_sorted=bool(os.environ.get("FRAG_SORTED")),
                                     nodes=int(os.environ["NODES"]) if os.environ.get("NODES") else None)
    sim = fleet.FleetSim(layout)
    acc = accel.Accel(layout.zones, **layout.capacities())
    stream = current_stream_handle()
    assert stream != 0
    prime = to_device(sim.next_interval())
    acc.run_interval(interval_from_tensors(prime, layout.sizes()), stream)
    # distinct input sets cycled like bench.py (no cache reuse between launches)
    n_distinct = int(os.environ.get("DISTINCT", "4"))
    dev = [to_device(sim.next_interval()) for _ in range(n_distinct)]
    if (frag > 0 or os.environ.get("SPAN")) and not os.environ.get("NO_SPAN"):
        span = to_device({"s": layout.proc_span()})["s"]
        for d in dev:
            d["node_proc_span"] = span
    # the bench's production flags (NO_STABLE=1: without KACC_F_STABLE_SLOT_NODES)
    flag = 0 if os.environ.get("KACC_LIB") else (layout.fast_flag() | accel.KACC_F_NODE_SLOT_RANGES
                                                 | (0 if os.environ.get("NO_STABLE") else accel.KACC_F_STABLE_SLOT_NODES))
    ivs = [interval_from_tensors(a, layout.sizes(), flag) for a in dev]
    it = ivs[0]
    Z = layout.zones
    sizes = layout.sizes()
    nbytes = accel.interval_bytes(Z, *[sizes[k] for k in ("n_nodes", "n_procs", "n_ctrs", "n_vms", "n_pods")], flag)
    times = {v: [] for v in variants}
    step_t = {v: [] for v in variants}
    off, slots = layout.namespace_csr()
    ns = to_device({"o": off, "s": slots})
    n_ns = len(off) - 1
    # STEP=1: bench.py's step, the variant followed by the cluster partials (namespace + node
    # totals, world 1) on the same stream; times both the variant alone and the pair
    step_mode = bool(os.environ.get("STEP"))
    if step_mode:
        cluster = accel.Cluster.join(acc, accel.Cluster.unique_id(), 1, 0)
        pe = torch.zeros(n_ns * Z, dtype=torch.int64, device="cuda")
        pp = torch.zeros(n_ns * Z, dtype=torch.float64, device="cuda")
        ne = torch.zeros(2 * Z, dtype=torch.int64, device="cuda")
        npw = torch.zeros(3 * Z, dtype=torch.float64, device="cuda")

    def partials():
        cluster.allreduce_namespaces(n_ns, [ns["o"].data_ptr()], [ns["s"].data_ptr()], [pe.data_ptr()],
                                     [pp.data_ptr()], [ne.data_ptr()], [npw.data_ptr()], streams=[stream],
                                     comm_streams=[stream])

    for v in variants:  # warm
        acc.run_variant(it, stream, v)
        if step_mode:
            partials()
    acc.sync(stream)
    launch = 0
    for _ in range(rounds):
        for v in variants:
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            it = ivs[launch % n_distinct]
            launch += 1
            e0.record()
            acc.run_variant(it, stream, v)
            e1.record()
            if step_mode:
                partials()
            e2.record()
            e2.synchronize()
            times[v].append(e0.elapsed_time(e1))
            step_t[v].append(e0.elapsed_time(e2))
    acc.sync(stream)
    oe = torch.zeros(n_ns * Z, dtype=torch.int64, device="cuda")
    op = torch.zeros(n_ns * Z, dtype=torch.float64, device="cuda")
    ns_t = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        acc.namespace_totals(n_ns, ns["o"].data_ptr(), ns["s"].data_ptr(), oe.data_ptr(), op.data_ptr(), stream)
        e1.record()
        e1.synchronize()
        ns_t.append(e0.elapsed_time(e1))
    acc.sync(stream)
    # same-box reference: a 1.28 GB device copy (torch copy_ kernel)
    src = torch.empty(160 * 1024 * 1024, dtype=torch.float64, device="cuda")
    dst = torch.empty_like(src)
    cp = []
    for _ in range(rounds + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        dst.copy_(src)
        e1.record()
        e1.synchronize()
        cp.append(e0.elapsed_time(e1))
    copy_gbps = 2 * src.numel() * 8 / (np.median(cp[2:]) * 1e-3) / 1e9
    out = {"config": cfg, "copy_GBps": copy_gbps, "sizes": sizes, "bytes_per_launch": nbytes,
           "variants": {str(v): {"median_ms": float(np.median(t)), "min_ms": float(np.min(t))} for v, t in times.items()},
           "namespace_ms": float(np.median(ns_t))}
    if step_mode:
        out["step_median_ms"] = {str(v): float(np.median(t)) for v, t in step_t.items()}
        out["partials_median_ms"] = {str(v): float(np.median(np.array(step_t[v]) - np.array(times[v])))
                                     for v in variants}
        cluster.close()
    if 0 in times:
        out["achieved_GBps_v0"] = nbytes / (np.median(times[0]) * 1e-3) / 1e9
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
