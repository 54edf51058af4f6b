#!/usr/bin/env python3
"""Ablations of the one-launch K-interval kernel (intervals_carry_kernel) on BASELINE config 2
(1k nodes x 1k procs, Z=2, K=60), against K single-interval launches.  Times one call of K
intervals with HIP events on the launch stream (median of ROUNDS); one JSON line.
Variants != 0 do not compute the reference results (timing only)."""

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from kepler_amd import accel, fleet
    from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device

    torch.cuda.set_stream(torch.cuda.Stream())
    K = int(os.environ.get("K", "60"))
    nodes = int(os.environ.get("NODES", "1000"))
    rounds = int(os.environ.get("ROUNDS", "5"))
    variants = [int(v) for v in os.environ.get("VARIANTS", "0,1,2,4,5").split(",")]
    L = fleet.config_layout(2, nodes=nodes)
    sim = fleet.FleetSim(L)
    prime = sim.next_interval()
    ivs = [sim.next_interval() for _ in range(K)]
    acc = accel.Accel(L.zones, **L.capacities())
    s = current_stream_handle()
    acc.run_interval(interval_from_tensors(to_device(prime), L.sizes()), s)
    if os.environ.get("SPAN", "1") == "1":  # kacc_slot_join's node_proc_span, as in production
        for a in ivs:
            a["node_proc_span"] = L.proc_span()
    dev = [to_device(a) for a in ivs]
    base = L.fast_flag()
    fused = [interval_from_tensors(t, L.sizes(), base | accel.KACC_F_NODE_SLOT_RANGES) for t in dev]
    plain = [interval_from_tensors(t, L.sizes(), base) for t in dev]

    def timed(fn):
        ts = []
        for _ in range(rounds + 1):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        return float(np.median(ts[1:]))

    out = {"K": K, "nodes": nodes, "sizes": L.sizes()}
    out["sequential_ms"] = timed(lambda: acc.run_intervals(plain, s))
    out["fused_ms"] = timed(lambda: acc.run_intervals(fused, s))
    for v in variants:
        out[f"variant_{v}_ms"] = timed(lambda: acc.run_intervals_variant(fused, s, v))
    if os.environ.get("STAMPS"):  # per-wave phase cycles (s_memtime), mean over nodes, per interval
        names = ["stage+prefetch", "bar1", "A+B+C", "bar2", "D+land", "E", "bar_end", "top"]
        buf = torch.zeros(nodes * 8 * 8, dtype=torch.int64, device="cuda")
        for v in (0, 2):
            acc.carry_stamps(fused, s, v, buf.data_ptr())
            acc.sync(s)
            a = buf.cpu().numpy().reshape(nodes, 8, 8).astype(np.float64) / K
            out[f"stamps_v{v}"] = {nm: [round(float(x)) for x in a[:, :, i].mean(axis=0)] for i, nm in enumerate(names)}
    acc.sync(s)
    per = accel.interval_bytes(L.zones, **L.sizes())
    carried = accel.intervals_bytes(L.zones, *[L.sizes()[k] for k in ("n_nodes", "n_procs", "n_ctrs", "n_vms", "n_pods")],
                                    K, True)
    out["us_per_interval"] = {k[:-3]: v * 1e3 / K for k, v in out.items() if k.endswith("_ms")}
    out["fused_TBps_carried_bytes"] = carried / (out["fused_ms"] * 1e-3) / 1e12
    out["fused_TBps_unfused_bytes"] = K * per / (out["fused_ms"] * 1e-3) / 1e12
    print(json.dumps(out))


if __name__ == "__main__":
    main()
