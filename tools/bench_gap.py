#!/usr/bin/env python3
"""Why the headline loop's interval kernel is slower than the same kernel back to back.

One config-3 context, the headline's inputs; interval-kernel time (HIP events on
the launch stream) in interleaved rounds of: the headline step (interval +
cluster partials), intervals back to back, intervals with a device sync between
them, and intervals with a cluster-partials launch before each one.  Prints JSON.
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from kepler_amd import accel, fleet
    from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device

    steps = int(os.environ.get("STEPS", "20"))
    rounds = int(os.environ.get("ROUNDS", "3"))
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    comm = torch.cuda.Stream()
    _, _, layout = fleet.config_shard(3, 1, 0, 10000)
    sim = fleet.FleetSim(layout, seed=fleet.SEED)
    sizes = layout.sizes()
    acc = accel.Accel(layout.zones, **layout.capacities())
    cluster = accel.Cluster.join(acc, accel.Cluster.unique_id(), 1, 0)
    stream = current_stream_handle()
    statics = to_device(layout.static_arrays())
    flags = layout.fast_flag() | accel.KACC_F_NODE_SLOT_RANGES
    prime = to_device(sim.next_interval())
    acc.run_interval(interval_from_tensors(prime, sizes), stream)
    del prime
    full = [to_device(sim.next_interval()) for _ in range(2)]
    ivs = []
    for k in range(steps + 1):
        t = dict(statics)
        t.update(full[k % 2])
        t.update(to_device({n: a for n, a in sim.next_node_inputs().items()
                            if n in ("node_ts_ns", "node_usage_ratio", "node_status", "zone_energy", "zone_max")}))
        ivs.append(interval_from_tensors(t, sizes, flags))
    ns_off, ns_slot = layout.namespace_csr()
    ns_t = to_device({"off": ns_off, "slot": ns_slot})
    n_ns = len(ns_off) - 1
    Z = layout.zones
    ns_e = torch.zeros(n_ns * Z, dtype=torch.int64, device="cuda")
    ns_p = torch.zeros(n_ns * Z, dtype=torch.float64, device="cuda")
    nd_e = torch.zeros(2 * Z, dtype=torch.int64, device="cuda")
    nd_p = torch.zeros(3 * Z, dtype=torch.float64, device="cuda")

    def partials():
        cluster.allreduce_namespaces(n_ns, [ns_t["off"].data_ptr()], [ns_t["slot"].data_ptr()],
                                     [ns_e.data_ptr()], [ns_p.data_ptr()], [nd_e.data_ptr()], [nd_p.data_ptr()],
                                     streams=[stream], comm_streams=[comm.cuda_stream])

    def timed(mode):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps + 1)]
        for i in range(steps + 1):
            if mode == "partials_before":
                partials()
            ev[i][0].record()
            acc.run_interval(ivs[i], stream)
            ev[i][1].record()
            if mode == "headline":
                partials()
            elif mode == "sync":
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        return [a.elapsed_time(b) for a, b in ev[1:]]

    if os.environ.get("CONTEXTS"):  # placement: several contexts, timed round-robin
        accs = [acc] + [accel.Accel(layout.zones, **layout.capacities()) for _ in range(int(os.environ["CONTEXTS"]) - 1)]
        p2 = to_device(sim.next_interval())
        for a2 in accs[1:]:
            a2.run_interval(interval_from_tensors(p2, sizes), stream)
        per = {i: [] for i in range(len(accs))}
        for _ in range(rounds * 2):
            for i, a2 in enumerate(accs):
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
                for j in range(steps):
                    ev[j][0].record()
                    a2.run_interval(ivs[j + 1], stream)
                    ev[j][1].record()
                torch.cuda.synchronize()
                per[i].append(round(float(np.mean([x.elapsed_time(y) for x, y in ev])), 4))
        print(json.dumps({"per_context_round_means_ms": per,
                          "tables": {i: [hex(a2.device_ptr(n)) for n in ("proc_energy", "proc_ratio")]
                                     for i, a2 in enumerate(accs)}}, indent=1))
        return
    modes = ["headline", "b2b", "sync", "partials_before"]
    res = {m: [] for m in modes}
    for _ in range(rounds):
        for m in modes:
            res[m] += timed(m)
    acc.sync(stream)
    out = {m: {"median_ms": float(np.median(v)), "mean_ms": float(np.mean(v)), "min_ms": float(np.min(v))}
           for m, v in res.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
