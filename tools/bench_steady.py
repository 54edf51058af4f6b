#!/usr/bin/env python3
"""The interval kernel on the slot layout the slot join actually produces.

A config-3 fleet (10k nodes x 2k procs, Z = 4) evolves under /proc-shaped churn:
each interval a CHURN fraction of the processes exits, and as many new ones
start in the same container (or VM / the node's pod-less rows); a new PID is
the largest of its node, so /proc lists it last in its container's rows
(informer.go:167-205 groups rows by container in listing order).  Every
interval goes through kacc_slot_join (the production join, optionally with
the terminated-slot reuse policy); after INTERVALS intervals the interval
kernel is timed on the join's slot words and spans, next to pristine slots
(slot = row) and the synthetic random fragmented layout, same box, same
inputs, back-to-back launches.  Prints one JSON object.
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

    intervals = int(os.environ.get("INTERVALS", "40"))
    churn = float(os.environ.get("CHURN", "0.02"))
    spare = float(os.environ.get("SPARE", "0.05"))
    policy = int(os.environ.get("POLICY", "0"))
    steps = int(os.environ.get("STEPS", "20"))
    nodes = int(os.environ.get("NODES", "10000"))
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    stream = current_stream_handle()
    t0 = time.time()
    layout = fleet.config_layout(3, nodes=nodes)
    sizes = layout.sizes()
    N, P = layout.n_nodes, sizes["n_procs"]
    off = layout.proc_off.astype(np.int64)
    rows = np.diff(off)
    slot_off = np.r_[0, np.cumsum(np.ceil(rows * (1 + spare)).astype(np.int64) + 8)].astype(np.uint32)
    caps = layout.capacities()
    caps["proc_slots"] = int(slot_off[-1])

    node_of_row = np.repeat(np.arange(N), rows)
    local = np.arange(P) - off[node_of_row]
    churner = fleet.ProcChurn(layout, churn=churn, seed=7)

    acc = accel.Accel(layout.zones, **caps)
    sm = accel.SlotMap(acc, accel.KACC_KIND_PROC, slot_off)
    if policy:
        sm.set_policy(policy)
    d_off = torch.from_numpy(layout.proc_off.view(np.int32)).cuda()
    d_slot = torch.zeros(P, dtype=torch.int32, device="cuda")
    tk = torch.zeros(int(slot_off[-1]), dtype=torch.int64, device="cuda")
    ts = torch.zeros(int(slot_off[-1]), dtype=torch.int32, device="cuda")
    cnt = torch.zeros(N, dtype=torch.int32, device="cuda")
    span = torch.zeros(2 * N, dtype=torch.int32, device="cuda")
    jms = []
    for it in range(intervals + 1):
        keys = churner.next_keys()
        d_keys = torch.from_numpy(keys.view(np.int32)).cuda()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        sm.join(P, d_off.data_ptr(), d_keys.data_ptr(), 0, d_slot.data_ptr(), tk.data_ptr(), ts.data_ptr(),
                cnt.data_ptr(), stream, span.data_ptr())
        e1.record()
        e1.synchronize()
        if it > 1:
            jms.append(e0.elapsed_time(e1))
        if it % 10 == 0:
            print(f"[steady] interval {it} ({time.time() - t0:.0f}s)", file=sys.stderr, flush=True)
    acc.sync(stream)
    slots = d_slot.cpu().numpy().view(np.uint32)
    spans = span.cpu().numpy().view(np.uint32)
    assert np.all(slots != 0xFFFFFFFF), "join errors"
    sl = (slots & np.uint32(accel.KACC_SLOT_MASK)).astype(np.int64)
    # layout statistics: rows whose slot follows the previous row's slot; span / rows
    same_node = np.r_[False, node_of_row[1:] == node_of_row[:-1]]
    seq = float(np.mean((sl[1:] == sl[:-1] + 1)[same_node[1:]]))
    lo = spans[0::2].astype(np.int64)
    hi = spans[1::2].astype(np.int64)
    span_over_rows = float(np.mean((hi - lo + 1) / rows))
    inv = np.argsort(sl, kind="stable")
    rank_disp = float(np.mean(np.abs(np.arange(P)[inv] - (np.arange(P)))))

    sim = fleet.FleetSim(layout, seed=fleet.SEED)
    statics = to_device(layout.static_arrays())
    prime = sim.next_interval()
    full = [sim.next_interval() for _ in range(2)]
    flags = layout.fast_flag() | accel.KACC_F_NODE_SLOT_RANGES

    # one context for every layout (contexts differ by up to 12 % on one box: table
    # placement), layouts timed in interleaved rounds
    a2 = accel.Accel(layout.zones, **caps)

    def make_ivs(proc_slot, span_arr):
        t = dict(statics)
        if span_arr is not None:
            t.update(to_device({"node_proc_span": span_arr}))
        ivs, keep = [], []
        for k in range(steps + 1):
            f = dict(full[k % 2])
            f["proc_slot"] = proc_slot
            tt = dict(t)
            tt.update(to_device({n: f[n] for n in ("proc_cpu_delta", "proc_slot", "ctr_slot", "vm_slot", "pod_slot",
                                                   "node_ts_ns", "node_usage_ratio", "node_status", "zone_energy",
                                                   "zone_max")}))
            keep.append(tt)
            ivs.append(interval_from_tensors(tt, sizes, flags))
        return ivs, keep

    def time_ivs(ivs):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in ivs]
        for k, iv in enumerate(ivs):
            ev[k][0].record()
            a2.run_interval(iv, stream)
            ev[k][1].record()
        torch.cuda.synchronize()
        return [x.elapsed_time(y) for x, y in ev[1:]]

    pristine = (slot_off[node_of_row].astype(np.int64) + local).astype(np.uint32)
    pristine_span = np.stack([slot_off[:-1], slot_off[:-1] + rows.astype(np.uint32) - 1], 1).reshape(-1).astype(np.uint32)
    res = {
        "config": "3 (10k nodes x 2k procs, Z=4)" if nodes == 10000 else f"3 shape, {nodes} nodes",
        "intervals": intervals, "churn": churn, "spare_slots": spare, "policy": policy,
        "join_ms_median": float(np.median(jms)) if jms else None,
        "steady_layout": {"rows_following_previous_slot": seq, "span_over_rows": span_over_rows,
                          "mean_rank_displacement": rank_disp},
        "kernel_ms": {},
    }
    tp = dict(statics)
    pr = dict(prime)
    pr["proc_slot"] = pristine
    tp.update(to_device(pr))
    a2.run_interval(interval_from_tensors(tp, sizes, flags), stream)
    frag = fleet.config_layout(3, nodes=nodes, fragment_slots=0.02)
    fslot = (slot_off[node_of_row].astype(np.int64) + (frag.proc_slot.astype(np.int64)
             - np.repeat(np.r_[0, np.cumsum((rows * 1.02).astype(np.int64) + 1)[:-1]], rows))).astype(np.uint32)
    fspan = np.zeros(2 * N, dtype=np.uint32)
    for_span = fslot.astype(np.int64)
    fspan[0::2] = np.minimum.reduceat(for_span, off[:-1])
    fspan[1::2] = np.maximum.reduceat(for_span, off[:-1])
    cases = {"pristine_no_span": make_ivs(pristine, None), "pristine_span": make_ivs(pristine, pristine_span),
             "join_steady_state_span": make_ivs(slots, spans), "synthetic_random_0.02_span": make_ivs(fslot, fspan)}
    times = {n: [] for n in cases}
    for _ in range(3):
        for n, (ivs, _) in cases.items():
            times[n] += time_ivs(ivs)
    a2.sync(stream)
    res["kernel_ms"] = {n: float(np.median(v)) for n, v in times.items()}
    k = res["kernel_ms"]
    res["steady_over_pristine"] = k["join_steady_state_span"] / k["pristine_no_span"]
    res["steady_over_pristine_span"] = k["join_steady_state_span"] / k["pristine_span"]
    res["synthetic_over_pristine_span"] = k["synthetic_random_0.02_span"] / k["pristine_span"]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
