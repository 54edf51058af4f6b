#!/usr/bin/env python3
"""Slot-join throughput at a BASELINE config (default 3: 10k nodes x 2k procs).

Times kacc_slot_join alone (HIP events on the launch stream) and the fused
interval step join -> interval kernel, with 2 % process churn per interval,
keys resident in HBM.  CPU reference: the oracle join (C++ unordered_map per
node, the Go-map shape) on a bounded node sample.  Prints one JSON object.

Algorithmic bytes of one join launch: per row the PID 4 B
read and the slot word 4 B written; per node its table read once (8-B packed
buckets); changed buckets written back (2 x churn x rows x 8 B).
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def node_buckets(s):
    """kacc_join.hip node_buckets: the smallest power of two >= 1.5 x the node's slots (a
    multiple of 64 instead — 8-22 % fewer table bytes — was 7 % slower: JOIN_POW2=0 gives that
    variant's bytes, profiles/r03/joinab)."""
    if os.environ.get("JOIN_POW2", "1") == "0":
        return max(64, (3 * s // 2 + 64) & ~63)
    h = 64
    while h * 2 < 3 * s:
        h <<= 1
    return h


def main():
    import torch

    from kepler_amd import accel, fleet
    from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device

    cfg = int(os.environ.get("CONFIG", "3"))
    steps = int(os.environ.get("STEPS", "20"))
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    stream = current_stream_handle()
    layout = fleet.config_layout(cfg)
    sizes = layout.sizes()
    rows = np.diff(layout.proc_off.astype(np.int64))
    slot_off = np.r_[0, np.cumsum(rows * 5 // 4 + 8)].astype(np.uint32)
    caps = layout.capacities()
    caps["proc_slots"] = int(slot_off[-1])
    acc = accel.Accel(layout.zones, **caps)
    sm = accel.SlotMap(acc, accel.KACC_KIND_PROC, slot_off)
    sim = fleet.FleetSim(layout, churn=0.0)
    keys_sim = fleet.KeyedChurn(layout.proc_off, churn=0.02)
    n_sets = 4
    key_sets = [torch.from_numpy(keys_sim.next_keys().astype(np.uint32).view(np.int32)).cuda() for _ in range(n_sets + 1)]
    a = sim.next_interval()
    t = to_device(a)
    t_next = [to_device({k: v for k, v in sim.next_interval().items() if k in ("node_ts_ns", "zone_energy", "node_usage_ratio")}) for _ in range(n_sets)]
    off = t["proc_off"]
    cap = int(slot_off[-1])
    tk = torch.zeros(cap, dtype=torch.int64, device="cuda")
    ts = torch.zeros(cap, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(layout.n_nodes, dtype=torch.int32, device="cuda")
    span = torch.zeros(2 * layout.n_nodes, dtype=torch.int32, device="cuda")
    t["node_proc_span"] = span  # the join's per-node slot spans: rows swept in slot order
    P = sizes["n_procs"]

    def join(k):
        sm.join(P, off.data_ptr(), key_sets[k].data_ptr(), 0, t["proc_slot"].data_ptr(), tk.data_ptr(),
                ts.data_ptr(), cnt.data_ptr(), stream, span.data_ptr())

    tr = accel.Tracker(acc, accel.KACC_KIND_PROC, 500, zone=0, min_energy=10 * 10**6)  # config.go:210-211

    def track():
        tr.add(sm, tk.data_ptr(), ts.data_ptr(), cnt.data_ptr(), stream)

    flag = layout.fast_flag()
    join(n_sets)  # first interval: every ID new
    acc.run_interval(interval_from_tensors(t, sizes, flag), stream)
    acc.sync(stream)
    tj, tall, ttr, tseq = [], [], [], []
    for s in range(steps):
        k = s % n_sets
        t.update(t_next[k])
        it = interval_from_tensors(t, sizes, flag)
        e0, e1, e2, e3 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
        e0.record()
        join(k)
        e1.record()
        # the tracker reads the terminated slots' final values (power derived from their
        # node's ActivePower) BEFORE the interval rewrites them: process.go:87-99 then :118-148
        if s % 2:  # an export every other interval: Clear() first (process.go:80-84)
            tr.clear(stream)
        track()
        e2.record()
        acc.run_interval(it, stream)
        e3.record()
        e3.synchronize()
        tj.append(e0.elapsed_time(e1))
        tall.append(e0.elapsed_time(e1) + e2.elapsed_time(e3))  # join + interval
        ttr.append(e1.elapsed_time(e2))
        tseq.append(e0.elapsed_time(e3))
    acc.sync(stream)
    # the same pipeline with the tracker on a second stream: it must read the
    # terminated slots' final values before the interval (a terminated process's
    # power is derived from its node's ActivePower, which the interval rewrites;
    # kacc_tracker_add's ordering rule), so the interval waits for it — the second
    # stream only moves the clear/add launches off the join's stream
    s2 = torch.cuda.Stream()
    tpipe = []
    for s in range(steps):
        k = s % n_sets
        t.update(t_next[k])
        it = interval_from_tensors(t, sizes, flag)
        e0, e3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        joined = torch.cuda.Event()
        e0.record()
        join(k)
        joined.record()
        s2.wait_event(joined)
        if s % 2:
            tr.clear(s2.cuda_stream)
        tr.add(sm, tk.data_ptr(), ts.data_ptr(), cnt.data_ptr(), s2.cuda_stream)
        torch.cuda.current_stream().wait_stream(s2)
        acc.run_interval(it, stream)
        e3.record()
        e3.synchronize()
        tpipe.append(e0.elapsed_time(e3))
    acc.sync(stream)
    # production order with KACC_JOIN_REUSE_TERMINATED: join -> tracker (reads the
    # terminated slots' final values) -> interval (rewrites them), one stream, keys
    # of /proc-shaped churn (fleet.ProcChurn); the interval runs on the join's spans
    sm2 = accel.SlotMap(acc, accel.KACC_KIND_PROC, slot_off)
    sm2.set_policy(accel.KACC_JOIN_REUSE_TERMINATED)
    pchurn = fleet.ProcChurn(layout, churn=0.02)
    pkeys = [torch.from_numpy(pchurn.next_keys().view(np.int32)).cuda() for _ in range(steps + n_sets + 1)]
    tr2 = accel.Tracker(acc, accel.KACC_KIND_PROC, 500, zone=0, min_energy=10 * 10**6)

    def join2(k):
        sm2.join(P, off.data_ptr(), pkeys[k].data_ptr(), 0, t["proc_slot"].data_ptr(), tk.data_ptr(),
                 ts.data_ptr(), cnt.data_ptr(), stream, span.data_ptr())

    for k in range(n_sets + 1):  # warm: the steady state of the first few intervals
        join2(k)
    acc.run_interval(interval_from_tensors(t, sizes, flag), stream)
    acc.sync(stream)
    treuse, treuse_j, treuse_i = [], [], []
    for s_ in range(steps):
        k = s_ % n_sets
        t.update(t_next[k])
        it = interval_from_tensors(t, sizes, flag)
        e0, e1, e2, e3 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
        e0.record()
        join2(n_sets + 1 + s_)  # consecutive intervals of churn
        e1.record()
        if s_ % 2:
            tr2.clear(stream)
        tr2.add(sm2, tk.data_ptr(), ts.data_ptr(), cnt.data_ptr(), stream)
        e2.record()
        acc.run_interval(it, stream)
        e3.record()
        e3.synchronize()
        treuse.append(e0.elapsed_time(e3))
        treuse_j.append(e0.elapsed_time(e1))
        treuse_i.append(e2.elapsed_time(e3))
    acc.sync(stream)
    n_term = int(cnt.sum().item())
    # exposition values of every process row x zone (kacc_format_values), energy and power
    nval = int(slot_off[-1]) * layout.zones
    fout = torch.empty(nval * accel.KACC_FMT_WIDTH, dtype=torch.uint8, device="cuda")
    flen = torch.empty(nval, dtype=torch.uint8, device="cuda")
    tf = []
    for rep in range(6):
        f0, f1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        f0.record()
        acc.format_values("proc_energy" if rep % 2 == 0 else "proc_power", 0, nval, fout.data_ptr(),
                          flen.data_ptr(), stream)
        f1.record()
        f1.synchronize()
        tf.append(f0.elapsed_time(f1))
    fmt_ms = float(np.median(tf[2:]))
    del fout, flen
    # phase ablation (kacc_debug_join_variant): each variant timed from the same state
    import ctypes
    lib = accel.load()
    lib.kacc_debug_join_variant.argtypes = [ctypes.c_void_p, ctypes.c_uint32] + [ctypes.c_void_p] * 7 + [ctypes.c_uint32]
    phases = {}
    for v in [int(x) for x in os.environ.get("STOPS", "1,2,3,4,5,0").split(",")]:
        ms = []
        for rep in range(4):
            sm.reset()
            join(0)
            join(1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = lib.kacc_debug_join_variant(sm.handle, P, ctypes.c_void_p(off.data_ptr()), ctypes.c_void_p(key_sets[2].data_ptr()),
                                             ctypes.c_void_p(t["proc_slot"].data_ptr()), ctypes.c_void_p(tk.data_ptr()),
                                             ctypes.c_void_p(ts.data_ptr()), ctypes.c_void_p(cnt.data_ptr()),
                                             ctypes.c_void_p(stream), v)
            e1.record()
            e1.synchronize()
            assert rc == 0
            ms.append(e0.elapsed_time(e1))
        phases[f"stop_after_{v}" if v else "full"] = float(np.median(ms))
    acc.sync(stream)
    H = sum(node_buckets(int(x)) for x in np.diff(slot_off.astype(np.int64)))
    join_bytes = 8 * P + 8 * H + int(2 * 0.02 * P) * 8
    jm, am = float(np.median(tj)), float(np.median(tall))

    # CPU reference: oracle join on the first 200 nodes (Go-map shape), bounded
    from oracle.oracle import OracleSlotMap

    nn = min(200, layout.n_nodes)
    sub_off = layout.proc_off[: nn + 1].astype(np.uint32)
    o = OracleSlotMap(slot_off[: nn + 1])
    ks = fleet.KeyedChurn(sub_off, churn=0.02)
    o.join(sub_off, ks.next_keys())
    t0, reps = time.time(), 0
    while time.time() - t0 < 5.0:
        o.join(sub_off, ks.next_keys())
        reps += 1
    cpu_rate = reps * int(sub_off[-1]) / (time.time() - t0)
    print(json.dumps({
        "config": cfg, "n_procs": P, "n_nodes": layout.n_nodes, "buckets": H,
        "join_ms": jm, "join_plus_interval_ms": am, "tracker_ms": float(np.median(ttr)),
        "tracker_items": int(tr.items()[0].size),
        "pipeline_ms": float(np.median(tseq)), "pipeline_tracker_beside_interval_ms": float(np.median(tpipe)),
        "pipeline_reuse_tracker_first_ms": float(np.median(treuse)),
        "pipeline_reuse_join_ms": float(np.median(treuse_j)), "pipeline_reuse_interval_ms": float(np.median(treuse_i)),
        "join_rows_per_s": P / (jm * 1e-3), "join_plus_interval_proc_attr_per_s": P / (am * 1e-3),
        "join_bytes": join_bytes, "join_GBps": join_bytes / (jm * 1e-3) / 1e9,
        "terminated_last": n_term, "phase_ms": phases,
        "format_values": nval, "format_ms": fmt_ms, "format_values_per_s": nval / (fmt_ms * 1e-3),
        "cpu_oracle_join_rows_per_s": cpu_rate, "cpu_sample": f"{nn} nodes, {reps} intervals, 1 thread",
    }, indent=1))


if __name__ == "__main__":
    main()
