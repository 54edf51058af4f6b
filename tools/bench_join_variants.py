#!/usr/bin/env python3
"""Slot-join variant A/B at a BASELINE config (default 3): every small-node join
variant (kacc_debug_set_join_variant) timed in interleaved rounds on the same box
from the same state, and its outputs (slot words, terminated lists, spans) checked
identical to the production variant's over a churn sequence.  Prints one JSON object.
"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from kepler_amd import accel, fleet
    from kepler_amd.torch_batch import current_stream_handle

    cfg = int(os.environ.get("CONFIG", "3"))
    # 31: round 2's kernel (8-B PID buckets); 63 / 127 / 255: + 6-B buckets, + seen marks
    # without return, + vector rows; 223: seen marks + vector rows on 8-B buckets; 511: 255 +
    # lookups reading four buckets per LDS read = production (-1); 1535: + DPP scans and
    # reductions (measured no faster: profiles/r04/join_group)
    variants = [int(x) for x in os.environ.get("VARIANTS", "31,127,1535,-1").split(",")]
    rounds = int(os.environ.get("ROUNDS", "3"))
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    stream = current_stream_handle()
    lib = accel.load()
    lib.kacc_debug_set_join_variant.argtypes = [ctypes.c_int]
    lib.kacc_debug_set_join_variant.restype = ctypes.c_int
    layout = fleet.config_layout(cfg)
    rows = np.diff(layout.proc_off.astype(np.int64))
    slot_off = np.r_[0, np.cumsum(rows * 5 // 4 + 8)].astype(np.uint32)
    caps = layout.capacities()
    caps["proc_slots"] = int(slot_off[-1])
    acc = accel.Accel(layout.zones, **caps)
    sm = accel.SlotMap(acc, accel.KACC_KIND_PROC, slot_off)
    keys_sim = fleet.KeyedChurn(layout.proc_off, churn=0.02)
    n_sets = 6
    key_sets = [torch.from_numpy(keys_sim.next_keys().astype(np.uint32).view(np.int32)).cuda() for _ in range(n_sets)]
    off = torch.from_numpy(layout.proc_off.astype(np.uint32).view(np.int32)).cuda()
    P = int(layout.proc_off[-1])
    cap = int(slot_off[-1])
    N = layout.n_nodes
    out = torch.zeros(P, dtype=torch.int32, device="cuda")
    tk = torch.zeros(cap, dtype=torch.int64, device="cuda")
    ts = torch.zeros(cap, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(N, dtype=torch.int32, device="cuda")
    span = torch.zeros(2 * N, dtype=torch.int32, device="cuda")

    def join(k):
        sm.join(P, off.data_ptr(), key_sets[k].data_ptr(), 0, out.data_ptr(), tk.data_ptr(), ts.data_ptr(),
                cnt.data_ptr(), stream, span.data_ptr())

    def run_seq(variant, timed):
        """reset, then joins over key sets 0..n_sets-1; times the last three."""
        lib.kacc_debug_set_join_variant(variant)
        sm.reset()
        ms, outs = [], []
        for k in range(n_sets):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            join(k)
            e1.record()
            e1.synchronize()
            if k >= 2:
                ms.append(e0.elapsed_time(e1))
            if not timed:
                c = cnt.cpu().numpy().astype(np.int64)
                terms = []
                s = slot_off[:-1].astype(np.int64)
                tkn, tsn = tk.cpu().numpy(), ts.cpu().numpy()
                for n in range(0, N, 97):  # a sample of nodes' terminated lists
                    terms.append((tkn[s[n]:s[n] + c[n]].copy(), tsn[s[n]:s[n] + c[n]].copy()))
                outs.append((out.cpu().numpy().copy(), c, span.cpu().numpy().copy(), terms))
        acc.sync(stream)
        return ms, outs

    ref = None
    checks = {}
    for v in variants:
        _, outs = run_seq(v, False)
        if ref is None:
            ref = outs
        same = all(np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
                   and all(np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1]) for x, y in zip(a[3], b[3]))
                   for a, b in zip(outs, ref))
        checks[str(v)] = same
    times = {str(v): [] for v in variants}
    for _ in range(rounds):
        for v in variants:
            ms, _ = run_seq(v, True)
            times[str(v)] += ms
    lib.kacc_debug_set_join_variant(-1)
    H = 0
    for s_ in np.diff(slot_off.astype(np.int64)):
        h = 64
        while h * 2 < 3 * s_:
            h <<= 1
        H += h
    join_bytes = 8 * P + 8 * H + int(2 * 0.02 * P) * 8
    res = {"config": cfg, "n_procs": P, "n_nodes": N, "join_bytes": join_bytes, "identical_to_first": checks,
           "join_ms": {v: float(np.median(t)) for v, t in times.items()},
           "frac_of_8TBs": {v: join_bytes / (float(np.median(t)) * 1e-3) / 8e12 for v, t in times.items()}}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
