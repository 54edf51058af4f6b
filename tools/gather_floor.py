#!/usr/bin/env python3
"""How fast can one GPU gather the namespace sums' pod records at config 3?  Times, on
the same device and buffers: a contiguous read of the pod table (0.7M x 64-B
[energy | power] records), torch.index_select of those records in a random order
(what the namespace CSR does: a namespace's pods sit at random slots) and in sorted
order, and kacc's cluster_partials launch itself for comparison (bench.py's
totals_compute_ms).  Diagnostic for DESIGN §4.2; prints one JSON object.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=20):
    import torch

    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = []
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        best.append(e0.elapsed_time(e1) * 1e3)
    best.sort()
    return best[len(best) // 2]


def main():
    import torch

    from kepler_amd import fleet

    L = fleet.config_layout(3)
    n_pods = L.n_pods
    rec = torch.randint(0, 1 << 40, (n_pods, 8), dtype=torch.int64, device="cuda")  # 64-B records
    off, slots = L.namespace_csr()
    idx = torch.from_numpy(slots.astype("int64")).cuda()
    srt = torch.sort(idx).values
    out = torch.empty_like(rec)
    red = torch.empty(n_pods // 8 + 1, 8, dtype=torch.int64, device="cuda")
    bytes_ = n_pods * 64
    res = {"n_pods": n_pods, "n_namespaces": int(L.n_namespaces), "record_bytes": 64}
    res["contiguous_sum_us"] = timed(lambda: torch.sum(rec, dim=0, out=red[0]))
    res["copy_us"] = timed(lambda: out.copy_(rec))
    res["gather_csr_order_us"] = timed(lambda: torch.index_select(rec, 0, idx, out=out))
    res["gather_sorted_us"] = timed(lambda: torch.index_select(rec, 0, srt, out=out))
    for k in ("contiguous_sum_us", "gather_csr_order_us", "gather_sorted_us"):
        res[k.replace("_us", "_read_GBps")] = bytes_ / (res[k] * 1e-6) / 1e9
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
