#!/usr/bin/env python3
"""Slot-join dispatches for rocprofv3 --pmc passes (tools/join_pmc.sh): config 3's small-node
PID join in its steady state (2 % churn, fleet.KeyedChurn), REPS joins per variant in
VARIANTS order (kacc_debug_set_join_variant; -1 = production), each variant from a reset
map and two warm-up joins; or, with STOPS=1,2,...,0, the production kernel stopped after each
phase (kacc_debug_join_variant), REPS times a reset + two full joins + the stopped join.  tools/join_pmc_summary.py averages the counters per kernel
instance (the variants are distinct template instances, so distinct kernel names)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from kepler_amd import accel, fleet
    from kepler_amd.torch_batch import current_stream_handle

    reps = int(os.environ.get("REPS", "6"))
    variants = [int(x) for x in os.environ.get("VARIANTS", "511,-1").split(",")]
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    stream = current_stream_handle()
    lib = accel.load()
    lib.kacc_debug_set_join_variant.argtypes = [ctypes.c_int]
    layout = fleet.config_layout(int(os.environ.get("CONFIG", "3")))
    rows = np.diff(layout.proc_off.astype(np.int64))
    slot_off = np.r_[0, np.cumsum(np.ceil(rows * 1.05).astype(np.int64) + 8)].astype(np.uint32)
    caps = layout.capacities()
    caps["proc_slots"] = int(slot_off[-1])
    acc = accel.Accel(layout.zones, **caps)
    sm = accel.SlotMap(acc, accel.KACC_KIND_PROC, slot_off)
    sm.set_policy(accel.KACC_JOIN_REUSE_TERMINATED)
    ks = fleet.KeyedChurn(layout.proc_off, churn=0.02)
    keys = [torch.from_numpy(ks.next_keys().astype(np.uint32).view(np.int32)).cuda() for _ in range(reps + 2)]
    off = torch.from_numpy(layout.proc_off.view(np.int32)).cuda()
    P = int(layout.proc_off[-1])
    cap = int(slot_off[-1])
    out = torch.zeros(P, dtype=torch.int32, device="cuda")
    tk = torch.zeros(cap, dtype=torch.int64, device="cuda")
    ts = torch.zeros(cap, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(layout.n_nodes, dtype=torch.int32, device="cuda")
    span = torch.zeros(2 * layout.n_nodes, dtype=torch.int32, device="cuda")
    stops = [int(x) for x in os.environ.get("STOPS", "").split(",") if x]
    if stops:  # per-phase counters of the production kernel: reset, two full joins, one stopped join
        lib.kacc_debug_join_variant.argtypes = [ctypes.c_void_p, ctypes.c_uint32] + [ctypes.c_void_p] * 7 + [ctypes.c_uint32]
        lib.kacc_debug_set_join_variant(-1)
        for s_ in stops:
            for _ in range(reps):
                sm.reset()
                for k in range(2):
                    sm.join(P, off.data_ptr(), keys[k].data_ptr(), 0, out.data_ptr(), tk.data_ptr(), ts.data_ptr(),
                            cnt.data_ptr(), stream, span.data_ptr())
                rc = lib.kacc_debug_join_variant(sm.handle, P, off.data_ptr(), keys[2].data_ptr(), out.data_ptr(),
                                                 tk.data_ptr(), ts.data_ptr(), cnt.data_ptr(), stream, s_)
                assert rc == 0, rc
        acc.sync(stream)
        variants = []
    for v in variants:
        lib.kacc_debug_set_join_variant(v)
        sm.reset()
        for k in range(reps + 2):
            sm.join(P, off.data_ptr(), keys[k].data_ptr(), 0, out.data_ptr(), tk.data_ptr(), ts.data_ptr(),
                    cnt.data_ptr(), stream, span.data_ptr())
        acc.sync(stream)
    lib.kacc_debug_set_join_variant(-1)
    print("done", flush=True)


if __name__ == "__main__":
    main()
