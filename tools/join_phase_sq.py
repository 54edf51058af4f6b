#!/usr/bin/env python3
"""Per-phase instruction counts of the small-node slot join at config 3: the
kacc_debug_join_variant stops (1 load ... 5 new slots, 0 full), each launched
REPS times from the same state, for rocprofv3 --pmc SQ_* passes (the counters
of each stop's dispatches, minus the previous stop's, are that phase's)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from kepler_amd import accel, fleet
    from kepler_amd.torch_batch import current_stream_handle

    reps = int(os.environ.get("REPS", "3"))
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    stream = current_stream_handle()
    lib = accel.load()
    lib.kacc_debug_join_variant.argtypes = [ctypes.c_void_p, ctypes.c_uint32] + [ctypes.c_void_p] * 7 + [ctypes.c_uint32]
    layout = fleet.config_layout(3)
    rows = np.diff(layout.proc_off.astype(np.int64))
    slot_off = np.r_[0, np.cumsum(rows * 5 // 4 + 8)].astype(np.uint32)
    caps = layout.capacities()
    caps["proc_slots"] = int(slot_off[-1])
    acc = accel.Accel(layout.zones, **caps)
    sm = accel.SlotMap(acc, accel.KACC_KIND_PROC, slot_off)
    ks = fleet.KeyedChurn(layout.proc_off, churn=0.02)
    keys = [torch.from_numpy(ks.next_keys().astype(np.uint32).view(np.int32)).cuda() for _ in range(3)]
    off = torch.from_numpy(layout.proc_off.view(np.int32)).cuda()
    P = int(layout.proc_off[-1])
    cap = int(slot_off[-1])
    out = torch.zeros(P, dtype=torch.int32, device="cuda")
    tk = torch.zeros(cap, dtype=torch.int64, device="cuda")
    ts = torch.zeros(cap, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(layout.n_nodes, dtype=torch.int32, device="cuda")
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    for stop in (1, 2, 3, 4, 5, 0):
        for _ in range(reps):
            sm.reset()
            for k in range(2):
                sm.join(P, off.data_ptr(), keys[k].data_ptr(), 0, out.data_ptr(), tk.data_ptr(), ts.data_ptr(),
                        cnt.data_ptr(), stream)
            rc = lib.kacc_debug_join_variant(sm.handle, P, ptr(off), ptr(keys[2]), ptr(out), ptr(tk), ptr(ts),
                                             ptr(cnt), ctypes.c_void_p(stream), stop)
            assert rc == 0
    acc.sync(stream)
    print("done", flush=True)


if __name__ == "__main__":
    main()
