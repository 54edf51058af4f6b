#!/usr/bin/env python3
"""Container-size skew at config-3 scale (10k nodes x 2k procs, Z=4): the container CPU-time
sum is one lane walking its rows in /proc order (Go sums in that order: bit-exactness forbids
reordering), so a node whose processes sit in ONE container serialises that lane.  Times
interval_kernel<4,0> (HIP events, median of ROUNDS back-to-back launches) for containers of
8 (BASELINE's shape), 64, 512 and ~2000 processes.  Prints one JSON object."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from kepler_amd import accel, fleet
    from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device

    torch.cuda.set_stream(torch.cuda.Stream())
    nodes = int(os.environ.get("NODES", "10000"))
    rounds = int(os.environ.get("ROUNDS", "10"))
    out = {"nodes": nodes, "procs_per_node": 2000, "zones": 4, "ms": {}}
    for ppc in (8, 64, 512, 2000):
        L = fleet.make_layout(nodes, 2000, 4, seed=7, procs_per_ctr=ppc, ctr_frac=0.99 if ppc >= 512 else 0.79)
        sim = fleet.FleetSim(L, seed=7)
        acc = accel.Accel(L.zones, **L.capacities())
        s = current_stream_handle()
        acc.run_interval(interval_from_tensors(to_device(sim.next_interval()), L.sizes(), L.fast_flag()), s)
        ivs = [interval_from_tensors(to_device(sim.next_interval()), L.sizes(), L.fast_flag()) for _ in range(2)]
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(rounds + 1)]
        for i in range(rounds + 1):
            ev[i][0].record()
            acc.run_interval(ivs[i % 2], s)
            ev[i][1].record()
        torch.cuda.synchronize()
        acc.sync(s)
        ms = float(np.median([a.elapsed_time(b) for a, b in ev[1:]]))
        out["ms"][f"procs_per_container_{ppc}"] = {"kernel_ms": ms, "containers": L.n_ctrs,
                                                   "max_container_rows": int(np.max(np.diff(np.r_[0, L.ctr_proc_end])))}
        acc.close()
        del ivs
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
