#!/usr/bin/env python3
"""PCIe-inclusive rate of the pinned host-batch path (the cgo caller's path).

The Go packer writes each interval into a pinned batch
(kacc_batch_alloc) and calls kacc_batch_submit / kacc_batch_wait.  This tool
times that path at a BASELINE config (default 3: 10k nodes x 2k procs, Z=4)
with the batches already filled (the packer writes in place), so what is timed
is: host layout validation (kacc_validate_host, multi-threaded) + H2D copies of
the interval's inputs over PCIe + the interval kernel.

  serial     submit(A); wait(A) per interval
  pipelined  two batches: submit(B); wait(A); ... -> the copies of one interval
             overlap the kernel of the previous one (copy stream + events)
  trusted    pipelined with KACC_F_TRUSTED_LAYOUT (slots from kacc_slot_join:
             no host layout check; the device range checks remain)

Also reported: the validation alone, a plain pinned->device copy of the same
bytes (torch, the PCIe ceiling), and the bytes per interval.  Prints one JSON
object.  This is never bench.py's `value` (inputs there are resident in HBM).
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

    cfg = int(os.environ.get("CONFIG", "3"))
    steps = int(os.environ.get("STEPS", "10"))
    torch.cuda.set_device(0)
    layout = fleet.config_layout(cfg)
    sizes = layout.sizes()
    sim = fleet.FleetSim(layout)
    acc = accel.Accel(layout.zones, **layout.capacities())
    ivs = [sim.next_interval() for _ in range(2 + steps)]
    batches = [accel.HostBatch.alloc(acc, **sizes) for _ in range(2)]

    def h2d_bytes(a):
        return int(sum(v.nbytes for k, v in a.items() if k in accel.INTERVAL_ARRAYS and v is not None))

    nbytes = h2d_bytes(ivs[0])

    # host validation alone (the first step of every submit)
    batches[0].fill(ivs[0])
    tv = []
    for _ in range(5):
        t0 = time.perf_counter()
        rc = acc.validate_host(batches[0].view.contents)
        tv.append(time.perf_counter() - t0)
        assert rc == 0, acc.last_error()

    # first read (untimed), then refill both batches with later intervals
    batches[0].submit()
    batches[0].wait()
    for b, a in zip(batches, ivs[1:3]):
        b.fill(a)

    def serial(k):
        t0 = time.perf_counter()
        for _ in range(k):
            batches[0].submit()
            batches[0].wait()
        return (time.perf_counter() - t0) / k

    def pipelined(k):
        t0 = time.perf_counter()
        batches[0].submit()
        for i in range(1, k):
            batches[i % 2].submit()
            batches[(i - 1) % 2].wait()
        batches[(k - 1) % 2].wait()
        return (time.perf_counter() - t0) / k

    serial(2)
    t_serial = serial(steps)
    pipelined(4)
    t_pipe = pipelined(steps)
    # packer slots from kacc_slot_join: host layout check skipped (device checks stay)
    for b, a in zip(batches, ivs[3:5]):
        b.fill(a, accel.KACC_F_TRUSTED_LAYOUT)
    pipelined(4)
    t_trusted = pipelined(steps)

    # the PCIe ceiling: one pinned -> device copy of the same byte count
    src = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    cps = []
    for _ in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        cps.append(time.perf_counter() - t0)
    t_copy = float(np.median(cps[1:]))

    for b in batches:
        b.free()
    acc.close()
    P = sizes["n_procs"]
    out = {
        "config": cfg,
        "sizes": sizes,
        "zones": layout.zones,
        "h2d_bytes_per_interval": nbytes,
        "validate_ms": 1e3 * float(np.median(tv)),
        "host_threads": min(16, os.cpu_count() or 1),
        "h2d_copy_ms": 1e3 * t_copy,
        "h2d_copy_GBps": nbytes / t_copy / 1e9,
        "serial_ms_per_interval": 1e3 * t_serial,
        "pipelined_ms_per_interval": 1e3 * t_pipe,
        "serial_proc_attr_per_s": P / t_serial,
        "pipelined_proc_attr_per_s": P / t_pipe,
        "pipelined_node_snapshots_per_s": sizes["n_nodes"] / t_pipe,
        "trusted_pipelined_ms_per_interval": 1e3 * t_trusted,
        "trusted_pipelined_proc_attr_per_s": P / t_trusted,
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
