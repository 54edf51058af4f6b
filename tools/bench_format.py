#!/usr/bin/env python3
"""Exposition throughput at config 3 (20M process slots, Z=4): kacc_format_values
(the VALUE fields) and kacc_format_lines (whole `NAME{LABELS,zone="Z"} VALUE` lines
of kepler_process_cpu_joules_total, 80M lines) on one MI355X.  Labels are synthetic
fixed-width rows (`comm="proc",container_id="",exe="/usr/bin/proc",pid="NNNNNNNN",
state="running",type="regular",vm_id=""`), uploaded once.  Prints one JSON object.
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from kepler_amd import accel
    from kepler_amd.torch_batch import current_stream_handle

    rows = int(os.environ.get("ROWS", "20000000"))
    Z = 4
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    s = current_stream_handle()
    acc = accel.Accel(Z, nodes=1, proc_slots=rows, ctr_slots=1, vm_slots=1, pod_slots=1)
    rng = np.random.default_rng(3)
    acc.upload("proc_energy", rng.integers(0, 2**42, size=rows * Z, dtype=np.uint64))

    pre = b'comm="proc",container_id="",exe="/usr/bin/proc",pid="'
    post = b'",state="running",type="regular",vm_id=""'
    L = len(pre) + 8 + len(post)
    lab = np.empty((rows, L), dtype=np.uint8)
    lab[:, : len(pre)] = np.frombuffer(pre, dtype=np.uint8)
    pid = np.arange(rows, dtype=np.int64) + 10_000_000
    for k in range(8):
        lab[:, len(pre) + k] = ord("0") + (pid // 10 ** (7 - k)) % 10
    lab[:, len(pre) + 8:] = np.frombuffer(post, dtype=np.uint8)
    d_lab = torch.from_numpy(lab.reshape(-1)).cuda()
    d_off = torch.from_numpy((np.arange(rows + 1, dtype=np.int64) * L)).cuda()
    del lab
    n = rows * Z
    d_line_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    zones = ["package", "core", "uncore", "dram"]
    metric = "kepler_process_cpu_joules_total"
    args = ("proc_energy", metric, 0, rows, zones, d_lab.data_ptr(), d_off.data_ptr(), d_line_off.data_ptr())
    total = acc.format_lines(*args, stream=s)
    out = torch.empty(total, dtype=torch.uint8, device="cuda")

    def timed(fn, reps=5):
        ms = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ms.append(e0.elapsed_time(e1))
        return float(np.median(ms[1:]))

    ms_lines = timed(lambda: acc.format_lines(*args, out_ptr=out.data_ptr(), out_cap=total, stream=s))
    ms_size = timed(lambda: acc.format_lines(*args, stream=s))  # the sizing call alone (lengths, scan, total)
    fv = torch.empty(n * accel.KACC_FMT_WIDTH, dtype=torch.uint8, device="cuda")
    fl = torch.empty(n, dtype=torch.uint8, device="cuda")
    ms_vals = timed(lambda: acc.format_values("proc_energy", 0, n, fv.data_ptr(), fl.data_ptr(), s))
    head = bytes(out[:400].cpu().numpy()).decode().splitlines()[:2]
    acc.close()
    print(json.dumps({
        "rows": rows, "zones": Z, "lines": n, "text_bytes": total,
        "format_lines_ms": ms_lines, "lines_per_s": n / (ms_lines * 1e-3),
        "text_GBps": total / (ms_lines * 1e-3) / 1e9,
        "sizing_call_ms": ms_size, "write_pass_ms": ms_lines - ms_size,
        "write_pass_text_GBps": total / ((ms_lines - ms_size) * 1e-3) / 1e9,
        "format_values_ms": ms_vals, "values_per_s": n / (ms_vals * 1e-3),
        "sample": head,
        "note": "format_lines = sizing pass (values + lengths + scan + total read back) and the write pass",
    }, indent=1))


if __name__ == "__main__":
    main()
