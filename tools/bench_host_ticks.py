#!/usr/bin/env python3
"""The CPU-tick end-to-end path (bench.py host_path_ticks) split: copies alone, kernels alone,
both with 2 and 3 staging buffers — where the interval time goes beyond the pinned copy.
Prints one JSON object."""
import json
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import bench

    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    args = types.SimpleNamespace(config=3, nodes=None)
    out = {}
    for nbuf, mode in ((2, "full"), (2, "copy"), (2, "compute"), (3, "full"), (4, "full")):
        r = bench.host_path_ticks_line(args, steps=10, nbuf=nbuf, mode=mode)
        out[f"{mode}_{nbuf}"] = {k: r[k] for k in ("ms_per_interval", "proc_attr_per_s", "pcie_copy_ms", "h2d_bytes_per_interval")}
        print(f"{mode} x{nbuf}: {r['ms_per_interval']:.3f} ms", file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
