#!/usr/bin/env python3
"""Host time of kacc_pack per 20M rows (BASELINE config 3's fleet as informer records).

The records are the config-3 fleet's rows with VM and regular processes
interleaved among the container processes (tests/test_packer.py's round trip),
packed into a pinned-size output at 1..T host threads; median of 5 runs after
a warm-up.  Prints one JSON line."""

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from kepler_amd import accel, fleet  # noqa: E402
from test_packer import _records_from_layout  # noqa: E402


def main():
    nodes = int(os.environ.get("NODES", "10000"))
    L = fleet.config_layout(3, nodes=nodes)
    t0 = time.time()
    _, r = _records_from_layout(L, seed=4)
    gen = time.time() - t0
    R = L.n_procs
    out = {n: np.zeros(max(R if not n.endswith("_off") else L.n_nodes + 1, 1), dtype=dt)
           for n, dt in accel.PACKED_ARRAYS}
    res = {"rows": R, "nodes": L.n_nodes, "records_generated_s": gen, "cpu_count": os.cpu_count()}
    for t in [int(x) for x in os.environ.get("THREADS", "1,4,8,16,32").split(",")]:
        accel.pack(threads=t, out=out, **r)  # warm-up
        ts = []
        for _ in range(5):
            t1 = time.perf_counter()
            accel.pack(threads=t, out=out, **r)
            ts.append(time.perf_counter() - t1)
        med = float(np.median(ts))
        res[f"threads_{t}"] = {"median_ms": med * 1e3, "ms_per_20M_rows": med * 1e3 * 20e6 / R,
                               "rows_per_s": R / med}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
