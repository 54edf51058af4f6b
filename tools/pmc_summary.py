#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into pmc_traffic.json.

usage: python tools/pmc_summary.py FETCH_DIR WRITE_DIR SOURCE_LABEL OUT.json [CONFIG [KERNEL [K]]]

KERNEL is a substring of the profiled kernel name (default "interval_kernel<4, 0>");
K > 1: the kernel is the one-launch K-interval carry kernel (entry "config<C>_k<K>",
algorithmic bytes kacc_intervals_bytes(carried), per-interval figures = per launch / K).
An existing OUT.json keeps its other configs' entries.

FETCH_SIZE is doubled (MI355X_MICROARCH.md §HBM: gfx950 tallies 128-B streaming
reads at 64 B); both counters are KiB.  Per launch of kacc::interval_kernel<Z,0>.
"""
import csv
import glob
import hashlib
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def values(d, counter, kernel="interval_kernel<4, 0>"):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                out.append(float(r["Counter_Value"]))
    return out


def main():
    fdir, wdir, label, out = sys.argv[1:5]
    cfg = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    kernel = sys.argv[6] if len(sys.argv) > 6 else "interval_kernel<4, 0>"
    K = int(sys.argv[7]) if len(sys.argv) > 7 else 1
    from kepler_amd import accel, fleet

    # PMC_SHARD_OF=W: rank 0's shard of the W-way split (bench.py --shard-of W); PMC_SUMS=1: the
    # launch also carries the previous interval's partial sums (bench.py --totals fused: entry
    # "config<C>_sums", algorithmic bytes + export_sums_bytes)
    shard_of = int(os.environ.get("PMC_SHARD_OF", "1"))
    sums = os.environ.get("PMC_SUMS", "0") == "1"
    if shard_of > 1:
        _, _, layout = fleet.config_shard(cfg, shard_of, 0, {1: 40000, 2: 1000, 3: 10000, 5: 1000}[cfg])
    else:
        layout = fleet.config_layout(cfg, nodes=40000 if cfg == 1 else None)  # bench.py --config 1 fleet
    s = layout.sizes()
    dims = [s[k] for k in ("n_nodes", "n_procs", "n_ctrs", "n_vms", "n_pods")]
    # the flags bench.py / tools/bench_variants.py run with
    flags = layout.fast_flag() | accel.KACC_F_NODE_SLOT_RANGES | accel.KACC_F_STABLE_SLOT_NODES
    alg = (accel.interval_bytes(layout.zones, *dims, flags) if K == 1 else
           accel.intervals_bytes(layout.zones, *dims, K, True, flags))
    if sums:
        from bench import export_sums_bytes

        alg += export_sums_bytes(layout.zones, s["n_nodes"], s["n_pods"], layout.n_namespaces)
    # KERNEL "a|b|c": the launches of one interval (config 5: interval_kernel + chunk_kernel +
    # pod_kernel), each kernel's median summed
    fm = wm = 0.0
    fv, wv = [], []
    for kn in kernel.split("|"):
        f1, w1 = values(fdir, "FETCH_SIZE", kn), values(wdir, "WRITE_SIZE", kn)
        if not f1 or not w1:
            raise SystemExit(f"no {kn} counter rows found")
        fm += statistics.median(f1)
        wm += statistics.median(w1)
        fv += f1
        wv += w1
    res = {}
    if os.path.exists(out):
        with open(out) as f:
            res = json.load(f)
    key = f"config{cfg}" + (f"_k{K}" if K > 1 else "") + ("_sums" if sums else "")
    res.update({
        key: {
            "n_procs": s["n_procs"],
            "shard_of": shard_of,
            "kernel": " + ".join("kacc::" + kn.replace(" ", "") for kn in kernel.split("|")),
            "fetch_size_kib_median": fm,
            "write_size_kib_median": wm,
            "hbm_bytes_per_launch": (2.0 * fm + wm) * 1024.0,
            "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over the "
            "config's command in tools/gpu_pmc_traffic.sh; FETCH_SIZE doubled per "
            "MI355X_MICROARCH.md §HBM (gfx950 tallies 128-B streaming reads at 64 B); values in KiB",
            "algorithmic_bytes_per_launch": alg,
            "intervals_per_launch": K,
            "hbm_bytes_per_interval": (2.0 * fm + wm) * 1024.0 / K,
            "algorithmic_bytes_per_interval": alg / K,
            "source": label,
            # the build the counters belong to: bench.py reports them only for this very library
            "lib_sha256": hashlib.sha256(open(accel.LIB_PATH, "rb").read()).hexdigest(),
            "raw_kib": {"FETCH_SIZE": fv, "WRITE_SIZE": wv},
        }
    })
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    r = res[key]
    print(f"traffic {r['hbm_bytes_per_launch']/1e9:.3f} GB/launch vs algorithmic {alg/1e9:.3f} GB")


if __name__ == "__main__":
    main()
