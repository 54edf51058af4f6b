#!/usr/bin/env python3
"""Summary of tools/gpu_regress_ab.sh: per run, the rocprofv3 mean duration of the
config's main kernel, the bench line's kernel_ms, and (when present) the PMC bytes per
launch of small_kernel<2> (FETCH_SIZE x 2 + WRITE_SIZE, KiB counters; MI355X_MICROARCH §HBM).
usage: python tools/regress_summary.py OUTDIR"""
import csv
import glob
import json
import os
import statistics
import sys


def kernel_mean_us(d, sub):
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Name"]:
                return float(r["AverageNs"]) / 1e3, int(r["Calls"])
    return None, 0


def pmc(d, counter, sub):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return statistics.median(vals) if vals else None


def main():
    o = sys.argv[1]
    rows = []
    for js in sorted(glob.glob(os.path.join(o, "c*_r*.json"))):
        name = os.path.basename(js)[:-5]
        d = json.load(open(js))
        sub = "small_kernel<2" if name.startswith("c1") else "intervals_carry_kernel"
        us, calls = kernel_mean_us(os.path.join(o, name), sub)
        K = d.get("config", {}).get("intervals_per_step", 1) or 1
        rows.append(dict(run=name, rocprof_kernel_us=us, per_interval_us=(us / K if us else None), calls=calls,
                         bench_kernel_ms=d.get("kernel_ms"), ms_per_step=d.get("ms_per_step"),
                         frac=d.get("roofline", {}).get("frac"),
                         bytes_per_interval=d.get("roofline", {}).get("bytes_per_interval")))
    for b in ("r2", "main"):
        f = pmc(os.path.join(o, f"pmc_{b}_FETCH_SIZE"), "FETCH_SIZE", "small_kernel<2")
        w = pmc(os.path.join(o, f"pmc_{b}_WRITE_SIZE"), "WRITE_SIZE", "small_kernel<2")
        if f is not None and w is not None:
            rows.append(dict(run=f"pmc_{b}", fetch_GB=2 * f * 1024 / 1e9, write_GB=w * 1024 / 1e9,
                             hbm_GB=(2 * f + w) * 1024 / 1e9))
    with open(os.path.join(o, "summary.json"), "w") as fh:
        json.dump(rows, fh, indent=1)
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
