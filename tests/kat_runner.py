"""Runs tests/golden/kat_cases.json against a backend (oracle or engine)."""

from __future__ import annotations

import json
import os

import numpy as np

from kepler_amd.accel import ARRAY_DTYPES

HERE = os.path.dirname(os.path.abspath(__file__))
KAT_PATH = os.path.join(HERE, "golden", "kat_cases.json")
GOLDEN_FLEET = os.path.join(HERE, "golden", "golden_fleet.npz")


def load_kats():
    with open(KAT_PATH) as f:
        return json.load(f)


def np_arrays(arrays: dict) -> dict:
    return {k: np.ascontiguousarray(np.array(v, dtype=ARRAY_DTYPES[k])) for k, v in arrays.items()}


def sizes_of(a: dict) -> dict:
    return dict(n_nodes=len(a["node_ts_ns"]), n_procs=len(a["proc_cpu_delta"]),
                n_ctrs=len(a["ctr_slot"]), n_vms=len(a["vm_slot"]), n_pods=len(a["pod_slot"]))


def check(exp: dict, T) -> None:
    """T(name) -> numpy table."""
    k = exp["kind"]
    where = f"{exp}"
    if k == "eq":
        got = T(exp["table"])[exp["index"]]
        assert got == type(got)(exp["value"]) if not isinstance(got, np.floating) else got == exp["value"], \
            f"{where}: got {got!r}"
    elif k == "near":
        got = float(T(exp["table"])[exp["index"]])
        assert abs(got - exp["value"]) <= exp["tol"], f"{where}: got {got!r}"
    elif k == "sum_eq":
        t = T(exp["table"])
        s = t.dtype.type(0)
        for i in exp["indices"]:
            s = s + t[i]
        assert s == exp["value"], f"{where}: got {s!r}"
    elif k in ("sum_eq_table", "sum_near_table"):
        t = T(exp["table"])
        s = 0.0
        for i in exp["indices"]:
            s = s + float(t[i])
        other = float(T(exp["other"])[exp["other_index"]]) * exp.get("scale", 1.0)
        if k == "sum_eq_table":
            assert s == other, f"{where}: {s!r} != {other!r}"
        else:
            assert abs(s - other) <= exp["tol"], f"{where}: {s!r} vs {other!r}"
    elif k == "ratio_eq_table":
        got = float(T(exp["table"])[exp["index"]])
        want = float(T(exp["other"])[exp["other_index"]]) * exp["scale"]
        assert got == want, f"{where}: {got!r} != {want!r}"
    elif k == "diff_eq_table":
        got = float(T(exp["table"])[exp["index"]])
        want = float(T(exp["a"])[exp["index"]]) - float(T(exp["b"])[exp["index"]])
        assert got == want, f"{where}: {got!r} != {want!r}"
    elif k == "le_table":
        got = float(T(exp["table"])[exp["index"]])
        assert 0 < got <= float(T(exp["other"])[exp["other_index"]]), where
    else:
        raise AssertionError(f"unknown expectation {k}")


def run_case(case: dict, backend_factory) -> None:
    """backend_factory(zones, caps) -> obj with upload(table, first, values),
    interval(arrays, sizes, flags), table(name)."""
    be = backend_factory(case["zones"], case["capacities"])
    for iv in case["intervals"]:
        for up in iv.get("upload", []):
            be.upload(up["table"], up["first"], up["values"])
        a = np_arrays(iv["arrays"])
        be.interval(a, sizes_of(a), iv["flags"])
        for exp in iv.get("expect", []):
            check(exp, be.table)
        for st in iv.get("expect_sum_tables", []):
            tot = sum(int(be.table(t)[st["index"]]) for t in st["tables"])
            assert tot == st["value"], st


def load_golden_fleet():
    d = np.load(GOLDEN_FLEET)
    zones = int(d["zones"])
    caps = {k.split("/")[1]: int(d[k]) for k in d.files if k.startswith("cap/")}
    sizes = {k.split("/")[1]: int(d[k]) for k in d.files if k.startswith("size/")}
    n_int = 1 + max(int(k.split("/")[0][2:]) for k in d.files if k.startswith("in"))
    intervals = []
    for k in range(n_int):
        ins = {f.split("/")[1]: d[f] for f in d.files if f.startswith(f"in{k}/")}
        outs = {f.split("/")[1]: d[f] for f in d.files if f.startswith(f"out{k}/")}
        intervals.append((ins, outs))
    return zones, caps, sizes, intervals
