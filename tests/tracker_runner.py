"""Runs the transcribed TerminatedResourceTracker KATs (tests/golden/tracker_kats.json)
against a backend: the oracle's Go heap (CPU) or the device tracker (GPU)."""

import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def load_tracker_kats():
    with open(os.path.join(HERE, "golden", "tracker_kats.json")) as f:
        return json.load(f)


def key_of(ids, name):
    """Resource ID string -> 64-bit key (stable per case)."""
    return ids.setdefault(name, len(ids) + 1)


def check(case, items, ids):
    """items: dict key -> per-zone energy array."""
    ex = case["expect"]
    name = case["name"]
    assert len(items) == ex["size"], (name, len(items), ex["size"])
    for i in ex.get("contains", []):
        assert key_of(ids, i) in items, (name, "missing", i)
    for i in ex.get("not_contains", []):
        assert key_of(ids, i) not in items, (name, "unexpected", i)
    for i, e in ex.get("energy", {}).items():
        assert int(items[key_of(ids, i)][0]) == e, (name, i)
    for i, e in ex.get("energy_other", {}).items():
        assert int(items[key_of(ids, i)][1]) == e, (name, i)
    if "energy_sum" in ex:
        assert sum(int(v[0]) for v in items.values()) == ex["energy_sum"], name
    if "min_energy_gt" in ex:
        assert min(int(v[0]) for v in items.values()) > ex["min_energy_gt"], name


def run_oracle_case(case, zones=2):
    from oracle.oracle import OracleTracker

    t = OracleTracker(case["max_size"], case["min_energy"], zones, 0)
    ids = {}
    for st in case["steps"]:
        if st["op"] == "clear":
            t.clear()
        else:
            t.add_one(0, key_of(ids, st["id"]), st["energy"])
    k, _, e, _ = t.items()
    check(case, {int(kk): ee for kk, ee in zip(k, e)}, ids)
