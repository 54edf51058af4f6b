#!/usr/bin/env python3
"""Transcribe the reference's TerminatedResourceTracker tests into tracker_kats.json.

Source: internal/monitor/terminated_resource_tracker_test.go (sthaha/kepler
@ 2025-08-24; file:line per case).  Each case: tracker parameters, a list of
steps ("add": one Add() call with a resource ID and its per-zone energy in µJ,
zone 0 = the tracked zone, zone 1 = the other zone of CreateTestZones; "clear"),
and the assertions the Go test makes (size, IDs contained / not contained,
energy of an ID, sum of tracked-zone energies, minimum energy > 0).  A
resource without the tracked zone has 0 µJ there (tracker.go:96-100).

Run: python tests/golden/make_tracker_kats.py  (writes tests/golden/tracker_kats.json)
"""
import json
import os

J = 1_000_000  # device.Joule in µJ


def add(i, e0, e1=0):
    return {"op": "add", "id": i, "energy": [int(e0), int(e1)]}


def case(name, ref, max_size, thr, steps, **expect):
    return {"name": name, "ref": "internal/monitor/terminated_resource_tracker_test.go:" + ref,
            "max_size": max_size, "min_energy": int(thr), "steps": steps, "expect": expect}


def cases():
    out = [
        case("New", "58-70", 10, 0, [], size=0),
        case("AddSingleResource", "72-85", 5, 6 * J, [add("resource-1", 1000 * J)], size=1,
             contains=["resource-1"]),
        case("AddResourceWithZeroEnergy", "87-98", 5, 1 * J, [add("resource-1", 0)], size=0),
        case("AddResourceWithoutTrackedZone", "100-112", 5, 1 * J, [add("resource-1", 0, 1000 * J)], size=0),
        case("AddMultipleResources", "114-142", 5, 10 * J,
             [add("resource-1", 1000 * J), add("resource-2", 2000 * J), add("resource-3", 500 * J)],
             size=3, contains=["resource-1", "resource-2", "resource-3"]),
        case("DuplicatesIgnored", "144-168", 5, 8 * J,
             [add("resource-1", 1000 * J), add("resource-1", 2000 * J)],
             size=1, energy={"resource-1": 1000 * J}),
        case("EvictOnCapactity", "170-209", 3, 7 * J,
             [add("low", 100 * J), add("medium", 500 * J), add("high", 1000 * J), add("new-medium", 300 * J)],
             size=3, contains=["medium", "high", "new-medium"], not_contains=["low"]),
        case("CapacityEvictionWithLowerEnergy", "211-244", 2, 9 * J,
             [add("high1", 1000 * J), add("high2", 2000 * J), add("low", 50 * J)],
             size=2, contains=["high1", "high2"], not_contains=["low"]),
        case("Clear", "246-267", 5, 12 * J,
             [add("resource-1", 1000 * J), add("resource-2", 2000 * J), {"op": "clear"}], size=0),
        case("MultiZoneResource", "269-293", 5, 15 * J, [add("multi-zone", 1000 * J, 5000 * J)],
             size=1, contains=["multi-zone"], energy={"multi-zone": 1000 * J},
             energy_other={"multi-zone": 5000 * J}),
        case("EdgeCases/zero capacity", "332-340", 0, 0, [add("resource-1", 1000 * J)], size=0),
        case("EdgeCases/negative capacity is unlimited", "342-354", -5, 0,
             [add(f"resource-{i}", (i + 1) * J) for i in range(100)], size=100),
        case("EdgeCases/unlimited capacity", "356-368", -1, 0,
             [add(f"resource-{i}", (i + 1) * J) for i in range(100)], size=100),
        case("EdgeCases/capacity of 1", "370-386", 1, 0,
             [add("resource-1", 1000 * J), add("resource-2", 2000 * J)], size=1, contains=["resource-2"]),
        case("EdgeCases/empty resource ID", "388-398", 5, 0, [add("", 1000 * J)], size=1, contains=[""]),
        case("HeapIntegrity", "401-431", 5, 20 * J,
             [add(f"resource-{i}", e * J) for i, e in enumerate([500, 1000, 100, 2000, 300])],
             size=5, energy_sum=3900 * J),
        case("RealWorldScenario", "433-490", 100, 25 * J,
             [add(f"process-{i}", (i + 1) * 100 * J) for i in range(50)]
             + [add(f"process-{50 + i}", (i + 1) * 50 * J) for i in range(75)],
             size=100, min_energy_gt=0),
        case("MinimumThreshold/below rejected", "496-514", 10, 100 * J,
             [add("below-1", 50 * J), add("below-2", 99 * J), add("below-3", 0)], size=0),
        case("MinimumThreshold/above accepted", "516-541", 10, 100 * J,
             [add("above-1", 100 * J), add("above-2", 101 * J), add("above-3", 500 * J)],
             size=3, contains=["above-1", "above-2", "above-3"]),
        case("MinimumThreshold/mixed", "543-577", 10, 200 * J,
             [add("reject-1", 50 * J), add("accept-1", 250 * J), add("reject-2", 199 * J),
              add("accept-2", 200 * J), add("reject-3", 0), add("accept-3", 1000 * J)],
             size=3, contains=["accept-1", "accept-2", "accept-3"],
             not_contains=["reject-1", "reject-2", "reject-3"]),
        case("MinimumThreshold/capacity eviction", "579-604", 2, 100 * J,
             [add("low-valid", 120 * J), add("high", 500 * J), add("medium", 300 * J)],
             size=2, contains=["high", "medium"], not_contains=["low-valid"]),
        case("MinimumThreshold/multi-zone above", "606-664", 10, 150 * J,
             [add("tracked-zone-above-threshold", 200 * J, 50 * J)], size=1,
             contains=["tracked-zone-above-threshold"]),
        case("MinimumThreshold/multi-zone below", "606-664", 10, 150 * J,
             [add("tracked-zone-below-threshold", 100 * J, 1000 * J)], size=0),
        case("MinimumThreshold/multi-zone at", "606-664", 10, 150 * J,
             [add("tracked-zone-at-threshold", 150 * J, 0)], size=1, contains=["tracked-zone-at-threshold"]),
        case("ThresholdEdgeCases/zero threshold", "670-693", 10, 0,
             [add("zero", 0), add("tiny", 1 * J), add("small", 10 * J), add("large", 1000 * J)],
             size=4, contains=["zero", "tiny", "small", "large"]),
        case("ThresholdEdgeCases/very high threshold", "695-723", 10, 10000 * J,
             [add("low", 1000 * J), add("medium", 5000 * J), add("high", 9999 * J),
              add("accepted", 10000 * J), add("very-high", 15000 * J)],
             size=2, contains=["accepted", "very-high"], not_contains=["low", "medium", "high"]),
        case("ThresholdEdgeCases/disabled", "725-735", 0, 100 * J, [add("valid", 200 * J)], size=0),
        case("ThresholdEdgeCases/unlimited", "737-755", -1, 50 * J,
             [add(f"resource-{i}", i * 10 * J) for i in range(100)], size=95),
        case("ThresholdEdgeCases/below-by-1", "757-791", 10, 500 * J, [add("below-by-1", 499 * J)], size=0),
        case("ThresholdEdgeCases/exact-threshold", "757-791", 10, 500 * J, [add("exact-threshold", 500 * J)],
             size=1, contains=["exact-threshold"]),
        case("ThresholdEdgeCases/above-by-1", "757-791", 10, 500 * J, [add("above-by-1", 501 * J)],
             size=1, contains=["above-by-1"]),
        case("ThresholdEdgeCases/missing tracked zone", "793-805", 10, 100 * J,
             [add("missing-zone", 0, 1000 * J)], size=0),
    ]
    return out


if __name__ == "__main__":
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tracker_kats.json")
    with open(path, "w") as f:
        json.dump({"source": "internal/monitor/terminated_resource_tracker_test.go", "zones": 2,
                   "cases": cases()}, f, indent=1)
    print(f"wrote {path}: {len(cases())} cases")
