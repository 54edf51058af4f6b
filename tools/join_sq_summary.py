#!/usr/bin/env python3
"""Per-phase SQ counters per wave of the small-node slot join from one rocprofv3 --pmc pass
over tools/join_phase_sq.py (its dispatch order: for each stop in 1 2 3 4 5 0, REPS x
(two full joins + the stopped join)).  Prints one JSON object: the cumulative counters per
wave at each stop and the increments (the phases).

  python tools/join_sq_summary.py gpurun_out/<dir>/sq/pmc/run_counter_collection.csv
"""
import collections
import csv
import json
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    disp = collections.OrderedDict()
    for r in rows:
        if "join_small" not in r["Kernel_Name"]:
            continue
        d = disp.setdefault(int(r["Dispatch_Id"]), {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = list(disp)
    stops = [1, 2, 3, 4, 5, 0]
    reps = len(ids) // (3 * len(stops))
    cum, i = {}, 0
    for st in stops:
        acc = collections.Counter()
        for _ in range(reps):
            i += 2  # the two full joins that set up the state
            for k, v in disp[ids[i]].items():
                acc[k] += v
            i += 1
        w = acc["SQ_WAVES"]
        cum["full" if st == 0 else f"stop_after_{st}"] = {k: v / w for k, v in sorted(acc.items()) if k != "SQ_WAVES"}
    names = list(cum)
    inc = {names[0]: cum[names[0]]}
    for a, b in zip(names, names[1:]):
        inc[b] = {k: cum[b][k] - cum[a][k] for k in cum[b]}
    print(json.dumps({"reps": reps, "per_wave_cumulative": cum, "per_wave_phase_increment": inc}, indent=1))


if __name__ == "__main__":
    main()
