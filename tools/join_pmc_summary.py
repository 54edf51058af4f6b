#!/usr/bin/env python3
"""Per-kernel-instance averages of rocprofv3 --pmc passes (tools/join_pmc.sh): for every
join kernel name, each counter summed per dispatch, then averaged over its dispatches (the
two warm-up joins of each variant dropped), plus per-wave values (÷ SQ_WAVES of the pass).

With STOPS (and REPS) as tools/join_pmc.py had them: per phase stop instead of per kernel.

  [STOPS=1,...,0 REPS=r] python tools/join_pmc_summary.py <pass csv> [<pass csv> ...]"""
import collections
import csv
import json
import sys


def main():
    import os

    out = collections.defaultdict(dict)
    stops = [int(x) for x in os.environ.get("STOPS", "").split(",") if x]
    reps = int(os.environ.get("REPS", "6"))
    for path in sys.argv[1:]:
        disp = collections.OrderedDict()
        names = {}
        for r in csv.DictReader(open(path)):
            if "join_" not in r["Kernel_Name"]:
                continue
            d = disp.setdefault(int(r["Dispatch_Id"]), collections.Counter())
            d[r["Counter_Name"]] += float(r["Counter_Value"])
            names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
        by_name = collections.defaultdict(list)
        for i, c in disp.items():
            by_name[names[i]].append(c)
        if stops:  # per phase: every third dispatch (after the two full joins), REPS per stop
            for name, lst in by_name.items():
                for i, st in enumerate(stops):
                    sel = lst[i * 3 * reps:(i + 1) * 3 * reps][2::3]
                    key = f"stop_after_{st}" if st else "full"
                    for k in sel[0] if sel else []:
                        v = sum(c[k] for c in sel) / len(sel)
                        out[key][k] = v
                        if k != "SQ_WAVES" and sel[0].get("SQ_WAVES"):
                            out[key][k + "_per_wave"] = v / (sum(c["SQ_WAVES"] for c in sel) / len(sel))
            continue
        for name, lst in by_name.items():
            lst = lst[2:]  # warm-up joins
            if not lst:
                continue
            short = name.split("(")[0]
            for k in lst[0]:
                v = sum(c[k] for c in lst) / len(lst)
                out[short][k] = v
                if k != "SQ_WAVES" and lst[0].get("SQ_WAVES"):
                    out[short][k + "_per_wave"] = v / (sum(c["SQ_WAVES"] for c in lst) / len(lst))
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
