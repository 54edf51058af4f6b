#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per interval_kernel variant (config 3): where the excess over
# the algorithmic bytes comes from (0 production, 1 no aggregates, 2 no process pass,
# 3 node phases only, 8 plain stores).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-pmcvar}
mkdir -p "$O"
export VARIANTS=${VARIANTS:-0,1,2,3,8} ROUNDS=2 CONFIG=3
for c in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$O/$c" -o run -- python3 "$R/tools/bench_variants.py") > "$O/$c.log" 2>&1 || exit $?
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections, statistics
d = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    per = collections.defaultdict(list)
    for f in glob.glob(f"{d}/{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "interval_kernel<4" in r["Kernel_Name"] and r["Counter_Name"] == c:
                per[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    for k, v in sorted(per.items()):
        m = statistics.median(v) * 1024 * (2 if c == "FETCH_SIZE" else 1) / 1e9
        print(c, k, "n=%d" % len(v), "GB/launch %.4f" % m)
PY
