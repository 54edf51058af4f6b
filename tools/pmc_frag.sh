#!/bin/bash
# PMC comparison of the interval kernel on pristine vs fragmented (2 %) slots.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
SQ="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES"
for F in 0 0.02; do
  cd /tmp
  FRAG=$F VARIANTS=0 ROUNDS=3 timeout -s KILL 90 rocprofv3 --pmc $SQ --output-format csv -d "$R/gpurun_out/pmc_sq_$F" -o run -- python "$R/tools/bench_variants.py" > "$R/gpurun_out/pmc_sq_$F.log" 2>&1 || exit $?
  FRAG=$F VARIANTS=0 ROUNDS=3 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_f_$F" -o run -- python "$R/tools/bench_variants.py" > "$R/gpurun_out/pmc_f_$F.log" 2>&1 || exit $?
  FRAG=$F VARIANTS=0 ROUNDS=3 timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_w_$F" -o run -- python "$R/tools/bench_variants.py" > "$R/gpurun_out/pmc_w_$F.log" 2>&1 || exit $?
  echo "frag $F done"
done
cd "$R"
python - <<'PY'
import csv, glob, statistics, collections
for F in ("0", "0.02"):
    vals = collections.defaultdict(list)
    for pat in (f"gpurun_out/pmc_sq_{F}", f"gpurun_out/pmc_f_{F}", f"gpurun_out/pmc_w_{F}"):
        for f in glob.glob(pat + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "interval_kernel<4, 0>" in r["Kernel_Name"]:
                    vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("frag", F, {k: statistics.median(v) for k, v in sorted(vals.items())})
PY
