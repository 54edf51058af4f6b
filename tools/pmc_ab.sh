#!/bin/bash
# WRITE_SIZE / FETCH_SIZE of interval_kernel<4,0> (config 3) for the in-tree build and an
# A/B build (KACC_LIB), each pass its own run.
set -u -o pipefail
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp VARIANTS=0 ROUNDS=3
O=$R/gpurun_out/pmc_ab
mkdir -p "$O"
step() { local n=$1 s=$2; shift 2; echo "== $n"; timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1; local rc=$?; echo "== $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
cd /tmp
step write_new 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write_new" -o run -- python3 "$R/tools/bench_variants.py"
export KACC_LIB=$R/kepler_amd/lib/alt/libkepler_accel.so
step write_old 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write_old" -o run -- python3 "$R/tools/bench_variants.py"
unset KACC_LIB
step write_new2 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write_new2" -o run -- python3 "$R/tools/bench_variants.py"
