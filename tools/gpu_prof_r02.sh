#!/bin/bash
# Round-2 profile set: kernel-trace stats of bench.py (config 3; config 2 x60), and
# FETCH_SIZE / WRITE_SIZE passes for interval_kernel<4,0> (config 3) and the
# carry kernel (config 2, K = 60).  Every step under its own limit; stops at the first failure.
set -u -o pipefail
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out/${PROF_DIR:-prof_r02}
mkdir -p "$O"
step() { local n=$1 s=$2; shift 2; echo "== $n"; timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1; local rc=$?; echo "== $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
cd /tmp
step stats_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats_c3" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --frag-line 0 --no-pipeline-line --json-out "$O/bench_c3_prof.json"
step stats_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats_c2" -o run -- python3 "$R/bench.py" --config 2 --intervals 60 --steps 10 --warmup 2 --no-cpu-baseline --frag-line 0 --json-out "$O/bench_c2_prof.json"
step stats_join 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats_join" -o run -- python3 "$R/tools/bench_join.py"
export VARIANTS=0 ROUNDS=3
step fetch_c3 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch_c3" -o run -- python3 "$R/tools/bench_variants.py"
step write_c3 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write_c3" -o run -- python3 "$R/tools/bench_variants.py"
step fetch_c2 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch_c2" -o run -- python3 "$R/tools/bench_carry.py"
step write_c2 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write_c2" -o run -- python3 "$R/tools/bench_carry.py"
cd "$R"
python3 tools/pmc_summary.py "$O/fetch_c3" "$O/write_c3" "profiles/r02/${PROF_DIR:-prof} (tools/gpu_prof_r02.sh)" "$O/pmc_traffic.json" 3 "interval_kernel<4, 0>"
python3 tools/pmc_summary.py "$O/fetch_c2" "$O/write_c2" "profiles/r02/${PROF_DIR:-prof} (tools/gpu_prof_r02.sh)" "$O/pmc_traffic.json" 2 "intervals_carry_kernel<2, 0, 256>" 60
