#!/bin/bash
# GPU run 2: parity, variant ablations, bench, rocprof stats + PMC traffic passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_variants.py > gpurun_out/variants.json 2> gpurun_out/variants.err || exit $?
cat gpurun_out/variants.json
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --json-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_stats" -o run -- python "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/prof_stats.log" 2>&1 || exit $?
echo "stats done"
VARIANTS=0 ROUNDS=3 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch" -o run -- python "$R/tools/bench_variants.py" > "$R/gpurun_out/pmc_fetch.log" 2>&1 || exit $?
echo "fetch done"
VARIANTS=0 ROUNDS=3 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write" -o run -- python "$R/tools/bench_variants.py" > "$R/gpurun_out/pmc_write.log" 2>&1 || exit $?
echo "write done"
