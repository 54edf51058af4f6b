#!/bin/bash
# Parity suite, config-1 fleet bench, and the small kernel's HBM traffic (separate
# FETCH_SIZE / WRITE_SIZE --pmc passes, MI355X_MICROARCH.md §HBM corrections).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_c1_fetch" -o run -- python "$R/bench.py" --config 1 --steps 5 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/pmc_c1_fetch.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_c1_write" -o run -- python "$R/bench.py" --config 1 --steps 5 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/pmc_c1_write.log" 2>&1 || exit $?
cd "$R"
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
python tools/pmc_summary.py gpurun_out/pmc_c1_fetch gpurun_out/pmc_c1_write run18 gpurun_out/pmc_traffic.json 1 "small_kernel<2>" || exit $?
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 400 python bench.py --config 1 --steps 20 --warmup 3 --no-cpu-baseline --json-out gpurun_out/bench_c1.json > gpurun_out/bench_c1.log 2>&1 || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c1.json'));print('bench_c1','value',round(d['value']/1e9,2),'G kernel_ms',round(d['kernel_ms'],4),'roofline',d['roofline'])"
