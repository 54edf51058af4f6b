#!/bin/bash
# Full GPU parity suite + config-3 headline bench + config-1 fleet (small-node kernel) bench and rocprof stats.
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
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --json-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --config 1 --steps 20 --warmup 3 --no-cpu-baseline --json-out gpurun_out/bench_c1.json > gpurun_out/bench_c1.log 2>&1 || exit $?
for f in bench bench_c1; do python -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f','value',round(d['value']/1e9,2),'G ms',round(d['ms_per_step'],4),'kernel_ms',round(d['kernel_ms'],4),'frac',round(d['roofline']['frac'],3),d['config']['workload'])"; done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_c1" -o run -- python "$R/bench.py" --config 1 --steps 10 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/prof_c1.log" 2>&1 || exit $?
cd "$R"
python - <<'PY'
import csv, glob
for f in glob.glob('gpurun_out/prof_c1/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print('c1prof', r['Name'][:60], r['Calls'], r['AverageNs'])
PY
