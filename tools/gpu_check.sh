#!/bin/bash
# Reusable GPU check: parity tests, variant ablations, bench (+ optional rocprof).
# usage: bash tools/gpu_check.sh [prof]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_variants.py > gpurun_out/variants.json 2> gpurun_out/variants.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/variants.json'));print({k:round(v['median_ms'],4) for k,v in d['variants'].items()}, 'ns', round(d['namespace_ms'],4), 'GB/s', round(d.get('achieved_GBps_v0',0)))"
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --json-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print('value',d['value'],'ms',d['ms_per_step'],'kernel_ms',d['kernel_ms'],'frac',d['roofline']['frac'])"
if [ "$1" = "prof" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_stats" -o run -- python "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/prof_stats.log" 2>&1 || exit $?
  echo "stats done"
  VARIANTS=0 ROUNDS=3 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch" -o run -- python "$R/tools/bench_variants.py" > "$R/gpurun_out/pmc_fetch.log" 2>&1 || exit $?
  VARIANTS=0 ROUNDS=3 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write" -o run -- python "$R/tools/bench_variants.py" > "$R/gpurun_out/pmc_write.log" 2>&1 || exit $?
  echo "pmc done"
fi
if [ "$1" = "configs" ] || [ "$2" = "configs" ]; then
  cd "$R"
  CONFIG=5 VARIANTS=${C5_VARIANTS:-0,32,1,2} ROUNDS=6 timeout -k 10 300 python tools/bench_variants.py > gpurun_out/variants_c5.json 2> gpurun_out/variants_c5.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/variants_c5.json'));print('c5 variants', {k:round(v['median_ms'],4) for k,v in d['variants'].items()})"
  timeout -k 10 400 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline --json-out gpurun_out/bench_c5.json > gpurun_out/bench_c5.log 2>&1 || exit $?
  timeout -k 10 400 python bench.py --config 5 --node-order --steps 10 --warmup 2 --no-cpu-baseline --json-out gpurun_out/bench_c5_lpt.json > gpurun_out/bench_c5_lpt.log 2>&1 || exit $?
  timeout -k 10 400 python bench.py --config 2 --steps 20 --warmup 3 --no-cpu-baseline --json-out gpurun_out/bench_c2.json > gpurun_out/bench_c2.log 2>&1 || exit $?
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_c5" -o run -- python "$R/bench.py" --config 5 --steps 10 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/prof_c5.log" 2>&1 || exit $?
  cd "$R"
  python - <<'PY'
import csv, glob
for f in glob.glob('gpurun_out/prof_c5/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print('c5prof', r['Name'][:60], r['Calls'], r['AverageNs'])
PY
  for f in bench_c5 bench_c5_lpt bench_c2; do python -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f', 'value',d['value'],'kernel_ms',d['kernel_ms'],'frac',d['roofline']['frac'],d['config']['workload'])"; done
fi
