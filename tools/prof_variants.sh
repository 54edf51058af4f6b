#!/bin/bash
# rocprof kernel stats of bench_variants (CONFIG / VARIANTS from the env)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_var" -o run -- python "$R/tools/bench_variants.py" > "$R/gpurun_out/prof_var.log" 2>&1 || exit $?
cd "$R"
python - <<'PY'
import csv, glob
for f in glob.glob('gpurun_out/prof_var/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'kacc' in r['Name']:
            print('prof', r['Name'][:70], r['Calls'], r['AverageNs'])
PY
