#!/bin/bash
# Round 4 close: the whole -m gpu suite and smoke() on the final build, its PMC traffic
# (configs 3, 1, 5: profiles/pmc_traffic.json is keyed by the library's sha256), then
# the default bench line (which then carries roofline.traffic).
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-final4}
mkdir -p gpurun_out/$O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/$O/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/$O/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$O/pytest_gpu.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/$O/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/$O/smoke.log
OUT=$O/pmc CONFIGS="3 1 5" bash tools/gpu_pmc_traffic.sh || exit $?
cp gpurun_out/$O/pmc/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 600 python bench.py --json-out gpurun_out/$O/bench_c3.json > gpurun_out/$O/bench_c3.log 2>&1 || exit $?
tail -1 gpurun_out/$O/bench_c3.log | cut -c1-600
