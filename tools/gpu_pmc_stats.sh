#!/bin/bash
# The PMC traffic passes (config 3 and 1) and the rocprofv3 kernel-trace summary of the
# config-3 bench for the current build: the second half of tools/gpu_full.sh.
#   OUT=<dir> tools/gpu_pmc_stats.sh
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-full}
mkdir -p gpurun_out/$O
OUT=$O/pmc CONFIGS="3 1" bash tools/gpu_pmc_traffic.sh || exit $?
(cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$O/stats_c3" -o run -- \
   python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --frag-line 0 --no-pipeline-line \
   --json-out "$GRAFT_REPO_ROOT/gpurun_out/$O/bench_c3_prof.json") > gpurun_out/$O/stats_c3.log 2>&1 || exit $?
python tools/trace_gaps.py gpurun_out/$O/stats_c3 interval_kernel cluster_partials | tee gpurun_out/$O/trace_gaps_c3.txt
