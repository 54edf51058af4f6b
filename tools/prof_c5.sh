#!/bin/bash
# rocprofv3 kernel-trace stats of config 5 (60 intervals per call): which launch of the
# big-node path (interval_kernel node phase, chunk_kernel, pod_kernel) costs what.
set -u
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out/${OUT:-prof_c5}
mkdir -p "$O"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o run -- \
  python3 "$R/bench.py" --config 5 --intervals 60 --steps 3 --warmup 1 --no-cpu-baseline --frag-line 0 \
  --json-out "$O/bench_c5_prof.json" > "$O/prof.log" 2>&1
