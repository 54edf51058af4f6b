#!/bin/bash
# rocprofv3 kernel trace of config 3 with the export path (interval kernel + comm-stream partials)
set -u
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out/${OUT:-prof_c3x}
mkdir -p "$O"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --frag-line 0 --no-pipeline-line \
  --totals ${TOTALS:-exports} --json-out "$O/bench.json" > "$O/prof.log" 2>&1
