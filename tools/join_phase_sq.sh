#!/bin/bash
set -u -o pipefail
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out/${OUT:-join_sq}
mkdir -p "$O"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH --output-format csv -d "$O/pmc" -o run -- python3 "$R/tools/join_phase_sq.py" > "$O/run.log" 2>&1
