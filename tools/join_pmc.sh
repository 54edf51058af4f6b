#!/bin/bash
# rocprofv3 counter passes over tools/join_pmc.py (one pass per counter group, each its own
# run), then the per-kernel averages: OUT=<dir> VARIANTS=511,-1 tools/join_pmc.sh
set -u -o pipefail
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out/${OUT:-join_pmc}
mkdir -p "$O"
cd /tmp
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
            "SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
            "SQ_WAVES SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD GRBM_COUNT"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d "$O/p$i" -o run -- python3 "$R/tools/join_pmc.py" \
    > "$O/p$i.log" 2>&1 || { echo "pass $i rc=$?"; tail -5 "$O/p$i.log"; }
done
python3 "$R/tools/join_pmc_summary.py" "$O"/p*/run_counter_collection.csv > "$O/summary.json" && cat "$O/summary.json"
