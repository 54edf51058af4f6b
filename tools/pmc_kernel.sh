#!/bin/bash
# Two SQ counter passes over a command; CSVs under gpurun_out/pmc_<name>/.
#   tools/pmc_kernel.sh NAME -- python3 tools/bench_x.py
set -u
export TMPDIR=/tmp
R=$PWD
name=$1; shift; shift
mkdir -p gpurun_out/pmc_$name
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $P -d $R/gpurun_out/pmc_$name/p$i -o run --output-format csv -- "$@") > gpurun_out/pmc_$name/p$i.log 2>&1 || exit $?
done
