#!/bin/bash
# Two SQ counter passes over tools/bench_carry.py (variant 0 only); CSVs under gpurun_out/pmc_carry/.
set -u
export TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out/pmc_carry
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  VARIANTS=0 ROUNDS=2 timeout -s KILL 120 rocprofv3 --pmc $P -d $R/gpurun_out/pmc_carry/p$i -o run --output-format csv -- python3 $R/tools/bench_carry.py || exit $?
done
