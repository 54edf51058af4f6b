#!/bin/bash
# Round 4 close: SQ counters of interval_kernel<4,0> at config 3 and at its 1/8 shard
# (planning data for the split-node work), two --pmc passes each.
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r04y}
mkdir -p gpurun_out/$O
VARIANTS=0 ROUNDS=3 bash tools/pmc_kernel.sh ${O}_c3 -- python3 "$GRAFT_REPO_ROOT/tools/bench_variants.py" || exit $?
NODES=1250 VARIANTS=0 ROUNDS=6 bash tools/pmc_kernel.sh ${O}_s8 -- python3 "$GRAFT_REPO_ROOT/tools/bench_variants.py" || exit $?
ls gpurun_out/pmc_${O}_c3 gpurun_out/pmc_${O}_s8
