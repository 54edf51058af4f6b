#!/bin/bash
# Slot-join A/B: production join_small (31) vs lane-strided rows (63), config 3,
# outputs checked identical, interleaved rounds.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/jstride
VARIANTS=31,63 ROUNDS=5 timeout -k 10 300 python tools/bench_join_variants.py > gpurun_out/jstride/ab.json 2> gpurun_out/jstride/ab.log || { tail -20 gpurun_out/jstride/ab.log; exit 1; }
cat gpurun_out/jstride/ab.json
