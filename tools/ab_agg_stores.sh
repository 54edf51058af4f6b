#!/bin/bash
# A/B of the aggregate-row store hint: HEAD (plain stores for containers / VMs /
# pods) against kepler_amd/lib/alt built with -DKACC_NT_AGG=1 (round-2 non-temporal
# stores), alternated per config; the GPU parity tests first on HEAD.
set -u
cd "$GRAFT_REPO_ROOT"
D=${OUT:-aggab}
mkdir -p gpurun_out/$D
OLD="KACC_LIB=$GRAFT_REPO_ROOT/kepler_amd/lib/alt/libkepler_accel.so"
B="python bench.py --no-cpu-baseline --frag-line 0 --no-pipeline-line"
tools/gpu_steps.sh $D/pytest 500 "python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_small.py tests/test_gpu_cluster.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider" \
  $D/variants 200 "env VARIANTS=0,4096 STEP=1 ROUNDS=30 python tools/bench_variants.py" \
  $D/c3_new1 200 "$B --json-out gpurun_out/$D/c3_new1.json" \
  $D/c3_old1 200 "env $OLD $B --json-out gpurun_out/$D/c3_old1.json" \
  $D/c3_new2 200 "$B --json-out gpurun_out/$D/c3_new2.json" \
  $D/c3_old2 200 "env $OLD $B --json-out gpurun_out/$D/c3_old2.json" \
  $D/c1_new 200 "$B --config 1 --json-out gpurun_out/$D/c1_new.json" \
  $D/c1_old 200 "env $OLD $B --config 1 --json-out gpurun_out/$D/c1_old.json" \
  $D/c2_new 200 "$B --config 2 --intervals 60 --json-out gpurun_out/$D/c2_new.json" \
  $D/c2_old 200 "env $OLD $B --config 2 --intervals 60 --json-out gpurun_out/$D/c2_old.json" \
  $D/c5_new 300 "$B --config 5 --intervals 60 --steps 10 --json-out gpurun_out/$D/c5_new.json" \
  $D/c5_old 300 "env $OLD $B --config 5 --intervals 60 --steps 10 --json-out gpurun_out/$D/c5_old.json"
