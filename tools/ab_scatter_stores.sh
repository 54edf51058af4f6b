#!/bin/bash
# A/B of the per-row scattered process-store hint: HEAD (plain stores) against
# kepler_amd/lib/alt built with -DKACC_NT_SCATTER=1 (round-2 non-temporal stores),
# on fragmented slot layouts and the held join policy's steady state.
set -u
cd "$GRAFT_REPO_ROOT"
D=${OUT:-scatab}
mkdir -p gpurun_out/$D
OLD="KACC_LIB=$GRAFT_REPO_ROOT/kepler_amd/lib/alt/libkepler_accel.so"
B="python bench.py --no-cpu-baseline --frag-line 0 --no-pipeline-line"
tools/gpu_steps.sh $D/pytest 500 "python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_small.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider" \
  $D/v_f10 200 "env FRAG=0.1 VARIANTS=0,8192 ROUNDS=20 python tools/bench_variants.py" \
  $D/v_f02 200 "env FRAG=0.02 VARIANTS=0,8192 ROUNDS=20 python tools/bench_variants.py" \
  $D/steady_held_new 300 "env POLICY=0 python tools/bench_steady.py" \
  $D/steady_held_old 300 "env $OLD POLICY=0 python tools/bench_steady.py" \
  $D/steady_reuse_new 300 "env POLICY=1 python tools/bench_steady.py" \
  $D/c2f_new 200 "$B --config 2 --intervals 60 --fragment 0.3 --json-out gpurun_out/$D/c2f_new.json" \
  $D/c2f_old 200 "env $OLD $B --config 2 --intervals 60 --fragment 0.3 --json-out gpurun_out/$D/c2f_old.json" \
  $D/c1f_new 200 "$B --config 1 --fragment 0.3 --json-out gpurun_out/$D/c1f_new.json" \
  $D/c1f_old 200 "env $OLD $B --config 1 --fragment 0.3 --json-out gpurun_out/$D/c1f_old.json"
