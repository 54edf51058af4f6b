#!/bin/bash
# A/B of plain aggregate stores in small_kernel / chunk_kernel / pod_kernel:
# kepler_amd/lib/alt built -DKACC_PLAIN_AGG_REST=1 (candidate) against HEAD,
# alternated three times per config (placement spread is per process).
set -u
cd "$GRAFT_REPO_ROOT"
D=${OUT:-aggrest}
mkdir -p gpurun_out/$D
NEW="KACC_LIB=$GRAFT_REPO_ROOT/kepler_amd/lib/alt/libkepler_accel.so"
B="python bench.py --no-cpu-baseline --frag-line 0 --no-pipeline-line"
args=()
for i in 1 2 3; do
  args+=($D/c1_head$i 200 "$B --config 1 --json-out gpurun_out/$D/c1_head$i.json")
  args+=($D/c1_new$i 200 "env $NEW $B --config 1 --json-out gpurun_out/$D/c1_new$i.json")
done
for i in 1 2; do
  args+=($D/c5_head$i 300 "$B --config 5 --intervals 60 --steps 10 --json-out gpurun_out/$D/c5_head$i.json")
  args+=($D/c5_new$i 300 "env $NEW $B --config 5 --intervals 60 --steps 10 --json-out gpurun_out/$D/c5_new$i.json")
done
tools/gpu_steps.sh "${args[@]}"
