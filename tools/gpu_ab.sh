#!/bin/bash
# A/B of the current build against a previous one staged in ab_prev/ (its own
# bench.py, kepler_amd/ package and libkepler_accel.so; not committed): the
# same bench lines alternated prev/new on one box, so box-to-box spread cancels.
#   OUT=<dir> CONFIGS="3 2k60 1 5k60 3s8" ROUNDS=2 tools/gpu_ab.sh
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-ab}
mkdir -p gpurun_out/$O
S=tools/gpu_steps.sh
args=()
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in ${CONFIGS:-3}; do
    case $c in
      3) a="--steps 30 --warmup 5" ;;
      2k60) a="--config 2 --intervals 60 --steps 10" ;;
      1) a="--config 1" ;;
      5k60) a="--config 5 --intervals 60 --steps 5" ;;
      3s8) a="--shard-of 8 --steps 50 --warmup 10" ;;
    esac
    common="--no-cpu-baseline --frag-line 0 --no-pipeline-line"
    args+=($O/prev_c${c}_r$r 300 "cd ab_prev && python bench.py $a $common --json-out ../gpurun_out/$O/prev_c${c}_r$r.json"
           $O/new_c${c}_r$r 300 "python bench.py $a $common --json-out gpurun_out/$O/new_c${c}_r$r.json")
  done
done
$S "${args[@]}"
