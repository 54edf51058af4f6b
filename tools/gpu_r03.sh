#!/bin/bash
# Round-3 check set: every GPU test, smoke(), the default bench (config 3 strong
# scaling at N = 1 with the CPU baseline, slot layouts, pipeline line), the
# per-GPU shard of a 2/4/8-way strong split (--shard-of), configs 1 / 2 x60 / 5 x60.
#   OUT=<dir> SETS="tests bench shards configs" tools/gpu_r03.sh
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r3}
mkdir -p gpurun_out/$O
S=tools/gpu_steps.sh
SETS=${SETS:-"tests bench shards configs"}
args=()
for set in $SETS; do
  case $set in
    tests) args+=($O/pytest_gpu 700 "python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -rA"
                  $O/smoke 200 "python -c 'import __graft_entry__ as g; g.smoke()'") ;;
    bench) args+=($O/bench_c3 600 "python bench.py --json-out gpurun_out/$O/bench_c3.json") ;;
    shards) for W in 2 4 8; do
              args+=($O/bench_c3_shard$W 300 "python bench.py --shard-of $W --steps 50 --warmup 10 --no-cpu-baseline --json-out gpurun_out/$O/bench_c3_shard$W.json")
            done ;;
    configs) args+=($O/bench_c1 400 "python bench.py --config 1 --no-cpu-baseline --frag-line 0 --json-out gpurun_out/$O/bench_c1.json"
                    $O/bench_c2_k60 300 "python bench.py --config 2 --intervals 60 --no-cpu-baseline --frag-line 0 --json-out gpurun_out/$O/bench_c2_k60.json"
                    $O/bench_c5_k60 400 "python bench.py --config 5 --intervals 60 --steps 10 --no-cpu-baseline --json-out gpurun_out/$O/bench_c5_k60.json") ;;
  esac
done
$S "${args[@]}"
