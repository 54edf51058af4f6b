#!/bin/bash
# Event-marker ablation (config 3 and its 1/8 shard): the timed loop with HIP
# events around interval + totals, around the interval only, and none (wall only);
# rocprofv3 kernel traces of the event-free shard loop (tools/trace_gaps.py).
#   OUT=<dir> tools/gpu_events.sh
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-events}
mkdir -p gpurun_out/$O
B="python bench.py --steps 60 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line"
args=()
for r in 1 2; do
  for e in launch markers none; do
    args+=($O/s8_${e}_r$r 300 "$B --shard-of 8 --step-events $e --json-out gpurun_out/$O/s8_${e}_r$r.json")
  done
done
for e in launch markers none; do
  args+=($O/c3_${e} 300 "$B --step-events $e --json-out gpurun_out/$O/c3_${e}.json")
done
args+=($O/trace_s8_launch 300 "cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$O/trace_s8_launch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --shard-of 8 --steps 60 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line --step-events launch")
args+=($O/trace_c3_launch 300 "cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$O/trace_c3_launch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 60 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line --json-out $GRAFT_REPO_ROOT/gpurun_out/$O/prof_c3_launch.json")
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', 'step', round(d['ms_per_step']*1e3,1), 'kernel', round(d['kernel_ms']*1e3,1), 'totals', round(d['totals_compute_ms']*1e3,1))"
done
for t in s8 c3; do python tools/trace_gaps.py gpurun_out/$O/trace_${t}_launch interval_kernel cluster_partials; done
