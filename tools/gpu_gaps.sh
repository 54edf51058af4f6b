#!/bin/bash
# Step-overhead study (config 3 and its 1/8 shard): the bench with and without the
# no-op cross-stream wait at one rank, and a rocprofv3 kernel trace of each shape
# (tools/trace_gaps.py: per-kernel durations and inter-kernel gaps).
#   OUT=<dir> tools/gpu_gaps.sh
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-gaps}
mkdir -p gpurun_out/$O
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line"
tools/gpu_steps.sh \
  $O/c3_auto 300 "$B --json-out gpurun_out/$O/c3_auto.json" \
  $O/c3_always 300 "$B --comm-wait always --json-out gpurun_out/$O/c3_always.json" \
  $O/s8_auto 300 "$B --shard-of 8 --json-out gpurun_out/$O/s8_auto.json" \
  $O/s8_always 300 "$B --shard-of 8 --comm-wait always --json-out gpurun_out/$O/s8_always.json" \
  $O/trace_c3 300 "cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$O/trace_c3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line" \
  $O/trace_s8 300 "cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$O/trace_s8 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --shard-of 8 --steps 40 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', 'step', round(d['ms_per_step']*1e3,1), 'kernel', round(d['kernel_ms']*1e3,1), 'totals', round(d['totals_compute_ms']*1e3,1))"
done
for t in c3 s8; do echo "== trace $t"; python tools/trace_gaps.py gpurun_out/$O/trace_$t interval_kernel cluster_partials; done
