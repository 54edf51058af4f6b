#!/bin/bash
# Bench with one cluster-total buffer per step (no cross-stream waits in the timed loop):
# config 3 and its 1/8 shard, in the default (event-free) timing mode.
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-perstep}
mkdir -p gpurun_out/$O
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line"
tools/gpu_steps.sh $O/c3 300 "$B --json-out gpurun_out/$O/c3.json" \
                   $O/s8 300 "$B --shard-of 8 --json-out gpurun_out/$O/s8.json" \
                   $O/s8x 300 "$B --shard-of 8 --totals exports --json-out gpurun_out/$O/s8x.json" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', 'value %.3g step %.1f kern %.1f tot %.1f' % (d['value'], d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3))"
done
