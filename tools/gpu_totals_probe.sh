#!/bin/bash
# Which half of the cluster partial sums bounds the step: namespace sums only, node
# totals only, both (config 3 and its 1/8 shard).
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-tprobe}
mkdir -p gpurun_out/$O
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line"
args=()
for p in both ns nodes; do
  args+=($O/c3_$p 300 "$B --totals-probe $p --json-out gpurun_out/$O/c3_$p.json")
  args+=($O/s8_$p 300 "$B --shard-of 8 --totals-probe $p --json-out gpurun_out/$O/s8_$p.json")
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', 'step %.1f kern %.1f tot %.1f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3))"
done
