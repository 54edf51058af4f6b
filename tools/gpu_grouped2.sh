#!/bin/bash
# bench.py with the precomputed all-reduce groups (allreduce_groups): 1/8 shard default and
# with the handoff emulated (--comm-wait always), config 3 default.
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-grouped2}
mkdir -p gpurun_out/$O
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line"
tools/gpu_steps.sh $O/s8_def 300 "$B --shard-of 8 --json-out gpurun_out/$O/s8_def.json" \
  $O/s8_hand8 300 "$B --shard-of 8 --comm-wait always --json-out gpurun_out/$O/s8_hand8.json" \
  $O/c3_def 300 "$B --json-out gpurun_out/$O/c3_def.json" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', 'step %.1f kern %.1f tot %.1f traffic %s' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3, d['roofline']['traffic']))"
done
