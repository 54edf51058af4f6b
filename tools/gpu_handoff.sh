#!/bin/bash
# Cost of the N > 1 stream handoff (an event on the compute stream after each step's
# partial sums, waited for by the comm stream) measured at one rank: --comm-wait always
# against the default, config 3 and its 1/8 shard, two interleaved rounds.
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-handoff}
mkdir -p gpurun_out/$O
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line"
args=()
for r in 1 2; do
  args+=($O/s8_off_r$r 300 "$B --shard-of 8 --json-out gpurun_out/$O/s8_off_r$r.json")
  args+=($O/s8_on_r$r 300 "$B --shard-of 8 --comm-wait always --json-out gpurun_out/$O/s8_on_r$r.json")
  args+=($O/c3_off_r$r 300 "$B --json-out gpurun_out/$O/c3_off_r$r.json")
  args+=($O/c3_on_r$r 300 "$B --comm-wait always --json-out gpurun_out/$O/c3_on_r$r.json")
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', 'step %.1f kern %.1f tot %.1f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3))"
done
