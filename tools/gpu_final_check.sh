#!/bin/bash
# End-of-round check of the committed tree: smoke, the default bench line, and the
# handoff-event A/B at the 1/8 shard (device-scope vs default event, one per step).
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-final}
mkdir -p gpurun_out/$O
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/$O/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/$O/smoke.log
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line --shard-of 8"
tools/gpu_steps.sh $O/c3 400 "python bench.py --json-out gpurun_out/$O/c3.json" \
  $O/s8_dev1 300 "$B --comm-wait always --allreduce-every 1 --json-out gpurun_out/$O/s8_dev1.json" \
  $O/s8_torch1 300 "$B --comm-wait always --allreduce-every 1 --handoff-event torch --json-out gpurun_out/$O/s8_torch1.json" \
  $O/s8_def 300 "$B --json-out gpurun_out/$O/s8_def.json" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', 'step %.1f kern %.1f tot %.1f traffic %s' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3, d['roofline']['traffic']))"
done
