#!/bin/bash
# Handoff events with a device-scope release (hipEventReleaseToDevice, a raw HIP event in
# bench.py) against a default (system-scope) torch event, at one rank with --comm-wait
# always; cluster GPU tests first; then this build's PMC traffic + rocprofv3 summary
# (tools/gpu_pmc_stats.sh, needed whenever the library changes).
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-relfence}
mkdir -p gpurun_out/$O
timeout -k 10 400 python -u -m pytest tests/test_gpu_cluster.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/$O/pt_cluster.log 2>&1; rc=$?
echo "cluster tests rc=$rc: $(tail -1 gpurun_out/$O/pt_cluster.log)"
[ $rc -eq 0 ] || { tail -30 gpurun_out/$O/pt_cluster.log; exit $rc; }
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line --shard-of 8"
args=()
for r in 1 2; do
  args+=($O/s8_def_r$r 300 "$B --json-out gpurun_out/$O/s8_def_r$r.json")
  args+=($O/s8_dev1_r$r 300 "$B --comm-wait always --allreduce-every 1 --json-out gpurun_out/$O/s8_dev1_r$r.json")
  args+=($O/s8_torch1_r$r 300 "$B --comm-wait always --allreduce-every 1 --handoff-event torch --json-out gpurun_out/$O/s8_torch1_r$r.json")
  args+=($O/s8_dev8_r$r 300 "$B --comm-wait always --json-out gpurun_out/$O/s8_dev8_r$r.json")
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', 'step %.1f kern %.1f tot %.1f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3))"
done
[ -n "${WITH_PMC:-}" ] && OUT=$O bash tools/gpu_pmc_stats.sh
true
