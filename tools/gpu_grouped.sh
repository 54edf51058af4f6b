#!/bin/bash
# Grouped cluster all-reduce (kacc_cluster_partials per step + one kacc_allreduce_sums per
# --allreduce-every steps): the cluster GPU tests, then the handoff cost at one rank with
# --comm-wait always at groups of 1 and 8, config 3 and its 1/8 shard.
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-grouped}
mkdir -p gpurun_out/$O
timeout -k 10 400 python -u -m pytest tests/test_gpu_cluster.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/$O/pt_cluster.log 2>&1; rc=$?
echo "cluster tests rc=$rc: $(tail -1 gpurun_out/$O/pt_cluster.log)"
[ $rc -eq 0 ] || { tail -30 gpurun_out/$O/pt_cluster.log; exit $rc; }
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line"
args=()
for r in 1 2; do
  args+=($O/s8_def_r$r 300 "$B --shard-of 8 --json-out gpurun_out/$O/s8_def_r$r.json")
  args+=($O/s8_hand8_r$r 300 "$B --shard-of 8 --comm-wait always --json-out gpurun_out/$O/s8_hand8_r$r.json")
  args+=($O/s8_hand1_r$r 300 "$B --shard-of 8 --comm-wait always --allreduce-every 1 --json-out gpurun_out/$O/s8_hand1_r$r.json")
  args+=($O/c3_def_r$r 300 "$B --json-out gpurun_out/$O/c3_def_r$r.json")
  args+=($O/c3_hand8_r$r 300 "$B --comm-wait always --json-out gpurun_out/$O/c3_hand8_r$r.json")
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', 'step %.1f kern %.1f tot %.1f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3))"
done
