#!/bin/bash
# Same-box ablation of the cluster-totals modes at config 3 and its 1/8 shard: the partial-sum
# launch (tables), the export stores alone (tables+writes), the sums in the next interval's
# launch over namespace-ordered exports (fused) and over batch-order exports (fused, rows).
#   OUT=<dir> tools/gpu_sums_ablation.sh
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-sums_ab}
mkdir -p gpurun_out/$O
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_export_sums.py tests/test_gpu_cluster.py} -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/$O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/$O/pytest.log; exit 1; }
tail -1 gpurun_out/$O/pytest.log
B="--no-cpu-baseline --frag-line 0 --no-pipeline-line --no-host-line"
args=()
for w in ${SIZES:-s8 s4 c3}; do
  case $w in
    s8) S="--shard-of 8 --steps 50 --warmup 10";;
    s4) S="--shard-of 4 --steps 40 --warmup 10";;
    s2) S="--shard-of 2 --steps 30 --warmup 5";;
    *) S="--steps 20 --warmup 3";;
  esac
  args+=($O/${w}_tables 300 "python bench.py $S $B --totals tables --json-out gpurun_out/$O/${w}_tables.json")
  args+=($O/${w}_writes 300 "python bench.py $S $B --totals tables+writes --json-out gpurun_out/$O/${w}_writes.json")
  args+=($O/${w}_fused_ns 300 "python bench.py $S $B --totals fused --json-out gpurun_out/$O/${w}_fused_ns.json")
  args+=($O/${w}_fused_rows 300 "python bench.py $S $B --totals fused --sums-order rows --json-out gpurun_out/$O/${w}_fused_rows.json")
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];t=d['totals_compute_ms'];print('$f', 'step %.2f us kern %.2f us tot %s frac %.3f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, ('%.2f us' % (t*1e3)) if t else '-', r['frac']))"
done
