#!/bin/bash
# Round 4: fused partial sums with the node blocks waiting at their start (default build)
# vs unfused, at config 3 and the 1/8 shard; then the join phase profile and the
# config-5 chunk-kernel A/B (tools/gpu_r04e.sh).
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r04f}
mkdir -p gpurun_out/$O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rA \
  tests/test_gpu_cluster.py -k "deferred or back_to_back or live_nodes" \
  > gpurun_out/$O/pytest_cluster.log 2>&1 || { echo "cluster tests failed rc=$?"; tail -40 gpurun_out/$O/pytest_cluster.log; exit 1; }
tail -1 gpurun_out/$O/pytest_cluster.log
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line --no-host-line"
args=()
for r in 1 2; do
  for f in on off; do
    args+=($O/c3_${f}_r$r 300 "$B --fuse-partials $f --json-out gpurun_out/$O/c3_${f}_r$r.json")
    args+=($O/s8_${f}_r$r 300 "$B --shard-of 8 --steps 50 --fuse-partials $f --json-out gpurun_out/$O/s8_${f}_r$r.json")
  done
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', 'step %.1f kern %.1f tot %.1f frac %.3f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3, r['frac']))"
done
OUT=$O/e bash tools/gpu_r04e.sh
