#!/bin/bash
# Round 4, fourth call: deferred partial sums fused into the interval launch (tests, then
# fused vs unfused at config 3 and its 1/8 shard, interleaved), config 2 x 60 (carry kernel
# without exports), then every GPU test.   OUT=<dir> tools/gpu_r04d.sh
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r04d}
mkdir -p gpurun_out/$O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rA \
  tests/test_gpu_cluster.py tests/test_gpu_cluster_ranks.py \
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
args+=($O/c2_k60 300 "python bench.py --config 2 --intervals 60 --steps 10 --no-cpu-baseline --frag-line 0 --json-out gpurun_out/$O/c2_k60.json")
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', 'step %.1f kern %.1f tot %.1f frac %.3f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3, r['frac']))"
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rA \
  > gpurun_out/$O/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/$O/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$O/pytest_gpu.log
