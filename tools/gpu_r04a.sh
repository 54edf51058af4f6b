#!/bin/bash
# Round 4, first GPU call: the new tests first (two-rank cluster over the loopback
# collectives, back-to-back node totals, empty batch), then every GPU test + smoke,
# then the default bench (config 3: CPU baseline, slot layouts, pipeline, host_path)
# and the 1/8 shard, config 1 and config 2 x 60 lines.
#   OUT=<dir> tools/gpu_r04a.sh
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r04a}
mkdir -p gpurun_out/$O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -rA \
  tests/test_gpu_cluster_ranks.py tests/test_gpu_cluster.py \
  > gpurun_out/$O/pytest_new.log 2>&1 || { echo "new tests failed rc=$?"; tail -60 gpurun_out/$O/pytest_new.log; exit 1; }
tail -3 gpurun_out/$O/pytest_new.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rA \
  > gpurun_out/$O/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/$O/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$O/pytest_gpu.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/$O/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/$O/smoke.log
tools/gpu_steps.sh \
  $O/bench_c3 600 "python bench.py --json-out gpurun_out/$O/bench_c3.json" \
  $O/bench_c3_shard8 300 "python bench.py --shard-of 8 --steps 50 --warmup 10 --no-cpu-baseline --json-out gpurun_out/$O/bench_c3_shard8.json" \
  $O/bench_c1 300 "python bench.py --config 1 --no-cpu-baseline --frag-line 0 --json-out gpurun_out/$O/bench_c1.json" \
  $O/bench_c2_k60 300 "python bench.py --config 2 --intervals 60 --no-cpu-baseline --frag-line 0 --json-out gpurun_out/$O/bench_c2_k60.json" \
  $O/s8_ns 300 "python bench.py --shard-of 8 --steps 40 --warmup 5 --no-cpu-baseline --totals-probe ns --json-out gpurun_out/$O/bench_s8_ns.json" \
  $O/s8_nodes 300 "python bench.py --shard-of 8 --steps 40 --warmup 5 --no-cpu-baseline --totals-probe nodes --json-out gpurun_out/$O/bench_s8_nodes.json" \
  $O/stamps 300 "python tools/bench_stamps.py > gpurun_out/$O/stamps.jsonl" || exit $?
for f in gpurun_out/$O/bench_c*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', 'value %.2fG step %.1f kern %.1f tot %.1f frac %.3f' % (d['value']/1e9, d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3, r['frac']))"
done
