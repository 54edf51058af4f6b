#!/bin/bash
# Full set on one box: every GPU test + smoke (stop on failure), the default
# bench (config 3 with CPU baseline, slot layouts, pipeline), the 2/4/8-way shards,
# then this build's HBM traffic (FETCH_SIZE / WRITE_SIZE passes -> pmc_traffic.json)
# and a rocprofv3 kernel-trace summary of the config-3 bench.
#   OUT=<dir> [SKIP_PMC=1] tools/gpu_full.sh
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-full}
mkdir -p gpurun_out/$O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -rA \
  > gpurun_out/$O/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/$O/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$O/pytest_gpu.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/$O/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/$O/smoke.log
tools/gpu_steps.sh \
  $O/bench_c3 600 "python bench.py --json-out gpurun_out/$O/bench_c3.json" \
  $O/bench_c3_shard2 300 "python bench.py --shard-of 2 --steps 50 --warmup 10 --no-cpu-baseline --json-out gpurun_out/$O/bench_c3_shard2.json" \
  $O/bench_c3_shard4 300 "python bench.py --shard-of 4 --steps 50 --warmup 10 --no-cpu-baseline --json-out gpurun_out/$O/bench_c3_shard4.json" \
  $O/bench_c3_shard8 300 "python bench.py --shard-of 8 --steps 50 --warmup 10 --no-cpu-baseline --json-out gpurun_out/$O/bench_c3_shard8.json" \
  $O/bench_c1 300 "python bench.py --config 1 --no-cpu-baseline --frag-line 0 --json-out gpurun_out/$O/bench_c1.json" \
  $O/bench_c2_k60 300 "python bench.py --config 2 --intervals 60 --no-cpu-baseline --frag-line 0 --json-out gpurun_out/$O/bench_c2_k60.json" \
  $O/bench_c2_k60_write 300 "python bench.py --config 2 --intervals 60 --no-cpu-baseline --frag-line 0 --slot-nodes write --json-out gpurun_out/$O/bench_c2_k60_write.json" \
  $O/bench_c5_k60 400 "python bench.py --config 5 --intervals 60 --steps 10 --no-cpu-baseline --json-out gpurun_out/$O/bench_c5_k60.json" || exit $?
if [ -z "${SKIP_PMC:-}" ]; then
  OUT=$O/pmc CONFIGS="${PMC_CONFIGS:-3 1 5}" bash tools/gpu_pmc_traffic.sh || exit $?
  (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$O/stats_c3" -o run -- \
     python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --frag-line 0 --no-pipeline-line \
     --no-host-line --json-out "$GRAFT_REPO_ROOT/gpurun_out/$O/bench_c3_prof.json") > gpurun_out/$O/stats_c3.log 2>&1 || exit $?
  python tools/trace_gaps.py gpurun_out/$O/stats_c3 interval_kernel cluster_partials
  (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$O/stats_s8" -o run -- \
     python3 "$GRAFT_REPO_ROOT/bench.py" --shard-of 8 --steps 50 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line \
     --no-host-line --json-out "$GRAFT_REPO_ROOT/gpurun_out/$O/bench_s8_prof.json") > gpurun_out/$O/stats_s8.log 2>&1 || exit $?
fi
for f in gpurun_out/$O/bench_c*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', 'value %.2fG step %.1f kern %.1f tot %.1f frac %.3f' % (d['value']/1e9, d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3, r['frac']))"
done
