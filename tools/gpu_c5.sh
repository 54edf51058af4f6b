#!/bin/bash
# Every GPU test (stop on failure), then config 5 x 60 (big-node chunk path) and
# config 3, with a rocprofv3 kernel-trace of config 5.
#   OUT=<dir> tools/gpu_c5.sh
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-c5}
mkdir -p gpurun_out/$O
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider -rf \
  > gpurun_out/$O/pytest_gpu.log 2>&1; rc=$?
tail -12 gpurun_out/$O/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
tools/gpu_steps.sh \
  $O/bench_c5_k60 400 "python bench.py --config 5 --intervals 60 --steps 10 --no-cpu-baseline --json-out gpurun_out/$O/bench_c5_k60.json" \
  $O/bench_c3 400 "python bench.py --no-cpu-baseline --frag-line 0 --no-pipeline-line --json-out gpurun_out/$O/bench_c3.json" \
  $O/stats_c5 300 "cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$O/stats_c5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 5 --intervals 60 --steps 3 --warmup 1 --no-cpu-baseline --frag-line 0" || exit $?
python tools/trace_gaps.py gpurun_out/$O/stats_c5 interval_kernel chunk_kernel pod_kernel items_kernel
for f in gpurun_out/$O/bench_c*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', 'value %.2fG step %.1f kern %.1f tot %.1f frac %.3f' % (d['value']/1e9, d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3, r['frac']))"
done
exit $rc
