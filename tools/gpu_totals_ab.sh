#!/bin/bash
# GPU tests, then a same-box interleaved A/B of the cluster-totals modes (tables: a
# partial-sum launch per step; fused: kacc_run_interval_sums, the previous step's sums in
# the interval's launch) at config 3 and its 1/8 shard.
#   OUT=<dir> [TESTS='tests -m gpu'] [REPS=2] tools/gpu_totals_ab.sh
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-totals_ab}
mkdir -p gpurun_out/$O
timeout -k 10 900 python -u -m pytest ${TESTS:-tests -m gpu} -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/$O/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/$O/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$O/pytest_gpu.log
B="--no-cpu-baseline --frag-line 0 --no-pipeline-line --no-host-line"
args=()
for r in $(seq 1 ${REPS:-2}); do
  for t in tables fused; do
    args+=($O/s8_${t}_r$r 300 "python bench.py --shard-of 8 --steps 50 --warmup 10 $B --totals $t --json-out gpurun_out/$O/s8_${t}_r$r.json")
    args+=($O/c3_${t}_r$r 300 "python bench.py --steps 20 --warmup 3 $B --totals $t --json-out gpurun_out/$O/c3_${t}_r$r.json")
  done
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*_r*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];t=d['totals_compute_ms'];print('$f', 'value %.2fG step %.2f us kern %.2f us tot %s frac %.3f' % (d['value']/1e9, d['ms_per_step']*1e3, d['kernel_ms']*1e3, ('%.2f us' % (t*1e3)) if t else '-', r['frac']))"
done
# the end-to-end lines: float64 batches (host_path) and the CPU-tick format (host_path_ticks)
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --frag-line 0 --no-pipeline-line --totals fused \
  --json-out gpurun_out/$O/c3_host.json > gpurun_out/$O/c3_host.log 2>&1 || { echo "host lines rc=$?"; tail -20 gpurun_out/$O/c3_host.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/$O/c3_host.json'));print({k: {x: d[k].get(x) for x in ('proc_attr_per_s','ms_per_interval','h2d_bytes_per_interval','frac_of_pcie_copy','error')} for k in ('host_path','host_path_ticks')})"
