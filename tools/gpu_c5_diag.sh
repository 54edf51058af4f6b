#!/bin/bash
# Config 5 (1000 big nodes x 60 intervals per kacc_run_intervals call): this build against
# kepler_amd/lib/ab/libkepler_accel_{base,nofuse}.so (KACC_LIB), then per-kernel rocprof
# statistics of each, so a change in the chunk path is split by kernel.
#   OUT=<dir> [REPS=2] tools/gpu_c5_diag.sh
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-c5_diag}
mkdir -p gpurun_out/$O
B="--config 5 --intervals 60 --no-cpu-baseline --frag-line 0 --no-pipeline-line --no-host-line"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/$O/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/$O/pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/$O/pytest_gpu.log
for v in fusedlate early; do
  KACC_LIB=kepler_amd/lib/ab/libkepler_accel_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_export_sums.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/$O/pytest_$v.log 2>&1 || { echo "$v pytest failed rc=$?"; tail -30 gpurun_out/$O/pytest_$v.log; exit 1; }
  tail -n 1 gpurun_out/$O/pytest_$v.log
done
args=()
for r in $(seq 1 ${REPS:-2}); do
  for v in base nofuse fusedlate early main; do
    L=""; [ $v != main ] && L="KACC_LIB=kepler_amd/lib/ab/libkepler_accel_$v.so"
    args+=($O/c5_${v}_r$r 400 "$L python bench.py --steps 6 --warmup 1 $B --json-out gpurun_out/$O/c5_${v}_r$r.json")
  done
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for v in base nofuse fusedlate early main; do
  if [ $v = main ]; then unset KACC_LIB; else export KACC_LIB=kepler_amd/lib/ab/libkepler_accel_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$O/prof_$v -o run -- \
    python bench.py --steps 2 --warmup 1 $B > gpurun_out/$O/prof_$v.log 2>&1 || { echo "rocprof $v rc=$?"; exit 1; }
done
unset KACC_LIB
for f in gpurun_out/$O/c5_*_r*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];K=d['config']['intervals_per_step'];print('$f', 'value %.2fG step/interval %.2f us kern %.2f us frac %.3f' % (d['value']/1e9, d['ms_per_step']*1e3/K, d['kernel_ms']*1e3, r['frac']))"
done
for v in base nofuse fusedlate early main; do
  echo "== $v"; s=$(find gpurun_out/$O/prof_$v -name '*kernel_stats.csv' | head -n 1); [ -n "$s" ] && head -n 8 "$s"
done
