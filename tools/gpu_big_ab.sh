#!/bin/bash
# GPU tests, then a same-box interleaved A/B of this build against kepler_amd/lib/ab/libkepler_accel_base.so
# (KACC_LIB) at config 5 x 60 intervals, config 3 and its 1/8 shard.
#   OUT=<dir> [TESTS='tests -m gpu'] [REPS=2] tools/gpu_big_ab.sh
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-big_ab}
mkdir -p gpurun_out/$O
timeout -k 10 900 python -u -m pytest ${TESTS:-tests -m gpu} -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/$O/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/$O/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$O/pytest_gpu.log
B="--no-cpu-baseline --frag-line 0 --no-pipeline-line --no-host-line"
args=()
for r in $(seq 1 ${REPS:-2}); do
  for v in base main; do
    L=""; [ $v = base ] && L="KACC_LIB=kepler_amd/lib/ab/libkepler_accel_base.so"
    args+=($O/c5_${v}_r$r 400 "$L python bench.py --config 5 --intervals 60 --steps 6 --warmup 1 $B --json-out gpurun_out/$O/c5_${v}_r$r.json")
    args+=($O/c3_${v}_r$r 300 "$L python bench.py --steps 20 --warmup 3 $B --json-out gpurun_out/$O/c3_${v}_r$r.json")
    args+=($O/s8_${v}_r$r 300 "$L python bench.py --shard-of 8 --steps 50 --warmup 10 $B --json-out gpurun_out/$O/s8_${v}_r$r.json")
  done
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*_r*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];K=d['config']['intervals_per_step'];print('$f', 'value %.2fG step/interval %.2f us kern %.2f us frac %.3f' % (d['value']/1e9, d['ms_per_step']*1e3/K, d['kernel_ms']*1e3, r['frac']))"
done
