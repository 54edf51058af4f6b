#!/bin/bash
# GPU tests, then a same-box interleaved A/B of this build against
# kepler_amd/lib/ab/libkepler_accel_base.so (KACC_LIB) on the bench lines CASES names.
#   OUT=<dir> [TESTS='tests -m gpu'] [REPS=2] CASES="c1 c3 s8 c5" tools/gpu_ab.sh
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-ab}
mkdir -p gpurun_out/$O
timeout -k 10 900 python -u -m pytest ${TESTS:-tests -m gpu} -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/$O/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/$O/pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/$O/pytest_gpu.log
B="--no-cpu-baseline --frag-line 0 --no-pipeline-line --no-host-line"
args=()
for r in $(seq 1 ${REPS:-2}); do
  for v in base main; do
    L=""; [ $v = base ] && L="KACC_LIB=kepler_amd/lib/ab/libkepler_accel_base.so"
    for c in ${CASES:-c1 c3 s8}; do
      case $c in
        c1) a="--config 1 --steps 20 --warmup 3" ;;
        c3) a="--steps 20 --warmup 3" ;;
        s8) a="--shard-of 8 --steps 50 --warmup 10" ;;
        c5) a="--config 5 --intervals 60 --steps 6 --warmup 1" ;;
        *) echo "unknown case $c"; exit 2 ;;
      esac
      args+=($O/${c}_${v}_r$r 400 "$L python bench.py $a $B --json-out gpurun_out/$O/${c}_${v}_r$r.json")
    done
  done
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*_r*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];K=d['config']['intervals_per_step'];print('$f', 'value %.2fG step/interval %.2f us kern %.2f us totals %s frac %.3f scrape %s' % (d['value']/1e9, d['ms_per_step']*1e3/K, d['kernel_ms']*1e3, d.get('totals_compute_ms'), r['frac'], (d.get('scrape_powers') or {}).get('ms')))"
done
