#!/bin/bash
# Chunk-kernel build A/B (geometry, aggregate store order / hints) on config 5 x 60 (kepler_amd/lib/nsvar builds with
# -DKACC_CHUNK_THREADS / -DKACC_CHUNK_WAVES), parity of each variant's big-node
# path first (random fleets, chunk edges, config-5 shape, adversarial, stable nodes).
#   OUT=<dir> LIBS="main c256w5" tools/gpu_chunk_geo.sh
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-geo}
mkdir -p gpurun_out/$O
L=${LIBS:-main cL cP cLP}
libpath() { [ "$1" = main ] && echo "" || echo "KACC_LIB=kepler_amd/lib/nsvar/libkepler_accel_$1.so"; }
for l in $L; do
  env $(libpath $l) timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layout.py -m gpu -q \
    -k "random_fleet or chunk_edges or config5 or adversarial or stable or run_intervals_matches" --timeout 240 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/$O/pt_$l.log 2>&1; rc=$?
  echo "parity $l rc=$rc: $(tail -1 gpurun_out/$O/pt_$l.log)"
  [ $rc -le 1 ] || exit $rc
done
args=()
for r in 1 2; do
  for l in $L; do
    args+=($O/c5_${l}_r$r 300 "env $(libpath $l) python bench.py --config 5 --intervals 60 --steps 5 --warmup 2 --no-cpu-baseline --json-out gpurun_out/$O/c5_${l}_r$r.json")
  done
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/c5_*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', 'step/interval %.1f kern %.1f frac %.3f' % (d['ms_per_step']*1e3/60, d['kernel_ms']*1e3, r['frac']))"
done
