#!/bin/bash
# Config-1 fleet (small_kernel) A/B of nsvar builds sA (slot-node flag ignored), sB (+ late
# aggregate stores), sC (late aggregate stores only) against the main build.
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-small2}
mkdir -p gpurun_out/$O
for l in sB; do
  env KACC_LIB=kepler_amd/lib/nsvar/libkepler_accel_$l.so timeout -k 10 300 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_layout.py -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/$O/pt_$l.log 2>&1; echo "$l pytest rc=$?: $(tail -1 gpurun_out/$O/pt_$l.log)"
done
B="python bench.py --config 1 --steps 30 --warmup 5 --no-cpu-baseline --frag-line 0"
args=()
for r in 1 2; do
  for l in main sA sB sC; do
    if [ $l = main ]; then e=""; else e="KACC_LIB=kepler_amd/lib/nsvar/libkepler_accel_$l.so"; fi
    args+=($O/c1_${l}_r$r 300 "env $e $B --json-out gpurun_out/$O/c1_${l}_r$r.json")
  done
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', 'step %.1f kern %.1f tot %.1f frac %.3f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3, r['frac']))"
done
