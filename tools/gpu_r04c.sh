#!/bin/bash
# Round 4, third call: interval_kernel residency A/B (lds2: 2 workgroups per CU via
# extra dynamic LDS; fw4: compiled for 4 waves per SIMD) against main at config 3
# and its 1/8 shard, then the config-1 / config-2 regression A/B against round 2's
# build (tools/gpu_regress_ab.sh, with the sstable variant and PMC).
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r04c}
mkdir -p gpurun_out/$O
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line --no-host-line"
args=()
for r in 1 2; do
  for l in main lds2 fw4; do
    if [ $l = main ]; then e=""; else e="KACC_LIB=kepler_amd/lib/r4var/libkepler_accel_$l.so"; fi
    args+=($O/c3_${l}_r$r 300 "env $e $B --json-out gpurun_out/$O/c3_${l}_r$r.json")
    args+=($O/s8_${l}_r$r 300 "env $e $B --shard-of 8 --steps 50 --json-out gpurun_out/$O/s8_${l}_r$r.json")
  done
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', 'step %.1f kern %.1f tot %.1f frac %.3f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3, r['frac']))"
done
OUT=$O/regab VARS="sstable" ROUNDS="1 2" bash tools/gpu_regress_ab.sh
