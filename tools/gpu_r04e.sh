#!/bin/bash
# Round 4: slot-join phase profile (tools/bench_join.py) and the config-5 chunk-kernel
# residency A/B (late previous totals: c5l1w6 / c5l2w6 at three workgroups per CU).
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r04e}
mkdir -p gpurun_out/$O
args=($O/join 300 "CONFIG=3 python tools/bench_join.py > gpurun_out/$O/join.json")
B="python bench.py --config 5 --intervals 60 --steps 6 --warmup 2 --no-cpu-baseline --frag-line 0"
for r in 1 2; do
  for l in main c5l1w6 c5l2w6; do
    if [ $l = main ]; then e=""; else e="KACC_LIB=kepler_amd/lib/r4var/libkepler_accel_$l.so"; fi
    args+=($O/c5_${l}_r$r 300 "env $e $B --json-out gpurun_out/$O/c5_${l}_r$r.json")
  done
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/c5*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', 'step %.1f kern %.1f frac %.3f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, r['frac']))"
done
python -c "import json;d=json.load(open('gpurun_out/$O/join.json'));print({k:d[k] for k in ('join_ms','phase_ms','pipeline_reuse_join_ms','pipeline_reuse_interval_ms','tracker_ms')})"
