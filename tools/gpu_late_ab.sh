#!/bin/bash
# Late-aggregate A/B (kepler_amd/lib/nsvar/libkepler_accel_late.so, -DKACC_LATE_AGG=1):
# every GPU test on the variant library, then bench.py config 3 and its 1/8 shard,
# interleaved with the main build.
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-late}
mkdir -p gpurun_out/$O
LV=KACC_LIB=kepler_amd/lib/nsvar/libkepler_accel_late.so
env $LV timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider -rf \
  > gpurun_out/$O/pytest_late.log 2>&1; rc=$?
echo "late pytest rc=$rc: $(tail -1 gpurun_out/$O/pytest_late.log)"
[ $rc -le 1 ] || exit $rc
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line"
args=()
for r in 1 2 3; do
  args+=($O/c3_main_r$r 300 "$B --json-out gpurun_out/$O/c3_main_r$r.json")
  args+=($O/c3_late_r$r 300 "env $LV $B --json-out gpurun_out/$O/c3_late_r$r.json")
done
args+=($O/s8_main 300 "$B --shard-of 8 --json-out gpurun_out/$O/s8_main.json")
args+=($O/s8_late 300 "env $LV $B --shard-of 8 --json-out gpurun_out/$O/s8_late.json")
args+=($O/c1_main 300 "python bench.py --config 1 --steps 20 --no-cpu-baseline --frag-line 0 --json-out gpurun_out/$O/c1_main.json")
args+=($O/c1_late 300 "env $LV python bench.py --config 1 --steps 20 --no-cpu-baseline --frag-line 0 --json-out gpurun_out/$O/c1_late.json")
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', 'step %.1f kern %.1f tot %.1f frac %.3f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3, r['frac']))"
done
