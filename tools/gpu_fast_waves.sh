#!/bin/bash
# interval_kernel occupancy A/B: 6 waves per SIMD (main, 3 workgroups per CU) against
# 8 (nsvar f8 build, -DKACC_FAST_WAVES=8: 4 workgroups per CU, some spills) on config 3
# and its 1/8 shard (1,250 nodes on 768 vs 1,024 resident workgroups); parity first.
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-fwaves}
mkdir -p gpurun_out/$O
V=KACC_LIB=kepler_amd/lib/nsvar/libkepler_accel_f8.so
env $V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layout.py -m gpu -q \
  -k "random_fleet or adversarial or stable or fast" --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/$O/pt_f8.log 2>&1; rc=$?
echo "parity f8 rc=$rc: $(tail -1 gpurun_out/$O/pt_f8.log)"
[ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line"
args=()
for r in 1 2; do
  args+=($O/c3_main_r$r 300 "$B --json-out gpurun_out/$O/c3_main_r$r.json")
  args+=($O/c3_f8_r$r 300 "env $V $B --json-out gpurun_out/$O/c3_f8_r$r.json")
  args+=($O/s8_main_r$r 300 "$B --shard-of 8 --json-out gpurun_out/$O/s8_main_r$r.json")
  args+=($O/s8_f8_r$r 300 "env $V $B --shard-of 8 --json-out gpurun_out/$O/s8_f8_r$r.json")
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', 'step %.1f kern %.1f tot %.1f frac %.3f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3, d['roofline']['frac']))"
done
