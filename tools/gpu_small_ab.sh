#!/bin/bash
# Config-1 fleet (small_kernel) A/B: late aggregate stores (nsvar slate build) and the
# slot-node flag; the C-ABI client test; config 3 on the main build.
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-small}
mkdir -p gpurun_out/$O
timeout -k 10 300 python -u -m pytest tests/test_c_client.py tests/test_gpu_small.py -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/$O/pt_main.log 2>&1; echo "main pytest rc=$?: $(tail -1 gpurun_out/$O/pt_main.log)"
LV=KACC_LIB=kepler_amd/lib/nsvar/libkepler_accel_slate.so
env $LV timeout -k 10 300 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_layout.py -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/$O/pt_slate.log 2>&1; echo "slate pytest rc=$?: $(tail -1 gpurun_out/$O/pt_slate.log)"
B="python bench.py --config 1 --steps 30 --warmup 5 --no-cpu-baseline --frag-line 0"
args=()
for r in 1 2; do
  args+=($O/c1_main_r$r 300 "$B --json-out gpurun_out/$O/c1_main_r$r.json")
  args+=($O/c1_write_r$r 300 "$B --slot-nodes write --json-out gpurun_out/$O/c1_write_r$r.json")
  args+=($O/c1_slate_r$r 300 "env $LV $B --json-out gpurun_out/$O/c1_slate_r$r.json")
done
args+=($O/c3_main 300 "python bench.py --steps 40 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line --json-out gpurun_out/$O/c3_main.json")
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', 'step %.1f kern %.1f tot %.1f frac %.3f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3, r['frac']))"
done
