#!/bin/bash
# Launch-latency A/B: HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device memory)
# on config 3 and its 1/8 shard, interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-karg}
mkdir -p gpurun_out/$O
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line"
args=()
for r in 1 2; do
  for m in 0 1; do
    args+=($O/c3_k${m}_r$r 300 "env HIP_FORCE_DEV_KERNARG=$m $B --json-out gpurun_out/$O/c3_k${m}_r$r.json")
    args+=($O/s8_k${m}_r$r 300 "env HIP_FORCE_DEV_KERNARG=$m $B --shard-of 8 --json-out gpurun_out/$O/s8_k${m}_r$r.json")
  done
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', 'step %.1f kern %.1f tot %.1f evpass %.1f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3, d['kernel_timing']['ms_per_step_timing_pass']*1e3))"
done
