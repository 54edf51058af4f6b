#!/bin/bash
# Round 4: namespace-sum geometry in the 64-VGPR cluster kernel — pods in flight per
# lane 4 (ab_prev/u4) and 8 lanes per namespace (ab_prev/l8) against 16 lanes x 2
# (main): config 3 and its 1/8 shard, interleaved, two rounds.
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r04x}
mkdir -p gpurun_out/$O
X="--no-cpu-baseline --frag-line 0 --no-pipeline-line --no-host-line"
args=()
for r in 1 2; do
  for b in main u4 l8; do
    d=.; [ $b != main ] && d=ab_prev/$b
    args+=($O/c3_${b}_r$r 300 "python $d/bench.py --steps 30 --warmup 5 $X --json-out gpurun_out/$O/c3_${b}_r$r.json")
    args+=($O/s8_${b}_r$r 300 "python $d/bench.py --shard-of 8 --steps 50 --warmup 5 $X --json-out gpurun_out/$O/s8_${b}_r$r.json")
  done
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', 'step %.2f kern %.2f tot %.2f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3))"
done
