#!/bin/bash
# Round 4: loads in flight per lane in the column-mode node totals past 4096 nodes
# (ab_prev/w8, ab_prev/w16 = this tree with kColLoadsWide 8 / 16; main = 32): the cluster
# kernel's VGPRs (64 / 82 / 166) set the namespace blocks' occupancy.  Config 1 (40k
# nodes), config 3 and the 1/8 shard, interleaved, two rounds.
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r04q}
mkdir -p gpurun_out/$O
X="--no-cpu-baseline --frag-line 0 --no-pipeline-line --no-host-line"
args=()
for r in 1 2; do
  for b in w8 w16 main; do
    d=.; [ $b != main ] && d=ab_prev/$b
    args+=($O/c1_${b}_r$r 300 "python $d/bench.py --config 1 --steps 30 --warmup 5 $X --json-out gpurun_out/$O/c1_${b}_r$r.json")
    args+=($O/c3_${b}_r$r 300 "python $d/bench.py --steps 30 --warmup 5 $X --json-out gpurun_out/$O/c3_${b}_r$r.json")
    args+=($O/s8_${b}_r$r 300 "python $d/bench.py --shard-of 8 --steps 50 --warmup 5 $X --json-out gpurun_out/$O/s8_${b}_r$r.json")
  done
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', 'step %.2f kern %.2f tot %.2f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3))"
done
