#!/bin/bash
# Same-box A/B of KACC_F_STABLE_SLOT_NODES (config 3 and its 1/8 shard), interleaved.
#   OUT=<dir> ROUNDS=2 tools/gpu_stable_ab.sh
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-stab}
mkdir -p gpurun_out/$O
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line"
args=()
for r in $(seq 1 ${ROUNDS:-2}); do
  for m in stable write; do
    args+=($O/c3_${m}_r$r 300 "$B --slot-nodes $m --json-out gpurun_out/$O/c3_${m}_r$r.json")
    args+=($O/s8_${m}_r$r 300 "$B --shard-of 8 --slot-nodes $m --json-out gpurun_out/$O/s8_${m}_r$r.json")
  done
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', 'step %.1f kern %.1f tot %.1f frac %.3f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3, r['frac']))"
done
