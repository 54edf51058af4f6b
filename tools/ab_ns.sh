#!/bin/bash
# Namespace-gather geometry A/B (config 3, cluster totals from the tables): the
# same bench line per variant library (kepler_amd/lib/variants/*, built with
# -DKACC_NS_LANES / -DKACC_NS_UNROLL / -DKACC_NS_PROBE_PAIRED), alternated over
# ROUNDS; bench.py reports totals_compute_ms (interval end -> partial sums end).
#   OUT=<dir> LIBS="main u8 l8u8 pair pairu8" ROUNDS=2 tools/ab_ns.sh
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-abns}
mkdir -p gpurun_out/$O
args=()
for r in $(seq 1 ${ROUNDS:-2}); do
  for l in ${LIBS:-main u8 l8u8 pair pairu8}; do
    if [ "$l" = main ]; then env=""; else env="KACC_LIB=kepler_amd/lib/variants/libkepler_accel_$l.so"; fi
    args+=($O/${l}_r$r 300 "env $env python bench.py --steps 30 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line --json-out gpurun_out/$O/${l}_r$r.json")
  done
done
tools/gpu_steps.sh "${args[@]}"
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', round(d['ms_per_step']*1e3,1), round(d['kernel_ms']*1e3,1), round(d['totals_compute_ms']*1e3,1))"
done
