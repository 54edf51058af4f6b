#!/bin/bash
# SQ counters (two passes) of config 5's chunk kernel and of config 3's interval
# kernel (tools/bench_variants.py, production variant), then the namespace-gather
# geometry A/B (kepler_amd/lib/nsvar builds) on config 3.
#   OUT=<dir> tools/gpu_sq_c5.sh
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-sq}
mkdir -p gpurun_out/$O
VARIANTS=0 ROUNDS=2 CONFIG=5 bash tools/pmc_kernel.sh ${O}_c5 -- python3 $GRAFT_REPO_ROOT/tools/bench_variants.py || exit $?
VARIANTS=0 ROUNDS=2 CONFIG=3 bash tools/pmc_kernel.sh ${O}_c3 -- python3 $GRAFT_REPO_ROOT/tools/bench_variants.py || exit $?
python3 tools/pmc_show.py gpurun_out/pmc_${O}_c5 2>/dev/null | head -40
python3 tools/pmc_show.py gpurun_out/pmc_${O}_c3 2>/dev/null | head -40
args=()
for r in 1 2; do
  for l in main u8 l8 l32 u2; do
    if [ "$l" = main ]; then env=""; else env="KACC_LIB=kepler_amd/lib/nsvar/libkepler_accel_$l.so"; fi
    args+=($O/ns_${l}_r$r 300 "env $env python bench.py --steps 30 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line --json-out gpurun_out/$O/ns_${l}_r$r.json")
  done
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/ns_*.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', round(d['ms_per_step']*1e3,1), round(d['kernel_ms']*1e3,1), round(d['totals_compute_ms']*1e3,1))"
done
