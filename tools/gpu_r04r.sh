#!/bin/bash
# Round 4: interval_kernel with the rows' previous totals loaded at the attribution
# (kVarLatePrev, 64 VGPRs: four workgroups per CU) against production (three), on
# config 3 and its 1/8 shard (1,250 nodes), pristine and with spans; interleaved.
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r04r}
mkdir -p gpurun_out/$O
tools/gpu_steps.sh \
  $O/c3 300 "VARIANTS=0,262144 ROUNDS=12 python tools/bench_variants.py > gpurun_out/$O/c3.json" \
  $O/s8 300 "NODES=1250 VARIANTS=0,262144 ROUNDS=30 python tools/bench_variants.py > gpurun_out/$O/s8.json" \
  $O/c3span 300 "SPAN=1 VARIANTS=0,262144 ROUNDS=12 python tools/bench_variants.py > gpurun_out/$O/c3span.json" \
  $O/s8span 300 "SPAN=1 NODES=1250 VARIANTS=0,262144 ROUNDS=30 python tools/bench_variants.py > gpurun_out/$O/s8span.json" || exit $?
for f in c3 s8 c3span s8span; do
  python -c "import json;d=json.load(open('gpurun_out/$O/$f.json'));print('$f', {k: round(v['median_ms']*1e3,1) for k,v in d['variants'].items()})"
done
