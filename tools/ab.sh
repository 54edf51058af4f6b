#!/bin/bash
# A/B two engine builds on the same box, interleaved runs (usage: bash tools/ab.sh libA.so [libB.so])
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
A=$1; B=${2:-kepler_amd/lib/libkepler_accel.so}
for r in ${AB_ROUNDS:-1 2}; do
  for L in $A $B; do
    KACC_LIB=$L VARIANTS=${VARIANTS:-0,1,2,3} ROUNDS=10 timeout -k 10 200 python tools/bench_variants.py > gpurun_out/ab.json 2> gpurun_out/ab.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$L', {k:round(v['median_ms'],4) for k,v in d['variants'].items()}, 'copy', round(d['copy_GBps']))"
  done
done
