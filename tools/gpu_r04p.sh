#!/bin/bash
# Round 4: config 5's big-node path — production (0) against temporal loads (16384: the
# chunks' Δ may hit the Infinity Cache the node pass just filled) and the node pass
# without its CPU-total sum (256, timing ablation), interleaved on one box.
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r04p}
mkdir -p gpurun_out/$O
tools/gpu_steps.sh \
  $O/var_c5 400 "CONFIG=5 VARIANTS=0,16384,256 ROUNDS=10 python tools/bench_variants.py > gpurun_out/$O/var_c5.json" || exit $?
python -c "
import json;d=json.load(open('gpurun_out/$O/var_c5.json'));print({k: round(v['median_ms']*1e3,1) for k,v in d['variants'].items()})"
