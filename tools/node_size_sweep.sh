#!/bin/bash
# Interval-kernel bandwidth vs processes per node (config-3 shape, Z=4, ~20M rows).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/nodesize
for pn in "${@:-2000:10000 1000:20000 500:40000 250:80000}"; do
  for x in $pn; do
    p=${x%%:*}; n=${x##*:}
    PROCS=$p NODES=$n VARIANTS=${VARIANTS:-0} ROUNDS=6 timeout -k 10 240 python tools/bench_variants.py \
      > gpurun_out/nodesize/p$p.json 2> gpurun_out/nodesize/p$p.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/nodesize/p$p.json'));print('procs/node',$p,'nodes',$n,{k:round(v['median_ms'],4) for k,v in d['variants'].items()},'GB/s',round(d['achieved_GBps_v0']),'copy',round(d['copy_GBps']))"
  done
done
