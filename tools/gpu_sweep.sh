#!/bin/bash
# GPU: all parity tests, then interval-kernel timing on pristine / fragmented slots
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/pytest_gpu.log | tail -8
[ $rc -ne 0 ] && exit $rc
for f in 0 0.02; do
  for ns in "" 1; do
    [ "$f" = "0" ] && [ -n "$ns" ] && continue
    FRAG=$f NO_SPAN=$ns VARIANTS=0,2048,32 ROUNDS=10 timeout -k 10 200 python tools/bench_variants.py > gpurun_out/v_$f$ns.json 2> gpurun_out/v_$f$ns.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/v_$f$ns.json'));print('frag=$f nospan=$ns', {k:round(v['median_ms'],4) for k,v in d['variants'].items()}, 'copy', round(d['copy_GBps']))"
  done
done
