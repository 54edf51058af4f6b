#!/bin/bash
# Slot-join A/B: the nsvar "jn" build (non-power-of-two per-node tables) against the
# main build: join / tracker / pipeline GPU tests on jn, then tools/bench_join.py
# interleaved (config 3, 2 % churn) and the bench pipeline line.
set -u
cd "$GRAFT_REPO_ROOT"
O=${OUT:-joinab}
mkdir -p gpurun_out/$O
JV=KACC_LIB=kepler_amd/lib/nsvar/libkepler_accel_jn.so
env $JV timeout -k 10 400 python -u -m pytest tests/test_gpu_join.py tests/test_gpu_tracker.py tests/test_gpu_packer.py -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/$O/pt_jn.log 2>&1; rc=$?
echo "jn pytest rc=$rc: $(tail -1 gpurun_out/$O/pt_jn.log)"
[ $rc -le 1 ] || exit $rc
args=()
for r in 1 2; do
  args+=($O/join_main_r$r 300 "env JOIN_POW2=1 python tools/bench_join.py > gpurun_out/$O/join_main_r$r.json")
  args+=($O/join_jn_r$r 300 "env $JV python tools/bench_join.py > gpurun_out/$O/join_jn_r$r.json")
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/join_*.json; do
  python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', {k: (round(v,4) if isinstance(v,float) else v) for k,v in d.items() if isinstance(v,(int,float))})"
done
