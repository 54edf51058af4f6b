#!/bin/bash
# Round 4: the terminated tracker's already-tracked check through an LDS hash set —
# tracker + join GPU tests, then tools/bench_join.py (tracker and pipeline timings) on
# this build and on the build before (ab_prev/trk0), interleaved, two rounds each.
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r04u}
mkdir -p gpurun_out/$O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_tracker.py tests/test_gpu_join.py > gpurun_out/$O/pytest.log 2>&1 \
  || { echo "tests failed rc=$?"; tail -60 gpurun_out/$O/pytest.log; exit 1; }
tail -1 gpurun_out/$O/pytest.log
args=()
for r in 1 2; do
  for b in trk0 main; do
    d=.; [ $b != main ] && d=ab_prev/$b
    args+=($O/join_${b}_r$r 400 "python $d/tools/bench_join.py > gpurun_out/$O/join_${b}_r$r.json")
  done
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/join_*.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', 'tracker %.4f pipeline %.4f reuse_first %.4f join %.4f' % (d['tracker_ms'], d['pipeline_ms'], d['pipeline_reuse_tracker_first_ms'], d['join_ms']))"
done
