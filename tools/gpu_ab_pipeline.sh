#!/bin/bash
# Tracker / production-pipeline A/B: the tracker tests, then bench.py's pipeline line for this
# build and kepler_amd/lib/ab/libkepler_accel_base.so (KACC_LIB), interleaved, REPS rounds.
#   OUT=<dir> [REPS=2] tools/gpu_ab_pipeline.sh
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-ab_pipeline}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tracker.py tests/test_gpu_join.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for r in $(seq 1 ${REPS:-2}); do
  for v in base main; do
    L=""; [ $v = base ] && L="kepler_amd/lib/ab/libkepler_accel_base.so"
    timeout -k 10 300 env ${L:+KACC_LIB=$L} python bench.py --steps 10 --warmup 2 --no-cpu-baseline --frag-line 0 --no-host-line \
      --json-out $O/${v}_r$r.json > $O/${v}_r$r.log 2>&1 || { echo "bench $v rc=$?"; tail -5 $O/${v}_r$r.log; exit 1; }
    python -c "import json;p=json.load(open('$O/${v}_r$r.json'))['pipeline'];print('$v', {k: round(p[k],4) for k in ('ms_per_interval','ms_per_interval_split','join_ms','tracker_ms','interval_ms')})"
  done
done
