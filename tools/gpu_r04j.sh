#!/bin/bash
# Round 4: slot-join lookups reading four buckets per LDS read (kJGroup, production) —
# join / packer / tracker parity, the variant A/B at config 3 (outputs identical), the
# per-phase stops, and the per-phase SQ counters of the production join.
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r04l}
mkdir -p gpurun_out/$O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_join.py tests/test_gpu_packer.py tests/test_gpu_tracker.py \
  > gpurun_out/$O/pytest.log 2>&1 || { echo "tests failed rc=$?"; tail -60 gpurun_out/$O/pytest.log; exit 1; }
tail -1 gpurun_out/$O/pytest.log
timeout -k 10 400 python -u tools/bench_join_variants.py > gpurun_out/$O/variants.json 2> gpurun_out/$O/variants.err \
  || { echo "variants rc=$?"; tail -30 gpurun_out/$O/variants.err; exit 1; }
cat gpurun_out/$O/variants.json
timeout -k 10 400 python -u tools/bench_join.py > gpurun_out/$O/join.json 2> gpurun_out/$O/join.err \
  || { echo "bench_join rc=$?"; tail -30 gpurun_out/$O/join.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/$O/join.json'));print(d['join_ms'], d['phase_ms'], d.get('pipeline_reuse_join_ms'))"
OUT=$O/sq tools/join_phase_sq.sh || { echo "sq rc=$?"; tail -20 gpurun_out/$O/sq/run.log; exit 1; }
ls gpurun_out/$O/sq
