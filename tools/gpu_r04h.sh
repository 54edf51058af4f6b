#!/bin/bash
# Round 4: the 6-B-bucket slot join (kJ6B / kJSeenNR / kJVec) — join parity tests and
# the join pipeline tests, the variant A/B at config 3 (outputs checked identical to
# round 2's kernel), the per-phase stops of the production join, and config 1 with
# the wide column-sum rounds.
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r04h}
mkdir -p gpurun_out/$O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_join.py tests/test_gpu_packer.py tests/test_gpu_tracker.py tests/test_gpu_cluster.py tests/test_gpu_cluster_ranks.py \
  > gpurun_out/$O/pytest.log 2>&1 || { echo "tests failed rc=$?"; tail -60 gpurun_out/$O/pytest.log; exit 1; }
tail -1 gpurun_out/$O/pytest.log
timeout -k 10 400 python -u tools/bench_join_variants.py > gpurun_out/$O/variants.json 2> gpurun_out/$O/variants.err \
  || { echo "variants rc=$?"; tail -30 gpurun_out/$O/variants.err; exit 1; }
cat gpurun_out/$O/variants.json
timeout -k 10 400 python -u tools/bench_join.py > gpurun_out/$O/join.json 2> gpurun_out/$O/join.err \
  || { echo "bench_join rc=$?"; tail -30 gpurun_out/$O/join.err; exit 1; }
X="--no-cpu-baseline --frag-line 0 --no-pipeline-line"
timeout -k 10 300 python bench.py --config 1 --steps 30 --warmup 5 $X --json-out gpurun_out/$O/c1.json > gpurun_out/$O/c1.log 2>&1 \
  || { echo "c1 rc=$?"; tail -30 gpurun_out/$O/c1.log; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 5 $X --json-out gpurun_out/$O/c3.json > gpurun_out/$O/c3.log 2>&1 \
  || { echo "c3 rc=$?"; tail -30 gpurun_out/$O/c3.log; exit 1; }
for f in gpurun_out/$O/c*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', 'step %.2f kern %.2f tot %.2f frac %.3f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3, r['frac']))"
done
python -c "import json;d=json.load(open('gpurun_out/$O/join.json'));print(d['join_ms'], d['phase_ms'], d.get('pipeline_reuse_join_ms'))"
