#!/bin/bash
# Round 4: same-box A/B of round 3's final build (ab_prev/r3 = git archive 176b537) against
# HEAD on config 3, its 1/8 shard, config 1, config 2 x 60 and config 5 x 60, after the
# cluster + parity tests of HEAD.
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r04g}
mkdir -p gpurun_out/$O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_cluster.py tests/test_gpu_cluster_ranks.py tests/test_gpu_parity.py \
  > gpurun_out/$O/pytest.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/$O/pytest.log; exit 1; }
tail -1 gpurun_out/$O/pytest.log
X="--no-cpu-baseline --frag-line 0 --no-pipeline-line"
args=()
for r in 1 2; do
  for b in r3 main; do
    d=.; [ $b = r3 ] && d=ab_prev/r3
    args+=($O/c3_${b}_r$r 300 "python $d/bench.py --steps 30 --warmup 5 $X --json-out gpurun_out/$O/c3_${b}_r$r.json")
    args+=($O/s8_${b}_r$r 300 "python $d/bench.py --shard-of 8 --steps 50 --warmup 5 $X --json-out gpurun_out/$O/s8_${b}_r$r.json")
    args+=($O/c1_${b}_r$r 300 "python $d/bench.py --config 1 --steps 30 --warmup 5 $X --json-out gpurun_out/$O/c1_${b}_r$r.json")
    args+=($O/c2_${b}_r$r 300 "python $d/bench.py --config 2 --intervals 60 --steps 10 --warmup 3 $X --json-out gpurun_out/$O/c2_${b}_r$r.json")
    args+=($O/c5_${b}_r$r 300 "python $d/bench.py --config 5 --intervals 60 --steps 6 --warmup 2 $X --json-out gpurun_out/$O/c5_${b}_r$r.json")
  done
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', 'step %.2f kern %.2f tot %.2f frac %.3f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3, r['frac']))"
done
