#!/bin/bash
# Round 4: the node CPU-total tree's first two levels by one wave (one workgroup barrier
# fewer in interval_node and big_node_prepare; bit-identical by construction) — the
# whole -m gpu suite, then config 3, its 1/8 shard and config 5 against the build
# before (ab_prev/base), interleaved, two rounds.
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r04v}
mkdir -p gpurun_out/$O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > gpurun_out/$O/pytest.log 2>&1 || { echo "tests failed rc=$?"; tail -60 gpurun_out/$O/pytest.log; exit 1; }
tail -1 gpurun_out/$O/pytest.log
X="--no-cpu-baseline --frag-line 0 --no-pipeline-line --no-host-line"
args=()
for r in 1 2; do
  for b in base main; do
    d=.; [ $b != main ] && d=ab_prev/$b
    args+=($O/c3_${b}_r$r 300 "python $d/bench.py --steps 30 --warmup 5 $X --json-out gpurun_out/$O/c3_${b}_r$r.json")
    args+=($O/s8_${b}_r$r 300 "python $d/bench.py --shard-of 8 --steps 50 --warmup 5 $X --json-out gpurun_out/$O/s8_${b}_r$r.json")
    args+=($O/c5_${b}_r$r 300 "python $d/bench.py --config 5 --steps 8 --warmup 2 $X --json-out gpurun_out/$O/c5_${b}_r$r.json")
  done
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/c*.json gpurun_out/$O/s*.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', 'step %.2f kern %.2f tot %.2f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3))"
done
