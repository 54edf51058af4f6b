#!/bin/bash
# Round 4: the whole -m gpu suite on the carry kernel without loop-carried row registers;
# config 2 x 60 against round 3's build (same box, interleaved); config 1 once.
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r04m}
mkdir -p gpurun_out/$O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > gpurun_out/$O/pytest.log 2>&1 || { echo "tests failed rc=$?"; tail -60 gpurun_out/$O/pytest.log; exit 1; }
tail -1 gpurun_out/$O/pytest.log
X="--no-cpu-baseline --frag-line 0 --no-pipeline-line"  # round 3's bench.py has no host line
args=()
for r in 1 2; do
  for b in r3 main; do
    d=.; h=--no-host-line; [ $b = r3 ] && { d=ab_prev/r3; h=; }
    args+=($O/c2_${b}_r$r 300 "python $d/bench.py --config 2 --intervals 60 --steps 10 --warmup 3 $X $h --json-out gpurun_out/$O/c2_${b}_r$r.json")
  done
done
args+=($O/c1_main 300 "python bench.py --config 1 --steps 30 --warmup 5 $X --no-host-line --json-out gpurun_out/$O/c1_main.json")
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/c*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', 'step %.2f kern %.2f tot %.2f frac %.3f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3, r['frac']))"
done
