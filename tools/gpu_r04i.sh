#!/bin/bash
# Round 4: the whole -m gpu suite on the 6-B join + carried zone totals in LDS; config 2 x 60
# against round 3's build (same box, interleaved); config 5 kernel stats (rocprofv3) and
# its PMC traffic (interval + chunk + pod kernels per interval).
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r04i}
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
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/c2*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', 'step %.2f kern %.2f frac %.3f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, r['frac']))"
done
OUT=$O/prof_c5 tools/prof_c5.sh || exit $?
OUT=$O/pmc CONFIGS="5" tools/gpu_pmc_traffic.sh || exit $?
