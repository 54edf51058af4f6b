#!/bin/bash
# Round 4, second call: column-mode node totals under the cluster tests + parity,
# then an interleaved A/B of write-through row stores (kepler_amd/lib/r4var: wtp
# process rows, wta aggregates, wtpa both) against the main build at config 3 and
# its 1/8 shard.   OUT=<dir> tools/gpu_r04b.sh
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r04b}
mkdir -p gpurun_out/$O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rA \
  tests/test_gpu_cluster.py tests/test_gpu_cluster_ranks.py tests/test_gpu_parity.py \
  > gpurun_out/$O/pytest.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/$O/pytest.log; exit 1; }
tail -1 gpurun_out/$O/pytest.log
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --frag-line 0 --no-pipeline-line --no-host-line"
args=()
for r in 1 2; do
  for l in main wtp wta wtpa; do
    if [ $l = main ]; then e=""; else e="KACC_LIB=kepler_amd/lib/r4var/libkepler_accel_$l.so"; fi
    args+=($O/c3_${l}_r$r 300 "env $e $B --json-out gpurun_out/$O/c3_${l}_r$r.json")
    args+=($O/s8_${l}_r$r 300 "env $e $B --shard-of 8 --steps 50 --json-out gpurun_out/$O/s8_${l}_r$r.json")
  done
done
tools/gpu_steps.sh "${args[@]}" || exit $?
for f in gpurun_out/$O/*.json; do
  python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', 'step %.1f kern %.1f tot %.1f frac %.3f' % (d['ms_per_step']*1e3, d['kernel_ms']*1e3, d['totals_compute_ms']*1e3, r['frac']))"
done
