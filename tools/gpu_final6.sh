#!/bin/bash
# Round 6 evidence of the current build: the whole -m gpu suite and smoke(); rocprofv3
# kernel statistics (csv) of configs 3, 1, 5 (x60 intervals) and the 1/8 shard; PMC traffic
# (configs 3, 1, 5 and the shard's fused launch; profiles/pmc_traffic.json is keyed by the
# library's sha256); then the bench lines (default = config 3, which carries
# roofline.traffic, cpu_baseline and the secondary lines).
#   OUT=<dir> [PART=a|b] [PMC=0] [JOIN=0] tools/gpu_final6.sh
# PART=a: tests, smoke, kernel stats, PMC traffic; PART=b: bench lines and the join evidence
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-final6}
mkdir -p gpurun_out/$O
sha=$(sha256sum kepler_amd/lib/libkepler_accel.so | cut -c1-16)
echo "lib sha256 $sha" | tee gpurun_out/$O/lib_sha256.txt
B="--no-cpu-baseline --frag-line 0 --no-pipeline-line --no-host-line"
if [ "${PART:-a}" = a ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/$O/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/$O/pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/$O/pytest_gpu.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/$O/smoke.log 2>&1 || exit $?
tail -n 1 gpurun_out/$O/smoke.log
prof() {  # NAME SECONDS bench-args...
  local n=$1 s=$2; shift 2
  echo "== prof $n"
  timeout -k 10 "$s" rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$O/prof_$n -o run -- \
    python3 bench.py "$@" --json-out gpurun_out/$O/prof_$n.json > gpurun_out/$O/prof_$n.log 2>&1 || { echo "prof $n rc=$?"; exit 1; }
  f=$(find gpurun_out/$O/prof_$n -name '*kernel_stats.csv' | head -n 1)
  cp "$f" gpurun_out/$O/kernel_stats_${n}_$sha.csv
  head -n 6 "$f" | cut -c1-200
}
prof c3 300 --steps 20 --warmup 3 $B
prof c1 300 --config 1 --steps 20 --warmup 3 $B
prof c5 400 --config 5 --intervals 60 --steps 4 --warmup 1 $B
prof s8 300 --shard-of 8 --steps 50 --warmup 10 $B
if [ "${PMC:-1}" = 1 ]; then
  OUT=$O/pmc PMC_ROUND=r06 CONFIGS="3 1 5 s8" bash tools/gpu_pmc_traffic.sh || exit $?
  cp gpurun_out/$O/pmc/pmc_traffic.json profiles/pmc_traffic.json
fi
fi
run() {  # NAME SECONDS bench-args...
  local n=$1 s=$2; shift 2
  echo "== bench $n"
  timeout -k 10 "$s" python bench.py "$@" --json-out gpurun_out/$O/bench_$n.json > gpurun_out/$O/bench_$n.log 2>&1 \
    || { echo "bench $n rc=$?"; tail -5 gpurun_out/$O/bench_$n.log; exit 1; }
  tail -n 1 gpurun_out/$O/bench_$n.log | cut -c1-400
}
if [ "${PART:-a}" = b ]; then
run c3 600
run c1 300 --config 1 --no-cpu-baseline
run c5 400 --config 5 --intervals 60 --no-cpu-baseline
run s8 300 --shard-of 8 --steps 50 --warmup 10 $B
run s8_handoff 300 --shard-of 8 --steps 48 --warmup 8 --comm-wait always --allreduce-every 8 $B
# the slot join: per-phase times (stops 1..8), the round-5 kernel (511) beside production (-1)
# and the first cuckoo build (25087), the per-wave SQ counters of the same three, then the
# production kernel's SQ counters per phase stop
if [ "${JOIN:-1}" = 1 ]; then
  echo "== join"
  timeout -k 10 400 env STOPS=1,2,3,4,5,6,7,8,0 python -u tools/bench_join.py > gpurun_out/$O/join.json 2>gpurun_out/$O/join.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/$O/join.json'));print(d['join_ms'], d['phase_ms'])"
  timeout -k 10 300 env VARIANTS=511,-1,25087 ROUNDS=5 python -u tools/bench_join_variants.py > gpurun_out/$O/variants.json 2>gpurun_out/$O/variants.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/$O/variants.json'));print(d['join_ms'], d['identical_to_first'])"
  OUT=$O/join_pmc VARIANTS=511,-1,25087 bash tools/join_pmc.sh > /dev/null || exit $?
  OUT=$O/join_phase_pmc STOPS=1,2,3,4,5,6,7,8,0 REPS=4 bash tools/join_pmc.sh > /dev/null || exit $?
fi
fi
