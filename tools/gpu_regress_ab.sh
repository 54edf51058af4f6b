#!/bin/bash
# Round-4 verdict item 4: same-box interleaved A/B of round 2's final build (0ca49db,
# its own tree under ab_prev/r2: the ABI changed since) against HEAD (and variants under
# kepler_amd/lib/r4var/) on config 1 (small_kernel<2>) and config 2 x 60 (carry kernel),
# each run under rocprofv3 --kernel-trace --stats (the kernel's own duration, whatever
# each bench's event method), then FETCH_SIZE / WRITE_SIZE passes of config 1 for r2 and
# HEAD.   OUT=<dir> VARS="sstable" ROUNDS="1 2" tools/gpu_regress_ab.sh
set -u -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R"
export TMPDIR=/tmp
O=$R/gpurun_out/${OUT:-regab}
mkdir -p "$O"
step() { local n=$1 s=$2; shift 2; echo "== $n"; (cd /tmp && timeout -k 10 "$s" "$@") > "$O/$n.log" 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -2 "$O/$n.log"; [ $rc -eq 0 ] || exit $rc; }
run() {  # name build config-args...
  local name=$1 build=$2; shift 2
  local dir=$R env=()
  case $build in
    r2) dir=$R/ab_prev/r2 ;;
    main) ;;
    *) env=(KACC_LIB=$R/kepler_amd/lib/r4var/libkepler_accel_$build.so) ;;
  esac
  step "$name" 300 env "${env[@]}" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$name" -o run -- \
    python3 "$dir/bench.py" "$@" --no-cpu-baseline --frag-line 0 --json-out "$O/$name.json"
}
for r in ${ROUNDS:-1 2}; do
  for b in r2 main ${VARS:-}; do
    run c1_${b}_r$r $b --config 1 --steps 30 --warmup 5
    run c2_${b}_r$r $b --config 2 --intervals 60 --steps 10 --warmup 3
  done
done
if [ -z "${SKIP_PMC:-}" ]; then
  for b in r2 main; do
    dir=$R; [ $b = r2 ] && dir=$R/ab_prev/r2
    for c in FETCH_SIZE WRITE_SIZE; do
      step pmc_${b}_$c 240 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_${b}_$c" -o run -- \
        python3 "$dir/bench.py" --config 1 --steps 5 --warmup 1 --no-cpu-baseline --frag-line 0
    done
  done
fi
python3 "$R/tools/regress_summary.py" "$O"
