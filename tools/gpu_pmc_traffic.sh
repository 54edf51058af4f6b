#!/bin/bash
# HBM traffic of the current build (separate FETCH_SIZE / WRITE_SIZE --pmc passes,
# MI355X_MICROARCH.md §HBM corrections via tools/pmc_summary.py), merged into a copy
# of profiles/pmc_traffic.json under gpurun_out/$OUT/ (entries carry the lib sha256).
#   OUT=<dir> CONFIGS="3 1" tools/gpu_pmc_traffic.sh
set -u -o pipefail
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out/${OUT:-pmc}
mkdir -p "$O"
cp "$R/profiles/pmc_traffic.json" "$O/pmc_traffic.json"
step() { local n=$1 s=$2; shift 2; echo "== $n"; (cd /tmp && timeout -k 10 "$s" "$@") > "$O/$n.log" 2>&1; local rc=$?; echo "== $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for c in ${CONFIGS:-3 1}; do
  case $c in
    3) kern="interval_kernel<4, 0>"; cmd=(python3 "$R/tools/bench_variants.py"); export VARIANTS=0 ROUNDS=3 CONFIG=3 ;;
    1) kern="small_kernel<2"; cmd=(python3 "$R/bench.py" --config 1 --steps 5 --warmup 1 --no-cpu-baseline --frag-line 0) ;;
    5) kern="interval_kernel<4, 0>|chunk_kernel<4, 0>|pod_kernel<4, 0>"
       cmd=(python3 "$R/bench.py" --config 5 --steps 3 --warmup 1 --no-cpu-baseline --frag-line 0 --no-pipeline-line --no-host-line) ;;
    s8) kern="interval_sums_kernel<4, 0>"  # rank 0's 1/8 shard, partial sums in the launch
       cmd=(python3 "$R/bench.py" --shard-of 8 --steps 20 --warmup 3 --no-cpu-baseline --frag-line 0 --no-pipeline-line --no-host-line) ;;
    *) echo "no PMC recipe for config $c"; exit 2 ;;
  esac
  step fetch_c$c 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch_c$c" -o run -- "${cmd[@]}"
  step write_c$c 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write_c$c" -o run -- "${cmd[@]}"
  cfg=$c; shard=1; sums=0; [ "$c" = s8 ] && { cfg=3; shard=8; sums=1; }
  (cd "$R" && PMC_SHARD_OF=$shard PMC_SUMS=$sums python3 tools/pmc_summary.py "$O/fetch_c$c" "$O/write_c$c" \
     "profiles/${PMC_ROUND:-r04}/${OUT:-pmc} (tools/gpu_pmc_traffic.sh)" "$O/pmc_traffic.json" "$cfg" "$kern") || exit $?
done
