#!/bin/bash
# Per-wave SQ counters (two passes, tools/pmc_kernel.sh) of the config-1 fleet's small_kernel<2>
# and config 5's chunk_kernel<4,0> / interval_kernel<4,0>, summarised per kernel.
#   OUT=<dir> tools/gpu_sq_profiles.sh
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-sq}
mkdir -p gpurun_out/$O
B="--no-cpu-baseline --frag-line 0 --no-pipeline-line --no-host-line"
bash tools/pmc_kernel.sh ${O}_c1 -- python3 "$GRAFT_REPO_ROOT/bench.py" --config 1 --steps 5 --warmup 1 $B || exit $?
python tools/sq_kernel_summary.py gpurun_out/pmc_${O}_c1 "small_kernel<2, false>" > gpurun_out/$O/sq_c1_small.json || exit $?
bash tools/pmc_kernel.sh ${O}_c5 -- python3 "$GRAFT_REPO_ROOT/bench.py" --config 5 --intervals 60 --steps 2 --warmup 1 $B || exit $?
python tools/sq_kernel_summary.py gpurun_out/pmc_${O}_c5 "chunk_kernel<4, 0>" > gpurun_out/$O/sq_c5_chunk.json || exit $?
python tools/sq_kernel_summary.py gpurun_out/pmc_${O}_c5 "interval_kernel<4, 0>" > gpurun_out/$O/sq_c5_interval.json || exit $?
for f in gpurun_out/$O/sq_*.json; do echo $f; python -c "import json;d=json.load(open('$f'));print(json.dumps({k: round(v, 1) for k, v in d['per_wave'].items()}), round(d['wait_any_over_wave_cycles'], 3), round(d['active_inst_over_wave_cycles'], 3))"; done
