#!/bin/bash
# Round-2 (session 3) check: every GPU test, smoke(), the default bench (config 3,
# CPU baseline, slot layouts, pipeline line) and the other configs.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/${OUT:-r2s3}
S=tools/gpu_steps.sh
$S ${OUT:-r2s3}/pytest_gpu 700 "python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider" \
   ${OUT:-r2s3}/smoke 200 "python -c 'import __graft_entry__ as g; g.smoke()'" \
   ${OUT:-r2s3}/bench_c3 600 "python bench.py --json-out gpurun_out/${OUT:-r2s3}/bench_c3.json" \
   ${OUT:-r2s3}/bench_c2_k60 300 "python bench.py --config 2 --intervals 60 --no-cpu-baseline --json-out gpurun_out/${OUT:-r2s3}/bench_c2_k60.json" \
   ${OUT:-r2s3}/bench_c5_k60 400 "python bench.py --config 5 --intervals 60 --steps 10 --no-cpu-baseline --json-out gpurun_out/${OUT:-r2s3}/bench_c5_k60.json" \
   ${OUT:-r2s3}/bench_c1 400 "python bench.py --config 1 --no-cpu-baseline --json-out gpurun_out/${OUT:-r2s3}/bench_c1.json" \
   ${OUT:-r2s3}/bench_c4 600 "python bench.py --config 4 --steps 5 --no-cpu-baseline --frag-line 0 --json-out gpurun_out/${OUT:-r2s3}/bench_c4.json" \
   ${OUT:-r2s3}/bench_join 300 "python tools/bench_join.py > gpurun_out/${OUT:-r2s3}/bench_join.json" \
   ${OUT:-r2s3}/bench_format 300 "python tools/bench_format.py > gpurun_out/${OUT:-r2s3}/bench_format.json"
