set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab1
OLD="KACC_LIB=$GRAFT_REPO_ROOT/kepler_amd/lib/alt/libkepler_accel.so"
B="python bench.py --no-cpu-baseline --frag-line 0 --no-pipeline-line"
tools/gpu_steps.sh ab1/pytest 400 "python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_small.py tests/test_gpu_join.py tests/test_gpu_tracker.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider" \
  ab1/c3_new1 200 "$B --json-out gpurun_out/ab1/c3_new1.json" \
  ab1/c3_old1 200 "$OLD $B --json-out gpurun_out/ab1/c3_old1.json" \
  ab1/c3_new2 200 "$B --json-out gpurun_out/ab1/c3_new2.json" \
  ab1/c3_old2 200 "$OLD $B --json-out gpurun_out/ab1/c3_old2.json" \
  ab1/c1_new 200 "$B --config 1 --json-out gpurun_out/ab1/c1_new.json" \
  ab1/c1_old 200 "$OLD $B --config 1 --json-out gpurun_out/ab1/c1_old.json" \
  ab1/c1_new2 200 "$B --config 1 --json-out gpurun_out/ab1/c1_new2.json" \
  ab1/c1_old2 200 "$OLD $B --config 1 --json-out gpurun_out/ab1/c1_old2.json" \
  ab1/join_new 200 "python tools/bench_join_variants.py > gpurun_out/ab1/join_new.json" \
  ab1/join_old 200 "$OLD python tools/bench_join_variants.py > gpurun_out/ab1/join_old.json"
