#!/bin/bash
# Round 4: the nranks > 1 cluster path with 2, 4 and 8 processes on the one GPU (loopback
# collectives): gather-v offsets and per-rank broadcasts at the driver's 8-GPU rank count.
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r04w}
mkdir -p gpurun_out/$O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_cluster_ranks.py > gpurun_out/$O/pytest.log 2>&1 || { echo "tests failed rc=$?"; tail -80 gpurun_out/$O/pytest.log; exit 1; }
tail -8 gpurun_out/$O/pytest.log
