cd $GRAFT_REPO_ROOT
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_join.py tests/test_gpu_format.py tests/test_gpu_config2_full.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_join.log 2>&1; rc=$?; tail -3 $O/pytest_join.log; [ $rc -ge 2 ] && exit $rc
rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
OUT=r06b/pmc VARIANTS=511,-1 bash tools/join_pmc.sh
