cd $GRAFT_REPO_ROOT
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_join.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_join.log 2>&1; rc=$?; tail -3 $O/pytest_join.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 env VARIANTS=511,2495,-1 ROUNDS=5 python -u tools/bench_join_variants.py > $O/variants.json 2>$O/variants.err || exit $?
cat $O/variants.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_format.py tests/test_gpu_config2_full.py tests/test_gpu_tracker.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_more.log 2>&1; rc=$?; tail -3 $O/pytest_more.log; [ $rc -ge 2 ] && exit $rc
OUT=r06c/pmc VARIANTS=511,2495,-1 bash tools/join_pmc.sh
