cd $GRAFT_REPO_ROOT
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_join.py tests/test_gpu_tracker.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_join.log 2>&1; rc=$?; tail -3 $O/pytest_join.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 env VARIANTS=511,-1 ROUNDS=5 python -u tools/bench_join_variants.py > $O/variants.json 2>$O/variants.err || exit $?
cat $O/variants.json
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --frag-line 0 --no-host-line --json-out $O/bench.json > $O/bench.log 2>&1 || exit $?
python -c "import json;d=json.load(open('$O/bench.json'));print(json.dumps(d.get('pipeline')))"
