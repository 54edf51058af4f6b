cd $GRAFT_REPO_ROOT
O=gpurun_out/r06l
mkdir -p $O
timeout -k 10 400 env STOPS=1,2,3,4,5,6,7,8,0 python -u tools/bench_join.py > $O/join.json 2>$O/join.err || exit $?
python -c "import json;d=json.load(open('$O/join.json'));print(d['join_ms'], d['phase_ms'])"
timeout -k 10 300 python -u -m pytest tests/test_gpu_join.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_join.log 2>&1; rc=$?; tail -2 $O/pytest_join.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 env VARIANTS=511,-1,90623,221695 ROUNDS=5 python -u tools/bench_join_variants.py > $O/variants.json 2>$O/variants.err || exit $?
python -c "import json;d=json.load(open('$O/variants.json'));print(d['join_ms'], d['identical_to_first'])"
