cd $GRAFT_REPO_ROOT
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_join.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_join.log 2>&1 || exit $?
timeout -k 10 300 env VARIANTS=511,-1,57855 ROUNDS=5 python -u tools/bench_join_variants.py > $O/variants.json 2>$O/variants.err || exit $?
cat $O/variants.json
OUT=r06h/pmc VARIANTS=511,-1,57855 bash tools/join_pmc.sh > /dev/null
timeout -k 10 400 python -u tools/bench_join.py > $O/join.json 2>$O/join.err || exit $?
python -c "import json;d=json.load(open('$O/join.json'));print(d['join_ms'], d['phase_ms'])"
