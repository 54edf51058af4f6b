cd $GRAFT_REPO_ROOT
O=gpurun_out/r06m
mkdir -p $O
timeout -k 10 300 env VARIANTS=511,-1,90623 ROUNDS=5 python -u tools/bench_join_variants.py > $O/variants.json 2>$O/variants.err || exit $?
python -c "import json;d=json.load(open('$O/variants.json'));print(d['join_ms'], d['identical_to_first'])"
timeout -k 10 300 python -u -m pytest tests/test_gpu_join.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_join.log 2>&1; rc=$?; tail -2 $O/pytest_join.log; [ $rc -ge 2 ] && exit $rc
OUT=r06m/pmc VARIANTS=-1,90623 bash tools/join_pmc.sh > /dev/null || exit $?
python tools/join_pmc_summary.py gpurun_out/r06m/pmc 2>/dev/null | head -5 || true
