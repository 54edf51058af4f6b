cd $GRAFT_REPO_ROOT
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 env VARIANTS=511,-1 ROUNDS=5 python -u tools/bench_join_variants.py > $O/variants.json 2>$O/variants.err || exit $?
cat $O/variants.json
timeout -k 10 600 python -u bench.py --json-out $O/bench.json > $O/bench.log 2>&1 || exit $?
python -c "import json;d=json.load(open('$O/bench.json'));print(json.dumps({k:d.get(k) for k in ('value','value_with_scrape','ms_per_step','kernel_ms','pipeline','roofline')}))"
OUT=r06g/pmc VARIANTS=511,-1 bash tools/join_pmc.sh > /dev/null
