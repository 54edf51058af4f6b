cd $GRAFT_REPO_ROOT
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 400 env STOPS=1,2,3,4,5,6,7,8,0 python -u tools/bench_join.py > $O/join.json 2>$O/join.err || exit $?
python -c "import json;d=json.load(open('$O/join.json'));print(d['join_ms'], d['phase_ms'])"
