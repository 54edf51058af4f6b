cd $GRAFT_REPO_ROOT
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 300 env VARIANTS=-1,221695,25087 ROUNDS=5 python -u tools/bench_join_variants.py > $O/variants.json 2>$O/variants.err || exit $?
python -c "import json;d=json.load(open('$O/variants.json'));print(d['join_ms'], d['identical_to_first'])"
