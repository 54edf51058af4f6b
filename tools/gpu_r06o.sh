cd $GRAFT_REPO_ROOT
O=gpurun_out/r06o
mkdir -p $O
timeout -k 10 60 python -c "
from kepler_amd import accel; import ctypes
lib = accel.load(); lib.kacc_debug_join_occupancy.argtypes = [ctypes.c_int]
print({v: lib.kacc_debug_join_occupancy(v) for v in (-1, 352767, 221695, 25087)})" || exit $?
timeout -k 10 300 env VARIANTS=-1,352767,221695 ROUNDS=5 python -u tools/bench_join_variants.py > $O/variants.json 2>$O/variants.err || exit $?
python -c "import json;d=json.load(open('$O/variants.json'));print(d['join_ms'], d['identical_to_first'])"
timeout -k 10 400 python -u -m pytest tests/test_gpu_join.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_join.log 2>&1; rc=$?; tail -3 $O/pytest_join.log; [ $rc -ge 2 ] && exit $rc
exit 0
