#!/bin/bash
# Round 4: the span sweep with slot-order staging (KACC_SLOT_STAGE, production) — the
# whole -m gpu suite, interleaved variant A/B on pristine slots with spans and on 2 %
# fragmented slots (0 = staged, 262144 = through s_inv, 2048 = no sweep), and the
# default bench line (slot layouts, production layout).
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-r04o}
mkdir -p gpurun_out/$O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > gpurun_out/$O/pytest.log 2>&1 || { echo "tests failed rc=$?"; tail -60 gpurun_out/$O/pytest.log; exit 1; }
tail -1 gpurun_out/$O/pytest.log
tools/gpu_steps.sh \
  $O/var_span 300 "SPAN=1 VARIANTS=0,262144,2048 ROUNDS=12 python tools/bench_variants.py > gpurun_out/$O/var_span.json" \
  $O/var_frag 300 "FRAG=0.02 VARIANTS=0,262144 ROUNDS=12 python tools/bench_variants.py > gpurun_out/$O/var_frag.json" \
  $O/bench 600 "python bench.py --no-cpu-baseline --json-out gpurun_out/$O/bench_c3.json" || exit $?
python - <<'PY'
import json
O="gpurun_out/r04o"
for f in ("var_span", "var_frag"):
    d = json.load(open(f"{O}/{f}.json"))
    print(f, {k: round(v["median_ms"] * 1e3, 1) for k, v in d["variants"].items()})
d = json.load(open(f"{O}/bench_c3.json"))
print("bench", round(d["kernel_ms"] * 1e3, 1), d["production_layout"]["over_pristine"],
      {k: (round(v["kernel_ms"] * 1e3, 1) if isinstance(v, dict) and "kernel_ms" in v else v) for k, v in d["slot_layouts"].items() if k != "note"})
PY
