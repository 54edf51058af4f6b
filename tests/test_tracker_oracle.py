"""TerminatedResourceTracker oracle (Go heap) against the reference's own tests — CPU."""

import numpy as np
import pytest

from tracker_runner import load_tracker_kats, run_oracle_case

KATS = load_tracker_kats()


@pytest.mark.parametrize("case", KATS["cases"], ids=[c["name"] for c in KATS["cases"]])
def test_tracker_oracle_kat(case):
    run_oracle_case(case, KATS["zones"])


def test_batch_order_is_a_go_order():
    """add_batch == add_one in descending-energy order (one of Go's map orders); one tracker
    per node."""
    from oracle.oracle import OracleTracker

    rng = np.random.default_rng(5)
    n, Z = 300, 2
    tab_e = rng.integers(0, 10**9, size=n * Z).astype(np.uint64)
    tab_p = rng.random(n * Z)
    slot = rng.permutation(n).astype(np.uint32)
    node = rng.integers(0, 4, size=n).astype(np.uint32)
    key = np.arange(n, dtype=np.uint64) + 7
    a, b = OracleTracker(50, 10**6, Z), OracleTracker(50, 10**6, Z)
    a.add_batch(node, key, slot, tab_e, tab_p)
    order = sorted(range(n), key=lambda i: (-int(tab_e[slot[i] * Z]), int(node[i]), int(slot[i])))
    for i in order:
        b.add_one(int(node[i]), int(key[i]), tab_e[slot[i] * Z: slot[i] * Z + Z], tab_p[slot[i] * Z: slot[i] * Z + Z])
    for x, y in zip(a.items(), b.items()):
        np.testing.assert_array_equal(x, y)
    k, nd, e, _ = a.items()
    # one tracker per node (monitor.go:123-144): each node keeps its own top 50 (distinct values)
    for n in range(4):
        elig = sorted((int(tab_e[slot[i] * Z]) for i in range(len(slot))
                       if node[i] == n and int(tab_e[slot[i] * Z]) >= 10**6), reverse=True)[:50]
        got = sorted(int(x) for x in e[nd == n, 0])
        assert got == sorted(elig), n
    assert k.size == sum(min(50, int(((node == n) & (tab_e[slot * Z] >= 10**6)).sum())) for n in range(4)) > 50
