"""The C++ oracle (kepler_oracle.cpp) against an independent pure-Python
restatement written in Go's shape (oracle/pyref.py) — CPU.

Every state table bit for bit, over multi-interval fleets with churn (new
slots), counter wraparound (fake-meter MaxEnergy 1e6), zero usage ratios,
read errors, empty and single-process nodes, VMs and pods; the C++ oracle in
listing-order summation mode (the Go map order replaced by /proc order).
"""

import numpy as np
import pytest

from kepler_amd import accel, fleet
from oracle.pyref import PyRef, duration_seconds, go_float64_to_uint64


def test_go_conversions():
    assert go_float64_to_uint64(1.9) == 1
    assert go_float64_to_uint64(-0.5) == 0
    assert go_float64_to_uint64(-1.5) == (1 << 64) - 1       # int64(-1) as uint64
    assert go_float64_to_uint64(float("nan")) == 1 << 63     # CVTTSD2SQ indefinite
    assert go_float64_to_uint64(2.0 ** 63) == 1 << 63
    assert go_float64_to_uint64(2.0 ** 64) == 1 << 63        # out of range -> indefinite | 1<<63
    assert duration_seconds(5_000_000_001) == 5.000000001
    assert duration_seconds(-1_500_000_000) == -1.5


FLEETS = [
    ("z2-small", dict(n_nodes=6, procs_per_node=[40, 0, 1, 300, 7, 64], zones=2, vm_frac=0.05, procs_per_vm=2)),
    ("z4-churn", dict(n_nodes=5, procs_per_node=[200, 150, 90, 3, 500], zones=4, shuffle_slots=True)),
    ("z3-odd", dict(n_nodes=4, procs_per_node=[33, 257, 1, 80], zones=3, vm_frac=0.1, procs_per_vm=3)),
]


@pytest.mark.parametrize("max_energy", [fleet.MAX_ENERGY_RAPL, fleet.MAX_ENERGY_FAKE], ids=["rapl", "wrap"])
@pytest.mark.parametrize("name,kw", FLEETS, ids=[f[0] for f in FLEETS])
def test_cpp_oracle_matches_python_restatement(name, kw, max_energy, oracle_lib):
    from oracle.oracle import KOR_SUM_LISTING, Oracle

    layout = fleet.make_layout(seed=5, **kw)
    caps = layout.capacities()
    sim = fleet.FleetSim(layout, seed=5, churn=0.1, read_error_frac=0.15, zero_ratio_frac=0.1,
                         max_energy=max_energy)
    ora = Oracle(layout.zones, **caps, sum_mode=KOR_SUM_LISTING)
    ref = PyRef(layout.zones)
    rng = np.random.default_rng(11)
    for k in range(5):
        a = sim.next_interval()
        if k:  # containers / VMs / pods recreated in their slots (no previous entry)
            for key in ("ctr_slot", "vm_slot", "pod_slot"):
                a[key] = a[key] | np.where(rng.random(a[key].size) < 0.2, np.uint32(accel.KACC_SLOT_NEW),
                                           np.uint32(0)).astype(np.uint32)
        ora.interval(a, layout.sizes())
        ref.interval(a)
        got = ref.tables(layout.n_nodes, caps)
        for tname in (t for t, _ in accel.TABLES if t not in accel.ENGINE_TABLES):
            np.testing.assert_array_equal(ora.state[tname], got[tname], err_msg=f"interval {k} {tname}")


def test_threaded_oracle_matches_serial(oracle_lib):
    """kor_interval_mt (the multi-core CPU baseline) == kor_interval, every table."""
    from oracle.oracle import Oracle

    layout = fleet.make_layout(37, [300, 2000, 1, 0, 700, 64, 5000] * 5 + [9, 9], 4, seed=8, shuffle_slots=True)
    caps = layout.capacities()
    sim = fleet.FleetSim(layout, seed=8, churn=0.05, read_error_frac=0.1)
    a_ser, a_mt = Oracle(layout.zones, **caps), Oracle(layout.zones, **caps)
    for _ in range(3):
        a = sim.next_interval()
        a_ser.interval(a, layout.sizes())
        a_mt.interval_mt(a, layout.sizes(), threads=5)
    for tname in (t for t, _ in accel.TABLES if t not in accel.ENGINE_TABLES):
        np.testing.assert_array_equal(a_mt.state[tname], a_ser.state[tname], err_msg=tname)


def bits(a: np.ndarray) -> np.ndarray:
    return a.view(np.uint64) if a.dtype == np.float64 else a


@pytest.mark.parametrize("name,kw", FLEETS + [("z4-big", dict(n_nodes=4, procs_per_node=[2500, 40, 700, 9],
                                                              zones=4))], ids=[f[0] for f in FLEETS] + ["z4-big"])
def test_adversarial_inputs_oracle_matches_python_restatement(name, kw, oracle_lib):
    """Reachable edge inputs (fleet.FleetSim.ADVERSARIAL: Δt = 0 and backward clock -> ±Inf / NaN
    power, unchanged counters, usage ratio 1 / > 1 / < 0 -> u64 idle wrap, negative CPU deltas
    -> Energy() of negatives and u64 total wrap, huge cancelling deltas -> Energy() out of
    range): the C++ oracle and the Python restatement agree bit for bit, NaN bits included
    (both evaluate on x86 SSE2, as Go on amd64 does)."""
    from oracle.oracle import KOR_SUM_LISTING, Oracle

    layout = fleet.make_layout(seed=7, **kw)
    caps = layout.capacities()
    sim = fleet.FleetSim(layout, seed=7, churn=0.05, read_error_frac=0.1, adversarial=0.6)
    ora = Oracle(layout.zones, **caps, sum_mode=KOR_SUM_LISTING)
    ref = PyRef(layout.zones)
    for k in range(6):
        a = sim.next_interval()
        ora.interval(a, layout.sizes())
        ref.interval(a)
        got = ref.tables(layout.n_nodes, caps)
        for tname in (t for t, _ in accel.TABLES if t not in accel.ENGINE_TABLES):
            np.testing.assert_array_equal(bits(ora.state[tname]), bits(got[tname]), err_msg=f"interval {k} {tname}")


def test_adversarial_scenarios_reach_their_edges(oracle_lib):
    """The adversarial mode really produces the edge values it is for."""
    from oracle.oracle import Oracle

    layout = fleet.make_layout(40, [300, 64, 1000, 5] * 10, 4, seed=3)
    caps = layout.capacities()
    sim = fleet.FleetSim(layout, seed=3, adversarial=0.9)
    ora = Oracle(layout.zones, **caps)
    seen = dict(inf=False, nan=False, neg_power=False, idle_wrap=False, out_of_range=False, neg_delta=False)
    prev_idle = None
    for k in range(8):
        a = sim.next_interval()
        seen["neg_delta"] |= bool((a["proc_cpu_delta"] < 0).any())
        ora.interval(a, layout.sizes())
        st = ora.state
        npow = np.concatenate([st["node_power"], st["proc_power"]])
        seen["inf"] |= bool(np.isinf(npow).any())
        seen["nan"] |= bool(np.isnan(np.concatenate([st["node_idle_power"], st["proc_power"]])).any())
        seen["neg_power"] |= bool((st["node_active_power"] < 0).any())
        seen["out_of_range"] |= bool((st["proc_energy"] == np.uint64(1 << 63)).any())
        idle = st["node_idle_total"].copy()
        if prev_idle is not None:
            seen["idle_wrap"] |= bool((idle < prev_idle).any())  # u64 modular add wrapped
        prev_idle = idle
    assert all(seen.values()), seen


@pytest.mark.parametrize("seed", [1, 2])
def test_any_go_map_order_within_documented_bound(seed, oracle_lib):
    """The engine fixes one order for the two sums Go takes over maps (the node's
    ProcessTotalCPUTimeDelta, informer.go:330-333; a pod's containers, :284-310).  Against
    the Python restatement summing both in random orders (one of Go's map orders per node
    and pod per interval), over 6 intervals with churn and pods of several containers:
    CPU-time deltas / totals within 1e-12 relative, energies within 1 µJ per interval per
    workload, powers within 1e-12 relative."""
    from oracle.oracle import Oracle

    layout = fleet.make_layout(8, [300, 1200, 64, 2000, 7, 900, 450, 1], 4, seed=seed, ctrs_per_pod=4.0)
    caps = layout.capacities()
    sim = fleet.FleetSim(layout, seed=seed, churn=0.05)
    ora = Oracle(layout.zones, **caps)
    ref = PyRef(layout.zones, map_order_rng=np.random.default_rng(100 + seed))
    K = 6
    for _ in range(K):
        a = sim.next_interval()
        ora.interval(a, layout.sizes())
        ref.interval(a)
    got = ref.tables(layout.n_nodes, caps)
    for tname in (t for t, _ in accel.TABLES if t not in accel.ENGINE_TABLES):
        want, have = ora.state[tname], got[tname]
        if want.dtype == np.float64:
            np.testing.assert_allclose(have, want, rtol=1e-12, atol=0, err_msg=tname)
        elif tname.endswith(("energy", "_total")) and want.dtype == np.uint64:
            diff = np.abs(have.astype(np.int64) - want.astype(np.int64))
            assert diff.max() <= K, (tname, int(diff.max()))
        else:
            np.testing.assert_array_equal(have, want, err_msg=tname)
    # the random orders did change some low bits (the test exercises the bound)
    assert any(not np.array_equal(got[t].view(np.uint64), ora.state[t].view(np.uint64))
               for t in ("node_cpu_delta", "pod_cpu_delta", "pod_cpu_total", "proc_energy", "pod_energy"))
