"""Table layout and the launch-timing hook of the C ABI — MI355X only.

The pod tables are stored as one [energy Z | power Z] record per slot
(kacc_table_row_stride 2Z; KACC_T_POD_POWER's device pointer is Z elements
after KACC_T_POD_ENERGY's); downloads, uploads and the device pointer must
still present the logical [slot*Z + z] tables.  kacc_time_next_launch puts a
start / stop event pair on the next launching call's dispatch packets.
"""

import ctypes

import numpy as np
import pytest
import torch

from kepler_amd import accel, fleet
from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu_ready():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    accel.load()
    torch.cuda.set_stream(torch.cuda.Stream())


@pytest.mark.parametrize("zones", [1, 2, 3, 4])
def test_pod_records_present_logical_tables(zones):
    layout = fleet.make_layout(6, [300, 40, 0, 900, 7, 1], zones, seed=7, shuffle_slots=True)
    sim = fleet.FleetSim(layout, seed=7, churn=0.05)
    caps = layout.capacities()
    acc = accel.Accel(zones, **caps)
    ora = Oracle(zones, **caps)
    s = current_stream_handle()
    for _ in range(3):
        a = sim.next_interval()
        acc.run_interval(interval_from_tensors(to_device(a), layout.sizes()), s)
        acc.sync(s)
        ora.interval(a, layout.sizes())
    assert acc.row_stride("pod_energy") == 2 * zones and acc.row_stride("pod_power") == 2 * zones
    assert acc.row_stride("ctr_energy") == zones and acc.row_stride("pod_cpu_delta") == 1
    assert acc.device_ptr("pod_power") - acc.device_ptr("pod_energy") == 8 * zones
    e, p = acc.download("pod_energy"), acc.download("pod_power")
    assert np.array_equal(e, ora.state["pod_energy"])
    assert np.array_equal(p, ora.state["pod_power"], equal_nan=True)
    # the device records themselves: slot s = energy row then power row
    n = caps["pod_slots"]
    raw = np.empty(2 * n * zones, dtype=np.uint64)
    torch.cuda.synchronize()
    lib = accel.load()  # dlsym through the library's handle finds its HIP runtime's hipMemcpy
    assert lib.hipMemcpy(ctypes.c_void_p(raw.ctypes.data), ctypes.c_void_p(acc.device_ptr("pod_energy")),
                         ctypes.c_size_t(raw.nbytes), 2) == 0  # hipMemcpyDeviceToHost
    rec = raw.reshape(n, 2, zones)
    assert np.array_equal(rec[:, 0, :].reshape(-1), e)
    assert np.array_equal(rec[:, 1, :].reshape(-1).view(np.float64), p, equal_nan=True)
    # partial-row uploads touch only their elements, in both halves of the records
    rng = np.random.default_rng(1)
    first, cnt = zones + 1 if zones > 1 else 1, 3 * zones + 1
    newp = rng.random(cnt)
    acc.upload("pod_power", newp, first)
    p2 = p.copy()
    p2[first:first + cnt] = newp
    assert np.array_equal(acc.download("pod_power"), p2, equal_nan=True)
    assert np.array_equal(acc.download("pod_energy"), e)
    newe = rng.integers(0, 2**63, cnt, dtype=np.uint64)
    acc.upload("pod_energy", newe, first)
    e2 = e.copy()
    e2[first:first + cnt] = newe
    assert np.array_equal(acc.download("pod_energy"), e2)
    assert np.array_equal(acc.download("pod_power"), p2, equal_nan=True)
    acc.close()


def test_time_next_launch_rides_on_the_dispatch():
    layout = fleet.make_layout(64, 2000, 4, seed=3)
    sim = fleet.FleetSim(layout, seed=3)
    caps = layout.capacities()
    acc = accel.Accel(4, **caps)
    s = current_stream_handle()
    ivs = [interval_from_tensors(to_device(sim.next_interval()), layout.sizes(), layout.fast_flag())
           for _ in range(3)]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for e in ev:  # torch creates the event on its first record
        e.record()
    acc.run_interval(ivs[0], s)
    acc.time_next_launch(ev[0].cuda_event, ev[1].cuda_event)
    acc.run_interval(ivs[1], s)
    acc.run_interval(ivs[2], s)  # the hook was consumed by the previous call
    acc.sync(s)
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1])
    assert 0.0 < ms < 100.0, ms
    acc.close()


@pytest.mark.parametrize("name,kw,shape", [
    # interval_kernel fast path: transposed 64-row groups and the per-row fallback
    ("z4-fast", dict(n_nodes=24, procs_per_node=[2000, 1500, 1, 0, 700, 64] * 4, zones=4), "fast"),
    ("z4-fast-shuffled", dict(n_nodes=12, procs_per_node=[2000, 900, 3, 64] * 3, zones=4, shuffle_slots=True), "fast"),
    # slot sweep (node_proc_span) over fragmented node ranges
    ("z4-sweep", dict(n_nodes=12, procs_per_node=[1900, 800, 1, 64] * 3, zones=4, fragment_slots=0.04), "fast"),
    ("z3-rowsweep", dict(n_nodes=12, procs_per_node=[1900, 800, 1, 64] * 3, zones=3, fragment_slots=0.04), "fast"),
    # small_kernel (one wavefront per node)
    ("z2-small", dict(n_nodes=36, procs_per_node=[500, 120, 1, 0, 512, 77] * 6, zones=2), "small"),
    ("z4-small-sweep", dict(n_nodes=36, procs_per_node=[480, 120, 1, 0, 500, 77] * 6, zones=4, fragment_slots=0.02),
     "small"),
    # big nodes: chunk_kernel
    ("z4-big", dict(n_nodes=6, procs_per_node=[9000, 300, 2049, 0, 5000, 12], zones=4), "generic"),
    # K intervals in one launch (intervals_carry_kernel)
    ("z2-carry", dict(n_nodes=24, procs_per_node=[1000, 700, 1, 0, 2048, 513] * 4, zones=2), "carry"),
    ("z2-carry-sweep", dict(n_nodes=12, procs_per_node=[1000, 700, 64, 3] * 3, zones=2, fragment_slots=0.05), "carry"),
])
@pytest.mark.parametrize("stable", [True, False])
def test_stable_slot_nodes_bit_exact(name, kw, shape, stable):
    """KACC_F_STABLE_SLOT_NODES: KACC_T_PROC_NODE is written only for NEW rows and on a node's
    first read; every table (the node ids and the powers derived through them included) stays
    bit-exact with the oracle, with churn (NEW rows), read errors (incl. skipped first reads)
    and adversarial inputs, in every kernel shape that stores process rows."""
    layout = fleet.make_layout(seed=31, **kw)
    sizes = layout.sizes()
    flags = layout.fast_flag() | accel.KACC_F_NODE_SLOT_RANGES | (accel.KACC_F_STABLE_SLOT_NODES if stable else 0)
    if shape == "fast" or shape == "carry":
        flags &= ~accel.KACC_F_SMALL_NODES
    if shape == "small":
        assert flags & accel.KACC_F_SMALL_NODES
    if shape == "generic":
        assert not flags & accel.KACC_F_FAST_NODES
    sim = fleet.FleetSim(layout, seed=31, churn=0.04, read_error_frac=0.1, max_energy=fleet.MAX_ENERGY_FAKE,
                         adversarial=0.1)
    acc = accel.Accel(layout.zones, **layout.capacities())
    ora = Oracle(layout.zones, **layout.capacities())
    s = current_stream_handle()
    K = 9
    ivs = [sim.next_interval() for _ in range(K)]
    if kw.get("fragment_slots"):
        for a in ivs:
            a["node_proc_span"] = layout.proc_span()
    dev = [to_device(a) for a in ivs]
    descs = [interval_from_tensors(t, sizes, flags) for t in dev]
    if shape == "carry":
        acc.run_intervals(descs[:2], s)
        acc.run_intervals(descs[2:], s)
    else:
        for d in descs:
            acc.run_interval(d, s)
    acc.sync(s)
    for a in ivs:
        ora.interval(a, sizes)
    bad = []
    # a derived power is defined for the slots rows use (table_check.LiveSlots): a free slot of a
    # fragmented range derives 0 x its node's ActivePower (NaN when that is +-Inf)
    used = np.zeros(layout.capacities()["proc_slots"], dtype=bool)
    used[layout.proc_slot] = True
    for tname, _ in accel.TABLES:
        got, want = acc.download(tname), ora.state[tname]
        if tname == "proc_power":
            m = np.repeat(used, layout.zones)
            got, want = got[m], want[m]
        if not np.array_equal(got, want, equal_nan=want.dtype.kind == "f"):
            neq = got != want
            if want.dtype.kind == "f":
                neq &= ~(np.isnan(got) & np.isnan(want))
            i = np.flatnonzero(neq)
            bad.append(f"{tname}: {i.size} differ, first {i[:4].tolist()} got {got[i[:4]].tolist()} "
                       f"want {want[i[:4]].tolist()}")
    assert not bad, f"{name} stable={stable}: " + "; ".join(bad)
    acc.close()
