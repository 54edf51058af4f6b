"""Parity of the HIP engine (through the C ABI) with the oracle — MI355X only.

Integer tables (energies, counters, statuses) must be bit-exact.  Float64
tables are bit-exact too against the oracle in the engine's canonical
summation order; against the listing-order sum (one of Go's map orders) the
tolerance is the north star's: <= 1e-12 relative on totals and <= 1 µJ per
workload.
"""

import numpy as np
import pytest
import torch

from kat_runner import load_golden_fleet, load_kats, run_case
from kepler_amd import accel, fleet
from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device

pytestmark = pytest.mark.gpu

KATS = load_kats()


@pytest.fixture(scope="module", autouse=True)
def gpu_ready():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    accel.load()  # raises if the HIP library is missing: no fallback
    torch.cuda.set_stream(torch.cuda.Stream())  # engine + copies on one explicit stream


class EngineBackend:
    """Device-pointer path: kacc_run_interval on torch's current stream."""

    def __init__(self, zones, caps):
        self.acc = accel.Accel(zones, **caps)

    def upload(self, table, first, values):
        self.acc.upload(table, np.array(values), first)

    def interval(self, arrays, sizes, flags):
        t = to_device(arrays)
        it = interval_from_tensors(t, sizes, flags)
        s = current_stream_handle()
        self.acc.run_interval(it, s)
        self.acc.sync(s)

    def table(self, name):
        return self.acc.download(name)


class HostBatchBackend(EngineBackend):
    """Pinned host path: kacc_batch_alloc / submit / wait (the cgo path)."""

    def interval(self, arrays, sizes, flags):
        b = accel.HostBatch.alloc(self.acc, **sizes)
        try:
            b.fill(arrays, flags)
            b.submit()
            b.wait()
        finally:
            b.free()


@pytest.mark.parametrize("case", KATS["cases"], ids=[c["name"] for c in KATS["cases"]])
def test_engine_kat(case):
    run_case(case, EngineBackend)


@pytest.mark.parametrize("case", KATS["cases"], ids=[c["name"] for c in KATS["cases"]])
def test_engine_kat_host_batch(case):
    run_case(case, HostBatchBackend)


def test_golden_fleet_bit_exact():
    zones, caps, sizes, intervals = load_golden_fleet()
    be = EngineBackend(zones, caps)
    for k, (ins, outs) in enumerate(intervals):
        be.interval(ins, sizes, 0)
        for name, want in outs.items():
            np.testing.assert_array_equal(be.table(name), want, err_msg=f"interval {k} {name}")


def run_both(layout, sim_kwargs, n_intervals, node_order=False, seed=1, span=False):
    from oracle.oracle import KOR_SUM_LISTING, Oracle

    caps = layout.capacities()
    sim = fleet.FleetSim(layout, seed=seed, **sim_kwargs)
    eng = EngineBackend(layout.zones, caps)
    ora = Oracle(layout.zones, **caps)
    lst = Oracle(layout.zones, **caps, sum_mode=KOR_SUM_LISTING)
    for _ in range(n_intervals):
        a = sim.next_interval()
        if node_order:
            a["node_order"] = layout.node_order_heaviest_first()
        if span:  # the slot join's per-node spans: rows moved in slot order
            a["node_proc_span"] = layout.proc_span()
        eng.interval(a, layout.sizes(), layout.fast_flag())  # skip empty big-node launches when possible
        ora.interval(a, layout.sizes())
        lst.interval(a, layout.sizes())
        for name, _ in accel.TABLES:
            np.testing.assert_array_equal(eng.table(name), ora.state[name], err_msg=name)
    return eng, ora, lst


FLEETS = [
    ("z1-small", dict(n_nodes=5, procs_per_node=[1, 0, 40, 300, 7], zones=1)),
    ("z2-config2-like", dict(n_nodes=64, procs_per_node=1000, zones=2)),
    ("z3-odd", dict(n_nodes=33, procs_per_node=257, zones=3, procs_per_vm=3, vm_frac=0.05)),
    ("z4-config3-like", dict(n_nodes=48, procs_per_node=2000, zones=4, shuffle_slots=True)),
    ("z8-max-zones", dict(n_nodes=9, procs_per_node=511, zones=8)),
    ("z4-skew", dict(n_nodes=6, procs_per_node=[10000, 50000, 12000, 31000, 10, 0], zones=4,
                     procs_per_vm=2, vm_frac=0.02)),
    # fast/generic path boundaries: 2048 rows staged in LDS, <= 512 aggregates per node
    ("z4-rows-boundary", dict(n_nodes=6, procs_per_node=[2047, 2048, 2049, 4096, 1, 0], zones=4)),
    ("z2-many-aggregates", dict(n_nodes=5, procs_per_node=[600, 700, 800, 2000, 300], zones=2,
                                procs_per_ctr=1, ctrs_per_pod=1.0, vm_frac=0.05)),
    # fragmented per-node slot ranges (the slot join's steady state), swept in slot order
    ("z4-fragmented", dict(n_nodes=12, procs_per_node=[2000, 1999, 1500, 64, 1, 0, 2005, 700, 3, 2040, 100, 1024],
                           zones=4, fragment_slots=0.02)),
    ("z4-fragmented-wide", dict(n_nodes=6, procs_per_node=[1600, 1200, 500, 17, 2048, 1000], zones=4,
                                fragment_slots=0.3)),
    ("z8-fragmented", dict(n_nodes=5, procs_per_node=[511, 300, 64, 1, 200], zones=8, fragment_slots=0.5)),
]
SPAN_FLEETS = {"z4-fragmented", "z4-fragmented-wide", "z8-fragmented", "z4-config3-like", "z3-odd"}


def test_fast_flag_rejects_oversized_node():
    """KACC_F_FAST_NODES is a promise: an oversized node raises KACC_ERANGE, nothing faults."""
    layout = fleet.make_layout(3, [100, 2049, 5], 4, seed=5)
    assert layout.fast_flag() == 0
    eng = EngineBackend(layout.zones, layout.capacities())
    a = fleet.FleetSim(layout, seed=5).next_interval()
    with pytest.raises(accel.AccelError) as ei:
        eng.interval(a, layout.sizes(), accel.KACC_F_FAST_NODES)
    assert ei.value.code == accel.KACC_ERANGE
    # the same batch without the promise runs (and the context is usable again)
    eng.interval(a, layout.sizes(), 0)


def test_row_outside_span_is_reported():
    """A row whose slot lies outside its node's node_proc_span raises KACC_ERANGE."""
    layout = fleet.make_layout(2, [300, 200], 4, seed=3, fragment_slots=0.1)
    eng = EngineBackend(layout.zones, layout.capacities())
    a = fleet.FleetSim(layout, seed=3).next_interval()
    span = layout.proc_span()
    span[1] = span[0] + 10  # node 0's span too narrow
    a["node_proc_span"] = span
    with pytest.raises(accel.AccelError) as ei:
        eng.interval(a, layout.sizes(), layout.fast_flag())
    assert ei.value.code == accel.KACC_ERANGE


@pytest.mark.parametrize("name,kw", FLEETS, ids=[f[0] for f in FLEETS])
def test_random_fleet_bit_exact(name, kw):
    layout = fleet.make_layout(seed=11, **kw)
    eng, ora, lst = run_both(layout, dict(churn=0.03, zero_ratio_frac=0.05, read_error_frac=0.05), 4,
                             span=name in SPAN_FLEETS)
    # listing-order (Go map order) oracle: <= 1e-12 relative on the node totals,
    # <= 1 µJ per workload energy
    nd_e, nd_l = eng.table("node_cpu_delta"), lst.state["node_cpu_delta"]
    np.testing.assert_allclose(nd_e, nd_l, rtol=1e-12, atol=0)
    for kind in ("proc", "ctr", "vm", "pod"):
        de = eng.table(f"{kind}_energy").astype(np.int64) - lst.state[f"{kind}_energy"].astype(np.int64)
        assert np.abs(de).max(initial=0) <= 1, kind
        np.testing.assert_allclose(eng.table(f"{kind}_power"), lst.state[f"{kind}_power"], rtol=1e-12, atol=1e-6)


def _chunk_edge_nodes():
    """Big-node chunking edges (chunks of 2048 rows, <= 512 aggregates per lane
    pass): segments and pods straddling chunks, a container longer than a
    chunk, > 512 (empty) containers owned by one chunk, empty pods at the end,
    a node with no rows but > 512 aggregates, and a fast-path node beside them."""
    rng = np.random.default_rng(21)
    # 1: 7000 rows; containers of 7 straddle chunk boundaries; pods of 3-5 containers
    c1 = [7] * 700
    p1 = list(rng.integers(3, 6, size=150))
    # 2: one 4500-row container (3 chunks), 600 empty containers in chunk 2, pods over all
    c2 = [4500] + [0] * 600 + [10] * 20
    p2 = [1, 300, 200, 100, 5, 0, 0]
    # 3: no rows, 700 empty containers, 5 empty VMs, 200 pods (> 512 aggregates)
    c3 = [0] * 700
    # 4: VMs straddling chunks, pod-less containers after the pods
    c4 = [30] * 100
    return [
        dict(rows=7000, ctr=c1, vm=[40, 40, 40], pod=p1),
        dict(rows=4700, ctr=c2, vm=[], pod=p2),
        dict(rows=0, ctr=c3, vm=[0] * 5, pod=[3] * 200 + [0, 0]),
        dict(rows=9000, ctr=c4, vm=[700] * 5 + [1] * 100, pod=[2] * 20),
        dict(rows=900, ctr=[9] * 80, vm=[3], pod=[4] * 20),
    ]


@pytest.mark.parametrize("zones,shuffle", [(4, False), (3, True), (8, False)])
def test_big_node_chunk_edges(zones, shuffle):
    layout = fleet.layout_from_sizes(zones, _chunk_edge_nodes(), seed=5, shuffle_slots=shuffle)
    run_both(layout, dict(churn=0.05, zero_ratio_frac=0.1), 4, node_order=shuffle, seed=7)


def test_wrapping_fake_meter_and_node_order():
    layout = fleet.make_layout(40, [0, 1, 2, 3, 500, 2000, 64, 65] * 5, 2, seed=3, shuffle_slots=True)
    run_both(layout, dict(max_energy=fleet.MAX_ENERGY_FAKE, churn=0.1), 5, node_order=True, seed=5)


def test_node_cpu_delta_given():
    layout = fleet.make_layout(16, 300, 2, seed=9)
    from oracle.oracle import Oracle

    caps = layout.capacities()
    sim = fleet.FleetSim(layout, seed=9)
    eng = EngineBackend(layout.zones, caps)
    ora = Oracle(layout.zones, **caps)
    for k in range(3):
        a = sim.next_interval()
        a["node_cpu_delta"] = np.full(layout.n_nodes, 1234.5 + k)
        eng.interval(a, layout.sizes(), accel.KACC_F_NODE_CPU_DELTA_GIVEN)
        ora.interval(a, layout.sizes(), accel.KACC_F_NODE_CPU_DELTA_GIVEN)
        for name, _ in accel.TABLES:
            np.testing.assert_array_equal(eng.table(name), ora.state[name], err_msg=name)


def test_namespace_totals_match_oracle():
    layout = fleet.make_layout(32, 800, 4, seed=13, n_namespaces=7)
    eng, ora, _ = run_both(layout, dict(churn=0.0), 3)
    off, slots = layout.namespace_csr()
    e_o, p_o = ora.namespace_totals(off, slots)
    d_off, d_slots = to_device({"o": off, "s": slots})["o"], to_device({"s": slots})["s"]
    out_e = torch.zeros(len(e_o), dtype=torch.int64, device="cuda")
    out_p = torch.zeros(len(p_o), dtype=torch.float64, device="cuda")
    s = current_stream_handle()
    eng.acc.namespace_totals(len(off) - 1, d_off.data_ptr(), d_slots.data_ptr(), out_e.data_ptr(),
                             out_p.data_ptr(), s)
    eng.acc.sync(s)
    np.testing.assert_array_equal(out_e.cpu().numpy().view(np.uint64), e_o)
    np.testing.assert_array_equal(out_p.cpu().numpy(), p_o)
    # against a plain list-order sum: <= 1e-12 relative (north-star totals bar)
    pp = ora.state["pod_power"].reshape(-1, layout.zones)
    ref = np.array([[sum(pp[s_, z] for s_ in slots[off[k]:off[k + 1]]) for z in range(layout.zones)]
                    for k in range(len(off) - 1)]).reshape(-1)
    np.testing.assert_allclose(out_p.cpu().numpy(), ref, rtol=1e-12, atol=0)


def test_out_of_range_slot_is_reported_not_faulted():
    layout = fleet.make_layout(4, 100, 2, seed=17)
    caps = layout.capacities()
    sim = fleet.FleetSim(layout, seed=17)
    eng = EngineBackend(layout.zones, caps)
    a = sim.next_interval()
    a["proc_slot"] = a["proc_slot"].copy()
    a["proc_slot"][5] = (caps["proc_slots"] + 100) | accel.KACC_SLOT_NEW
    t = to_device(a)
    it = interval_from_tensors(t, layout.sizes())
    s = current_stream_handle()
    eng.acc.run_interval(it, s)
    with pytest.raises(accel.AccelError) as ei:
        eng.acc.sync(s)
    assert ei.value.code == accel.KACC_ERANGE
    # host validation rejects the same batch before it reaches the GPU
    assert eng.acc.validate_host(accel.make_interval(a, layout.sizes())) == accel.KACC_EINVAL


@pytest.mark.slow
def test_config3_full_size_properties_and_sampled_parity():
    """10k nodes x 2k procs, Z=4 (BASELINE config 3) through 3 intervals:
    size-independent properties on every node + oracle parity on a sample."""
    from oracle.oracle import Oracle

    layout = fleet.config_layout(3)
    Z = layout.zones
    sim = fleet.FleetSim(layout, seed=21)
    eng = EngineBackend(Z, layout.capacities())
    rng = np.random.default_rng(0)
    sample = np.sort(rng.choice(layout.n_nodes, 40, replace=False))
    ora = None
    for k in range(3):
        a = sim.next_interval()
        eng.interval(a, layout.sizes(), 0)
        sub, sub_sizes, maps = fleet.subset_interval(a, sample, Z)
        if ora is None:
            ora = Oracle(Z, nodes=len(sample), proc_slots=sub_sizes["n_procs"], ctr_slots=sub_sizes["n_ctrs"],
                         vm_slots=sub_sizes["n_vms"], pod_slots=sub_sizes["n_pods"])
        ora.interval(sub, sub_sizes)
    # sampled parity (bit exact)
    for name, _ in accel.TABLES:
        kind = name.split("_")[0]
        full = eng.table(name)
        per = len(full) // (layout.n_nodes if kind == "node" else layout.capacities()[f"{kind}_slots"])
        idx = maps[kind]
        got = full.reshape(-1, per)[idx].reshape(-1)
        want = ora.state[name]
        if name in accel.NODE_INDEX_TABLES:  # the sample's node indices -> the fleet's
            want = maps["node"][want]
        np.testing.assert_array_equal(got, want, err_msg=name)
    # conservation on every node: sum of process power == ActivePower (rel 1e-9),
    # sum of process interval energy within [aE - rows, aE]
    ap = eng.table("node_active_power").reshape(-1, Z)
    pp = eng.table("proc_power").reshape(-1, Z)
    off = layout.proc_off.astype(np.int64)
    sums = np.add.reduceat(pp[layout.proc_slot], off[:-1], axis=0)
    nd = eng.table("node_cpu_delta")
    ok = (nd != 0)[:, None] & (ap != 0)
    assert np.all(np.abs(sums - ap)[ok] <= 1e-9 * np.abs(ap)[ok])


def test_host_batch_pipelined_bit_exact():
    """Two pinned batches in flight (submit B, wait A): copies overlap the previous
    kernel, intervals still apply in submission order, bit-exact vs the oracle."""
    from oracle.oracle import Oracle

    layout = fleet.make_layout(24, [2000, 700, 1, 0, 1500, 2048] * 4, 4, seed=77, shuffle_slots=True)
    sizes = layout.sizes()
    sim = fleet.FleetSim(layout, seed=77, churn=0.05, read_error_frac=0.05)
    acc = accel.Accel(layout.zones, **layout.capacities())
    ora = Oracle(layout.zones, **layout.capacities())
    bs = [accel.HostBatch.alloc(acc, **sizes) for _ in range(2)]
    try:
        ivs = [sim.next_interval() for _ in range(6)]
        bs[0].fill(ivs[0])
        bs[0].submit()
        for k in range(1, len(ivs)):
            # the other batch is still in flight; odd intervals skip the host check
            bs[k % 2].fill(ivs[k], accel.KACC_F_TRUSTED_LAYOUT if k % 2 else 0)
            bs[k % 2].submit()
            bs[(k - 1) % 2].wait()
        bs[(len(ivs) - 1) % 2].wait()
        for a in ivs:
            ora.interval(a, sizes)
        for name, _ in accel.TABLES:
            np.testing.assert_array_equal(acc.download(name), ora.state[name], err_msg=name)
    finally:
        for b in bs:
            b.free()
        acc.close()


def test_host_batch_rejects_bad_layout():
    """kacc_batch_submit validates on the host (multi-threaded for big batches):
    a duplicate slot, an out-of-range slot and a container past its node's rows
    are KACC_EINVAL before anything is copied or launched."""
    layout = fleet.make_layout(64, 5000, 2, seed=9)  # 320k rows: the threaded checks run
    sizes = layout.sizes()
    acc = accel.Accel(layout.zones, **layout.capacities())
    b = accel.HostBatch.alloc(acc, **sizes)
    try:
        good = fleet.FleetSim(layout, seed=9).next_interval()
        for mutate, msg in (
            (lambda a: a["proc_slot"].__setitem__(300001, a["proc_slot"][7]), "used twice"),
            (lambda a: a["proc_slot"].__setitem__(250000, layout.capacities()["proc_slots"]), ">= capacity"),
            (lambda a: a["ctr_proc_end"].__setitem__(len(a["ctr_proc_end"]) - 1, sizes["n_procs"] + 1),
             "outside node"),
        ):
            a = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in good.items()}
            mutate(a)
            b.fill(a)
            with pytest.raises(accel.AccelError) as ei:
                b.submit()
            assert ei.value.code == accel.KACC_EINVAL and msg in str(ei.value), str(ei.value)
        b.fill(good)  # the context is usable afterwards
        b.submit()
        b.wait()
    finally:
        b.free()
        acc.close()


@pytest.mark.parametrize("name,kw", [
    ("z4-wrap", dict(n_nodes=16, procs_per_node=[2000, 300, 1, 0] * 4, zones=4)),
    ("z4-skew-chunked", dict(n_nodes=5, procs_per_node=[10000, 50000, 12, 0, 2049], zones=4,
                             procs_per_vm=2, vm_frac=0.02)),
])
def test_run_intervals_matches_sequential(name, kw):
    """kacc_run_intervals over K intervals == K interval calls == the oracle (BASELINE
    config 5's batched intervals with counter wraparound: fake-meter MaxEnergy 1e6)."""
    from oracle.oracle import Oracle

    layout = fleet.make_layout(seed=21, **kw)
    sizes = layout.sizes()
    sim = fleet.FleetSim(layout, seed=21, churn=0.03, read_error_frac=0.05, max_energy=fleet.MAX_ENERGY_FAKE)
    acc = accel.Accel(layout.zones, **layout.capacities())
    ora = Oracle(layout.zones, **layout.capacities())
    ivs = [sim.next_interval() for _ in range(12)]
    dev = [to_device(a) for a in ivs]
    descs = [interval_from_tensors(t, sizes) for t in dev]
    s = current_stream_handle()
    acc.run_intervals(descs[:1], s)  # first read alone, then 11 in one call
    acc.run_intervals(descs[1:], s)
    acc.sync(s)
    for a in ivs:
        ora.interval(a, sizes)
    for tname, _ in accel.TABLES:
        np.testing.assert_array_equal(acc.download(tname), ora.state[tname], err_msg=tname)
    acc.close()


@pytest.mark.parametrize("flags_mask", [~0, ~accel.KACC_F_SMALL_NODES], ids=["small_kernel", "interval_kernel"])
@pytest.mark.parametrize("nodes", [None, 96], ids=["single-node", "fleet-96"])
def test_config1_exact_layout_bit_exact(nodes, flags_mask):
    """BASELINE config 1 exactly: fleet.config_layout(1) — package + dram (Z = 2), the fake CPU
    power meter's MaxEnergy 1e6 (counters wrap), 500 processes -> 50 containers -> 20 pods per
    node — over 8 intervals with churn, every table bit-exact against the oracle; one node (the
    reference's own case) and a fleet of such nodes, through the one-wavefront-per-node kernel
    and the workgroup-per-node kernel."""
    from oracle.oracle import Oracle

    layout = fleet.config_layout(1, nodes=nodes)
    assert layout.zones == 2 and np.all(np.diff(layout.proc_off.astype(np.int64)) == 500)
    assert np.all(np.diff(layout.ctr_off.astype(np.int64)) == 50) and np.all(np.diff(layout.pod_off.astype(np.int64)) == 20)
    flags = layout.fast_flag() & flags_mask
    assert flags & accel.KACC_F_FAST_NODES
    sim = fleet.FleetSim(layout, seed=31, churn=0.03, max_energy=fleet.MAX_ENERGY_FAKE, read_error_frac=0.05)
    eng = EngineBackend(layout.zones, layout.capacities())
    ora = Oracle(layout.zones, **layout.capacities())
    wrapped = 0
    prev = None
    for k in range(8):
        a = sim.next_interval()
        wrapped += 0 if prev is None else int(np.count_nonzero(a["zone_energy"] < prev))
        prev = a["zone_energy"].copy()
        eng.interval(a, layout.sizes(), flags)
        ora.interval(a, layout.sizes())
        for name, _ in accel.TABLES:
            assert_table_equal(eng.table(name), ora.state[name], f"interval {k} {name}")
    assert wrapped > 0  # the fake meter's counters wrapped at least once


@pytest.mark.parametrize("shared", [False, True], ids=["own-arrays", "one-layout"])
@pytest.mark.timeout(300)
def test_config5_shape_60_intervals_one_call_bit_exact(shared):
    """BASELINE config 5's shape: heavy-tailed nodes of 10k-50k processes, Z = 4, VMs +
    containers + pods, 60 intervals in ONE kacc_run_intervals call with counter wraparound
    (fake-meter MaxEnergy 1e6), churn, read errors and adversarial inputs: every table
    bit-exact against the oracle after the call (and after the first-read call before it).
    one-layout: every descriptor points at the SAME offset arrays, so the call generates the
    big nodes' chunk items once and reuses them (items_kernel), and the chunk kernel must skip
    the items of nodes skipped (read error) in their interval."""
    from oracle.oracle import Oracle

    procs = [10000, 50000, 23000, 12000, 31000, 10000, 17500]
    layout = fleet.make_layout(len(procs), procs, 4, seed=55, procs_per_vm=2, vm_frac=0.02)
    assert layout.fast_flag() == 0  # big nodes: the chunked path
    sizes = layout.sizes()
    sim = fleet.FleetSim(layout, seed=55, churn=0.02, read_error_frac=0.03, max_energy=fleet.MAX_ENERGY_FAKE,
                         adversarial=0.05)
    acc = accel.Accel(layout.zones, **layout.capacities())
    ora = Oracle(layout.zones, **layout.capacities())
    s = current_stream_handle()
    first = sim.next_interval()
    t0 = to_device(first)
    acc.run_intervals([interval_from_tensors(t0, sizes)], s)
    ora.interval(first, sizes)
    ivs = [sim.next_interval() for _ in range(60)]
    if shared:
        statics = to_device(layout.static_arrays())
        dev = []
        for a in ivs:
            t = to_device({k: v for k, v in a.items() if k not in statics})
            t.update(statics)
            dev.append(t)
        assert sum(int((a["node_status"] & accel.KACC_NODE_READ_ERROR).any()) for a in ivs) > 3
    else:
        dev = [to_device(a) for a in ivs]
    acc.run_intervals([interval_from_tensors(t, sizes) for t in dev], s)
    acc.sync(s)
    for a in ivs:
        ora.interval(a, sizes)
    for tname, _ in accel.TABLES:
        assert_table_equal(acc.download(tname), ora.state[tname], tname)
    acc.close()


@pytest.mark.parametrize("name,kw,K", [
    ("z2-config2-like", dict(n_nodes=64, procs_per_node=[1000, 700, 1, 0, 2048, 513] * 10 + [9] * 4, zones=2), 12),
    ("z2-fragmented", dict(n_nodes=16, procs_per_node=[2000, 900, 64, 3] * 4, zones=2, fragment_slots=0.05), 9),
    ("z1-shuffled", dict(n_nodes=20, procs_per_node=[1500, 600, 0, 77] * 5, zones=1, shuffle_slots=True), 7),
    ("z4-not-fused", dict(n_nodes=12, procs_per_node=[2000, 600, 0, 77] * 3, zones=4), 5),
    # more intervals than one LDS chunk of node inputs (kCarryChunk = 63): two refills
    ("z2-long", dict(n_nodes=6, procs_per_node=[300, 1200, 5, 0, 64, 2048], zones=2), 140),
    ("z1-long-fragmented", dict(n_nodes=4, procs_per_node=[700, 90, 1, 2000], zones=1, fragment_slots=0.1), 66),
    # KACC_F_MEDIUM_NODES (every node <= 1024 rows, <= 256 aggregates): 256-thread workgroups,
    # 31 intervals per LDS chunk of node inputs
    ("z2-medium", dict(n_nodes=48, procs_per_node=[1000, 700, 1, 0, 1024, 513] * 8, zones=2), 12),
    ("z2-medium-long", dict(n_nodes=5, procs_per_node=[1024, 300, 7, 0, 999], zones=2), 70),
    ("z1-medium-fragmented", dict(n_nodes=8, procs_per_node=[900, 64, 3, 1024] * 2, zones=1, fragment_slots=0.05), 33),
])
def test_fused_run_intervals_bit_exact(name, kw, K):
    """kacc_run_intervals as ONE launch (KACC_F_FAST_NODES | KACC_F_NODE_SLOT_RANGES: every
    workgroup carries its node through K intervals) == the oracle interval by interval, with
    churn, read errors, zero ratios, counter wraparound and adversarial inputs."""
    from oracle.oracle import Oracle

    layout = fleet.make_layout(seed=23, **kw)
    flags = layout.fast_flag() & ~accel.KACC_F_SMALL_NODES
    assert flags & accel.KACC_F_FAST_NODES
    assert bool(flags & accel.KACC_F_MEDIUM_NODES) == ("medium" in name), name
    flags |= accel.KACC_F_NODE_SLOT_RANGES
    sizes = layout.sizes()
    sim = fleet.FleetSim(layout, seed=23, churn=0.03, read_error_frac=0.05, max_energy=fleet.MAX_ENERGY_FAKE,
                         adversarial=0.1)
    acc = accel.Accel(layout.zones, **layout.capacities())
    ora = Oracle(layout.zones, **layout.capacities())
    ivs = [sim.next_interval() for _ in range(K)]
    if kw.get("fragment_slots"):
        for a in ivs:
            a["node_proc_span"] = layout.proc_span()
    dev = [to_device(a) for a in ivs]
    descs = [interval_from_tensors(t, sizes, flags) for t in dev]
    s = current_stream_handle()
    acc.run_intervals(descs[:1], s)  # first read alone, then K-1 in one launch
    acc.run_intervals(descs[1:], s)
    acc.sync(s)
    for a in ivs:
        ora.interval(a, sizes)
    for tname, _ in accel.TABLES:
        assert_table_equal(acc.download(tname), ora.state[tname], tname)
    acc.close()


@pytest.mark.parametrize("medium", [False, True])
def test_fused_span_toggles_bit_exact(medium):
    """One launch whose intervals give node_proc_span only sometimes: the carried totals switch
    between row keys and the slot window (and back) mid-launch; fragmented slots with churn,
    read errors and adversarial inputs; nodes whose span exceeds the window stay in row order."""
    from oracle.oracle import Oracle

    procs = [1000, 700, 1, 0, 1024, 513] if medium else [2000, 1500, 1, 0, 1990, 64]
    layout = fleet.make_layout(n_nodes=12, procs_per_node=procs * 2, zones=2, seed=29, fragment_slots=0.03)
    flags = (layout.fast_flag() & ~accel.KACC_F_SMALL_NODES) | accel.KACC_F_NODE_SLOT_RANGES
    assert bool(flags & accel.KACC_F_MEDIUM_NODES) == medium
    sizes = layout.sizes()
    sim = fleet.FleetSim(layout, seed=29, churn=0.05, read_error_frac=0.08, max_energy=fleet.MAX_ENERGY_FAKE,
                         adversarial=0.1)
    acc = accel.Accel(layout.zones, **layout.capacities())
    ora = Oracle(layout.zones, **layout.capacities())
    pattern = [0, 1, 1, 0, 1, 0, 0, 1, 1, 1, 0, 1]
    ivs = [sim.next_interval() for _ in pattern]
    for a, given in zip(ivs, pattern):
        if given:
            a["node_proc_span"] = layout.proc_span()
    dev = [to_device(a) for a in ivs]
    descs = [interval_from_tensors(t, sizes, flags) for t in dev]
    s = current_stream_handle()
    acc.run_intervals(descs[:1], s)
    acc.run_intervals(descs[1:], s)
    acc.sync(s)
    for a in ivs:
        ora.interval(a, sizes)
    for tname, _ in accel.TABLES:
        assert_table_equal(acc.download(tname), ora.state[tname], tname)
    acc.close()


@pytest.mark.parametrize("procs", [[1000, 1025, 3], [200, 220, 3]])
def test_medium_flag_rejects_oversized_node(procs):
    """KACC_F_MEDIUM_NODES is a promise: under the one-launch path a node over 1024 rows
    (or over 256 aggregates) raises KACC_ERANGE and nothing faults."""
    kw = {} if max(procs) > 1024 else dict(procs_per_ctr=1, ctr_frac=0.95, ctrs_per_pod=1.0)
    layout = fleet.make_layout(3, procs, 2, seed=6, **kw)
    assert layout.fast_flag() & accel.KACC_F_FAST_NODES and not layout.fast_flag() & accel.KACC_F_MEDIUM_NODES
    flags = accel.KACC_F_FAST_NODES | accel.KACC_F_MEDIUM_NODES | accel.KACC_F_NODE_SLOT_RANGES
    acc = accel.Accel(layout.zones, **layout.capacities())
    sim = fleet.FleetSim(layout, seed=6)
    dev = [to_device(sim.next_interval()) for _ in range(3)]
    s = current_stream_handle()
    with pytest.raises(accel.AccelError) as ei:
        acc.run_intervals([interval_from_tensors(t, layout.sizes(), flags) for t in dev], s)
        acc.sync(s)
    assert ei.value.code == accel.KACC_ERANGE
    acc.close()


def test_recreated_aggregates_bit_exact():
    """Containers / VMs / pods recreated in their slots (NEW on aggregate slot
    words after the first interval): totals restart, CPU caches reset."""
    from oracle.oracle import Oracle

    layout = fleet.make_layout(12, [300, 2000, 1, 0, 700, 64] * 2, 4, seed=13, vm_frac=0.05, procs_per_vm=2)
    sim = fleet.FleetSim(layout, seed=13, churn=0.05, read_error_frac=0.05)
    eng = EngineBackend(layout.zones, layout.capacities())
    ora = Oracle(layout.zones, **layout.capacities())
    rng = np.random.default_rng(3)
    for k in range(5):
        a = sim.next_interval()
        if k:
            for key in ("ctr_slot", "vm_slot", "pod_slot"):
                a[key] = a[key] | np.where(rng.random(a[key].size) < 0.2, np.uint32(accel.KACC_SLOT_NEW),
                                           np.uint32(0)).astype(np.uint32)
        eng.interval(a, layout.sizes(), layout.fast_flag())
        ora.interval(a, layout.sizes())
        for name, _ in accel.TABLES:
            np.testing.assert_array_equal(eng.table(name), ora.state[name], err_msg=f"interval {k} {name}")


def assert_table_equal(got, want, msg):
    """Bit-exact, except that any NaN equals any NaN: Go formats every NaN alike ("NaN" in
    strconv and the Prometheus text format) and the NaN bits are not an observable of the
    reference; x86 SSE2 (Go on amd64, the oracle) produces the default NaN with the sign
    bit set where gfx950 produces it without."""
    if want.dtype == np.float64:
        gb, wb = got.view(np.uint64), want.view(np.uint64)
        both_nan = np.isnan(got) & np.isnan(want)
        bad = (gb != wb) & ~both_nan
        assert not bad.any(), f"{msg}: {int(bad.sum())} differ, first at {int(np.flatnonzero(bad)[0])}: " \
                              f"{got[bad][0]!r} vs {want[bad][0]!r}"
    else:
        np.testing.assert_array_equal(got, want, err_msg=msg)


ADV_FLEETS = [
    ("z4-fast-shuffled", dict(n_nodes=40, procs_per_node=[2000, 300, 1, 0, 1500] * 8, zones=4,
                              shuffle_slots=True)),
    ("z2-small-kernel", dict(n_nodes=64, procs_per_node=[500, 64, 3, 0] * 16, zones=2)),
    ("z4-small-kernel", dict(n_nodes=32, procs_per_node=[512, 200, 1, 77] * 8, zones=4)),
    ("z4-big-nodes", dict(n_nodes=6, procs_per_node=[10000, 3000, 12, 0, 2049, 700], zones=4, vm_frac=0.02,
                          procs_per_vm=2)),
    ("z3-odd", dict(n_nodes=30, procs_per_node=257, zones=3, vm_frac=0.05, procs_per_vm=3)),
    ("z4-fragmented-span", dict(n_nodes=24, procs_per_node=[2000, 1200, 64, 5] * 6, zones=4, fragment_slots=0.05)),
]


@pytest.mark.parametrize("name,kw", ADV_FLEETS, ids=[f[0] for f in ADV_FLEETS])
def test_adversarial_inputs_bit_exact(name, kw):
    """Reachable edge inputs (fleet.FleetSim.ADVERSARIAL), every table against the oracle:
    Δt = 0 / backward clock (node.go:34 -> ±Inf / NaN node and workload power), unchanged
    counters (ΔE = 0 with a nonzero ratio), usage ratio 1 / > 1 / < 0 (u64 idle wrap,
    negative ActivePower), negative CPU deltas (informer.go:518, PID reuse in a cached
    entry: Energy() of negatives, u64 EnergyTotal wrap, process.go:136) and huge cancelling
    deltas (Energy() out of range, process.go:130), with churn and read errors, on every
    kernel path (fast, small, chunked big nodes, odd Z, slot sweep)."""
    from oracle.oracle import Oracle

    layout = fleet.make_layout(seed=19, **kw)
    caps = layout.capacities()
    sim = fleet.FleetSim(layout, seed=19, churn=0.04, read_error_frac=0.05, adversarial=0.5)
    eng = EngineBackend(layout.zones, caps)
    ora = Oracle(layout.zones, **caps)
    edges = 0
    for k in range(6):
        a = sim.next_interval()
        if kw.get("fragment_slots"):
            a["node_proc_span"] = layout.proc_span()
        eng.interval(a, layout.sizes(), layout.fast_flag())
        ora.interval(a, layout.sizes())
        for tname, _ in accel.TABLES:
            assert_table_equal(eng.table(tname), ora.state[tname], f"interval {k} {tname}")
        st = ora.state
        edges += int((~np.isfinite(st["node_power"])).sum() + (st["node_active_power"] < 0).sum()
                     + (st["proc_energy"] >= np.uint64(1 << 63)).sum() + (a["proc_cpu_delta"] < 0).sum())
    assert edges > 0  # the edges were exercised
