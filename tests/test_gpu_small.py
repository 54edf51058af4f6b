"""Small-node kernel (KACC_F_SMALL_NODES: one wavefront per node) — MI355X only.

The reference's own single-node case is 500 procs -> 50 containers -> 20 pods
(BASELINE config 1); fleets of such nodes run one node per wavefront.  The
small kernel must be bit-identical to the oracle and to the workgroup-per-node
kernel on every table, over the edges of its two 256-row batches, slot
sweeps, VMs, NEW aggregates, read errors and first reads.
"""

import numpy as np
import pytest
import torch

from kepler_amd import accel, fleet
from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device

pytestmark = pytest.mark.gpu

SMALL = accel.KACC_F_SMALL_NODES | accel.KACC_F_FAST_NODES


@pytest.fixture(scope="module", autouse=True)
def gpu_ready():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    accel.load()  # raises if the HIP library is missing: no fallback
    torch.cuda.set_stream(torch.cuda.Stream())


def _fits_small(layout):
    rows = np.diff(layout.proc_off.astype(np.int64))
    agg = (np.diff(layout.ctr_off.astype(np.int64)) + np.diff(layout.vm_off.astype(np.int64))
           + np.diff(layout.pod_off.astype(np.int64)))
    return bool(np.all(rows <= accel.KACC_SMALL_MAX_PROCS) and np.all(agg <= accel.KACC_SMALL_MAX_AGGREGATES))


def _run(acc, a, sizes, flags):
    t = to_device(a)
    s = current_stream_handle()
    acc.run_interval(interval_from_tensors(t, sizes, flags), s)
    acc.sync(s)


EDGES = [0, 1, 2, 63, 64, 65, 127, 128, 255, 256, 257, 300, 383, 384, 385, 448, 500, 510, 511, 512]
ODD = [257, 500, 3, 0, 64, 130, 511, 200, 1] * 2 + [400]
SMALL_FLEETS = [
    ("z4-config1-like", dict(n_nodes=40, procs_per_node=500, zones=4)),
    ("z4-edges", dict(n_nodes=len(EDGES), procs_per_node=EDGES, zones=4)),
    ("z4-edges-shuffled", dict(n_nodes=len(EDGES), procs_per_node=EDGES[::-1], zones=4, shuffle_slots=True)),
    ("z2-edges", dict(n_nodes=len(EDGES), procs_per_node=EDGES, zones=2)),
    ("z3-odd-vms", dict(n_nodes=len(ODD), procs_per_node=ODD, zones=3, procs_per_vm=3, vm_frac=0.05)),
    ("z8-max-zones", dict(n_nodes=9, procs_per_node=[511, 512, 256, 1, 0, 64, 300, 65, 129], zones=8)),
    ("z1", dict(n_nodes=7, procs_per_node=[1, 0, 40, 300, 7, 512, 257], zones=1)),
    ("z4-fragmented", dict(n_nodes=12, procs_per_node=[500, 499, 300, 64, 1, 0, 495, 256, 3, 460, 100, 257],
                           zones=4, fragment_slots=0.02)),
    ("z4-fragmented-wide", dict(n_nodes=6, procs_per_node=[300, 200, 250, 17, 320, 128], zones=4,
                                fragment_slots=0.5)),
    ("z6-fragmented", dict(n_nodes=5, procs_per_node=[400, 300, 64, 1, 200], zones=6, fragment_slots=0.2)),
    ("z4-many-aggregates", dict(n_nodes=6, procs_per_node=[60, 64, 30, 50, 10, 0], zones=4, procs_per_ctr=1,
                                ctrs_per_pod=1.0, ctr_frac=0.95, vm_frac=0.05)),
]
SPAN = {"z4-fragmented", "z4-fragmented-wide", "z6-fragmented", "z4-edges-shuffled"}


@pytest.mark.parametrize("name,kw", SMALL_FLEETS, ids=[f[0] for f in SMALL_FLEETS])
def test_small_kernel_bit_exact(name, kw):
    """small kernel == oracle == workgroup-per-node kernel, every table, 5 intervals."""
    from oracle.oracle import Oracle

    layout = fleet.make_layout(seed=31, **kw)
    assert _fits_small(layout), "fleet must fit the small kernel"
    caps = layout.capacities()
    sizes = layout.sizes()
    sim = fleet.FleetSim(layout, seed=31, churn=0.05, zero_ratio_frac=0.05, read_error_frac=0.05)
    small = accel.Accel(layout.zones, **caps)
    wide = accel.Accel(layout.zones, **caps)
    ora = Oracle(layout.zones, **caps)
    rng = np.random.default_rng(5)
    for k in range(5):
        a = sim.next_interval()
        if name in SPAN:
            a["node_proc_span"] = layout.proc_span()
        if k == 3:  # recreated aggregates (NEW on their slot words)
            for key in ("ctr_slot", "vm_slot", "pod_slot"):
                a[key] = a[key] | np.where(rng.random(a[key].size) < 0.2, np.uint32(accel.KACC_SLOT_NEW),
                                           np.uint32(0)).astype(np.uint32)
        if k == 4:  # a shuffled node order
            a["node_order"] = rng.permutation(layout.n_nodes).astype(np.uint32)
        _run(small, a, sizes, SMALL)
        _run(wide, a, sizes, accel.KACC_F_FAST_NODES)
        ora.interval(a, sizes)
        for tname, _ in accel.TABLES:
            got = small.download(tname)
            np.testing.assert_array_equal(got, ora.state[tname], err_msg=f"interval {k} {tname} vs oracle")
            np.testing.assert_array_equal(got, wide.download(tname), err_msg=f"interval {k} {tname} vs wide")
    small.close()
    wide.close()


def test_small_kernel_node_cpu_delta_given_and_wrap():
    from oracle.oracle import Oracle

    layout = fleet.make_layout(24, [500, 0, 1, 257] * 6, 4, seed=9)
    caps = layout.capacities()
    sim = fleet.FleetSim(layout, seed=9, max_energy=fleet.MAX_ENERGY_FAKE, churn=0.1)
    acc = accel.Accel(layout.zones, **caps)
    ora = Oracle(layout.zones, **caps)
    for k in range(4):
        a = sim.next_interval()
        flags = SMALL
        if k % 2:
            a["node_cpu_delta"] = np.full(layout.n_nodes, 1234.5 + k)
            flags |= accel.KACC_F_NODE_CPU_DELTA_GIVEN
        _run(acc, a, layout.sizes(), flags)
        ora.interval(a, layout.sizes(), flags & accel.KACC_F_NODE_CPU_DELTA_GIVEN)
        for tname, _ in accel.TABLES:
            np.testing.assert_array_equal(acc.download(tname), ora.state[tname], err_msg=f"interval {k} {tname}")
    acc.close()


@pytest.mark.parametrize("sizes_", [[100, 513, 5], [100, 200, 5]])
def test_small_flag_rejects_oversized_node(sizes_):
    """KACC_F_SMALL_NODES is a promise: a node over 512 rows or 128 aggregates
    raises KACC_ERANGE, nothing faults, and the batch runs without the flag."""
    kw = {} if sizes_[1] > 512 else dict(procs_per_ctr=1, ctr_frac=0.95, ctrs_per_pod=1.0)
    layout = fleet.make_layout(3, sizes_, 4, seed=5, **kw)
    assert not _fits_small(layout)
    acc = accel.Accel(layout.zones, **layout.capacities())
    a = fleet.FleetSim(layout, seed=5).next_interval()
    with pytest.raises(accel.AccelError) as ei:
        _run(acc, a, layout.sizes(), SMALL)
    assert ei.value.code == accel.KACC_ERANGE
    _run(acc, a, layout.sizes(), 0)
    acc.close()


def test_small_kernel_run_intervals_and_host_batch():
    """kacc_run_intervals and the pinned host path (which sets KACC_F_SMALL_NODES
    by itself) on a config-1-shaped fleet == the oracle."""
    from oracle.oracle import Oracle

    layout = fleet.make_layout(64, 500, 2, seed=17)
    sizes = layout.sizes()
    caps = layout.capacities()
    sim = fleet.FleetSim(layout, seed=17, churn=0.03, read_error_frac=0.05, max_energy=fleet.MAX_ENERGY_FAKE)
    ivs = [sim.next_interval() for _ in range(8)]
    acc = accel.Accel(layout.zones, **caps)
    ora = Oracle(layout.zones, **caps)
    dev = [to_device(a) for a in ivs[:5]]
    s = current_stream_handle()
    acc.run_intervals([interval_from_tensors(t, sizes, SMALL) for t in dev], s)
    acc.sync(s)
    for a in ivs[:5]:
        ora.interval(a, sizes)
    for a in ivs[5:]:
        b = accel.HostBatch.alloc(acc, **sizes)
        try:
            b.fill(a, 0)
            b.submit()
            b.wait()
        finally:
            b.free()
        ora.interval(a, sizes)
    for tname, _ in accel.TABLES:
        np.testing.assert_array_equal(acc.download(tname), ora.state[tname], err_msg=tname)
    acc.close()
