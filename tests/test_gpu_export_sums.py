"""Cluster partial sums of an interval inside the NEXT interval's launch — MI355X only.

kacc_run_interval_sums(interval k, sums of interval k-1's exports) and the standalone
kacc_run_export_sums against kacc_cluster_partials over the tables interval k-1 left
(bit-exact: the same per-lane orders), for every kernel shape the interval can take (workgroup
per node with the sums blocks in its tail; wavefront per node and big-node chunks, whose sums
run as a launch of their own), with exports in batch order (ns_pod_row) and in namespace order
(kacc_interval.pod_export_pos: contiguous records per namespace).  The interval's own tables
stay bit-exact against the oracle, and the namespace totals against the oracle's
kor_namespace_totals.
"""

import numpy as np
import pytest
import torch

from kepler_amd import accel, fleet
from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device
from oracle.oracle import Oracle
from table_check import assert_tables_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu_ready():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    accel.load()
    torch.cuda.set_stream(torch.cuda.Stream())


FLEETS = [
    # (name, layout kwargs, node order) — fast: the sums blocks ride in interval_sums_kernel
    ("fast-z4", dict(n_nodes=40, procs_per_node=[2000, 300, 1, 0, 1500] * 8, zones=4, shuffle_slots=True,
                     n_namespaces=13), False),
    ("fast-z4-order", dict(n_nodes=33, procs_per_node=[64, 2000, 7, 1200] * 8 + [5], zones=4, n_namespaces=300),
     True),
    ("fast-z2-many-ns", dict(n_nodes=24, procs_per_node=[900, 20, 2000] * 8, zones=2, n_namespaces=2000), False),
    # wavefront per node (KACC_F_SMALL_NODES): interval, then the sums as their own launch
    ("small-z2", dict(n_nodes=64, procs_per_node=[500, 64, 3, 0] * 16, zones=2, n_namespaces=7), False),
    # big nodes: interval_sums_kernel + chunk / pod kernels
    ("big-z4", dict(n_nodes=6, procs_per_node=[10000, 3000, 12, 0, 2049, 700], zones=4, vm_frac=0.02,
                    procs_per_vm=2, n_namespaces=5), False),
]


def _outs(n_ns, Z):
    return [torch.zeros(n, dtype=dt, device="cuda") for n, dt in ((max(n_ns * Z, 1), torch.int64),
                                                                 (max(n_ns * Z, 1), torch.float64),
                                                                 (2 * Z, torch.int64), (3 * Z, torch.float64))]


def _sums(L, d, ordered, pex, nex, outs, nodes=True):
    s = accel.KaccExportSums()
    s.n_ns = L.n_namespaces
    s.n_pods = L.n_pods
    s.n_nodes = L.n_nodes
    s.ns_ordered = 1 if ordered else 0
    s.ns_pod_off = d["o"].data_ptr()
    s.ns_pod_row = None if ordered else d["r"].data_ptr()
    s.pod_export = pex.data_ptr()
    s.node_export = nex.data_ptr() if nodes else None
    s.out_energy, s.out_power = outs[0].data_ptr(), outs[1].data_ptr()
    s.out_node_energy = outs[2].data_ptr() if nodes else None
    s.out_node_power = outs[3].data_ptr() if nodes else None
    return s


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


@pytest.mark.parametrize("ordered", [False, True], ids=["rows", "ns-ordered"])
@pytest.mark.parametrize("name,kw,node_order", FLEETS, ids=[f[0] for f in FLEETS])
def test_interval_sums_match_table_partials(name, kw, node_order, ordered):
    L = fleet.make_layout(seed=31, **kw)
    Z = L.zones
    n_ns = L.n_namespaces
    acc = accel.Accel(Z, **L.capacities())
    cl = accel.Cluster.join(acc, accel.Cluster.unique_id(), 1, 0)
    ora = Oracle(Z, **L.capacities())
    sim = fleet.FleetSim(L, seed=31, churn=0.03, read_error_frac=0.1, adversarial=0.05,
                         max_energy=fleet.MAX_ENERGY_FAKE)
    s = current_stream_handle()
    flags = L.fast_flag()
    off, slots_ns = L.namespace_csr()
    _, rows_ns = L.namespace_csr_rows()
    pos = np.zeros(max(L.n_pods, 1), dtype=np.uint32)
    pos[rows_ns] = np.arange(len(rows_ns), dtype=np.uint32)  # pod q's place in namespace order
    d = to_device({"o": off, "s": slots_ns, "r": rows_ns, "pos": pos})
    order = to_device({"x": L.node_order_heaviest_first()})["x"] if node_order else None
    pex = [torch.zeros(max(L.n_pods, 1) * 2 * Z, dtype=torch.int64, device="cuda") for _ in range(2)]
    nex = [torch.zeros(L.n_nodes * 5 * Z, dtype=torch.int64, device="cuda") for _ in range(2)]
    n_iv = 4
    fused = [_outs(n_ns, Z) for _ in range(n_iv)]  # interval k's sums, computed in launch k + 1
    ref = [_outs(n_ns, Z) for _ in range(n_iv)]    # interval k's sums from the tables it left
    keep = []
    for k in range(n_iv):
        a = sim.next_interval()
        ora.interval(a, L.sizes())
        t = to_device(a)
        t["pod_export"], t["node_export"] = pex[k % 2], nex[k % 2]
        if ordered:
            t["pod_export_pos"] = d["pos"]
        if order is not None:
            t["node_order"] = order
        keep.append(t)
        iv = interval_from_tensors(t, L.sizes(), flags)
        prev = _sums(L, d, ordered, pex[(k - 1) % 2], nex[(k - 1) % 2], fused[k - 1]) if k else None
        acc.run_interval_sums(iv, prev, s)
        cl.partials(n_ns, [d["o"].data_ptr()], [d["s"].data_ptr()], [ref[k][0].data_ptr()], [ref[k][1].data_ptr()],
                    [ref[k][2].data_ptr()], [ref[k][3].data_ptr()], streams=[s])
        acc.sync(s)
        assert_tables_equal(acc.download, ora.state, f"{name} interval {k}")
    acc.export_sums(_sums(L, d, ordered, pex[(n_iv - 1) % 2], nex[(n_iv - 1) % 2], fused[n_iv - 1]), s)
    acc.sync(s)
    for k in range(n_iv):
        for j, (f_, r_) in enumerate(zip(fused[k], ref[k])):
            np.testing.assert_array_equal(_u64(f_), _u64(r_), err_msg=f"{name} interval {k} output {j}")
    e_o, p_o = ora.namespace_totals(off, slots_ns)  # the last interval, pinned by the oracle's own order
    np.testing.assert_array_equal(_u64(fused[-1][0])[: n_ns * Z], e_o)
    np.testing.assert_array_equal(fused[-1][1].cpu().numpy()[: n_ns * Z].view(np.uint64), p_o.view(np.uint64))
    assert np.count_nonzero(e_o) > 0
    cl.close()
    acc.close()


def test_ns_ordered_export_is_the_permuted_batch_export():
    """pod_export_pos writes pod q's record at row pos[q]: the namespace-ordered export is the
    batch-order export permuted (and node exports unchanged)."""
    L = fleet.make_layout(20, [700, 2000, 3, 0, 1200] * 4, 4, seed=5, n_namespaces=9)
    Z = L.zones
    _, rows_ns = L.namespace_csr_rows()
    pos = np.zeros(L.n_pods, dtype=np.uint32)
    pos[rows_ns] = np.arange(len(rows_ns), dtype=np.uint32)
    outs = []
    for use_pos in (False, True):
        acc = accel.Accel(Z, **L.capacities())
        sim = fleet.FleetSim(L, seed=5, churn=0.02, read_error_frac=0.1)
        s = current_stream_handle()
        pex = torch.zeros(L.n_pods * 2 * Z, dtype=torch.int64, device="cuda")
        nex = torch.zeros(L.n_nodes * 5 * Z, dtype=torch.int64, device="cuda")
        keep = []
        for _ in range(3):
            t = to_device(sim.next_interval())
            t["pod_export"], t["node_export"] = pex, nex
            if use_pos:
                t["pod_export_pos"] = to_device({"p": pos})["p"]
            keep.append(t)
            acc.run_interval(interval_from_tensors(t, L.sizes(), L.fast_flag()), s)
        acc.sync(s)
        outs.append((_u64(pex).reshape(-1, 2 * Z), _u64(nex)))
        acc.close()
    (pe0, ne0), (pe1, ne1) = outs
    np.testing.assert_array_equal(pe1[pos], pe0)
    np.testing.assert_array_equal(ne1, ne0)


def test_interval_sums_argument_errors():
    L = fleet.make_layout(8, [100, 50] * 4, 2, seed=3, n_namespaces=3)
    Z = L.zones
    acc = accel.Accel(Z, **L.capacities())
    s = current_stream_handle()
    off, slots_ns = L.namespace_csr()
    _, rows_ns = L.namespace_csr_rows()
    d = to_device({"o": off, "r": rows_ns})
    pex = torch.zeros(L.n_pods * 2 * Z, dtype=torch.int64, device="cuda")
    nex = torch.zeros(L.n_nodes * 5 * Z, dtype=torch.int64, device="cuda")
    sim = fleet.FleetSim(L, seed=3)
    t = to_device(sim.next_interval())
    t["pod_export"], t["node_export"] = pex, nex
    iv = interval_from_tensors(t, L.sizes(), L.fast_flag())
    outs = _outs(L.n_namespaces, Z)
    with pytest.raises(accel.AccelError) as ei:  # reading the exports this interval writes
        acc.run_interval_sums(iv, _sums(L, d, False, pex, nex, outs), s)
    assert ei.value.code == accel.KACC_EINVAL
    bad = _sums(L, d, False, pex, nex, outs)
    bad.out_node_power = None  # node totals need both outputs
    with pytest.raises(accel.AccelError) as ei:
        acc.export_sums(bad, s)
    assert ei.value.code == accel.KACC_EINVAL
    # an export row out of range raises ERANGE on the device and is not written
    t2 = to_device(sim.next_interval())
    pex2 = torch.zeros_like(pex)
    t2["pod_export"] = pex2
    p = np.arange(L.n_pods, dtype=np.uint32)
    p[0] = L.n_pods + 5
    t2["pod_export_pos"] = to_device({"p": p})["p"]
    keep = [t, t2]
    acc.run_interval(interval_from_tensors(t2, L.sizes(), L.fast_flag()), s)
    with pytest.raises(accel.AccelError) as ei:
        acc.sync(s)
    assert ei.value.code == accel.KACC_ERANGE
    del keep
    acc.close()
