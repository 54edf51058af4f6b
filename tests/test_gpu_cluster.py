"""Multi-GPU path through the C ABI (BASELINE config 4) — MI355X only.

A fleet is cut into node shards by shard.plan_node_ranges (shard.shard), every
shard runs in its own engine context, and the cluster totals cross the shards
through kacc_create_multi / kacc_allreduce_namespaces / kacc_gather_pods: the
real RCCL path, here with several shards on the one GPU of the box (their
partial vectors are added on the GPU, then all-reduced over a one-rank
communicator).  Nodes are independent, so every shard's state must equal the
unsharded oracle's (bit-exact); namespace totals: u64 bit-exact, f64 <= 1e-12
relative (the north star's totals bar: the sum order differs from one
context's); gathered pods: bit-exact.
"""

import numpy as np
import pytest
import torch

from kepler_amd import accel, fleet, shard
from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu_ready():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    accel.load()
    torch.cuda.set_stream(torch.cuda.Stream())


def _gather_rows(acc, name, idx, per):
    """Rows idx (each `per` elements) of a device table, one download per consecutive run."""
    idx = np.asarray(idx, dtype=np.int64)
    if not len(idx):
        return np.zeros(0, dtype=dict(accel.TABLES)[name])
    cuts = np.flatnonzero(np.diff(idx) != 1) + 1
    parts = []
    for run in np.split(idx, cuts):
        parts.append(acc.download(name, int(run[0]) * per, len(run) * per))
    return np.concatenate(parts)


def _check_shard_tables(shard_acc, sl, lo, hi, maps, want_state, zones, nodes_total):
    """Shard tables (compact slots) == the unsharded tables at the original slots / nodes."""
    for name, _ in accel.TABLES:
        kind = name.split("_")[0]
        got = shard_acc.download(name)
        full = want_state[name]
        n_rows = (hi - lo) if kind == "node" else sl.capacities()[f"{kind}_slots"]
        per = len(got) // max(n_rows, 1) if n_rows else 1
        if kind == "node":
            idx = np.arange(lo, hi)
        else:
            idx = maps[kind]
        if len(idx) == 0:
            continue
        want = full.reshape(-1, per)[idx]
        g = got.reshape(-1, per)[: len(idx)]
        if name in accel.NODE_INDEX_TABLES:  # shard-local node indices -> the fleet's
            g = g + lo
        np.testing.assert_array_equal(g, want, err_msg=f"shard [{lo},{hi}) {name}")


def _namespace_csr_device(layouts):
    out = []
    for sl in layouts:
        off, slots = sl.namespace_csr()
        out.append(to_device({"o": off, "s": slots}))
    return out


@pytest.mark.parametrize("world", [8, 3])
def test_sharded_fleet_matches_unsharded_oracle(world):
    """One fleet (skewed, VMs, churn, read errors, Z = 4) cut `world` ways; each shard in its
    own context; namespace + cluster node totals through kacc_allreduce_namespaces and the
    pods through kacc_gather_pods, against the unsharded oracle."""
    from oracle.oracle import Oracle

    L = fleet.make_layout(96, [2000, 300, 0, 1, 4096, 700, 12000, 64] * 12, 4, seed=41, n_namespaces=13,
                          vm_frac=0.03, procs_per_vm=2, shuffle_slots=True)
    shards = shard.shard(L, world)
    cl = accel.Cluster.create_multi([0] * world, L.zones, [sl.capacities() for _, _, sl in shards])
    assert cl.info() == (1, 0, world)  # one GPU: one RCCL rank holding `world` shards
    ora = Oracle(L.zones, **L.capacities())
    sim = fleet.FleetSim(L, seed=41, churn=0.04, read_error_frac=0.05)
    s = current_stream_handle()
    for k in range(4):
        a = sim.next_interval()
        ora.interval(a, L.sizes())
        keep = []
        for (lo, hi, sl), acc in zip(shards, cl.shards):
            sub, sizes, maps = fleet.subset_interval(a, np.arange(lo, hi), L.zones)
            t = to_device(sub)
            keep.append(t)
            acc.run_interval(interval_from_tensors(t, sizes, sl.fast_flag()), s)
        for acc in cl.shards:
            acc.sync(s)
    for (lo, hi, sl), acc in zip(shards, cl.shards):
        _, _, maps = fleet.subset_interval(a, np.arange(lo, hi), L.zones)
        _check_shard_tables(acc, sl, lo, hi, maps, ora.state, L.zones, L.n_nodes)

    Z = L.zones
    n_ns = L.n_namespaces
    csr = _namespace_csr_device([sl for _, _, sl in shards])
    oe = [torch.zeros(n_ns * Z, dtype=torch.int64, device="cuda") for _ in range(world)]
    op = [torch.zeros(n_ns * Z, dtype=torch.float64, device="cuda") for _ in range(world)]
    ne = [torch.zeros(2 * Z, dtype=torch.int64, device="cuda") for _ in range(world)]
    npw = [torch.zeros(3 * Z, dtype=torch.float64, device="cuda") for _ in range(world)]
    comm = torch.cuda.Stream()
    cl.allreduce_namespaces(n_ns, [c["o"].data_ptr() for c in csr], [c["s"].data_ptr() for c in csr],
                            [x.data_ptr() for x in oe], [x.data_ptr() for x in op],
                            [x.data_ptr() for x in ne], [x.data_ptr() for x in npw],
                            streams=[s] * world, comm_streams=[comm.cuda_stream] * world)
    torch.cuda.synchronize()
    e_o, p_o = ora.namespace_totals(*L.namespace_csr())
    assert np.count_nonzero(e_o) > 0 and np.count_nonzero(p_o) > 0
    for r in range(world):  # every shard holds the cluster result
        np.testing.assert_array_equal(oe[r].cpu().numpy().view(np.uint64), e_o, err_msg=f"shard {r}")
        np.testing.assert_allclose(op[r].cpu().numpy(), p_o, rtol=1e-12, atol=0, err_msg=f"shard {r}")
    # cluster node totals: Σ over every node of the unsharded tables
    st = ora.state
    want_e = np.concatenate([st[t].reshape(-1, Z).sum(axis=0, dtype=np.uint64)
                             for t in ("node_active_total", "node_idle_total")])
    want_p = np.concatenate([st[t].reshape(-1, Z).sum(axis=0)
                             for t in ("node_power", "node_active_power", "node_idle_power")])
    for r in range(world):
        np.testing.assert_array_equal(ne[r].cpu().numpy().view(np.uint64), want_e)
        np.testing.assert_allclose(npw[r].cpu().numpy(), want_p, rtol=1e-12, atol=0)

    # pod gather: every shard receives all pods in (shard, pod) order = the fleet's pod order
    slots = [to_device({"s": sl.pod_slot})["s"] for _, _, sl in shards]
    ge = [torch.zeros(L.n_pods * Z, dtype=torch.int64, device="cuda") for _ in range(world)]
    gp = [torch.zeros(L.n_pods * Z, dtype=torch.float64, device="cuda") for _ in range(world)]
    total, first = cl.gather_pods([sl.n_pods for _, _, sl in shards], [x.data_ptr() for x in slots], L.n_pods,
                                  [x.data_ptr() for x in ge], [x.data_ptr() for x in gp], streams=[s] * world)
    torch.cuda.synchronize()
    assert total == L.n_pods
    assert first == [int(L.pod_off[lo]) for lo, _, _ in shards]
    want_pe = st["pod_energy"].reshape(-1, Z)[L.pod_slot].reshape(-1)
    want_pp = st["pod_power"].reshape(-1, Z)[L.pod_slot].reshape(-1)
    for r in range(world):
        np.testing.assert_array_equal(ge[r].cpu().numpy().view(np.uint64), want_pe)
        np.testing.assert_array_equal(gp[r].cpu().numpy().view(np.uint64), want_pp.view(np.uint64))
    # a too-small output is refused, not overrun
    with pytest.raises(accel.AccelError) as ei:
        cl.gather_pods([sl.n_pods for _, _, sl in shards], [x.data_ptr() for x in slots], L.n_pods - 1,
                       [x.data_ptr() for x in ge], [x.data_ptr() for x in gp])
    assert ei.value.code == accel.KACC_ERANGE
    cl.close()


def test_batched_allreduce_matches_per_interval():
    """kacc_cluster_partials per interval into back-to-back [K][n_ns*Z + 2Z] / [K][n_ns*Z + 3Z]
    rows, then ONE kacc_allreduce_sums over all K intervals == kacc_allreduce_namespaces after
    each interval (bit-exact: the same shard partials, shard-order combine, the same collective)."""
    L = fleet.make_layout(40, [2000, 300, 0, 1, 700, 64, 1500, 9] * 5, 4, seed=43, n_namespaces=11,
                          shuffle_slots=True)
    world, K = 3, 4
    shards = shard.shard(L, world)
    cl = accel.Cluster.create_multi([0] * world, L.zones, [sl.capacities() for _, _, sl in shards])
    sim = fleet.FleetSim(L, seed=43, churn=0.04, read_error_frac=0.05)
    s = current_stream_handle()
    comm = torch.cuda.Stream()
    Z, n_ns = L.zones, L.n_namespaces
    csr = _namespace_csr_device([sl for _, _, sl in shards])
    ne, npw = n_ns * Z + 2 * Z, n_ns * Z + 3 * Z
    te = [torch.zeros(K, ne, dtype=torch.int64, device="cuda") for _ in range(world)]
    tp = [torch.zeros(K, npw, dtype=torch.float64, device="cuda") for _ in range(world)]
    ref = []
    keep = []
    for k in range(K):
        a = sim.next_interval()
        for (lo, hi, sl), acc in zip(shards, cl.shards):
            sub, sizes, _ = fleet.subset_interval(a, np.arange(lo, hi), L.zones)
            t = to_device(sub)
            keep.append(t)
            acc.run_interval(interval_from_tensors(t, sizes, sl.fast_flag()), s)
        r = ([torch.zeros(n_ns * Z, dtype=torch.int64, device="cuda") for _ in range(world)],
             [torch.zeros(n_ns * Z, dtype=torch.float64, device="cuda") for _ in range(world)],
             [torch.zeros(2 * Z, dtype=torch.int64, device="cuda") for _ in range(world)],
             [torch.zeros(3 * Z, dtype=torch.float64, device="cuda") for _ in range(world)])
        cl.allreduce_namespaces(n_ns, [c["o"].data_ptr() for c in csr], [c["s"].data_ptr() for c in csr],
                                *[[x.data_ptr() for x in v] for v in r], streams=[s] * world,
                                comm_streams=[comm.cuda_stream] * world)
        ref.append(r)
        cl.partials(n_ns, [c["o"].data_ptr() for c in csr], [c["s"].data_ptr() for c in csr],
                    [x[k].data_ptr() for x in te], [x[k].data_ptr() for x in tp],
                    [x[k, n_ns * Z:].data_ptr() for x in te], [x[k, n_ns * Z:].data_ptr() for x in tp],
                    streams=[s] * world)
    cl.allreduce_sums([x.data_ptr() for x in te], K * ne, [x.data_ptr() for x in tp], K * npw,
                      streams=[s] * world, comm_streams=[comm.cuda_stream] * world)
    torch.cuda.synchronize()
    for acc in cl.shards:
        acc.sync(s)
    for k in range(K):
        oe, op, nde, ndp = ref[k]
        for r in range(world):
            e, p = te[r][k].cpu().numpy(), tp[r][k].cpu().numpy()
            np.testing.assert_array_equal(e[:n_ns * Z], oe[r].cpu().numpy(), err_msg=f"interval {k} shard {r}")
            np.testing.assert_array_equal(e[n_ns * Z:], nde[r].cpu().numpy())
            np.testing.assert_array_equal(p[:n_ns * Z].view(np.uint64), op[r].cpu().numpy().view(np.uint64))
            np.testing.assert_array_equal(p[n_ns * Z:].view(np.uint64), ndp[r].cpu().numpy().view(np.uint64))
    assert np.count_nonzero(ref[-1][0][0].cpu().numpy()) > 0  # (the first interval is a first read: zeros)
    with pytest.raises(accel.AccelError) as ei:  # a missing shard vector is refused
        cl.allreduce_sums([te[0].data_ptr(), 0, te[2].data_ptr()], ne, [x.data_ptr() for x in tp], npw)
    assert ei.value.code == accel.KACC_EINVAL
    cl.close()


def test_cluster_join_one_rank():
    """The one-process-per-GPU entry (kacc_cluster_unique_id + kacc_cluster_join, what
    bench.py --gpus N uses) with a one-rank communicator == the context's own totals."""
    from oracle.oracle import Oracle

    L = fleet.make_layout(20, [500, 2000, 3, 0] * 5, 2, seed=5, n_namespaces=4)
    acc = accel.Accel(L.zones, **L.capacities())
    ora = Oracle(L.zones, **L.capacities())
    sim = fleet.FleetSim(L, seed=5)
    s = current_stream_handle()
    for _ in range(3):
        a = sim.next_interval()
        t = to_device(a)
        acc.run_interval(interval_from_tensors(t, L.sizes(), L.fast_flag()), s)
        ora.interval(a, L.sizes())
    acc.sync(s)
    cl = accel.Cluster.join(acc, accel.Cluster.unique_id(), 1, 0)
    assert cl.info() == (1, 0, 1)
    # the RCCL the collectives run with: major version of the build's headers, a real file
    import os
    version, path = accel.Cluster.rccl()
    print(f"RCCL {version} at {path}", flush=True)
    assert version // 10000 == 2 and os.path.exists(path)
    off, slots = L.namespace_csr()
    d = to_device({"o": off, "s": slots})
    Z = L.zones
    oe = torch.zeros(L.n_namespaces * Z, dtype=torch.int64, device="cuda")
    op = torch.zeros(L.n_namespaces * Z, dtype=torch.float64, device="cuda")
    cl.allreduce_namespaces(L.n_namespaces, [d["o"].data_ptr()], [d["s"].data_ptr()], [oe.data_ptr()],
                            [op.data_ptr()], streams=[s])
    torch.cuda.synchronize()
    e_o, p_o = ora.namespace_totals(off, slots)
    np.testing.assert_array_equal(oe.cpu().numpy().view(np.uint64), e_o)
    np.testing.assert_array_equal(op.cpu().numpy(), p_o)  # one shard: the namespace kernel's own order
    cl.close()
    acc.close()


@pytest.mark.timeout(900)
def test_config4_full_size_sharded_8_ways():
    """BASELINE config 4 at full size on one GPU: a 100k-node x 2k-process fleet (200M rows,
    Z = 4) cut 8 ways by plan_node_ranges into 8 contexts, 2 intervals.  Size-independent
    properties: every shard's tables == the unsharded context's tables at the same nodes /
    slots (sharding invariance, bit-exact); the all-reduced namespace totals == the
    unsharded context's (u64 exact, f64 <= 1e-12); oracle parity on a node sample."""
    from oracle.oracle import Oracle

    L = fleet.config_layout(4, nodes=100_000)
    Z = L.zones
    world = 8
    shards = shard.shard(L, world)
    assert [hi - lo for lo, hi, _ in shards] == [12_500] * 8
    full = accel.Accel(Z, **L.capacities())
    cl = accel.Cluster.create_multi([0] * world, Z, [sl.capacities() for _, _, sl in shards])
    sim = fleet.FleetSim(L, seed=44)
    rng = np.random.default_rng(4)
    sample = np.sort(rng.choice(L.n_nodes, 24, replace=False))
    ora = None
    s = current_stream_handle()
    for k in range(2):
        a = sim.next_interval()
        t = to_device(a)
        full.run_interval(interval_from_tensors(t, L.sizes(), L.fast_flag()), s)
        full.sync(s)
        del t
        for (lo, hi, sl), acc in zip(shards, cl.shards):
            sub, sizes, _ = fleet.subset_interval(a, np.arange(lo, hi), Z)
            ts = to_device(sub)
            acc.run_interval(interval_from_tensors(ts, sizes, sl.fast_flag()), s)
            acc.sync(s)
            del ts
        osub, osizes, omaps = fleet.subset_interval(a, sample, Z)
        if ora is None:
            ora = Oracle(Z, nodes=len(sample), proc_slots=osizes["n_procs"], ctr_slots=osizes["n_ctrs"],
                         vm_slots=osizes["n_vms"], pod_slots=osizes["n_pods"])
        ora.interval(osub, osizes)
        print(f"config4 interval {k} done", flush=True)
    # sharding invariance (slots are consecutive per node in config 4: shard slot i = slot p0 + i)
    for (lo, hi, sl), acc in zip(shards, cl.shards):
        base = {"node": lo, "proc": int(L.proc_off[lo]), "ctr": int(L.ctr_off[lo]), "vm": int(L.vm_off[lo]),
                "pod": int(L.pod_off[lo])}
        for name, _ in accel.TABLES:
            kind = name.split("_")[0]
            got = acc.download(name)
            if not len(got):
                continue
            n_rows = (hi - lo) if kind == "node" else sl.capacities()[f"{kind}_slots"]
            per = len(got) // n_rows
            want = full.download(name, base[kind] * per, len(got))
            if name in accel.NODE_INDEX_TABLES:  # shard-local node indices -> the fleet's
                got = got + lo
            np.testing.assert_array_equal(got, want, err_msg=f"shard [{lo},{hi}) {name}")
    # sampled oracle parity of the unsharded context
    for name, _ in accel.TABLES:
        kind = name.split("_")[0]
        cap = L.n_nodes if kind == "node" else L.capacities()[f"{kind}_slots"]
        per = full.table_info(name)[1] // cap
        got = _gather_rows(full, name, omaps[kind], per)
        want = ora.state[name]
        if name in accel.NODE_INDEX_TABLES:  # the sample's node indices -> the fleet's
            want = omaps["node"][want]
        np.testing.assert_array_equal(got, want, err_msg=name)
    # cluster namespace totals (RCCL path) == one context's namespace kernel
    n_ns = L.n_namespaces
    csr = _namespace_csr_device([sl for _, _, sl in shards])
    oe = [torch.zeros(n_ns * Z, dtype=torch.int64, device="cuda") for _ in range(world)]
    op = [torch.zeros(n_ns * Z, dtype=torch.float64, device="cuda") for _ in range(world)]
    cl.allreduce_namespaces(n_ns, [c["o"].data_ptr() for c in csr], [c["s"].data_ptr() for c in csr],
                            [x.data_ptr() for x in oe], [x.data_ptr() for x in op], streams=[s] * world)
    off, slots = L.namespace_csr()
    d = to_device({"o": off, "s": slots})
    fe = torch.zeros(n_ns * Z, dtype=torch.int64, device="cuda")
    fp = torch.zeros(n_ns * Z, dtype=torch.float64, device="cuda")
    full.namespace_totals(n_ns, d["o"].data_ptr(), d["s"].data_ptr(), fe.data_ptr(), fp.data_ptr(), s)
    torch.cuda.synchronize()
    for r in (0, world - 1):
        np.testing.assert_array_equal(oe[r].cpu().numpy(), fe.cpu().numpy())
        np.testing.assert_allclose(op[r].cpu().numpy(), fp.cpu().numpy(), rtol=1e-12, atol=0)
    cl.close()
    full.close()


def test_cluster_node_totals_follow_the_live_nodes():
    """Cluster node totals sum the nodes of the LAST interval run on the context: when a
    shard's batch shrinks, the nodes that left stop counting (Kepler: a node that is gone
    stops exporting, so PromQL's sum drops it), although their state rows are kept."""
    L = fleet.make_layout(12, [300, 40, 900, 5] * 3, 2, seed=9, n_namespaces=3)
    acc = accel.Accel(L.zones, **L.capacities())
    sim = fleet.FleetSim(L, seed=9)
    s = current_stream_handle()
    cl = accel.Cluster.join(acc, accel.Cluster.unique_id(), 1, 0)
    Z = L.zones
    ne = torch.zeros(2 * Z, dtype=torch.int64, device="cuda")
    npw = torch.zeros(3 * Z, dtype=torch.float64, device="cuda")

    def totals():
        cl.allreduce_namespaces(0, None, None, None, None, [ne.data_ptr()], [npw.data_ptr()], streams=[s])
        torch.cuda.synchronize()
        return ne.cpu().numpy().view(np.uint64).copy(), npw.cpu().numpy().copy()

    e0, p0 = totals()  # nothing run yet: zero
    assert not e0.any() and not p0.any()

    def want(n):
        st = {t: acc.download(t).reshape(-1, Z)[:n] for t in ("node_active_total", "node_idle_total", "node_power",
                                                            "node_active_power", "node_idle_power")}
        return (np.concatenate([st[t].sum(axis=0, dtype=np.uint64) for t in ("node_active_total", "node_idle_total")]),
                np.concatenate([st[t].sum(axis=0) for t in ("node_power", "node_active_power", "node_idle_power")]))

    for _ in range(3):
        t = to_device(sim.next_interval())
        acc.run_interval(interval_from_tensors(t, L.sizes(), L.fast_flag()), s)
    acc.sync(s)
    e, p = totals()
    we, wp = want(L.n_nodes)
    np.testing.assert_array_equal(e, we)
    np.testing.assert_allclose(p, wp, rtol=1e-12, atol=0)
    assert we.any()
    # the batch shrinks to its first 9 nodes
    keep = np.arange(9)
    sub, sizes, _ = fleet.subset_interval(sim.next_interval(), keep, Z)
    t = to_device(sub)
    acc.run_interval(interval_from_tensors(t, sizes, L.fast_flag()), s)
    acc.sync(s)
    e, p = totals()
    we, wp = want(9)
    np.testing.assert_array_equal(e, we)
    np.testing.assert_allclose(p, wp, rtol=1e-12, atol=0)
    assert not np.array_equal(we, want(L.n_nodes)[0])  # the 3 nodes that left counted before
    # the batch empties: no node counts any more (the early return of an empty
    # kacc_run_interval re-arms the live-node count too)
    acc.run_interval(accel.KaccInterval(), s)
    acc.sync(s)
    e, p = totals()
    assert not e.any() and not p.any()
    cl.close()
    acc.close()


def test_cluster_node_totals_back_to_back_launches():
    """The cluster node totals under back-to-back launches with no host sync: 24 intervals of
    changing node data, each followed by its partial sums into its own row.  20k nodes: past
    kColSplitFrom, so every column is split over 5 blocks whose partials the last-arriving
    block adds (and re-arms the arrival count for the next launch); a stale partial, a
    count left armed or a mixed-up total would show against the oracle."""
    from oracle.oracle import Oracle

    n, Z, K = 20000, 2, 24
    L = fleet.make_layout(n, [3, 1, 0, 2, 5] * (n // 5), Z, seed=21, n_namespaces=1)
    acc = accel.Accel(Z, **L.capacities())
    ora = Oracle(Z, **L.capacities())
    sim = fleet.FleetSim(L, seed=21, read_error_frac=0.02)
    s = current_stream_handle()
    cl = accel.Cluster.join(acc, accel.Cluster.unique_id(), 1, 0)
    ne = torch.zeros(K, 2 * Z, dtype=torch.int64, device="cuda")
    npw = torch.zeros(K, 3 * Z, dtype=torch.float64, device="cuda")
    want_e, want_p, keep = [], [], []
    for k in range(K):
        a = sim.next_interval()
        t = to_device(a)
        keep.append(t)
        acc.run_interval(interval_from_tensors(t, L.sizes(), L.fast_flag()), s)
        cl.partials(0, None, None, None, None, [ne[k].data_ptr()], [npw[k].data_ptr()], streams=[s])
        ora.interval(a, L.sizes())
        st = {x: ora.state[x].reshape(-1, Z) for x in ("node_active_total", "node_idle_total", "node_power",
                                                       "node_active_power", "node_idle_power")}
        want_e.append(np.concatenate([st[x].sum(axis=0, dtype=np.uint64)
                                      for x in ("node_active_total", "node_idle_total")]))
        want_p.append(np.concatenate([st[x].sum(axis=0) for x in ("node_power", "node_active_power",
                                                                  "node_idle_power")]))
    acc.sync(s)
    got_e = ne.cpu().numpy().view(np.uint64)
    got_p = npw.cpu().numpy()
    for k in range(K):
        np.testing.assert_array_equal(got_e[k], want_e[k], err_msg=f"interval {k}")
        np.testing.assert_allclose(got_p[k], want_p[k], rtol=1e-12, atol=0, err_msg=f"interval {k}")
    assert len({tuple(x) for x in want_e}) == K  # the data did change every interval
    cl.close()
    acc.close()


EXPORT_FLEETS = [
    ("fast-z4", dict(n_nodes=40, procs_per_node=[2000, 300, 1, 0, 1500] * 8, zones=4, shuffle_slots=True), 0),
    ("small-z2", dict(n_nodes=64, procs_per_node=[500, 64, 3, 0] * 16, zones=2), 0),
    ("big-z4", dict(n_nodes=6, procs_per_node=[10000, 3000, 12, 0, 2049, 700], zones=4, vm_frac=0.02,
                    procs_per_vm=2), 0),
    ("carry-z2", dict(n_nodes=48, procs_per_node=[1000, 700, 1, 0, 1024, 513] * 8, zones=2), 5),
]


@pytest.mark.parametrize("name,kw,K", EXPORT_FLEETS, ids=[f[0] for f in EXPORT_FLEETS])
def test_interval_exports_match_tables_and_totals(name, kw, K):
    """kacc_interval.pod_export / node_export, written by every kernel shape (workgroup per
    node, wavefront per node, big-node chunks + deferred pods, the K-interval carry kernel)
    == the state tables after the interval (a skipped node: its unchanged values; a pod with
    an out-of-range slot: zeros); kacc_allreduce_exports on the comm stream ==
    kacc_allreduce_namespaces from the tables, bit for bit (same sum order)."""
    L = fleet.make_layout(seed=19, **kw)
    Z = L.zones
    acc = accel.Accel(Z, **L.capacities())
    sim = fleet.FleetSim(L, seed=19, churn=0.03, read_error_frac=0.15, adversarial=0.1,
                         max_energy=fleet.MAX_ENERGY_FAKE)
    s = current_stream_handle()
    flags = L.fast_flag()
    if K:
        flags = (flags & ~accel.KACC_F_SMALL_NODES) | accel.KACC_F_NODE_SLOT_RANGES
    pex = [torch.zeros(max(L.n_pods, 1) * 2 * Z, dtype=torch.int64, device="cuda") for _ in range(max(K, 1))]
    nex = [torch.zeros(L.n_nodes * 5 * Z, dtype=torch.int64, device="cuda") for _ in range(max(K, 1))]
    keep = []
    for it in range(3):
        ivs = [sim.next_interval() for _ in range(max(K, 1))]
        if it == 2:  # a node skipped in the last interval (read error): exported unchanged
            ivs[-1]["node_status"] = ivs[-1]["node_status"] | np.where(np.arange(L.n_nodes) == 1, 1, 0).astype(np.uint32)
        descs = []
        for k, a in enumerate(ivs):
            t = to_device(a)
            t["pod_export"], t["node_export"] = pex[k], nex[k]
            keep.append(t)
            descs.append(interval_from_tensors(t, L.sizes(), flags))
        acc.run_intervals(descs, s)
        acc.sync(s)
    # the last interval's exports against the tables
    last = ivs[-1]
    pe = pex[-1].cpu().numpy().view(np.uint64).reshape(-1, 2 * Z)[: L.n_pods]
    ne = nex[-1].cpu().numpy().view(np.uint64).reshape(-1, 5 * Z)
    st = {t: acc.download(t) for t in ("pod_energy", "pod_power", "node_active_total", "node_idle_total",
                                       "node_power", "node_active_power", "node_idle_power")}
    slots = (last["pod_slot"] & np.uint32(accel.KACC_SLOT_MASK)).astype(np.int64)
    np.testing.assert_array_equal(pe[:, :Z], st["pod_energy"].reshape(-1, Z)[slots])
    np.testing.assert_array_equal(pe[:, Z:], st["pod_power"].reshape(-1, Z)[slots].view(np.uint64))
    want_ne = np.concatenate([st["node_active_total"].reshape(-1, Z), st["node_idle_total"].reshape(-1, Z)]
                             + [st[t].reshape(-1, Z).view(np.uint64) for t in ("node_power", "node_active_power",
                                                                                "node_idle_power")], axis=1)
    np.testing.assert_array_equal(ne, want_ne)
    assert last["node_status"][1] & accel.KACC_NODE_READ_ERROR  # a skipped node was exported too
    # cluster totals from the exports (comm stream) == from the tables
    cl = accel.Cluster.join(acc, accel.Cluster.unique_id(), 1, 0)
    n_ns = L.n_namespaces
    off, slots_ns = L.namespace_csr()
    _, rows_ns = L.namespace_csr_rows()
    d = to_device({"o": off, "s": slots_ns, "r": rows_ns})
    outs = [[torch.zeros(n, dtype=dt, device="cuda") for n, dt in ((n_ns * Z, torch.int64), (n_ns * Z, torch.float64),
                                                                  (2 * Z, torch.int64), (3 * Z, torch.float64))]
            for _ in range(2)]
    cl.allreduce_namespaces(n_ns, [d["o"].data_ptr()], [d["s"].data_ptr()], [outs[0][0].data_ptr()],
                            [outs[0][1].data_ptr()], [outs[0][2].data_ptr()], [outs[0][3].data_ptr()], streams=[s])
    comm = torch.cuda.Stream()
    cl.allreduce_exports(n_ns, [d["o"].data_ptr()], [d["r"].data_ptr()], [L.n_pods], [pex[-1].data_ptr()],
                         [outs[1][0].data_ptr()], [outs[1][1].data_ptr()], n_nodes=[L.n_nodes],
                         node_export=[nex[-1].data_ptr()], out_node_energy=[outs[1][2].data_ptr()],
                         out_node_power=[outs[1][3].data_ptr()], streams=[s], comm_streams=[comm.cuda_stream])
    torch.cuda.synchronize()
    acc.sync(s)
    for a_, b_ in zip(outs[0], outs[1]):
        np.testing.assert_array_equal(a_.cpu().numpy().view(np.uint64), b_.cpu().numpy().view(np.uint64))
    assert outs[0][0].abs().sum().item() > 0
    cl.close()
    acc.close()


def test_allreduce_exports_sharded_matches_tables():
    """Several shards on one GPU (kacc_create_multi): kacc_allreduce_exports (partials of
    every shard on the comm streams, combined, all-reduced) == kacc_allreduce_namespaces."""
    L = fleet.make_layout(48, [2000, 300, 1, 0, 700, 64] * 8, 4, seed=23, n_namespaces=11)
    world = 3
    shards = shard.shard(L, world)
    cl = accel.Cluster.create_multi([0] * world, L.zones, [sl.capacities() for _, _, sl in shards])
    Z = L.zones
    sim = fleet.FleetSim(L, seed=23, read_error_frac=0.1)
    s = current_stream_handle()
    comm = torch.cuda.Stream()
    pex = [torch.zeros(max(sl.n_pods, 1) * 2 * Z, dtype=torch.int64, device="cuda") for _, _, sl in shards]
    nex = [torch.zeros(sl.n_nodes * 5 * Z, dtype=torch.int64, device="cuda") for _, _, sl in shards]
    keep = []
    for _ in range(3):
        a = sim.next_interval()
        for r, ((lo, hi, sl), acc) in enumerate(zip(shards, cl.shards)):
            sub, sizes, _ = fleet.subset_interval(a, np.arange(lo, hi), Z)
            t = to_device(sub)
            t["pod_export"], t["node_export"] = pex[r], nex[r]
            keep.append(t)
            acc.run_interval(interval_from_tensors(t, sizes, sl.fast_flag()), s)
    n_ns = L.n_namespaces
    csr = [to_device({"o": sl.namespace_csr()[0], "s": sl.namespace_csr()[1], "r": sl.namespace_csr_rows()[1]})
           for _, _, sl in shards]
    mk = lambda n, dt: [torch.zeros(n, dtype=dt, device="cuda") for _ in range(world)]  # noqa: E731
    o_tab = [mk(n_ns * Z, torch.int64), mk(n_ns * Z, torch.float64), mk(2 * Z, torch.int64), mk(3 * Z, torch.float64)]
    o_exp = [mk(n_ns * Z, torch.int64), mk(n_ns * Z, torch.float64), mk(2 * Z, torch.int64), mk(3 * Z, torch.float64)]
    P = lambda xs: [x.data_ptr() for x in xs]  # noqa: E731
    cl.allreduce_namespaces(n_ns, [c["o"].data_ptr() for c in csr], [c["s"].data_ptr() for c in csr], *map(P, o_tab),
                            streams=[s] * world)
    cl.allreduce_exports(n_ns, [c["o"].data_ptr() for c in csr], [c["r"].data_ptr() for c in csr],
                         [sl.n_pods for _, _, sl in shards], P(pex), P(o_exp[0]), P(o_exp[1]),
                         n_nodes=[sl.n_nodes for _, _, sl in shards], node_export=P(nex),
                         out_node_energy=P(o_exp[2]), out_node_power=P(o_exp[3]), streams=[s] * world,
                         comm_streams=[comm.cuda_stream] * world)
    torch.cuda.synchronize()
    for acc in cl.shards:
        acc.sync(s)
    for a_, b_ in zip(o_tab, o_exp):
        for r in range(world):
            np.testing.assert_array_equal(a_[r].cpu().numpy().view(np.uint64), b_[r].cpu().numpy().view(np.uint64))
    cl.close()
