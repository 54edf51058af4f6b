"""Host logic: fleet layout invariants, node subsets, sharding plan (CPU)."""

import numpy as np
import pytest

from kepler_amd import accel, fleet, shard


def check_layout(L):
    """Python restatement of kacc_validate_host's layout rules."""
    for off, n in ((L.proc_off, L.n_procs), (L.ctr_off, L.n_ctrs), (L.vm_off, L.n_vms), (L.pod_off, L.n_pods)):
        assert off[0] == 0 and off[-1] == n and np.all(np.diff(off.astype(np.int64)) >= 0)
    for nd in range(L.n_nodes):
        p0, p1 = L.proc_off[nd], L.proc_off[nd + 1]
        prev = p0
        for c in range(L.ctr_off[nd], L.ctr_off[nd + 1]):
            assert prev < L.ctr_proc_end[c] <= p1  # every container has >= 1 process
            prev = L.ctr_proc_end[c]
        for v in range(L.vm_off[nd], L.vm_off[nd + 1]):
            assert prev < L.vm_proc_end[v] <= p1
            prev = L.vm_proc_end[v]
        cprev = L.ctr_off[nd]
        for q in range(L.pod_off[nd], L.pod_off[nd + 1]):
            assert cprev < L.pod_ctr_end[q] <= L.ctr_off[nd + 1]
            cprev = L.pod_ctr_end[q]
    for s in (L.proc_slot, L.ctr_slot, L.vm_slot, L.pod_slot):
        assert len(np.unique(s)) == len(s)


@pytest.mark.parametrize("cfg", [1, 2, 5])
def test_config_layouts(cfg):
    L = fleet.config_layout(cfg, nodes=50 if cfg != 1 else None)
    check_layout(L)


def test_config3_shape():
    L = fleet.config_layout(3, nodes=100)
    assert L.n_procs == 100 * 2000 and L.zones == 4
    per = L.sizes()
    assert per["n_ctrs"] == 100 * 197 and per["n_vms"] == 100 * 20
    check_layout(L)


def test_edge_layouts():
    check_layout(fleet.make_layout(6, [0, 1, 2, 9, 10, 100], 3, shuffle_slots=True, procs_per_vm=2, vm_frac=0.2))


def test_subset_matches_full_fleet(oracle_lib):
    from oracle.oracle import Oracle

    L = fleet.make_layout(12, [50, 0, 300, 7, 128, 1, 64, 900, 33, 2, 500, 20], 2, seed=4, shuffle_slots=True)
    sim = fleet.FleetSim(L, seed=4, churn=0.1, read_error_frac=0.1)
    full = Oracle(L.zones, **L.capacities())
    nodes = np.array([0, 2, 5, 7, 11])
    sub = None
    for _ in range(3):
        a = sim.next_interval()
        full.interval(a, L.sizes())
        s, sizes, maps = fleet.subset_interval(a, nodes, L.zones)
        if sub is None:
            sub = Oracle(L.zones, nodes=len(nodes), proc_slots=max(sizes["n_procs"], 1),
                         ctr_slots=max(sizes["n_ctrs"], 1), vm_slots=max(sizes["n_vms"], 1),
                         pod_slots=max(sizes["n_pods"], 1))
        sub.interval(s, sizes)
    for name in full.state.t:
        kind = name.split("_")[0]
        f = full.state[name]
        per = len(f) // (L.n_nodes if kind == "node" else L.capacities()[f"{kind}_slots"])
        got = f.reshape(-1, per)[maps[kind]].reshape(-1)
        want = sub.state[name][: len(got)]
        if name in accel.NODE_INDEX_TABLES:  # node indices of the subset -> the fleet's
            want = maps["node"][want]
        np.testing.assert_array_equal(got, want, err_msg=name)


def test_plan_node_ranges_balanced():
    rng = np.random.default_rng(1)
    p = rng.pareto(1.5, 1000) * 1000 + 10
    for world in (1, 2, 4, 8):
        b = shard.plan_node_ranges(p, world)
        assert b[0] == 0 and b[-1] == 1000 and np.all(np.diff(b) >= 0)
        loads = np.array([p[b[r]:b[r + 1]].sum() for r in range(world)])
        assert loads.max() <= p.sum() / world + p.max()


def test_shards_reproduce_full_fleet(oracle_lib):
    """Node-sharded computation == whole-fleet computation (no cross-shard data)."""
    from oracle.oracle import Oracle

    L = fleet.make_layout(20, [100, 400, 3, 0, 250] * 4, 2, seed=8, shuffle_slots=True, n_namespaces=5)
    sim = fleet.FleetSim(L, seed=8, churn=0.05)
    full = Oracle(L.zones, **L.capacities())
    parts = shard.shard(L, 3)
    ors = [Oracle(L.zones, **sl.capacities()) for _, _, sl in parts]
    for _ in range(3):
        a = sim.next_interval()
        full.interval(a, L.sizes())
        for (lo, hi, sl), o in zip(parts, ors):
            s, sizes, _ = fleet.subset_interval(a, np.arange(lo, hi), L.zones)
            o.interval(s, sizes)
    # namespace totals: sum of per-shard partials == whole-fleet totals (u64 exact)
    e_full, p_full = full.namespace_totals(*L.namespace_csr())
    e_sum = np.zeros_like(e_full)
    p_sum = np.zeros_like(p_full)
    for (_, _, sl), o in zip(parts, ors):
        e, p = o.namespace_totals(*sl.namespace_csr())
        e_sum += e
        p_sum += p
    np.testing.assert_array_equal(e_sum, e_full)
    np.testing.assert_allclose(p_sum, p_full, rtol=1e-12)


def test_namespace_order_close_to_list_order(oracle_lib):
    from oracle.oracle import Oracle

    L = fleet.make_layout(30, 700, 4, seed=2, n_namespaces=3)
    sim = fleet.FleetSim(L, seed=2)
    o = Oracle(L.zones, **L.capacities())
    for _ in range(3):
        o.interval(sim.next_interval(), L.sizes())
    off, slots = L.namespace_csr()
    e, p = o.namespace_totals(off, slots)
    pe = o.state["pod_energy"].reshape(-1, L.zones)
    pp = o.state["pod_power"].reshape(-1, L.zones)
    for k in range(len(off) - 1):
        sl = slots[off[k]:off[k + 1]]
        assert np.array_equal(e.reshape(-1, L.zones)[k], pe[sl].sum(axis=0, dtype=np.uint64))
        ref = np.array([sum(pp[s, z] for s in sl) for z in range(L.zones)])
        np.testing.assert_allclose(p.reshape(-1, L.zones)[k], ref, rtol=1e-12)


def test_proc_churn_model_keeps_groups_and_listing_order():
    """ProcChurn: PIDs unique per node, ascending inside every container / VM / rest group
    (/proc listing order), the CSR fixed; with KACC_JOIN_REUSE_TERMINATED the oracle join
    keeps every node on exactly its first `rows` slots."""
    from oracle.oracle import OracleSlotMap

    layout = fleet.make_layout(6, [300, 1000, 40, 0, 2000, 7], 2, seed=4)
    off = layout.proc_off.astype(np.int64)
    ch = fleet.ProcChurn(layout, churn=0.05, seed=3)
    rows = np.diff(off)
    slot_off = np.r_[0, np.cumsum(rows + 4)].astype(np.uint32)
    join = OracleSlotMap(slot_off, policy=1)
    ends = np.unique(np.concatenate([layout.ctr_proc_end, layout.vm_proc_end, off[1:]]).astype(np.int64))
    starts = np.r_[0, ends[:-1]]
    changed = 0
    prev = None
    for _ in range(12):
        keys = ch.next_keys()
        for n in range(layout.n_nodes):
            assert len(np.unique(keys[off[n]:off[n + 1]])) == rows[n]
        for a, b in zip(starts, ends):
            assert np.all(np.diff(keys[a:b].astype(np.int64)) > 0)
        if prev is not None:
            changed += int(np.sum(~np.isin(keys, prev)))
        prev = keys
        rc, out, _, _, _ = join.join(layout.proc_off, keys)
        assert rc == 0
        for n in range(layout.n_nodes):
            s = np.sort((out[off[n]:off[n + 1]] & 0x7FFFFFFF) - slot_off[n])
            np.testing.assert_array_equal(s, np.arange(rows[n]))
    assert 0.03 < changed / (11 * off[-1]) < 0.07
