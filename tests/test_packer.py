"""Host packer (kacc_pack) — CPU.

1. The reference's own fixture, CreateTestResources (internal/monitor/
   mock_utils.go:227-391): six processes in /proc order, container-1 = {123,
   1231} in pod-1, container-2 = {456} without a pod, vm-1 / vm-2, one regular
   process; the packed batch then attributes through the oracle to the
   fixture's known CPU-time sums (container-1 40 %, container-2 20 %, pod-1
   40 %, vm-1 20 %, vm-2 5 % of the 200 s node total).
2. Round trip: the rows of a synthetic fleet (kepler_amd/fleet.py), handed
   over as records with VM and regular processes interleaved among the
   container processes (listing order kept per segment), pack back to
   exactly the fleet's layout.
3. Random nodes against an independent Python restatement (oracle/pack_ref):
   interleaved containers, pods shared by several containers, containers
   without a pod, VMs with several processes — bit-identical.
"""

import numpy as np
import pytest

from kepler_amd import accel, fleet
from oracle.pack_ref import pack_ref

E = accel.KACC_KEY_EMPTY
C, V, R = accel.KACC_PROC_CONTAINER, accel.KACC_PROC_VM, accel.KACC_PROC_REGULAR


def test_create_test_resources_fixture(oracle_lib):
    from oracle.oracle import Oracle

    node_delta = 200.0  # mock_utils.go:230 nodeCpuTimeDelta
    # procfs lists PIDs in ascending order
    pids = [123, 456, 789, 1001, 1002, 1231]
    frac = {123: 0.3, 1231: 0.1, 456: 0.20, 789: 0.15, 1001: 0.20, 1002: 0.05}
    delta = [frac[p] * node_delta for p in pids]
    types = [C, C, R, V, V, C]
    c1, c2, vm1, vm2, pod1 = 0xC1, 0xC2, 0xF1, 0xF2, 0xB1
    ctr = [c1, c2, 0, 0, 0, c1]
    vms = [0, 0, 0, vm1, vm2, 0]
    pods = [pod1, E, E, E, E, pod1]  # container-2 has no pod (mock_utils.go:269-274)
    p = accel.pack([0, 6], pids, delta, types, ctr, vms, pods, [0] * 6)
    assert (p["n_procs"], p["n_ctrs"], p["n_vms"], p["n_pods"]) == (6, 2, 2, 1)
    np.testing.assert_array_equal(p["proc_key"], [123, 1231, 456, 1001, 1002, 789])
    np.testing.assert_array_equal(p["row_record"], [0, 5, 1, 3, 4, 2])
    np.testing.assert_array_equal(p["ctr_key"], [c1, c2])  # pod-1's container first, ContainersNoPod last
    np.testing.assert_array_equal(p["ctr_proc_end"], [2, 3])
    np.testing.assert_array_equal(p["vm_key"], [vm1, vm2])
    np.testing.assert_array_equal(p["vm_proc_end"], [4, 5])
    np.testing.assert_array_equal(p["pod_key"], [pod1])
    np.testing.assert_array_equal(p["pod_ctr_end"], [1])
    # attribute the packed batch (usage 0.5, 100 J package per interval) through the oracle
    Z = 1
    o = Oracle(Z, nodes=1, proc_slots=6, ctr_slots=2, vm_slots=2, pod_slots=1)
    batch = {k: p[k] for k in ("proc_off", "ctr_off", "vm_off", "pod_off", "proc_cpu_delta", "ctr_proc_end",
                                "vm_proc_end", "pod_ctr_end")}
    for k, ts, e in ((0, 10**9, 10**9), (1, 6 * 10**9, 10**9 + 10**8)):
        flag = np.uint32(accel.KACC_SLOT_NEW) if k == 0 else np.uint32(0)
        batch.update(node_ts_ns=np.array([ts], np.int64), node_usage_ratio=np.array([0.5]),
                     node_status=np.zeros(1, np.uint32), zone_energy=np.array([e], np.uint64),
                     zone_max=np.array([10**12], np.uint64),
                     proc_slot=np.arange(6, dtype=np.uint32) | flag, ctr_slot=np.arange(2, dtype=np.uint32) | flag,
                     vm_slot=np.arange(2, dtype=np.uint32) | flag, pod_slot=np.arange(1, dtype=np.uint32) | flag)
        o.interval(batch, dict(n_nodes=1, n_procs=6, n_ctrs=2, n_vms=2, n_pods=1))
    st = o.state
    assert st["node_cpu_delta"][0] == node_delta
    assert list(st["ctr_cpu_delta"]) == [0.3 * node_delta + 0.1 * node_delta, 0.2 * node_delta]  # mock_utils.go:342-343
    assert list(st["pod_cpu_delta"]) == [0.3 * node_delta + 0.1 * node_delta]                   # :369
    assert list(st["vm_cpu_delta"]) == [0.2 * node_delta, 0.05 * node_delta]                    # :360-361
    # 100 J x 0.5 active = 50 J; container-1 gets 40 % of it (container.go:106-140)
    assert st["ctr_energy"][0] == 20 * 10**6 and st["ctr_energy"][1] == 10 * 10**6


def _records_from_layout(L: fleet.FleetLayout, seed: int):
    """The fleet's rows as informer records: per node the container rows in row order, with
    VM and regular rows interleaved at random positions (each segment keeps its order)."""
    rng = np.random.default_rng(seed)
    ctr_of_row = np.full(L.n_procs, -1, np.int64)
    vm_of_row = np.full(L.n_procs, -1, np.int64)
    for n in range(L.n_nodes):
        c0, c1 = int(L.ctr_off[n]), int(L.ctr_off[n + 1])
        prev = int(L.proc_off[n])
        for c in range(c0, c1):
            ctr_of_row[prev:int(L.ctr_proc_end[c])] = c
            prev = int(L.ctr_proc_end[c])
        for v in range(int(L.vm_off[n]), int(L.vm_off[n + 1])):
            vm_of_row[prev:int(L.vm_proc_end[v])] = v
            prev = int(L.vm_proc_end[v])
    pod_of_ctr = np.full(L.n_ctrs, -1, np.int64)
    for n in range(L.n_nodes):
        prev = int(L.ctr_off[n])
        for q in range(int(L.pod_off[n]), int(L.pod_off[n + 1])):
            pod_of_ctr[prev:int(L.pod_ctr_end[q])] = q
            prev = int(L.pod_ctr_end[q])
    order = []
    for n in range(L.n_nodes):
        rows = np.arange(int(L.proc_off[n]), int(L.proc_off[n + 1]))
        is_c = ctr_of_row[rows] >= 0
        cont, other = rows[is_c], rows[~is_c]
        # random merge of the two sequences, each keeping its order
        pick = np.zeros(rows.size, bool)
        pick[rng.choice(rows.size, cont.size, replace=False)] = True
        merged = np.empty(rows.size, np.int64)
        merged[pick], merged[~pick] = cont, other
        order.append(merged)
    rec_rows = np.concatenate(order) if order else np.zeros(0, np.int64)
    ptype = np.where(ctr_of_row[rec_rows] >= 0, C, np.where(vm_of_row[rec_rows] >= 0, V, R)).astype(np.uint8)
    ctr_key = np.where(ctr_of_row[rec_rows] >= 0, ctr_of_row[rec_rows] + 1000, 0).astype(np.uint64)
    vm_key = np.where(vm_of_row[rec_rows] >= 0, vm_of_row[rec_rows] + 10**7, 0).astype(np.uint64)
    q = np.where(ctr_of_row[rec_rows] >= 0, pod_of_ctr[np.maximum(ctr_of_row[rec_rows], 0)], -1)
    pod_key = np.where(q >= 0, q + 5 * 10**7, E).astype(np.uint64)
    pod_ns = np.where(q >= 0, L.pod_ns[np.maximum(q, 0)], 0).astype(np.uint32)
    pid = (rec_rows + 300).astype(np.uint32)
    delta = np.random.default_rng(seed + 1).random(L.n_procs)[rec_rows]
    return rec_rows, dict(rec_off=L.proc_off, pid=pid, cpu_delta=delta, ptype=ptype, ctr_key=ctr_key,
                          vm_key=vm_key, pod_key=pod_key, pod_ns=pod_ns)


@pytest.mark.parametrize("threads", [1, 5])
def test_fleet_layout_round_trip(threads):
    L = fleet.make_layout(30, [2000, 500, 1, 0, 64, 700] * 5, 4, seed=9, vm_frac=0.03, procs_per_vm=3)
    rec_rows, r = _records_from_layout(L, seed=4)
    p = accel.pack(threads=threads, **r)
    for k in ("proc_off", "ctr_off", "vm_off", "pod_off", "ctr_proc_end", "vm_proc_end", "pod_ctr_end"):
        np.testing.assert_array_equal(p[k], getattr(L, k), err_msg=k)
    np.testing.assert_array_equal(rec_rows[p["row_record"]], np.arange(L.n_procs))  # row r <- layout row r
    np.testing.assert_array_equal(p["proc_cpu_delta"], r["cpu_delta"][p["row_record"]])
    np.testing.assert_array_equal(p["ctr_key"], np.arange(L.n_ctrs) + 1000)
    np.testing.assert_array_equal(p["vm_key"], np.arange(L.n_vms) + 10**7)
    np.testing.assert_array_equal(p["pod_key"], np.arange(L.n_pods) + 5 * 10**7)
    np.testing.assert_array_equal(p["pod_ns"], L.pod_ns)


def random_records(n_nodes, seed, max_rows=400):
    rng = np.random.default_rng(seed)
    rows = rng.integers(0, max_rows, size=n_nodes)
    rows[::7] = 0
    rec_off = np.r_[0, np.cumsum(rows)].astype(np.uint32)
    Rn = int(rec_off[-1])
    ptype = rng.choice([R, C, C, C, V], size=Rn).astype(np.uint8)
    node = np.repeat(np.arange(n_nodes), rows)
    ctr_key = (node * 1000 + rng.integers(0, 25, size=Rn)).astype(np.uint64) * (ptype == C)
    vm_key = (node * 1000 + rng.integers(0, 4, size=Rn)).astype(np.uint64) * (ptype == V)
    # a container's pod: a function of the container (some have none)
    pod_of = lambda k: np.where(k % 5 == 0, E, (k // 3) * 7 + 11)  # noqa: E731
    pod_key = np.where(ptype == C, pod_of(ctr_key), E).astype(np.uint64)
    pod_ns = (pod_key % 13).astype(np.uint32)
    pid = rng.permutation(Rn).astype(np.uint32) + 1
    delta = rng.random(Rn) * 100
    return dict(rec_off=rec_off, pid=pid, cpu_delta=delta, ptype=ptype, ctr_key=ctr_key, vm_key=vm_key,
                pod_key=pod_key, pod_ns=pod_ns)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_nodes_match_python_restatement(seed):
    r = random_records(40, seed)
    p = accel.pack(threads=3, **r)
    want = pack_ref(r["rec_off"], r["pid"], r["cpu_delta"], r["ptype"], r["ctr_key"], r["vm_key"], r["pod_key"],
                    r["pod_ns"])
    for k, v in want.items():
        got = p[k]
        np.testing.assert_array_equal(got, v, err_msg=k)
        assert got.dtype == v.dtype or k.endswith("_off"), k


def test_capacity_and_bad_input():
    r = random_records(8, 5)
    p = accel.pack(**r)
    small = {n: np.zeros(max(p[n].size - (1 if n == "ctr_key" else 0), 1), dtype=dt)
             for n, dt in accel.PACKED_ARRAYS}
    for n in ("proc_off", "ctr_off", "vm_off", "pod_off"):
        small[n] = np.zeros(9, np.uint32)
    with pytest.raises(accel.AccelError) as ei:
        accel.pack(out=small, **r)
    assert ei.value.code == accel.KACC_ERANGE and "needs" in str(ei.value)
    bad = dict(r)
    bad["ptype"] = r["ptype"].copy()
    bad["ptype"][3] = 9
    with pytest.raises(accel.AccelError) as ei:
        accel.pack(**bad)
    assert "unknown process type" in str(ei.value)
