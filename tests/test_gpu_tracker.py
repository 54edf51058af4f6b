"""Device TerminatedResourceTracker (kacc_tracker_*) — MI355X only.

1. The reference's own tracker tests (tracker_kats.json, one Add() = one batch
   of one terminated workload) through the C ABI.
2. Whole fleets: slot join -> interval -> tracker on the device against the
   oracle join -> oracle interval -> Go-heap tracker fed the same batches in
   the device's map order; the retained sets (IDs and frozen energy / power)
   must be identical.  Energies are wide-range u64, so the retention boundary
   is untied and every Go map order gives this set.
"""

import numpy as np
import pytest
import torch

from kepler_amd import accel, fleet
from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device
from oracle.oracle import Oracle, OracleSlotMap, OracleTracker
from tracker_runner import check, key_of, load_tracker_kats

pytestmark = pytest.mark.gpu

KATS = load_tracker_kats()


@pytest.fixture(scope="module", autouse=True)
def gpu_ready():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    accel.load()
    torch.cuda.set_stream(torch.cuda.Stream())


@pytest.mark.parametrize("case", KATS["cases"], ids=[c["name"] for c in KATS["cases"]])
def test_tracker_kat_on_device(case):
    Z = KATS["zones"]
    adds = [s for s in case["steps"] if s["op"] == "add"]
    S = max(len(adds), 1)
    acc = accel.Accel(Z, nodes=1, proc_slots=S, ctr_slots=1, vm_slots=1, pod_slots=1)
    sm = accel.SlotMap(acc, accel.KACC_KIND_PROC, np.array([0, S], dtype=np.uint32))
    tr = accel.Tracker(acc, accel.KACC_KIND_PROC, case["max_size"], zone=0, min_energy=case["min_energy"],
                       capacity=256)
    tk = torch.zeros(S, dtype=torch.int64, device="cuda")
    ts = torch.zeros(S, dtype=torch.int32, device="cuda")
    tc = torch.ones(1, dtype=torch.int32, device="cuda")
    ids, slot = {}, 0
    s = current_stream_handle()
    for st in case["steps"]:
        if st["op"] == "clear":
            tr.clear(s)
            continue
        acc.upload("proc_energy", np.array(st["energy"], dtype=np.uint64), slot * Z)
        tk[0] = key_of(ids, st["id"])
        ts[0] = slot
        tr.add(sm, tk.data_ptr(), ts.data_ptr(), tc.data_ptr(), s)
        slot += 1
    acc.sync(s)
    k, nd, e, _ = tr.items()
    assert np.all(nd == 0)
    check(case, {int(kk): ee for kk, ee in zip(k, e)}, ids)
    # highest energy first
    assert np.all(np.diff(e[:, 0].astype(np.float64)) <= 0) if len(k) > 1 else True


FLEETS = [
    ("small", [40, 0, 300, 7, 1000, 64], 2, 0.1, 25),
    ("many-nodes-top3", [60, 200, 5, 0, 90, 400] * 6, 2, 0.1, 3),
    ("config3-like", [2000] * 16, 4, 0.02, 500),
    ("unlimited", [500, 200, 1500], 2, 0.05, -1),
    ("big-node", [12000, 300, 2500], 4, 0.03, 200),
    ("five-zones", [700, 300, 1300], 5, 0.05, 100),  # the kernel instance that carries 8 zones
    ("config3-shape-1k-nodes", [2000] * 1000, 4, 0.02, 500),  # 2M rows: the production pipeline's scale per node
]


@pytest.mark.parametrize("concurrent", [False, True, "reuse"],
                         ids=["one-stream", "tracker-second-stream", "reuse-tracker-first"])
@pytest.mark.parametrize("name,sizes,Z,churn,max_size", FLEETS, ids=[f[0] for f in FLEETS])
def test_tracker_fleet_matches_go_heap(name, sizes, Z, churn, max_size, concurrent):
    """One tracker per node (every node's PowerMonitor owns one): each node keeps its own top
    max_size, against one Go heap per node.  The tracker adds an interval's terminated batch
    after the join and BEFORE the interval kernel, as calculateProcessPower does
    (process.go:87-99 precede :118-148): a process's power is derived from its ratio and its
    node's tables (kacc_derive.hpp), which the interval rewrites.  concurrent: the tracker
    runs on a second stream (the interval waits for it) and clears only the odd nodes (a
    per-node export); otherwise every node.  "reuse": the join hands terminated slots to new
    rows at once (KACC_JOIN_REUSE_TERMINATED)."""
    reuse = concurrent == "reuse"
    concurrent = concurrent is True
    layout = fleet.make_layout(len(sizes), sizes, Z, seed=31)
    sizes_d = layout.sizes()
    rows = np.diff(layout.proc_off.astype(np.int64))
    slot_off = np.r_[0, np.cumsum(rows * 5 // 4 + 8)].astype(np.uint32)
    caps = layout.capacities()
    caps["proc_slots"] = int(slot_off[-1])
    acc = accel.Accel(Z, **caps)
    sm = accel.SlotMap(acc, accel.KACC_KIND_PROC, slot_off)
    if reuse:
        sm.set_policy(accel.KACC_JOIN_REUSE_TERMINATED)
    thr = 2 * 10**6  # 2 J
    tr = accel.Tracker(acc, accel.KACC_KIND_PROC, max_size, zone=0, min_energy=thr, capacity=200_000)
    ojoin, ora = OracleSlotMap(slot_off, int(reuse)), Oracle(Z, **caps)
    otr = OracleTracker(max_size, thr, Z, 0)
    sim = fleet.FleetSim(layout, seed=31, churn=0.0, read_error_frac=0.05)
    keys_sim = (fleet.ProcChurn(layout, churn=churn, seed=31) if reuse  # the production pairing
                else fleet.KeyedChurn(layout.proc_off, seed=31, churn=churn))
    cap = int(slot_off[-1])
    tk = torch.zeros(cap, dtype=torch.int64, device="cuda")
    ts = torch.zeros(cap, dtype=torch.int32, device="cuda")
    tc = torch.zeros(layout.n_nodes, dtype=torch.int32, device="cuda")
    span = torch.zeros(2 * layout.n_nodes, dtype=torch.int32, device="cuda")
    s = current_stream_handle()
    s2 = torch.cuda.Stream()
    ts2 = s2.cuda_stream if concurrent else s
    for it in range(6):
        a = sim.next_interval()
        keys = keys_sim.next_keys()
        rc, want_slots, otk, ots, ocnt = ojoin.join(layout.proc_off, keys, a["node_status"])
        assert rc == 0
        a_ora = dict(a)
        a_ora["proc_slot"] = want_slots
        t = to_device(a)
        d_keys = torch.from_numpy(keys.astype(np.uint32).view(np.int32)).cuda()
        sm.join(layout.n_procs, t["proc_off"].data_ptr(), d_keys.data_ptr(), t["node_status"].data_ptr(),
                t["proc_slot"].data_ptr(), tk.data_ptr(), ts.data_ptr(), tc.data_ptr(), s, span.data_ptr())
        t["node_proc_span"] = span
        if concurrent:  # the tracker waits for the join only
            joined = torch.cuda.Event()
            joined.record(torch.cuda.current_stream())
            s2.wait_event(joined)
        if it == 3:  # an export happened: Clear() before this interval's adds (process.go:80-84)
            if concurrent:  # only the odd nodes exported
                mask = (np.arange(layout.n_nodes) % 2).astype(np.int32)
                d_mask = torch.from_numpy(mask).cuda()
                tr.clear(ts2, d_mask.data_ptr())
                otr.clear(np.flatnonzero(mask))
            else:
                tr.clear(ts2)
                otr.clear()
        tr.add(sm, tk.data_ptr(), ts.data_ptr(), tc.data_ptr(), ts2)
        if concurrent:  # the interval (and the next join) after the tracker's reads
            torch.cuda.current_stream().wait_stream(s2)
        acc.run_interval(interval_from_tensors(t, sizes_d, layout.fast_flag()), s)
        acc.sync(s)
        # the oracle tracker reads the same final values: the tables before this interval
        pre_e, pre_p = ora.state["proc_energy"].copy(), ora.state["proc_power"].copy()
        ora.interval(a_ora, sizes_d)
        # oracle: the same terminated batch (per-node segments), values from the oracle tables
        nodes, kk, ss = [], [], []
        for n, c in enumerate(ocnt.tolist()):
            s0 = int(slot_off[n])
            nodes += [n] * c
            kk += otk[s0:s0 + c].tolist()
            ss += ots[s0:s0 + c].tolist()
        otr.add_batch(nodes, kk, ss, pre_e, pre_p)
        gk, gn, ge, gp = tr.items()
        order = np.lexsort((gk, gn))
        ok_, on_, oe_, op_ = otr.items()
        assert gk.size == ok_.size, (it, gk.size, ok_.size)
        np.testing.assert_array_equal(gn[order], on_, err_msg=f"interval {it}")
        np.testing.assert_array_equal(gk[order], ok_, err_msg=f"interval {it}")
        np.testing.assert_array_equal(ge[order], oe_, err_msg=f"interval {it}")
        np.testing.assert_array_equal(gp[order], op_, err_msg=f"interval {it}")
