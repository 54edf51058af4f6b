"""Device slot join (kacc_slot_join) against the oracle — MI355X only.

Slot words are integer results: bit-exact against oracle/kor_join.cpp, which
is itself checked against a Go-map restatement on CPU (test_join_oracle.py).
The terminated list is a set (node segments land in any order; the
reference iterates a Go map, informer.go:206-212 / process.go:89): compared
sorted.  The end-to-end test feeds the joined slot words to the interval
kernel and checks every state table against the oracle fed the oracle's.
"""

import numpy as np
import pytest
import torch

from kepler_amd import accel, fleet
from table_check import LiveSlots, assert_tables_equal
from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device
from oracle.oracle import Oracle, OracleSlotMap

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu_ready():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    accel.load()
    torch.cuda.set_stream(torch.cuda.Stream())


class GpuJoin:
    def __init__(self, acc, kind, slot_off, policy=0):
        self.acc = acc
        self.kind = kind
        self.m = accel.SlotMap(acc, kind, slot_off)
        if policy:
            self.m.set_policy(policy)
        self.slot_off = slot_off
        cap = max(int(slot_off[-1]), 1)
        self.tk = torch.zeros(cap, dtype=torch.int64, device="cuda")
        self.ts = torch.zeros(cap, dtype=torch.int32, device="cuda")
        self.cnt = torch.zeros(max(len(slot_off) - 1, 1), dtype=torch.int32, device="cuda")
        self.span = torch.zeros(2 * max(len(slot_off) - 1, 1), dtype=torch.int32, device="cuda")

    def join(self, row_off, keys, status=None, out=None, sync=True):
        d_off = torch.from_numpy(row_off.astype(np.int32)).cuda()
        if self.kind == accel.KACC_KIND_PROC:  # PIDs are u32 keys
            d_keys = torch.from_numpy(keys.astype(np.uint32).view(np.int32)).cuda()
        else:
            d_keys = torch.from_numpy(keys.view(np.int64)).cuda()
        d_st = None if status is None else torch.from_numpy(status.astype(np.int32)).cuda()
        n_rows = int(row_off[-1])
        if out is None:
            out = torch.zeros(max(n_rows, 1), dtype=torch.int32, device="cuda")
        s = current_stream_handle()
        self.m.join(n_rows, d_off.data_ptr(), d_keys.data_ptr(), 0 if d_st is None else d_st.data_ptr(),
                    out.data_ptr(), self.tk.data_ptr(), self.ts.data_ptr(), self.cnt.data_ptr(), s,
                    self.span.data_ptr())
        if not sync:
            return out
        self.acc.sync(s)
        got = out[:n_rows].cpu().numpy().view(np.uint32)
        span = self.span.cpu().numpy().view(np.uint32)
        for n in range(len(self.slot_off) - 1):  # {min, max} slot of the node's rows
            if status is not None and status[n]:
                continue
            w = got[row_off[n]:row_off[n + 1]] & 0x7FFFFFFF
            want = (int(w.min()), int(w.max())) if w.size else (1, 0)
            assert (int(span[2 * n]), int(span[2 * n + 1])) == want, n
        tk = self.tk.cpu().numpy().view(np.uint64)
        ts = self.ts.cpu().numpy().view(np.uint32)
        term = []  # node segments, ascending by slot
        for n, c in enumerate(self.cnt.cpu().numpy()[: len(self.slot_off) - 1].tolist()):
            if status is not None and status[n]:
                continue
            s0 = int(self.slot_off[n])
            term += list(zip(tk[s0:s0 + c].tolist(), ts[s0:s0 + c].tolist()))
        return got, term


def caps_for(slot_off):
    n = int(slot_off[-1])
    return dict(nodes=len(slot_off) - 1, proc_slots=max(n, 1), ctr_slots=max(n, 1), vm_slots=1, pod_slots=1)


JOIN_FLEETS = [
    ("tiny", [0, 1, 2, 17, 64], 0.2, "proc"),
    ("config3-like", [2000] * 24, 0.02, "proc"),
    ("lds-edge", [2700, 2731, 2184, 1820], 0.05, "proc"),  # 4096-bucket LDS path boundary
    ("big-nodes", [10000, 50000, 3, 0, 12000], 0.03, "proc"),  # global-table path
    ("container-ids", [250, 180, 0, 520], 0.1, "ctr"),
]


@pytest.mark.parametrize("policy", [0, accel.KACC_JOIN_REUSE_TERMINATED], ids=["held", "reuse"])
@pytest.mark.parametrize("name,sizes,churn,kind", JOIN_FLEETS, ids=[f[0] for f in JOIN_FLEETS])
def test_join_bit_exact(name, sizes, churn, kind, policy):
    row_off = np.r_[0, np.cumsum(sizes)].astype(np.uint32)
    slot_off = np.r_[0, np.cumsum([int(s * 1.2) + 4 for s in sizes])].astype(np.uint32)
    acc = accel.Accel(1, **caps_for(slot_off))
    gpu = GpuJoin(acc, accel.KACC_KIND_PROC if kind == "proc" else accel.KACC_KIND_CTR, slot_off, policy)
    ora = OracleSlotMap(slot_off, policy)
    sim = fleet.KeyedChurn(row_off, seed=7, churn=churn, kind=kind)
    rng = np.random.default_rng(2)
    for it in range(5):
        keys = sim.next_keys()
        status = None
        if it >= 2:
            status = np.where(rng.random(len(sizes)) < 0.2, accel.KACC_NODE_READ_ERROR, 0).astype(np.uint32)
        rc, want, tk, ts, cnt = ora.join(row_off, keys, status)
        assert rc == 0
        want_term = ora.terminated(tk, ts, cnt)
        got, term = gpu.join(row_off, keys, status)
        if status is not None:  # rows of skipped nodes are not produced by either side
            keep = np.repeat(status == 0, np.diff(row_off.astype(np.int64)))
            got, want = got[keep], want[keep]
        np.testing.assert_array_equal(got, want, err_msg=f"interval {it}")
        assert term == want_term, f"interval {it}"


@pytest.fixture(params=[-1, 90623, 57855, 511], ids=["production", "cuckoo-shift", "cuckoo-1.5S", "round5-linear"])
def join_variant(request):
    """The production join (the cuckoo table), its A/B variant with a table of 1.5 S buckets, and
    round 5's linear-probing kernel (tools/bench_join_variants.py), set for the test's maps
    (kacc_debug_set_join_variant, read at reset)."""
    import ctypes

    lib = accel.load()
    lib.kacc_debug_set_join_variant.argtypes = [ctypes.c_int]
    lib.kacc_debug_set_join_variant.restype = ctypes.c_int
    prev = lib.kacc_debug_set_join_variant(request.param)
    yield request.param
    lib.kacc_debug_set_join_variant(prev)


@pytest.mark.parametrize("policy", [0, accel.KACC_JOIN_REUSE_TERMINATED], ids=["held", "reuse"])
@pytest.mark.parametrize("churn", [0.02, 0.1, 0.3])
def test_join_long_churn_bit_exact(churn, policy, join_variant):
    """30 intervals of churn, bit-exact every interval: at 2-10 % the small nodes take the
    one-wave tail (kJEasy) until tombstones crowd their tables, then one block-wide
    interval rebuilds them and the tail resumes; at 30 % the 2000-row nodes have more
    than 512 new rows per interval (block-wide path) and the small ones stay on the tail.
    Read errors skip nodes (their tables unchanged) every few intervals."""
    sizes = [2000, 2000, 1500, 300, 40, 0, 2700, 5, 2400, 64]
    row_off = np.r_[0, np.cumsum(sizes)].astype(np.uint32)
    # room for the held policy: rows + this interval's terminated (+ a skipped interval's)
    # slots; a 2000-row node stays on a 4096-bucket (LDS) table, 2400 / 2700 go global
    slot_off = np.r_[0, np.cumsum([int(s * 1.35) + 8 for s in sizes])].astype(np.uint32)
    acc = accel.Accel(1, **caps_for(slot_off))
    gpu = GpuJoin(acc, accel.KACC_KIND_PROC, slot_off, policy)
    ora = OracleSlotMap(slot_off, policy)
    sim = fleet.KeyedChurn(row_off, seed=11, churn=churn, kind="proc")
    rng = np.random.default_rng(5)
    for it in range(30):
        keys = sim.next_keys()
        status = None
        if it % 4 == 3 and churn <= 0.1:
            status = np.where(rng.random(len(sizes)) < 0.3, accel.KACC_NODE_READ_ERROR, 0).astype(np.uint32)
        rc, want, tk, ts, cnt = ora.join(row_off, keys, status)
        assert rc == 0
        want_term = ora.terminated(tk, ts, cnt)
        got, term = gpu.join(row_off, keys, status)
        if status is not None:
            keep = np.repeat(status == 0, np.diff(row_off.astype(np.int64)))
            got, want = got[keep], want[keep]
        np.testing.assert_array_equal(got, want, err_msg=f"interval {it}")
        assert term == want_term, f"interval {it}"


@pytest.mark.parametrize("policy", [0, accel.KACC_JOIN_REUSE_TERMINATED], ids=["held", "reuse"])
@pytest.mark.parametrize("churn", [0.02, 0.1])
def test_join_uniform_map_bit_exact(churn, policy, join_variant):
    """A map whose every node has a 4096-bucket table (1,100-2,000 rows, 1.3 x rows + 8
    slots: room for the held policy's terminated slots; the config-3 shape), where the production join loads each node's table before its
    node words (kJUni); 20 intervals of churn with read errors, bit-exact every interval."""
    rng = np.random.default_rng(17)
    sizes = rng.integers(1100, 2001, size=24).tolist()
    row_off = np.r_[0, np.cumsum(sizes)].astype(np.uint32)
    slot_off = np.r_[0, np.cumsum([s * 13 // 10 + 8 for s in sizes])].astype(np.uint32)
    acc = accel.Accel(1, **caps_for(slot_off))
    gpu = GpuJoin(acc, accel.KACC_KIND_PROC, slot_off, policy)
    ora = OracleSlotMap(slot_off, policy)
    sim = fleet.KeyedChurn(row_off, seed=23, churn=churn, kind="proc")
    for it in range(20):
        keys = sim.next_keys()
        status = None
        if it % 5 == 4:
            status = np.where(rng.random(len(sizes)) < 0.25, accel.KACC_NODE_READ_ERROR, 0).astype(np.uint32)
        rc, want, tk, ts, cnt = ora.join(row_off, keys, status)
        assert rc == 0
        want_term = ora.terminated(tk, ts, cnt)
        got, term = gpu.join(row_off, keys, status)
        if status is not None:
            keep = np.repeat(status == 0, np.diff(row_off.astype(np.int64)))
            got, want = got[keep], want[keep]
        np.testing.assert_array_equal(got, want, err_msg=f"interval {it}")
        assert term == want_term, f"interval {it}"


def test_join_errors_raise_erange():
    slot_off = np.array([0, 8, 10], dtype=np.uint32)
    acc = accel.Accel(1, **caps_for(slot_off))
    gpu = GpuJoin(acc, accel.KACC_KIND_PROC, slot_off)
    row_off = np.array([0, 3, 6], dtype=np.uint32)
    with pytest.raises(accel.AccelError) as ei:  # duplicate ID in node 0; 4 IDs for 2 slots... in node 1
        gpu.join(row_off, np.array([5, 5, 6, 1, 2, 3], dtype=np.uint64))
    assert ei.value.code == accel.KACC_ERANGE
    gpu.m.reset()
    with pytest.raises(accel.AccelError):  # reserved PID 0xffffffff
        gpu.join(row_off, np.array([1, 0xFFFFFFFF, 2, 1, 2, 3], dtype=np.uint64))
    gpu.m.reset()
    with pytest.raises(accel.AccelError):  # a new ID given twice
        gpu.join(np.array([0, 3, 3], dtype=np.uint32), np.array([9, 4, 9], dtype=np.uint64))
    gpu.m.reset()  # and a valid batch afterwards
    got, term = gpu.join(np.array([0, 3, 5], dtype=np.uint32), np.array([1, 2, 3, 7, 8], dtype=np.uint64))
    np.testing.assert_array_equal(got & 0x7FFFFFFF, [0, 1, 2, 8, 9])
    assert term == []


def test_join_found_duplicate_and_overfull_small_table():
    """The 6-B small-table PID join's own error paths: an ID already in the table given
    twice in one call (found twice: caught by counting the found rows against the held,
    not-terminated slots, then re-marked) and a small-table node (<= 4096 buckets) with
    more rows than join_small holds (3100 > its 2700 slots: ERANGE in join_small, never
    join_big)."""
    slot_off = np.array([0, 100, 2800], dtype=np.uint32)  # node 1: 2700 slots, 4096 buckets
    acc = accel.Accel(1, **caps_for(slot_off))
    gpu = GpuJoin(acc, accel.KACC_KIND_PROC, slot_off)
    ora = OracleSlotMap(slot_off, 0)
    row_off = np.array([0, 50, 2050], dtype=np.uint32)
    keys = np.r_[np.arange(1, 51), np.arange(1000, 3000)].astype(np.uint64)
    rc, want, _, _, _ = ora.join(row_off, keys, None)
    assert rc == 0
    got, term = gpu.join(row_off, keys)
    np.testing.assert_array_equal(got, want)
    dup = np.r_[np.arange(1, 51), [7], np.arange(1000, 3000)].astype(np.uint64)  # 7 found twice
    with pytest.raises(accel.AccelError) as ei:
        gpu.join(np.array([0, 51, 2051], dtype=np.uint32), dup)
    assert ei.value.code == accel.KACC_ERANGE
    gpu.m.reset()
    big = np.r_[np.arange(1, 51), np.arange(5000, 8100)].astype(np.uint64)  # node 1: 3100 rows
    with pytest.raises(accel.AccelError) as ei:
        gpu.join(np.array([0, 50, 3150], dtype=np.uint32), big)
    assert ei.value.code == accel.KACC_ERANGE
    gpu.m.reset()  # and the same valid batch afterwards, from empty tables
    ora = OracleSlotMap(slot_off, 0)
    rc, want, _, _, _ = ora.join(row_off, keys, None)
    got, term = gpu.join(row_off, keys)
    np.testing.assert_array_equal(got, want)
    assert term == []


@pytest.mark.parametrize("kind", [accel.KACC_KIND_CTR, accel.KACC_KIND_POD])
def test_join_overfull_small_table_u64_kinds(kind):
    """A small-table node (<= 4096 buckets) with more rows than join_small holds, for
    the u64-keyed kinds of a map with no big node (join_big is never launched): the
    call raises ERANGE and the node's slot words are written invalid — none is left
    stale — and the map still joins a valid batch afterwards."""
    slot_off = np.array([0, 100, 2800], dtype=np.uint32)  # node 1: 2700 slots, 4096 buckets
    acc = accel.Accel(1, nodes=2, proc_slots=1, ctr_slots=2800, vm_slots=1, pod_slots=2800)
    gpu = GpuJoin(acc, kind, slot_off)
    big = np.r_[np.arange(1, 51), np.arange(5000, 8100)].astype(np.uint64)  # node 1: 3100 rows
    out = torch.full((3150,), 0x1234, dtype=torch.int32, device="cuda")
    with pytest.raises(accel.AccelError) as ei:
        gpu.join(np.array([0, 50, 3150], dtype=np.uint32), big, out=out)
    assert ei.value.code == accel.KACC_ERANGE
    words = out.cpu().numpy().view(np.uint32)
    assert (words[50:] == 0xFFFFFFFF).all()  # join_small's invalid word on every row of node 1
    assert int(gpu.cnt[1].item()) == 0
    gpu.m.reset()
    ora = OracleSlotMap(slot_off, 0)
    row_off = np.array([0, 50, 2050], dtype=np.uint32)
    keys = np.r_[np.arange(1, 51), np.arange(1000, 3000)].astype(np.uint64)
    rc, want, _, _, _ = ora.join(row_off, keys, None)
    assert rc == 0
    got, term = gpu.join(row_off, keys)
    np.testing.assert_array_equal(got, want)
    assert term == []


@pytest.mark.parametrize("churn_model", ["keyed", "proc"])
@pytest.mark.parametrize("policy", [0, accel.KACC_JOIN_REUSE_TERMINATED], ids=["held", "reuse"])
def test_join_feeds_interval_bit_exact(policy, churn_model):
    """Keyed fleet: device join -> interval kernel == oracle join -> oracle interval.
    churn_model "proc": /proc-shaped churn (fleet.ProcChurn: newcomers listed last in
    their container), the layout the reuse policy keeps near row order."""
    layout = fleet.make_layout(12, [1500, 2000, 40, 0, 700, 2048] * 2, 4, seed=21)
    sizes = layout.sizes()
    P = layout.n_procs
    proc_slot_off = np.r_[0, np.cumsum(np.diff(layout.proc_off.astype(np.int64)) * 5 // 4 + 8)].astype(np.uint32)
    caps = layout.capacities()
    caps["proc_slots"] = int(proc_slot_off[-1])
    acc = accel.Accel(layout.zones, **caps)
    gpu = GpuJoin(acc, accel.KACC_KIND_PROC, proc_slot_off, policy)
    ojoin = OracleSlotMap(proc_slot_off, policy)
    ora = Oracle(layout.zones, **caps)
    sim = fleet.FleetSim(layout, seed=21, churn=0.0, read_error_frac=0.1)
    keys_sim = (fleet.KeyedChurn(layout.proc_off, seed=21, churn=0.04) if churn_model == "keyed"
                else fleet.ProcChurn(layout, churn=0.04, seed=21))
    stream = current_stream_handle()
    live = LiveSlots(proc_slot_off)
    for it in range(4):
        a = sim.next_interval()
        keys = keys_sim.next_keys()
        # CPU deltas restart for new IDs (informer.go:518: prevTotal 0 for a new PID)
        _, want_slots, _, _, _ = ojoin.join(layout.proc_off, keys, a["node_status"])
        live.update(layout.proc_off, want_slots, a["node_status"])
        a_ora = dict(a)
        a_ora["proc_slot"] = want_slots
        t = to_device(a)
        out = t["proc_slot"]  # the join writes the batch's slot words in place
        gpu.join(layout.proc_off, keys, a["node_status"], out=out, sync=False)
        t["node_proc_span"] = gpu.span  # rows swept in slot order
        acc.run_interval(interval_from_tensors(t, sizes, layout.fast_flag()), stream)
        acc.sync(stream)
        ora.interval(a_ora, sizes)
        # terminated slots left the batch: their derived power is not compared (table_check.py)
        assert_tables_equal(acc.download, ora.state, f"interval {it}", live=live, zones=layout.zones)
    assert P > 0
