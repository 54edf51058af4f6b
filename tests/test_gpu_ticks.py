"""CPU-tick input format on the device (kacc_tickmap / kacc_ticks_delta) — MI355X only.

Per interval the host sends each process row's tick increment (u16, escapes as int64) and the
device writes Go's CPUTimeDelta into the batch's proc_cpu_delta from its per-slot tick map.  The
expected Δ is the informer's own arithmetic (populateProcessFields, informer.go:512-524;
procWrapper.CPUTime, procfs_reader.go:75-82) kept on the host per row; the Δ must be bit-exact,
and the interval fed with the device's Δ must leave every state table bit-exact against the
oracle fed with Go's Δ.  Cases: first readings (NEW) of long-lived processes (big tick counts,
escapes), 16-bit overflow, negative increments (a reused PID in a cached entry), u64 tick
wrap, ticks past 2^53 (float64 rounds them), read-error nodes (Refresh skipped: neither the
informer nor the tick map moves), and churn (a NEW row of a reused slot starts from 0).
"""

import numpy as np
import pytest
import torch

from kepler_amd import accel, fleet
from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device
from oracle.oracle import Oracle
from table_check import assert_tables_equal

pytestmark = pytest.mark.gpu

U64 = np.uint64((1 << 64) - 1)


@pytest.fixture(scope="module", autouse=True)
def gpu_ready():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    accel.load()
    torch.cuda.set_stream(torch.cuda.Stream())


def _readings(rng, prev, new, k):
    """This interval's cumulative ticks per row (u64)."""
    P = prev.size
    inc = rng.integers(0, 2500, size=P).astype(np.int64)
    inc[rng.random(P) < 0.05] = 0
    big = rng.random(P) < 0.02
    inc[big] = rng.integers(0xFFFF, 5 * 10**6, size=int(big.sum()))
    back = rng.random(P) < 0.01  # a reused PID in a cached entry: the new process has fewer ticks
    now = prev + inc.astype(np.uint64)
    now[back] = prev[back] // np.uint64(3)
    first = np.where(new)[0]  # a process's first reading: everything it ran so far
    long_lived = rng.random(first.size) < 0.3
    now[first] = rng.integers(0, 60000, size=first.size).astype(np.uint64)
    now[first[long_lived]] = rng.integers(1 << 33, 1 << 60, size=int(long_lived.sum()), dtype=np.uint64)
    if k == 0:  # a few counters about to wrap, some past 2^53
        w = rng.choice(P, size=max(P // 200, 1), replace=False)
        now[w] = U64 - rng.integers(0, 4000, size=w.size).astype(np.uint64)
        b = rng.choice(P, size=max(P // 200, 1), replace=False)
        now[b] = rng.integers(1 << 53, 1 << 62, size=b.size, dtype=np.uint64)
    return now


def test_ticks_delta_matches_go_and_feeds_the_interval():
    L = fleet.make_layout(30, [2000, 700, 1, 0, 1500, 64] * 5, 4, seed=13, n_namespaces=5)
    Z, P, N = L.zones, L.n_procs, L.n_nodes
    acc = accel.Accel(Z, **L.capacities())
    tm = accel.TickMap(acc)
    ora = Oracle(Z, **L.capacities())
    sim = fleet.FleetSim(L, seed=13, read_error_frac=0.15, churn=0.03)
    rng = np.random.default_rng(13)
    s = current_stream_handle()
    node_of = np.repeat(np.arange(N), np.diff(L.proc_off.astype(np.int64)))
    slots = (L.proc_slot & np.uint32(accel.KACC_SLOT_MASK)).astype(np.int64)
    ticks = np.zeros(P, dtype=np.uint64)   # the informer's ticks per row (its PID)
    total = np.zeros(P, dtype=np.float64)  # p.CPUTotalTime
    keep = []
    n_esc = 0
    for k in range(6):
        a = sim.next_interval()
        good = (a["node_status"][node_of] & accel.KACC_NODE_READ_ERROR) == 0
        new = (a["proc_slot"] & np.uint32(accel.KACC_SLOT_NEW)) != 0
        now = _readings(rng, ticks, new, k)
        now[~good] = ticks[~good]  # a skipped node is not read (any increment: the device skips it)
        base = np.where(new, np.uint64(0), ticks)
        dticks, esc_off, esc_row, esc_ticks = accel.encode_ticks(L.proc_off, now, base)
        n_esc += esc_row.size
        # Go: cpuTotalTime = float64(ticks)/100; CPUTimeDelta = cpuTotalTime - p.CPUTotalTime
        go_total = now.astype(np.float64) / 100.0
        go_delta = go_total - np.where(new, 0.0, total)
        d = to_device({"dt": dticks.view(np.int16), "eo": esc_off, "er": esc_row, "ev": esc_ticks})
        t = to_device(a)
        t["proc_cpu_delta"] = torch.full((max(P, 1),), float("nan"), dtype=torch.float64, device="cuda")
        tk = accel.KaccTicks(N, P, esc_row.size, 0, t["proc_off"].data_ptr(), t["node_status"].data_ptr(),
                             t["proc_slot"].data_ptr(), d["dt"].data_ptr(), d["eo"].data_ptr(),
                             d["er"].data_ptr() if esc_row.size else None,
                             d["ev"].data_ptr() if esc_row.size else None, t["proc_cpu_delta"].data_ptr())
        tm.delta(tk, s)
        acc.run_interval(interval_from_tensors(t, L.sizes(), L.fast_flag()), s)
        keep.append((t, d))
        acc.sync(s)
        got = t["proc_cpu_delta"].cpu().numpy()
        np.testing.assert_array_equal(got[good].view(np.uint64), go_delta[good].view(np.uint64),
                                      err_msg=f"interval {k}")
        a["proc_cpu_delta"] = go_delta
        ora.interval(a, L.sizes())
        assert_tables_equal(acc.download, ora.state, f"interval {k}")
        ticks = np.where(good, now, ticks)
        total = np.where(good, go_total, total)
    assert n_esc > 0
    np.testing.assert_array_equal(tm.download()[slots], ticks)
    tm.close()
    acc.close()


def test_ticks_errors_raise_erange():
    L = fleet.make_layout(4, [100, 50, 3, 20], 2, seed=2, n_namespaces=2)
    acc = accel.Accel(L.zones, **L.capacities())
    tm = accel.TickMap(acc)
    s = current_stream_handle()
    P = L.n_procs
    slot = to_device({"w": L.proc_slot | np.uint32(accel.KACC_SLOT_NEW), "o": L.proc_off})
    out = torch.zeros(P, dtype=torch.float64, device="cuda")
    dt = np.zeros(P, dtype=np.uint16)
    dt[5] = accel.KACC_TICKS_ESCAPED  # an escaped row without an escape
    d = to_device({"dt": dt.view(np.int16), "eo": np.zeros(L.n_nodes + 1, dtype=np.uint32)})
    tk = accel.KaccTicks(L.n_nodes, P, 0, 0, slot["o"].data_ptr(), None, slot["w"].data_ptr(), d["dt"].data_ptr(),
                         None, None, None, out.data_ptr())
    tm.delta(tk, s)
    with pytest.raises(accel.AccelError) as ei:
        acc.sync(s)
    assert ei.value.code == accel.KACC_ERANGE
    assert out[5].item() == 0.0
    # escapes out of order inside a node
    dt[6] = accel.KACC_TICKS_ESCAPED
    esc_off = np.array([0, 2, 2, 2, 2], dtype=np.uint32)
    d2 = to_device({"dt": dt.view(np.int16), "eo": esc_off, "er": np.array([6, 5], dtype=np.uint32),
                    "ev": np.array([70000, 80000], dtype=np.int64)})
    tk2 = accel.KaccTicks(L.n_nodes, P, 2, 0, slot["o"].data_ptr(), None, slot["w"].data_ptr(), d2["dt"].data_ptr(),
                          d2["eo"].data_ptr(), d2["er"].data_ptr(), d2["ev"].data_ptr(), out.data_ptr())
    tm.delta(tk2, s)
    with pytest.raises(accel.AccelError) as ei:
        acc.sync(s)
    assert ei.value.code == accel.KACC_ERANGE
    # the same escapes in order: clean, Δ = ticks / 100 for these NEW rows
    d3 = to_device({"er": np.array([5, 6], dtype=np.uint32), "ev": np.array([80000, 70000], dtype=np.int64)})
    tm.reset()
    tk3 = accel.KaccTicks(L.n_nodes, P, 2, 0, slot["o"].data_ptr(), None, slot["w"].data_ptr(), d2["dt"].data_ptr(),
                          d2["eo"].data_ptr(), d3["er"].data_ptr(), d3["ev"].data_ptr(), out.data_ptr())
    tm.delta(tk3, s)
    acc.sync(s)
    assert out[5].item() == 800.0 and out[6].item() == 700.0
    tm.close()
    acc.close()
