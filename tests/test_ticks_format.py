"""The CPU-tick input format on the host (no GPU): the encoder's increments / escapes decode to
the readings, and the float64 arithmetic the device performs — float64(now)/100 -
float64(prev)/100 — is Go's CPUTimeDelta (oracle/pyref.Informer, a restatement of
populateProcessFields, informer.go:512-524, and procWrapper.CPUTime, procfs_reader.go:75-82),
including u64 tick wrap, increments past 16 bits, negative increments (a reused PID in a cached
entry) and first readings of long-lived processes."""

import numpy as np

from kepler_amd import accel
from oracle.pyref import Informer, go_cpu_time

U64 = (1 << 64) - 1


def _cases(rng, n):
    prev = rng.integers(0, 10**6, size=n, dtype=np.uint64)
    inc = rng.integers(0, 3000, size=n).astype(np.int64)
    k = n // 8
    inc[:k] = rng.integers(0xFFFF, 10**7, size=k)                       # past 16 bits: escapes
    inc[k:2 * k] = -rng.integers(1, 10**5, size=k)                        # a reused PID: ticks go back
    prev[2 * k:3 * k] = np.uint64(U64) - rng.integers(0, 500, size=k).astype(np.uint64)  # u64 tick wrap
    prev[3 * k:4 * k] = rng.integers(1 << 53, 1 << 62, size=k, dtype=np.uint64)  # float64 rounds the ticks
    inc[4 * k:4 * k + 3] = [0, 0xFFFE, 0xFFFF]                            # the 16-bit boundary
    now = prev + inc.astype(np.uint64)                                    # mod 2^64 (numpy wraps)
    return prev, now


def test_encoder_round_trip_and_escapes():
    rng = np.random.default_rng(7)
    proc_off = np.array([0, 100, 100, 1000, 4000], dtype=np.uint32)
    prev, now = _cases(rng, 4000)
    dticks, esc_off, esc_row, esc_ticks = accel.encode_ticks(proc_off, now, prev)
    assert dticks.dtype == np.uint16 and esc_ticks.dtype == np.int64
    esc = dticks == accel.KACC_TICKS_ESCAPED
    np.testing.assert_array_equal(np.flatnonzero(esc), esc_row)
    assert (dticks[~esc] < 0xFFFF).all()
    for n in range(len(proc_off) - 1):  # every escape of node n lies in its rows, ascending
        r = esc_row[esc_off[n]:esc_off[n + 1]]
        assert ((r >= proc_off[n]) & (r < proc_off[n + 1])).all() and (np.diff(r.astype(np.int64)) > 0).all()
    dec = prev + dticks.astype(np.uint64)                     # the device's decode, in numpy
    dec[esc_row] = prev[esc_row] + esc_ticks.astype(np.uint64)
    np.testing.assert_array_equal(dec, now)


def test_device_arithmetic_is_gos_cpu_time_delta():
    rng = np.random.default_rng(11)
    prev, now = _cases(rng, 20000)
    new = rng.random(prev.size) < 0.1  # a new process: p.CPUTotalTime = 0 (its whole ticks are the increment)
    p = np.where(new, np.uint64(0), prev)
    got = now.astype(np.float64) / 100.0 - p.astype(np.float64) / 100.0
    inf = Informer()
    want = np.empty(prev.size)
    for i in range(prev.size):
        if not new[i]:
            inf.read(i, int(prev[i]), True)  # the previous reading of the same PID
        want[i] = inf.read(i, int(now[i]), bool(new[i]))
    np.testing.assert_array_equal(got.view(np.uint64), want.view(np.uint64))
    # float64(uint64) is correctly rounded in both (numpy's cast and Python's float(int))
    big = rng.integers(1 << 53, 1 << 63, size=5000, dtype=np.uint64) | np.uint64(1 << 63)
    np.testing.assert_array_equal(big.astype(np.float64), np.array([float(int(x)) for x in big]))
    assert go_cpu_time(U64 + 5) == go_cpu_time(4)  # the uint sum wraps like Go's
