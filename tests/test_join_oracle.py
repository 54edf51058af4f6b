"""Slot-join oracle (oracle/kor_join.cpp) against the reference's semantics — CPU.

The reference decides "running total or new" with ``prev.Processes[pid]``
(process.go:132-138) and builds the terminated set as cached-before minus
running-now (informer.go:206-212).  An independent pure-Python restatement
(dicts keyed by ID, as the Go maps) checks the C++ oracle, including the
engine's slot numbering rule (lowest slot free at the start of the interval,
new rows in row order).
"""

import numpy as np
import pytest

from kepler_amd import fleet
from kepler_amd.accel import KACC_KEY_EMPTY, KACC_NODE_READ_ERROR, KACC_SLOT_NEW
from oracle.oracle import OracleSlotMap

KACC_ERANGE = -4


class PySlotMap:
    """Go-map restatement: per node dict ID -> slot."""

    def __init__(self, slot_off, reuse=False):
        self.off = [int(x) for x in slot_off]
        self.live = [dict() for _ in range(len(self.off) - 1)]
        self.reuse = reuse  # KACC_JOIN_REUSE_TERMINATED

    def join(self, row_off, keys, node_status=None):
        out = np.zeros(int(row_off[-1]), dtype=np.uint32)
        term = []
        for n, prev in enumerate(self.live):
            if node_status is not None and node_status[n] & KACC_NODE_READ_ERROR:
                continue
            s0, S = self.off[n], self.off[n + 1] - self.off[n]
            held = set(prev.values())
            free = [s for s in range(S) if s not in held]
            if self.reuse:  # the slots of IDs absent from this batch first, ascending
                now = set(int(k) for k in keys[int(row_off[n]):int(row_off[n + 1])])
                free = sorted(s for k, s in prev.items() if k not in now) + free
            cur = {}
            for r in range(int(row_off[n]), int(row_off[n + 1])):
                k = int(keys[r])
                if k in prev:  # process.go:134 — the running total continues
                    cur[k] = prev[k]
                    out[r] = s0 + prev[k]
                else:
                    s = free.pop(0)
                    cur[k] = s
                    out[r] = (s0 + s) | KACC_SLOT_NEW
            # informer.go:206-212; the node's segment ascending by slot
            term += sorted(((k, s0 + s) for k, s in prev.items() if k not in cur), key=lambda x: x[1])
            self.live[n] = cur
        return out, term


def ranges(sizes, slack=1.25):
    row_off = np.r_[0, np.cumsum(sizes)].astype(np.uint32)
    slot_off = np.r_[0, np.cumsum([int(np.ceil(s * slack)) + 2 for s in sizes])].astype(np.uint32)
    return row_off, slot_off


@pytest.mark.parametrize("kind,reuse", [("proc", False), ("ctr", False), ("proc", True), ("ctr", True)])
def test_oracle_join_matches_go_maps(kind, reuse):
    sizes = [0, 1, 7, 64, 300, 1000]
    row_off, slot_off = ranges(sizes)
    sim = fleet.KeyedChurn(row_off, seed=3, churn=0.1, kind=kind)
    ora, py = OracleSlotMap(slot_off, policy=int(reuse)), PySlotMap(slot_off, reuse)
    rng = np.random.default_rng(1)
    live_slot = {}
    for it in range(6):
        keys = sim.next_keys()
        status = np.where(rng.random(len(sizes)) < 0.15, KACC_NODE_READ_ERROR, 0).astype(np.uint32) if it else None
        rc, out, tk, ts, cnt = ora.join(row_off, keys, status)
        assert rc == 0
        want, want_term = py.join(row_off, keys, status)
        np.testing.assert_array_equal(out, want)
        assert ora.terminated(tk, ts, cnt) == want_term
        ts = np.array([s for _, s in want_term], dtype=np.uint32)
        # properties: slots in range and unique per node; a live key keeps its slot
        for n in range(len(sizes)):
            if status is not None and status[n]:
                continue
            r0, r1 = row_off[n], row_off[n + 1]
            s = out[r0:r1] & 0x7FFFFFFF
            assert np.all((s >= slot_off[n]) & (s < slot_off[n + 1]))
            assert len(np.unique(s)) == s.size
            for k, w in zip(keys[r0:r1].tolist(), out[r0:r1].tolist()):
                if (n, k) in live_slot and not (w & KACC_SLOT_NEW):
                    assert live_slot[(n, k)] == w & 0x7FFFFFFF
                live_slot[(n, k)] = w & 0x7FFFFFFF
        new_slots = set((out[(out & KACC_SLOT_NEW) != 0] & 0x7FFFFFFF).tolist())
        if reuse:  # KeyedChurn: as many new rows as terminated IDs -> the terminated slots exactly
            assert set(ts.tolist()) <= new_slots or status is not None
        else:  # terminated slots are not handed to new rows in the same interval
            assert not new_slots & set(ts.tolist())


def test_oracle_join_reuse_keeps_slot_order():
    """/proc-shaped churn (a newcomer listed where an exited process was): with
    KACC_JOIN_REUSE_TERMINATED every node keeps exactly slots 0..rows-1 in row order."""
    row_off, slot_off = ranges([40, 300, 1000])
    sim = fleet.KeyedChurn(row_off, seed=5, churn=0.05)
    ora = OracleSlotMap(slot_off, policy=1)
    for _ in range(8):
        rc, out, _, _, cnt = ora.join(row_off, sim.next_keys())
        assert rc == 0
        for n in range(3):
            s = (out[row_off[n]:row_off[n + 1]] & 0x7FFFFFFF) - slot_off[n]
            np.testing.assert_array_equal(s, np.arange(row_off[n + 1] - row_off[n]))
    assert cnt.sum() > 0


def test_oracle_join_first_interval_consecutive():
    row_off, slot_off = ranges([5, 3])
    rc, out, _, _, cnt = OracleSlotMap(slot_off).join(row_off, np.arange(8, dtype=np.uint64))
    assert rc == 0 and cnt.sum() == 0
    np.testing.assert_array_equal(out & 0x7FFFFFFF, [0, 1, 2, 3, 4, slot_off[1], slot_off[1] + 1, slot_off[1] + 2])
    assert np.all(out & KACC_SLOT_NEW)


def test_oracle_join_errors():
    row_off = np.array([0, 3], dtype=np.uint32)
    # duplicate ID inside a node, reserved key
    rc, out, _, _, _ = OracleSlotMap(np.array([0, 8], dtype=np.uint32)).join(row_off, np.array([5, 5, 6], dtype=np.uint64))
    assert rc == KACC_ERANGE and out[1] == 0xFFFFFFFF
    rc, out, _, _, _ = OracleSlotMap(np.array([0, 8], dtype=np.uint32)).join(
        row_off, np.array([1, KACC_KEY_EMPTY, 2], dtype=np.uint64))
    assert rc == KACC_ERANGE and out[1] == 0xFFFFFFFF
    # range overflow: 3 live IDs, 2 slots
    rc, out, _, _, _ = OracleSlotMap(np.array([0, 2], dtype=np.uint32)).join(row_off, np.array([1, 2, 3], dtype=np.uint64))
    assert rc == KACC_ERANGE and out[2] == 0xFFFFFFFF
    # terminated slots stay held for one interval: 2 slots, full turnover -> overflow now, fine next time
    m = OracleSlotMap(np.array([0, 2], dtype=np.uint32))
    two = np.array([0, 2], dtype=np.uint32)
    assert m.join(two, np.array([1, 2], dtype=np.uint64))[0] == 0
    rc, out, tk, ts, cnt = m.join(two, np.array([3, 4], dtype=np.uint64))
    assert rc == KACC_ERANGE and m.terminated(tk, ts, cnt) == [(1, 0), (2, 1)]
