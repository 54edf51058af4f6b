"""Helpers for comparing engine state tables with the oracle's.

KACC_T_PROC_POWER is derived (ABI 3, kacc_derive.hpp): a slot's power is its ratio times
its node's ActivePower of the node's LAST processed interval.  For a slot that left its
node's batch (a terminated process under the held join policy, or one its node no longer
lists) the derived value is not Go's (Go drops the process from the snapshot; its final
power lives in the tracker, read before the node's next interval), so table comparisons
with the oracle restrict proc_power to the slots whose node attributed them at that node's
last processed interval.
"""

import numpy as np

from kepler_amd import accel


class LiveSlots:
    """Per-slot validity of the derived process power across intervals (node-private slot
    ranges slot_off[n] .. slot_off[n+1])."""

    def __init__(self, slot_off):
        self.slot_off = np.asarray(slot_off, dtype=np.int64)
        self.valid = np.zeros(int(self.slot_off[-1]), dtype=bool)

    def update(self, proc_off, slot_words, node_status=None):
        """After an interval: a processed node's slots are valid iff its batch rows hold them."""
        proc_off = np.asarray(proc_off, dtype=np.int64)
        n_nodes = len(proc_off) - 1
        ok = np.ones(n_nodes, dtype=bool) if node_status is None else \
            (np.asarray(node_status) & accel.KACC_NODE_READ_ERROR) == 0
        for n in np.flatnonzero(ok):
            self.valid[self.slot_off[n]:self.slot_off[n + 1]] = False
        rows = np.repeat(ok, np.diff(proc_off))
        s = (np.asarray(slot_words, dtype=np.uint32)[rows] & np.uint32(accel.KACC_SLOT_MASK)).astype(np.int64)
        self.valid[s] = True


def assert_tables_equal(get, want_state, msg="", live=None, zones=None):
    """Every table of accel.TABLES: get(name) == want_state[name] (NaN == NaN); proc_power only
    at live.valid slots when `live` is given."""
    for name, _ in accel.TABLES:
        got, want = get(name), want_state[name]
        if name == "proc_power" and live is not None:
            m = np.repeat(live.valid, zones)
            got, want = got[: m.size][m], want[: m.size][m]
        if want.dtype == np.float64:
            bad = (got.view(np.uint64) != want.view(np.uint64)) & ~(np.isnan(got) & np.isnan(want))
            assert not bad.any(), f"{msg} {name}: {int(bad.sum())} differ, first at {int(np.flatnonzero(bad)[0])}"
        else:
            np.testing.assert_array_equal(got, want, err_msg=f"{msg} {name}")
