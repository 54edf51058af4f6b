"""Multi-GPU plan: node snapshots shard across GPUs; namespace totals all-reduce.

Node snapshots are independent (node.go / process.go only read the node's own
zones and totals), so a fleet is split into contiguous node ranges balanced
by process count (prefix-sum cuts; needed for skewed fleets, BASELINE
config 5).  No data-path collective is needed; the only cross-GPU quantity is
the cluster-wide per-namespace total (north star), summed with one RCCL
all-reduce of u64 energy (modular, exact, order independent) and f64 power.
"""

from __future__ import annotations

from typing import List, Tuple

import numpy as np

from .fleet import FleetLayout


def plan_node_ranges(procs_per_node: np.ndarray, world: int) -> np.ndarray:
    """Boundaries b[0..world] so rank r owns nodes [b[r], b[r+1]) with ~equal rows."""
    p = np.asarray(procs_per_node, dtype=np.int64)
    n = len(p)
    prefix = np.concatenate([[0], np.cumsum(p)])
    total = prefix[-1]
    targets = (total * np.arange(1, world)) / world
    cuts = np.searchsorted(prefix, targets, side="left")
    # choose the closer of the two candidate cut points
    cuts = np.where((cuts > 0) & (np.abs(prefix[np.maximum(cuts - 1, 0)] - targets) < np.abs(prefix[cuts] - targets)),
                    cuts - 1, cuts)
    b = np.concatenate([[0], np.clip(cuts, 0, n), [n]]).astype(np.int64)
    return np.maximum.accumulate(b)


def shard_layout(layout: FleetLayout, lo: int, hi: int) -> FleetLayout:
    """The sub-fleet of nodes [lo, hi) with compact offsets and slots."""
    po, co, vo, qo = (layout.proc_off.astype(np.int64), layout.ctr_off.astype(np.int64),
                      layout.vm_off.astype(np.int64), layout.pod_off.astype(np.int64))
    p0, p1, c0, c1, v0, v1, q0, q1 = po[lo], po[hi], co[lo], co[hi], vo[lo], vo[hi], qo[lo], qo[hi]
    u32 = lambda a: np.ascontiguousarray(a, dtype=np.uint32)  # noqa: E731

    def compact(slots):
        # a shard's slot tables are private: slots are the rows' positions
        # (the same compaction fleet.subset_interval applies)
        return np.arange(len(slots), dtype=np.int64)

    return FleetLayout(
        zones=layout.zones, n_nodes=hi - lo,
        proc_off=u32(po[lo:hi + 1] - p0), ctr_off=u32(co[lo:hi + 1] - c0),
        vm_off=u32(vo[lo:hi + 1] - v0), pod_off=u32(qo[lo:hi + 1] - q0),
        ctr_proc_end=u32(layout.ctr_proc_end[c0:c1].astype(np.int64) - p0),
        vm_proc_end=u32(layout.vm_proc_end[v0:v1].astype(np.int64) - p0),
        pod_ctr_end=u32(layout.pod_ctr_end[q0:q1].astype(np.int64) - c0),
        proc_slot=u32(compact(layout.proc_slot[p0:p1])), ctr_slot=u32(compact(layout.ctr_slot[c0:c1])),
        vm_slot=u32(compact(layout.vm_slot[v0:v1])), pod_slot=u32(compact(layout.pod_slot[q0:q1])),
        pod_ns=layout.pod_ns[q0:q1].copy(), n_namespaces=layout.n_namespaces,
    )


def shard(layout: FleetLayout, world: int) -> List[Tuple[int, int, FleetLayout]]:
    b = plan_node_ranges(np.diff(layout.proc_off.astype(np.int64)), world)
    return [(int(b[r]), int(b[r + 1]), shard_layout(layout, int(b[r]), int(b[r + 1]))) for r in range(world)]
