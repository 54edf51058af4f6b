"""Synthetic fleet generator and SoA batch layout.

A *fleet* is N node snapshots.  Each node has Z RAPL zones and a process
table laid out as the engine expects (include/kepler_accel.h): container
processes grouped by container, then VM processes grouped by VM, then the
other processes; containers grouped by pod.  Workloads keep stable slots in
the device-resident tables; a process that is new this interval carries
KACC_SLOT_NEW (process.go:133-138: no previous snapshot entry).

Inputs are generated the way the Go side would produce them:
  * zone counters advance by P(W)·dt µJ and wrap at MaxEnergy
    (fake_cpu_power_meter.go:57 / node.go:87-98);
  * timestamps are monotonic ns, dt = 5 s ± jitter (config.go:206 interval);
  * per-process CPUTimeDelta = f64(ticks)/100 − previous total, exactly the
    informer formula (procfs_reader.go:75-82, informer.go:518);
  * the usage ratio is U[0.05, 0.95] with 1 % exact zeros (exercises the
    zero-ActivePower skip, process.go:124).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Optional

import numpy as np

from .accel import KACC_NODE_READ_ERROR, KACC_SLOT_NEW

SEED = 0x4B45504C
# internal/device/testdata/sys/.../max_energy_range_uj
MAX_ENERGY_RAPL = 262143328850
# fake_cpu_power_meter.go:135 (the wrap configs)
MAX_ENERGY_FAKE = 1_000_000
ZONE_NAMES = {
    1: ["package"],
    2: ["package", "dram"],
    3: ["package", "core", "dram"],
    4: ["package", "core", "uncore", "dram"],
    5: ["package", "core", "uncore", "dram", "psys"],
    6: ["package", "core", "uncore", "dram", "psys", "pp0"],
    7: ["package", "core", "uncore", "dram", "psys", "pp0", "pp1"],
    8: ["package", "core", "uncore", "dram", "psys", "pp0", "pp1", "package-1"],
}


@dataclass
class FleetLayout:
    zones: int
    n_nodes: int
    proc_off: np.ndarray
    ctr_off: np.ndarray
    vm_off: np.ndarray
    pod_off: np.ndarray
    ctr_proc_end: np.ndarray
    vm_proc_end: np.ndarray
    pod_ctr_end: np.ndarray
    proc_slot: np.ndarray
    ctr_slot: np.ndarray
    vm_slot: np.ndarray
    pod_slot: np.ndarray
    pod_ns: np.ndarray
    n_namespaces: int

    @property
    def n_procs(self) -> int:
        return int(self.proc_off[-1])

    @property
    def n_ctrs(self) -> int:
        return int(self.ctr_off[-1])

    @property
    def n_vms(self) -> int:
        return int(self.vm_off[-1])

    @property
    def n_pods(self) -> int:
        return int(self.pod_off[-1])

    def sizes(self) -> Dict[str, int]:
        return dict(n_nodes=self.n_nodes, n_procs=self.n_procs, n_ctrs=self.n_ctrs,
                    n_vms=self.n_vms, n_pods=self.n_pods)

    def capacities(self) -> Dict[str, int]:
        return dict(
            nodes=self.n_nodes,
            proc_slots=max(int(self.proc_slot.max(initial=0)) + 1, 1),
            ctr_slots=max(int(self.ctr_slot.max(initial=0)) + 1, 1),
            vm_slots=max(int(self.vm_slot.max(initial=0)) + 1, 1),
            pod_slots=max(int(self.pod_slot.max(initial=0)) + 1, 1),
        )

    def proc_span(self) -> np.ndarray:
        """node_proc_span [2N]: {min, max} process slot per node ({1, 0} when empty)."""
        out = np.zeros(2 * self.n_nodes, dtype=np.uint32)
        rows = np.diff(self.proc_off.astype(np.int64))
        nz = rows > 0
        starts = self.proc_off[:-1][nz].astype(np.int64)
        out[0::2][~nz], out[1::2][~nz] = 1, 0
        if nz.any():
            out[0::2][nz] = np.minimum.reduceat(self.proc_slot, starts)
            out[1::2][nz] = np.maximum.reduceat(self.proc_slot, starts)
        return out

    def fast_flag(self) -> int:
        """KACC_F_FAST_NODES when every node fits the fast path (| KACC_F_MEDIUM_NODES /
        KACC_F_SMALL_NODES when every node also fits those shapes), else 0."""
        from .accel import (KACC_F_FAST_NODES, KACC_F_MEDIUM_NODES, KACC_F_SMALL_NODES, KACC_FAST_MAX_AGGREGATES,
                            KACC_FAST_MAX_PROCS, KACC_MEDIUM_MAX_AGGREGATES, KACC_MEDIUM_MAX_PROCS,
                            KACC_SMALL_MAX_AGGREGATES, KACC_SMALL_MAX_PROCS)

        rows = np.diff(self.proc_off.astype(np.int64))
        agg = (np.diff(self.ctr_off.astype(np.int64)) + np.diff(self.vm_off.astype(np.int64))
               + np.diff(self.pod_off.astype(np.int64)))
        if not (np.all(rows <= KACC_FAST_MAX_PROCS) and np.all(agg <= KACC_FAST_MAX_AGGREGATES)):
            return 0
        small = bool(np.all(rows <= KACC_SMALL_MAX_PROCS) and np.all(agg <= KACC_SMALL_MAX_AGGREGATES))
        medium = bool(np.all(rows <= KACC_MEDIUM_MAX_PROCS) and np.all(agg <= KACC_MEDIUM_MAX_AGGREGATES))
        return KACC_F_FAST_NODES | (KACC_F_SMALL_NODES if small else 0) | (KACC_F_MEDIUM_NODES if medium else 0)

    def static_arrays(self) -> Dict[str, np.ndarray]:
        return dict(proc_off=self.proc_off, ctr_off=self.ctr_off, vm_off=self.vm_off,
                    pod_off=self.pod_off, ctr_proc_end=self.ctr_proc_end,
                    vm_proc_end=self.vm_proc_end, pod_ctr_end=self.pod_ctr_end)

    def namespace_csr(self):
        """ns_pod_off [n_ns+1], ns_pod_slot [Q]: pods grouped by namespace (stable)."""
        order = np.argsort(self.pod_ns, kind="stable")
        counts = np.bincount(self.pod_ns, minlength=self.n_namespaces)
        off = np.zeros(self.n_namespaces + 1, dtype=np.uint32)
        np.cumsum(counts, out=off[1:])
        return off, self.pod_slot[order].astype(np.uint32)

    def namespace_csr_rows(self):
        """ns_pod_off [n_ns+1], ns_pod_row [Q]: the same grouping over batch pod ROWS (the
        index space of an interval's pod export, kacc_allreduce_exports): the same order."""
        order = np.argsort(self.pod_ns, kind="stable")
        off, _ = self.namespace_csr()
        return off, order.astype(np.uint32)

    def node_order_heaviest_first(self) -> np.ndarray:
        rows = np.diff(self.proc_off.astype(np.int64))
        return np.argsort(-rows, kind="stable").astype(np.uint32)


def _split(rng, totals: np.ndarray, parts: np.ndarray) -> np.ndarray:
    """Split totals[n] into parts[n] segments of size >= 1 (random), flattened."""
    totals = totals.astype(np.int64)
    parts = parts.astype(np.int64)
    assert np.all(parts <= np.maximum(totals, 0)) and np.all((parts > 0) | (totals == 0))
    n_seg = int(parts.sum())
    sizes = np.ones(n_seg, dtype=np.int64)
    extra = totals - parts
    seg_base = np.zeros(len(parts), dtype=np.int64)
    np.cumsum(parts[:-1], out=seg_base[1:])
    n_extra = int(extra.sum())
    if n_extra > 0:
        owner = np.repeat(np.arange(len(parts)), extra)
        pick = seg_base[owner] + (rng.random(n_extra) * parts[owner]).astype(np.int64)
        sizes += np.bincount(pick, minlength=n_seg)
    return sizes


def make_layout(n_nodes: int, procs_per_node, zones: int, seed: int = SEED,
                ctr_frac: float = 0.79, procs_per_ctr: int = 8, vm_frac: float = 0.01,
                procs_per_vm: int = 1, ctrs_per_pod: float = 2.5, pod_frac: float = 0.9,
                n_namespaces: Optional[int] = None, shuffle_slots: bool = False,
                fragment_slots: float = 0.0, fragment_sorted: bool = False) -> FleetLayout:
    """Synthetic fleet.  Process slots: consecutive per node (default), a global
    permutation (``shuffle_slots``), or, with ``fragment_slots`` = f > 0, each
    node's processes on a random subset of its own slot range of (1 + f) x rows
    in random order — the steady state the slot join reaches under churn
    (``fragment_sorted``: the same subsets in increasing slot order).
    """
    rng = np.random.default_rng(seed)
    P = np.broadcast_to(np.asarray(procs_per_node, dtype=np.int64), (n_nodes,)).copy()
    Vp = np.floor(P * vm_frac).astype(np.int64)  # VM processes
    W = np.where(Vp > 0, np.maximum(Vp // max(procs_per_vm, 1), 1), 0)  # VMs
    T = np.minimum(np.floor(P * ctr_frac).astype(np.int64), P - Vp)  # container processes
    C = np.where(T > 0, np.maximum(T // procs_per_ctr, 1), 0)
    ctr_sizes = _split(rng, T, C)
    vm_sizes = _split(rng, Vp, W)
    podded = np.floor(C * pod_frac).astype(np.int64)
    Q = np.where(podded > 0, np.maximum(np.floor(podded / ctrs_per_pod).astype(np.int64), 1), 0)
    pod_sizes = _split(rng, podded, Q)

    def offsets(counts):
        off = np.zeros(n_nodes + 1, dtype=np.int64)
        np.cumsum(counts, out=off[1:])
        return off

    proc_off, ctr_off, vm_off, pod_off = offsets(P), offsets(C), offsets(W), offsets(Q)
    # container c ends at node base + cumulative size within node
    node_of_ctr = np.repeat(np.arange(n_nodes), C)
    csum = np.cumsum(ctr_sizes)
    ctr_base = np.repeat(np.concatenate([[0], csum])[ctr_off[:-1]], C)
    ctr_proc_end = proc_off[node_of_ctr] + (csum - ctr_base)
    node_of_vm = np.repeat(np.arange(n_nodes), W)
    vsum = np.cumsum(vm_sizes)
    vm_base = np.repeat(np.concatenate([[0], vsum])[vm_off[:-1]], W)
    vm_proc_end = proc_off[node_of_vm] + T[node_of_vm] + (vsum - vm_base)
    node_of_pod = np.repeat(np.arange(n_nodes), Q)
    qsum = np.cumsum(pod_sizes)
    pod_base = np.repeat(np.concatenate([[0], qsum])[pod_off[:-1]], Q)
    pod_ctr_end = ctr_off[node_of_pod] + (qsum - pod_base)

    n_procs, n_ctrs, n_vms, n_pods = int(proc_off[-1]), int(ctr_off[-1]), int(vm_off[-1]), int(pod_off[-1])
    if fragment_slots > 0:
        rng_f = np.random.default_rng(seed ^ 0xF4A6)
        cap = (P * (1.0 + fragment_slots)).astype(np.int64) + 1
        slot_base = np.concatenate([[0], np.cumsum(cap)[:-1]])
        pick = (lambda x: np.sort(x)) if fragment_sorted else (lambda x: x)
        proc_slot = np.concatenate([slot_base[n] + pick(rng_f.permutation(int(cap[n]))[: int(P[n])])
                                    for n in range(n_nodes)]) if n_procs else np.zeros(0, np.int64)
        ctr_slot, vm_slot, pod_slot = np.arange(n_ctrs), np.arange(n_vms), np.arange(n_pods)
    elif shuffle_slots:
        proc_slot = rng.permutation(n_procs)
        ctr_slot = rng.permutation(n_ctrs)
        vm_slot = rng.permutation(n_vms)
        pod_slot = rng.permutation(n_pods)
    else:
        proc_slot, ctr_slot = np.arange(n_procs), np.arange(n_ctrs)
        vm_slot, pod_slot = np.arange(n_vms), np.arange(n_pods)
    if n_namespaces is None:
        n_namespaces = max(n_nodes, 1)
    pod_ns = rng.integers(0, n_namespaces, size=n_pods)
    u32 = lambda a: np.ascontiguousarray(a, dtype=np.uint32)  # noqa: E731
    return FleetLayout(
        zones=zones, n_nodes=n_nodes,
        proc_off=u32(proc_off), ctr_off=u32(ctr_off), vm_off=u32(vm_off), pod_off=u32(pod_off),
        ctr_proc_end=u32(ctr_proc_end), vm_proc_end=u32(vm_proc_end), pod_ctr_end=u32(pod_ctr_end),
        proc_slot=u32(proc_slot), ctr_slot=u32(ctr_slot), vm_slot=u32(vm_slot), pod_slot=u32(pod_slot),
        pod_ns=u32(pod_ns), n_namespaces=n_namespaces,
    )


def layout_from_sizes(zones: int, nodes, seed: int = SEED, shuffle_slots: bool = False) -> FleetLayout:
    """Layout with explicit per-node segment sizes (edge-case fleets).

    ``nodes`` is a list of dicts: ``rows`` (processes), ``ctr`` (processes per
    container, listing order), ``vm`` (processes per VM) and ``pod``
    (containers per pod; pods take containers from the front, the rest stay
    pod-less).  Rows are laid out [container procs][VM procs][rest].
    """
    rng = np.random.default_rng(seed)
    proc_off, ctr_off, vm_off, pod_off = [0], [0], [0], [0]
    ctr_end, vm_end, pod_end = [], [], []
    for nd in nodes:
        base, cbase = proc_off[-1], ctr_off[-1]
        ctr, vm, pod = list(nd.get("ctr", [])), list(nd.get("vm", [])), list(nd.get("pod", []))
        rows = int(nd["rows"])
        assert sum(ctr) + sum(vm) <= rows and sum(pod) <= len(ctr)
        ctr_end += list(base + np.cumsum(ctr, dtype=np.int64)) if ctr else []
        vm_end += list(base + sum(ctr) + np.cumsum(vm, dtype=np.int64)) if vm else []
        pod_end += list(cbase + np.cumsum(pod, dtype=np.int64)) if pod else []
        proc_off.append(base + rows)
        ctr_off.append(cbase + len(ctr))
        vm_off.append(vm_off[-1] + len(vm))
        pod_off.append(pod_off[-1] + len(pod))
    n_procs, n_ctrs, n_vms, n_pods = proc_off[-1], ctr_off[-1], vm_off[-1], pod_off[-1]
    slots = [(rng.permutation(k) if shuffle_slots else np.arange(k)) for k in (n_procs, n_ctrs, n_vms, n_pods)]
    u32 = lambda a: np.ascontiguousarray(a, dtype=np.uint32)  # noqa: E731
    n_ns = max(len(nodes), 1)
    return FleetLayout(
        zones=zones, n_nodes=len(nodes),
        proc_off=u32(proc_off), ctr_off=u32(ctr_off), vm_off=u32(vm_off), pod_off=u32(pod_off),
        ctr_proc_end=u32(ctr_end), vm_proc_end=u32(vm_end), pod_ctr_end=u32(pod_end),
        proc_slot=u32(slots[0]), ctr_slot=u32(slots[1]), vm_slot=u32(slots[2]), pod_slot=u32(slots[3]),
        pod_ns=u32(rng.integers(0, n_ns, size=n_pods)), n_namespaces=n_ns,
    )


def config_layout(config: int, seed: int = SEED, nodes: Optional[int] = None,
                  fragment_slots: float = 0.0, fragment_sorted: bool = False,
                  n_namespaces: Optional[int] = None) -> FleetLayout:
    """Layouts of BASELINE.json configs (2: 1k×1k Z=2, 3: 10k×2k Z=4, 5: skewed).

    ``fragment_slots`` > 0 places each node's processes on a random subset of
    its own slot range (the slot join's steady state under churn).
    ``n_namespaces``: the fleet's namespace count (default: one per node; a
    shard of a bigger fleet passes the whole fleet's, config_shard)."""
    if config == 1:  # single node, 500 procs -> 50 containers -> 20 pods, package+dram
        # (``nodes``: a fleet of such nodes — the small-node kernel's workload)
        return make_layout(nodes or 1, 500, 2, seed, ctr_frac=0.8, procs_per_ctr=8, ctrs_per_pod=2.5,
                           pod_frac=1.0, n_namespaces=n_namespaces or (4 if not nodes else None),
                           fragment_slots=fragment_slots)
    if config == 2:
        return make_layout(nodes or 1000, 1000, 2, seed, fragment_slots=fragment_slots, n_namespaces=n_namespaces)
    if config in (3, 4):
        return make_layout(nodes or 10000, 2000, 4, seed, fragment_slots=fragment_slots,
                           fragment_sorted=fragment_sorted, n_namespaces=n_namespaces)
    if config == 5:
        p = config_procs_per_node(5, nodes or 1000, seed)
        return make_layout(len(p), p, 4, seed, procs_per_vm=2, vm_frac=0.02)
    raise ValueError(config)


def config_procs_per_node(config: int, nodes: int, seed: int = SEED) -> np.ndarray:
    """Processes per node of a BASELINE config's fleet of ``nodes`` nodes (cheap: no layout)."""
    if config == 5:
        # truncated Pareto(alpha=1.5) on [10k, 50k] procs per node
        rng = np.random.default_rng(seed ^ 5)
        u = rng.random(nodes)
        a, lo, hi = 1.5, 10_000.0, 50_000.0
        return (lo / (1 - u * (1 - (lo / hi) ** a)) ** (1 / a)).astype(np.int64)
    per = {1: 500, 2: 1000, 3: 2000, 4: 2000}[config]
    return np.full(nodes, per, dtype=np.int64)


def config_shard(config: int, world: int, rank: int, nodes: int, seed: int = SEED,
                 fragment_slots: float = 0.0):
    """Rank `rank`'s node range of a `nodes`-node fleet of BASELINE config `config`, cut by
    shard.plan_node_ranges over the fleet's per-node process counts (balanced rows; config 5
    is skewed).  Each rank generates only its own nodes (seeded by the range start), so a
    100k-node fleet is never materialised on one host.  Returns (lo, hi, layout)."""
    from .shard import plan_node_ranges

    b = plan_node_ranges(config_procs_per_node(config, nodes, seed), world)
    lo, hi = int(b[rank]), int(b[rank + 1])
    s = seed + lo
    # every shard indexes the whole fleet's namespaces (one per node, as an unsharded fleet)
    if config == 5:
        p = config_procs_per_node(5, nodes, seed)[lo:hi]
        return lo, hi, make_layout(hi - lo, p, 4, s, procs_per_vm=2, vm_frac=0.02, fragment_slots=fragment_slots,
                                   n_namespaces=max(nodes, 1))
    return lo, hi, config_layout(config, seed=s, nodes=hi - lo, fragment_slots=fragment_slots,
                                 n_namespaces=max(nodes, 1))


@dataclass
class FleetSim:
    """Per-interval dynamic inputs for a layout (host numpy arrays)."""

    layout: FleetLayout
    seed: int = SEED
    max_energy: int = MAX_ENERGY_RAPL
    dt_ns: int = 5_000_000_000
    jitter_ns: int = 50_000_000
    zero_ratio_frac: float = 0.01
    churn: float = 0.02
    read_error_frac: float = 0.0
    # fraction of nodes per interval given one adversarial-but-reachable input (see
    # ADVERSARIAL): zero / backward clock steps, unchanged counters, usage ratio 1 / > 1 /
    # < 0, negative CPU deltas (PID reuse in a cached entry), huge cancelling deltas
    adversarial: float = 0.0
    interval: int = 0
    _rng: np.random.Generator = field(init=False, repr=False)

    # adversarial scenarios: (name, reference line the input exercises)
    ADVERSARIAL = (
        ("dt_zero", "node.go:34 now.Sub(prev).Seconds() == 0 -> p = ΔE/0 = +Inf or NaN"),
        ("clock_backward", "node.go:34 negative Seconds() -> negative / -Inf power"),
        ("energy_unchanged", "node.go:50-56 ΔE = 0 with a nonzero ratio -> activeEnergy 0, zones skipped"),
        ("energy_unchanged_one_zone", "node.go:50-56 one zone's ΔE = 0"),
        ("ratio_one", "node.go:56 usage ratio exactly 1: idle = 0"),
        ("ratio_above_one", "procfs_reader.go:137-139 (dIdle+dIowait < 0) -> ratio > 1: u64 idle wraps"),
        ("ratio_negative", "ratio < 0 -> Energy(negative) wraps, negative ActivePower"),
        ("negative_cpu_delta", "informer.go:518 a reused PID in a cached entry: Δ = total - prev < 0"),
        ("huge_cancelling_deltas", "process.go:130 ratio = Δ/ΔcpuNode huge -> Energy() out of range"),
    )

    def __post_init__(self):
        L = self.layout
        self._rng = np.random.default_rng(self.seed ^ 0x51)
        Z, N = L.zones, L.n_nodes
        self.zone_max = np.full(N * Z, self.max_energy, dtype=np.uint64)
        self.counters = (self._rng.random(N * Z) * self.max_energy).astype(np.uint64)
        self.ts = (1_000_000_000_000 + self._rng.integers(0, 10**9, size=N)).astype(np.int64)
        self.cum_ticks = self._rng.integers(0, 10_000, size=L.n_procs).astype(np.int64)
        self.prev_total = np.zeros(L.n_procs, dtype=np.float64)  # informer cache starts empty
        # a process born while its node's reads fail is first seen (NEW) at the node's next
        # good interval: Refresh is skipped when calculateNodePower fails (monitor.go:399-408)
        self.pending_new = np.zeros(L.n_procs, dtype=bool)
        self.node_of_proc = np.repeat(np.arange(N), np.diff(L.proc_off.astype(np.int64)))
        self.last_status = np.zeros(N, dtype=np.uint32)
        self.last_scenario = np.full(N, -1, dtype=np.int64)
        pkg = self._rng.uniform(50.0, 400.0, size=N)
        dram = self._rng.uniform(5.0, 40.0, size=N)
        watts = {"package": pkg, "core": 0.6 * pkg, "uncore": 0.1 * pkg, "dram": dram,
                 "psys": 1.3 * pkg + dram, "pp0": 0.55 * pkg, "pp1": 0.05 * pkg, "package-1": 0.9 * pkg}
        self.zone_watts = np.stack([watts[z] for z in ZONE_NAMES[Z]], axis=1).reshape(-1)

    def next_node_inputs(self) -> Dict[str, np.ndarray]:
        """Advance the node-level inputs (clock, counters, usage ratio) one interval."""
        L, rng = self.layout, self._rng
        N, Z = L.n_nodes, L.zones
        dt = self.dt_ns + rng.integers(-self.jitter_ns, self.jitter_ns + 1, size=N)
        dts = np.repeat(dt, Z).astype(np.float64) / 1e9
        watts = self.zone_watts * rng.uniform(0.8, 1.2, size=N * Z)
        de = np.round(watts * dts * 1e6).astype(np.uint64)
        ratio = rng.uniform(0.05, 0.95, size=N)
        ratio[rng.random(N) < self.zero_ratio_frac] = 0.0
        scen = np.full(N, -1, dtype=np.int64)
        if self.adversarial > 0 and self.interval > 0:
            # a separate stream: the ordinary inputs stay those of a non-adversarial sim
            arng = np.random.default_rng([self.seed, 0xAD, self.interval])
            hit = arng.random(N) < self.adversarial
            scen[hit] = arng.integers(0, len(self.ADVERSARIAL), size=int(hit.sum()))
            names = [s[0] for s in self.ADVERSARIAL]
            is_ = lambda name: scen == names.index(name)  # noqa: E731
            # the counters advance with real time; only the clock reading is off
            dt = np.where(is_("dt_zero"), 0, dt)
            dt = np.where(is_("clock_backward"), -arng.integers(1, 5 * 10**9, size=N), dt)
            de = de.reshape(N, Z)
            de[is_("energy_unchanged")] = 0
            one = np.flatnonzero(is_("energy_unchanged_one_zone"))
            de[one, arng.integers(0, Z, size=one.size)] = 0
            de = de.reshape(-1)
            ratio = np.where(is_("ratio_one"), 1.0, ratio)
            ratio = np.where(is_("ratio_above_one"), 1.0 + arng.uniform(0.01, 1.0, size=N), ratio)
            ratio = np.where(is_("ratio_negative"), -arng.uniform(0.01, 0.5, size=N), ratio)
        self.ts = self.ts + dt
        self.counters = (self.counters + de) % self.zone_max
        status = np.zeros(N, dtype=np.uint32)
        if self.read_error_frac > 0 and self.interval > 0:
            status[rng.random(N) < self.read_error_frac] = KACC_NODE_READ_ERROR
        self.last_status = status
        self.last_scenario = scen
        return dict(node_ts_ns=self.ts.astype(np.int64), node_usage_ratio=ratio, node_status=status,
                    zone_energy=self.counters.copy(), zone_max=self.zone_max)

    def next_interval(self) -> Dict[str, np.ndarray]:
        L, rng = self.layout, self._rng
        P = L.n_procs
        first = self.interval == 0
        out = self.next_node_inputs()
        # processes: cumulative ticks -> Go's CPUTimeDelta = ticks/100 - prev
        dticks = np.where(rng.random(P) < 0.3, 0,
                          np.minimum(rng.lognormal(3.0, 1.5, size=P), 50_000.0)).astype(np.int64)
        proc_slot = L.proc_slot.copy()
        # rows of nodes whose read fails this interval: the reference skips Refresh
        # (monitor.go:399-408), so their informer cache (prev totals) stays and a process
        # born meanwhile is first seen at the node's next good interval
        skipped = (self.last_status[self.node_of_proc] & KACC_NODE_READ_ERROR) != 0
        if first:
            proc_slot |= np.uint32(KACC_SLOT_NEW)
        elif self.churn > 0:
            born = rng.random(P) < self.churn  # PID reuse of the slot by a new process
            self.cum_ticks[born] = 0
            self.prev_total[born] = 0.0
            self.pending_new |= born
        if not first:
            show = self.pending_new & ~skipped
            proc_slot[show] |= np.uint32(KACC_SLOT_NEW)
            self.pending_new &= skipped
        self.cum_ticks += dticks
        if self.adversarial > 0 and not first:
            arng = np.random.default_rng([self.seed, 0xAE, self.interval])
            scen = self.last_scenario[self.node_of_proc]
            names = [s[0] for s in self.ADVERSARIAL]
            # a reused PID in a cached entry: the new process's cumulative time is below the
            # old one's, and the entry is not new (informer.go:512-520) -> Δ < 0
            reuse = (scen == names.index("negative_cpu_delta")) & (arng.random(P) < 0.3)
            self.cum_ticks[reuse] = arng.integers(0, 50, size=int(reuse.sum()))
            # long-lived processes with huge cumulative times whose deltas cancel: ΔcpuNode is
            # tiny next to single deltas, ratios are huge, Energy() goes out of range
            cached = (proc_slot & np.uint32(KACC_SLOT_NEW)) == 0  # entries the informer already had
            huge = np.flatnonzero((scen == names.index("huge_cancelling_deltas")) & (arng.random(P) < 0.05) & cached)
            if huge.size:  # alternately +M (a long runner) and -M (a reused PID of one), M = 1e13 s
                up, down = huge[0::2], huge[1::2]
                self.cum_ticks[up] += 10**15
                self.prev_total[down] += 1e13
        total = self.cum_ticks.astype(np.float64) / 100.0
        cpu_delta = total - self.prev_total
        self.prev_total = np.where(skipped, self.prev_total, total)
        flag = np.uint32(KACC_SLOT_NEW) if first else np.uint32(0)
        self.interval += 1
        out.update(
            proc_cpu_delta=cpu_delta,
            proc_slot=proc_slot,
            ctr_slot=L.ctr_slot | flag,
            vm_slot=L.vm_slot | flag,
            pod_slot=L.pod_slot | flag,
        )
        out.update(L.static_arrays())
        return out


def _ranges(off: np.ndarray, nodes: np.ndarray):
    off = off.astype(np.int64)
    lo, hi = off[nodes], off[nodes + 1]
    idx = np.concatenate([np.arange(a, b) for a, b in zip(lo, hi)]) if len(nodes) else np.zeros(0, np.int64)
    new_off = np.zeros(len(nodes) + 1, dtype=np.int64)
    np.cumsum(hi - lo, out=new_off[1:])
    return idx.astype(np.int64), lo, new_off


def subset_interval(a: Dict[str, np.ndarray], nodes: np.ndarray, zones: int):
    """Extract the given nodes of a batch into a compact batch.

    Node snapshots are independent, so the oracle can check a sample of a
    full-size fleet.  Returns (arrays, sizes, maps) where maps[kind] are the
    original slot ids in compact-slot order (compact slot i <-> original
    maps[kind][i]) and maps["node"] the original node ids.
    """
    nodes = np.asarray(nodes, dtype=np.int64)
    out: Dict[str, np.ndarray] = {}
    pidx, p_lo, p_new = _ranges(a["proc_off"], nodes)
    cidx, c_lo, c_new = _ranges(a["ctr_off"], nodes)
    vidx, _, v_new = _ranges(a["vm_off"], nodes)
    qidx, _, q_new = _ranges(a["pod_off"], nodes)
    u32 = lambda x: np.ascontiguousarray(x, dtype=np.uint32)  # noqa: E731
    zidx = (nodes[:, None] * zones + np.arange(zones)[None, :]).reshape(-1)
    for name in ("node_ts_ns", "node_usage_ratio", "node_status", "node_cpu_delta"):
        if a.get(name) is not None:
            out[name] = np.ascontiguousarray(a[name][nodes])
    out["zone_energy"] = np.ascontiguousarray(a["zone_energy"][zidx])
    out["zone_max"] = np.ascontiguousarray(a["zone_max"][zidx])
    out["proc_off"], out["ctr_off"] = u32(p_new), u32(c_new)
    out["vm_off"], out["pod_off"] = u32(v_new), u32(q_new)
    out["proc_cpu_delta"] = np.ascontiguousarray(a["proc_cpu_delta"][pidx])
    # row shifts per node
    shift_p = np.repeat(p_new[:-1] - p_lo, np.diff(c_new))
    out["ctr_proc_end"] = u32(a["ctr_proc_end"][cidx].astype(np.int64) + shift_p)
    shift_pv = np.repeat(p_new[:-1] - p_lo, np.diff(v_new))
    out["vm_proc_end"] = u32(a["vm_proc_end"][vidx].astype(np.int64) + shift_pv)
    shift_c = np.repeat(c_new[:-1] - c_lo, np.diff(q_new))
    out["pod_ctr_end"] = u32(a["pod_ctr_end"][qidx].astype(np.int64) + shift_c)
    maps = {"node": nodes}
    for kind, idx in (("proc", pidx), ("ctr", cidx), ("vm", vidx), ("pod", qidx)):
        w = a[f"{kind}_slot"][idx].astype(np.uint32)
        orig = (w & np.uint32(0x7FFFFFFF)).astype(np.int64)
        out[f"{kind}_slot"] = u32(np.arange(len(idx), dtype=np.int64) | (w & np.uint32(0x80000000)))
        maps[kind] = orig
    sizes = dict(n_nodes=len(nodes), n_procs=len(pidx), n_ctrs=len(cidx), n_vms=len(vidx), n_pods=len(qidx))
    return out, sizes, maps


@dataclass
class KeyedChurn:
    """Per-row workload IDs with churn, for the slot join (kacc_slot_join).

    Row r of node n holds one live ID; each interval a ``churn`` fraction of
    rows is taken over by a new ID (the old one terminates), as PIDs turn over
    in /proc.  IDs are node-local PIDs (``kind='proc'``) or random 64-bit IDs
    (container / VM / pod string IDs hashed by the packer).
    """

    row_off: np.ndarray
    seed: int = SEED
    churn: float = 0.02
    kind: str = "proc"
    _rng: np.random.Generator = field(init=False, repr=False)

    def __post_init__(self):
        self._rng = np.random.default_rng(self.seed ^ 0x4A4F494E)
        off = self.row_off.astype(np.int64)
        n_rows = int(off[-1])
        self.node_of_row = np.repeat(np.arange(len(off) - 1), np.diff(off))
        if self.kind == "proc":
            # node-local PIDs: distinct per node, ascending-ish like /proc
            local = np.arange(n_rows) - off[self.node_of_row]
            self.keys = (300 + 3 * local + self._rng.integers(0, 3, size=n_rows)).astype(np.uint64)
            self.next_pid = np.full(len(off) - 1, 1 << 22, dtype=np.int64)
        else:
            self.keys = self._new_ids(n_rows)

    def _new_ids(self, k: int) -> np.ndarray:
        x = self._rng.integers(0, 2**63 - 1, size=k, dtype=np.int64).astype(np.uint64)
        return x * np.uint64(2) + np.uint64(1) - np.uint64(2) * (x == np.uint64(2**63 - 1))

    def next_keys(self) -> np.ndarray:
        """Advance one interval (churned rows get new IDs); returns the keys."""
        born = np.flatnonzero(self._rng.random(self.keys.size) < self.churn)
        if born.size:
            if self.kind == "proc":
                nodes = self.node_of_row[born]
                # new PIDs, increasing per node (never reused within the run)
                order = np.argsort(nodes, kind="stable")
                nb = nodes[order]
                first = np.r_[0, np.flatnonzero(np.diff(nb)) + 1]
                rank = np.arange(nb.size) - np.repeat(first, np.diff(np.r_[first, nb.size]))
                pids = self.next_pid[nb] + rank
                np.add.at(self.next_pid, nb, 1)
                self.keys[born[order]] = pids.astype(np.uint64)
            else:
                self.keys[born] = self._new_ids(born.size)
        return self.keys.copy()


class ProcChurn:
    """PIDs of a fleet's process rows under /proc-shaped churn, for the slot join.

    Rows are grouped by container (then VM, then the node's pod-less rest) in
    /proc listing order (informer.go:167-205), i.e. ascending PID inside a
    group.  Each interval a ``churn`` fraction of the processes exits and as
    many new ones start in the same group, each with a PID above every PID
    its node has used, so /proc lists it last in its group: the group sizes,
    hence the layout's CSR, stay fixed while rows shift inside the groups.
    """

    def __init__(self, layout: "FleetLayout", churn: float = 0.02, seed: int = SEED):
        self.rng = np.random.default_rng(seed ^ 0x50524F43)
        self.churn = churn
        off = layout.proc_off.astype(np.int64)
        self.n_rows = int(off[-1])
        self.node_of_row = np.repeat(np.arange(layout.n_nodes), np.diff(off))
        ends = np.unique(np.concatenate([layout.ctr_proc_end.astype(np.int64),
                                         layout.vm_proc_end.astype(np.int64), off[1:]]))
        # a row's group = the first segment end after it
        self.group = np.searchsorted(ends, np.arange(self.n_rows), side="right").astype(np.int64)
        local = np.arange(self.n_rows) - off[self.node_of_row]
        self.keys = (300 + 3 * local + self.rng.integers(0, 3, size=self.n_rows)).astype(np.uint32)
        self.next_pid = np.full(layout.n_nodes, 1 << 22, dtype=np.int64)
        self.started = False

    def next_keys(self) -> np.ndarray:
        """The keys of the next interval (the first call: the initial processes)."""
        if self.started:
            die = self.rng.random(self.n_rows) < self.churn
            k = np.flatnonzero(die)
            nd = self.node_of_row[k]  # ascending, as k is
            rank = np.arange(k.size) - np.searchsorted(nd, nd)
            keys = self.keys.copy()
            keys[k] = (self.next_pid[nd] + rank).astype(np.uint32)
            np.add.at(self.next_pid, nd, 1)
            # survivors keep their order, newcomers go last in their group
            self.keys = keys[np.argsort(self.group * 2 + die, kind="stable")]
        self.started = True
        return self.keys.copy()
