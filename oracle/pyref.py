"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product.

An independent pure-Python restatement of one collection interval, written
from the Go sources in Go's own shape (per-node NodeUsage zones, snapshots of
workloads keyed by ID, the informer's container / pod caches), not from the
C++ restatement in kepler_oracle.cpp.  It cross-checks that restatement on
small fleets (tests/test_pyref.py): every table bit for bit in the
listing-order summation mode (KOR_SUM_LISTING), i.e. Go's map iteration
replaced by the /proc listing order.

Inputs are the batch arrays of kepler_amd.fleet (a slot word stands for the
workload's ID; KACC_SLOT_NEW = the ID has no entry in the previous snapshot).
Python floats are IEEE doubles, and like Go on amd64 (GOAMD64=v1) Python
never fuses a*b+c, so every expression below rounds as Go's does.
"""

from __future__ import annotations

import numpy as np

SLOT_NEW = 0x80000000
SLOT_MASK = 0x7FFFFFFF
NODE_READ_ERROR = 0x1
NODE_OK, NODE_FIRST_READ, NODE_SKIPPED = 0, 1, 2
U64 = (1 << 64) - 1
TWO63 = float(1 << 63)


def cvttsd2sq(x: float) -> int:
    """amd64 CVTTSD2SQ: truncate toward zero; NaN / out of range -> INT64_MIN."""
    if not (-TWO63 <= x < TWO63):
        return -(1 << 63)
    return int(x)  # int() truncates toward zero


def go_float64_to_uint64(x: float) -> int:
    """cmd/compile ssagen float64ToUint64 (the Energy(...) conversions)."""
    if x < TWO63:
        return cvttsd2sq(x) & U64
    return (cvttsd2sq(x - TWO63) | (1 << 63)) & U64


def go_fdiv(a: float, b: float) -> float:
    """Go float64 division: IEEE, x/0 = ±Inf, 0/0 = NaN (no panic, unlike Python's `/`)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        return float(np.float64(a) / np.float64(b))


def go_trunc_divmod(d: int, m: int):
    """Go integer division and remainder (truncated toward zero)."""
    q = abs(d) // m
    q = q if d >= 0 else -q
    return q, d - q * m


def duration_seconds(d: int) -> float:
    """time.Duration.Seconds(): float64(d/1e9) + float64(d%1e9)/1e9."""
    sec, nsec = go_trunc_divmod(d, 1_000_000_000)
    return float(sec) + float(nsec) / 1e9


def sub_mono(t: int, u: int) -> int:
    """time.Time.Sub on monotonic readings, saturating."""
    d = t - u
    return max(min(d, (1 << 63) - 1), -(1 << 63))


def energy_delta(cur: int, prev: int, max_e: int) -> int:
    """node.go:87-98 calculateEnergyDelta (uint64 arithmetic)."""
    if cur >= prev:
        return cur - prev
    if max_e > 0:
        return ((max_e - prev) + cur) & U64
    return 0


USER_HZ = 100  # procfs_reader.go:73 userHZ


def go_cpu_time(ticks: int) -> float:
    """procWrapper.CPUTime (procfs_reader.go:75-82): float64(st.STime+st.UTime) / userHZ — the uint
    sum wraps mod 2^64, float64(uint64) rounds once (Python's float(int) rounds half to even), one
    IEEE division."""
    return float(ticks & U64) / USER_HZ


class Informer:
    """The informer's per-process CPU-time fields (populateProcessFields, informer.go:512-524) keyed
    by an ID: p.CPUTotalTime of the PID's previous reading, 0 for a process the cache does not hold.
    The tick format's oracle: feed it the same readings as the device tick map."""

    def __init__(self):
        self.total = {}  # ID -> p.CPUTotalTime (float64)

    def read(self, pid, ticks: int, new: bool) -> float:
        """One reading: returns p.CPUTimeDelta and updates p.CPUTotalTime.  ``new``: the cache has no
        entry for this process (a new Process, p.CPUTotalTime = 0)."""
        now = go_cpu_time(ticks)
        prev = 0.0 if new else self.total.get(pid, 0.0)
        self.total[pid] = now
        return now - prev


class PyRef:
    """Go-shaped state of a fleet of PowerMonitors (one per node)."""

    def __init__(self, zones: int, map_order_rng=None):
        """map_order_rng: a numpy Generator — sum the node's processes (informer.go:330-333)
        and each pod's containers (:284-310) in a random order, as Go's map iteration may;
        None = listing order."""
        self.Z = zones
        self.rng = map_order_rng
        self.node = {}         # n -> dict(ts, zones=[NodeUsage dict] , ratio, cpu_delta, status)
        self.snap = {k: {} for k in ("proc", "ctr", "vm", "pod")}  # kind -> {slot: [(E, P)] * Z}
        self.ctr_cache = {}    # slot -> [CPUTimeDelta, CPUTotalTime]  (informer containerCache)
        self.pod_cache = {}    # slot -> [CPUTimeDelta, CPUTotalTime]  (informer podCache)
        self.vm_cache = {}     # slot -> CPUTimeDelta
        self.node_status = {}  # n -> NODE_*

    # -- node.go -----------------------------------------------------------------
    def _node(self, n, a):
        Z = self.Z
        prev = self.node.get(n)
        ratio = float(a["node_usage_ratio"][n])
        now = int(a["node_ts_ns"][n])
        zones = []
        if prev is None:  # firstNodeRead, node.go:101-131
            for z in range(Z):
                e = int(a["zone_energy"][n * Z + z])
                active = go_float64_to_uint64(float(e) * ratio)
                zones.append(dict(EnergyTotal=e, ActiveEnergyTotal=active, IdleEnergyTotal=(e - active) & U64,
                                  activeEnergy=active, Power=0.0, ActivePower=0.0, IdlePower=0.0))
            self.node[n] = dict(ts=now, zones=zones, UsageRatio=0.0)
            return True
        dt = duration_seconds(sub_mono(now, prev["ts"]))  # node.go:34
        for z in range(Z):  # calculateNodePower, node.go:46-68
            pz = prev["zones"][z]
            e = int(a["zone_energy"][n * Z + z])
            delta = energy_delta(e, pz["EnergyTotal"], int(a["zone_max"][n * Z + z]))
            active = go_float64_to_uint64(float(delta) * ratio)
            idle = (delta - active) & U64
            p = go_fdiv(float(delta), dt)
            ap = p * ratio
            zones.append(dict(EnergyTotal=e, ActiveEnergyTotal=(pz["ActiveEnergyTotal"] + active) & U64,
                              IdleEnergyTotal=(pz["IdleEnergyTotal"] + idle) & U64, activeEnergy=active,
                              Power=p, ActivePower=ap, IdlePower=p - ap))
        self.node[n] = dict(ts=now, zones=zones, UsageRatio=ratio)
        return False

    # -- process.go / container.go / vm.go / pod.go ------------------------------
    def _attribute(self, kind, slot_word, cpu_delta, node_delta, zones, first, pod):
        s = slot_word & SLOT_MASK
        prev = None if (slot_word & SLOT_NEW) else self.snap[kind].get(s)
        out = []
        for z, nz in enumerate(zones):
            guard = nz["ActivePower"] if (first or not pod) else nz["Power"]  # pod.go:96 vs :23
            if guard == 0 or nz["activeEnergy"] == 0 or node_delta == 0:
                out.append((0, 0.0))  # newProcess's zero Usage
                continue
            ratio = cpu_delta / node_delta
            if pod:  # pod.go:102
                e = go_float64_to_uint64(float(nz["activeEnergy"]) * ratio)
            else:    # process.go:129
                e = go_float64_to_uint64(ratio * float(nz["activeEnergy"]))
            if first:  # first*Read: Power(0), EnergyTotal = interval energy
                out.append((e, 0.0))
                continue
            if prev is not None:
                e = (e + prev[z][0]) & U64
            out.append((e, ratio * nz["ActivePower"]))
        return s, out

    def interval(self, a: dict) -> None:
        Z = self.Z
        N = len(a["node_ts_ns"])
        po, co, vo, qo = (np.asarray(a[k], dtype=np.int64) for k in ("proc_off", "ctr_off", "vm_off", "pod_off"))
        d = a["proc_cpu_delta"]
        new_snap = {k: {} for k in self.snap}
        for n in range(N):
            status = int(a["node_status"][n]) if a.get("node_status") is not None else 0
            if status & NODE_READ_ERROR:  # node.go:39-44 -> previous snapshot kept, no Refresh
                self.node_status[n] = NODE_SKIPPED
                continue
            first = self._node(n, a)
            self.node_status[n] = NODE_FIRST_READ if first else NODE_OK
            zones = self.node[n]["zones"]
            p0, p1, c0, c1, v0, v1, q0, q1 = po[n], po[n + 1], co[n], co[n + 1], vo[n], vo[n + 1], qo[n], qo[n + 1]
            # Refresh (informer.go:223-345): containers in /proc listing order
            ctr_delta = {}
            begin = p0
            for c in range(c0, c1):
                w = int(a["ctr_slot"][c])
                s = w & SLOT_MASK
                cache = [0.0, 0.0] if (w & SLOT_NEW) else list(self.ctr_cache.get(s, [0.0, 0.0]))
                cache[0] = 0.0  # resetCPUTime on the container's first process
                for i in range(begin, int(a["ctr_proc_end"][c])):
                    cache[0] += float(d[i])
                    cache[1] += float(d[i])
                begin = int(a["ctr_proc_end"][c])
                self.ctr_cache[s] = cache
                ctr_delta[c] = cache
            for v in range(v0, v1):  # updateVMCache: last writer wins
                w = int(a["vm_slot"][v])
                delta = 0.0
                for i in range(begin, int(a["vm_proc_end"][v])):
                    delta = float(d[i])
                begin = int(a["vm_proc_end"][v])
                self.vm_cache[w & SLOT_MASK] = delta
            cbeg = c0
            for q in range(q0, q1):  # updatePodCache over the pod's containers
                w = int(a["pod_slot"][q])
                s = w & SLOT_MASK
                cache = [0.0, 0.0] if (w & SLOT_NEW) else list(self.pod_cache.get(s, [0.0, 0.0]))
                cache[0] = 0.0
                members = list(range(cbeg, int(a["pod_ctr_end"][q])))
                if self.rng is not None:
                    self.rng.shuffle(members)
                for c in members:
                    cache[0] += ctr_delta[c][0]
                    cache[1] += ctr_delta[c][1]  # quirk: the container's running total
                cbeg = int(a["pod_ctr_end"][q])
                self.pod_cache[s] = cache
            node_delta = 0.0  # refreshNode: Σ over running processes (a map in Go)
            order = np.arange(p0, p1)
            if self.rng is not None:
                self.rng.shuffle(order)
            for i in order:
                node_delta += float(d[i])
            self.node[n]["cpu_delta"] = node_delta
            for kind, rows, slots, deltas, pod in (
                ("proc", range(p0, p1), a["proc_slot"], lambda i: float(d[i]), False),
                ("ctr", range(c0, c1), a["ctr_slot"], lambda c: ctr_delta[c][0], False),
                ("vm", range(v0, v1), a["vm_slot"], lambda v: self.vm_cache[int(a["vm_slot"][v]) & SLOT_MASK], False),
                ("pod", range(q0, q1), a["pod_slot"], lambda q: self.pod_cache[int(a["pod_slot"][q]) & SLOT_MASK][0], True),
            ):
                got = {}
                for r in rows:
                    s, out = self._attribute(kind, int(slots[r]), deltas(r), node_delta, zones, first, pod)
                    got[s] = out
                new_snap[kind].update(got)
        for k in self.snap:  # a terminated workload keeps its last values in the tables
            self.snap[k].update(new_snap[k])

    # -- tables in the engine's layout -------------------------------------------
    def tables(self, nodes: int, caps: dict) -> dict:
        Z = self.Z
        t = {}
        for name, key in (("node_energy_total", "EnergyTotal"), ("node_active_energy", "activeEnergy"),
                          ("node_active_total", "ActiveEnergyTotal"), ("node_idle_total", "IdleEnergyTotal")):
            arr = np.zeros(nodes * Z, dtype=np.uint64)
            for n, st in self.node.items():
                for z in range(Z):
                    arr[n * Z + z] = st["zones"][z][key]
            t[name] = arr
        for name, key in (("node_power", "Power"), ("node_active_power", "ActivePower"),
                          ("node_idle_power", "IdlePower")):
            arr = np.zeros(nodes * Z, dtype=np.float64)
            for n, st in self.node.items():
                for z in range(Z):
                    arr[n * Z + z] = st["zones"][z][key]
            t[name] = arr
        t["node_ts"] = np.array([self.node[n]["ts"] if n in self.node else 0 for n in range(nodes)], dtype=np.int64)
        t["node_has_prev"] = np.array([1 if n in self.node else 0 for n in range(nodes)], dtype=np.uint32)
        t["node_usage_ratio"] = np.array([self.node[n]["UsageRatio"] if n in self.node else 0.0
                                          for n in range(nodes)], dtype=np.float64)
        t["node_cpu_delta"] = np.array([self.node[n].get("cpu_delta", 0.0) if n in self.node else 0.0
                                        for n in range(nodes)], dtype=np.float64)
        t["node_status"] = np.array([self.node_status.get(n, 0) for n in range(nodes)], dtype=np.uint32)
        for kind, cap in (("proc", "proc_slots"), ("ctr", "ctr_slots"), ("vm", "vm_slots"), ("pod", "pod_slots")):
            e = np.zeros(caps[cap] * Z, dtype=np.uint64)
            p = np.zeros(caps[cap] * Z, dtype=np.float64)
            for s, zs in self.snap[kind].items():
                for z, (ez, pz) in enumerate(zs):
                    e[s * Z + z] = ez
                    p[s * Z + z] = pz
            t[f"{kind}_energy"], t[f"{kind}_power"] = e, p
        for kind, cache, cap in (("ctr", self.ctr_cache, "ctr_slots"), ("pod", self.pod_cache, "pod_slots")):
            dd = np.zeros(caps[cap], dtype=np.float64)
            tt = np.zeros(caps[cap], dtype=np.float64)
            for s, (x, y) in cache.items():
                dd[s], tt[s] = x, y
            t[f"{kind}_cpu_delta"], t[f"{kind}_cpu_total"] = dd, tt
        vd = np.zeros(caps["vm_slots"], dtype=np.float64)
        for s, x in self.vm_cache.items():
            vd[s] = x
        t["vm_cpu_delta"] = vd
        return t

