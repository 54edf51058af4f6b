"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/build/libkepler_oracle.so, the CPU restatement of
Kepler's attribution path.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg import this module, as the checker or the CPU
baseline; the product path (kepler_amd) never does.
"""

from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_double, c_int, c_int64, c_uint8, c_uint32, c_uint64, c_void_p

import numpy as np

from kepler_amd.accel import TABLES, KaccInterval, make_interval

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libkepler_oracle.so")

KOR_SUM_TREE256 = 0
KOR_SUM_LISTING = 1


class KorState(ctypes.Structure):
    _fields_ = [("zones", c_uint32), ("reserved0", c_uint32), ("nodes", c_uint64),
                ("proc_slots", c_uint64), ("ctr_slots", c_uint64), ("vm_slots", c_uint64),
                ("pod_slots", c_uint64)] + [(name, c_void_p) for name, _ in TABLES]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    lib = ctypes.CDLL(LIB_PATH)
    lib.kor_go_f64_to_u64.argtypes = [c_double]
    lib.kor_go_f64_to_u64.restype = c_uint64
    lib.kor_go_duration_seconds.argtypes = [c_int64]
    lib.kor_go_duration_seconds.restype = c_double
    lib.kor_calculate_energy_delta.argtypes = [c_uint64, c_uint64, c_uint64]
    lib.kor_calculate_energy_delta.restype = c_uint64
    lib.kor_interval.argtypes = [POINTER(KorState), POINTER(KaccInterval), c_int]
    lib.kor_interval_mt.argtypes = [POINTER(KorState), POINTER(KaccInterval), c_int, c_int]
    lib.kor_namespace_totals.argtypes = [POINTER(KorState), c_uint32, c_void_p, c_void_p, c_void_p, c_void_p]
    lib.kor_aggregated_max.argtypes = [c_uint32, c_void_p]
    lib.kor_aggregated_max.restype = c_uint64
    lib.kor_aggregated_energy.argtypes = [c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_uint64]
    lib.kor_aggregated_energy.restype = c_uint64
    lib.kor_slotmap_create.argtypes = [c_uint32, c_void_p]
    lib.kor_slotmap_create.restype = c_void_p
    lib.kor_slotmap_set_policy.argtypes = [c_void_p, c_uint32]
    lib.kor_slotmap_set_policy.restype = None
    lib.kor_slotmap_destroy.argtypes = [c_void_p]
    lib.kor_slotmap_destroy.restype = None
    lib.kor_slot_join.argtypes = [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_void_p]
    lib.kor_tracker_create.argtypes = [ctypes.c_int64, c_uint64, c_uint32, c_uint32]
    lib.kor_tracker_create.restype = c_void_p
    lib.kor_tracker_destroy.argtypes = [c_void_p]
    lib.kor_tracker_destroy.restype = None
    lib.kor_tracker_clear.argtypes = [c_void_p]
    lib.kor_tracker_clear.restype = None
    lib.kor_tracker_clear_node.argtypes = [c_void_p, c_uint32]
    lib.kor_tracker_clear_node.restype = None
    lib.kor_tracker_add_one.argtypes = [c_void_p, c_uint32, c_uint64, c_void_p, c_void_p]
    lib.kor_tracker_add_one.restype = None
    lib.kor_tracker_add_batch.argtypes = [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
    lib.kor_tracker_add_batch.restype = None
    lib.kor_tracker_items.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
    lib.kor_tracker_items.restype = c_uint32
    lib.kor_aggregated_energy_st.argtypes = [c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                             c_void_p, c_uint64, c_void_p]
    lib.kor_gf_create.argtypes = [c_uint32]
    lib.kor_gf_create.restype = c_void_p
    lib.kor_gf_destroy.argtypes = [c_void_p]
    lib.kor_gf_destroy.restype = None
    lib.kor_gf_interval.argtypes = [c_void_p, POINTER(KorState), POINTER(KaccInterval)]
    _lib = lib
    return lib


def go_f64_to_u64(x: float) -> int:
    return int(load().kor_go_f64_to_u64(x))


def go_duration_seconds(ns: int) -> float:
    return float(load().kor_go_duration_seconds(ns))


def calculate_energy_delta(cur: int, prev: int, max_j: int) -> int:
    return int(load().kor_calculate_energy_delta(cur, prev, max_j))


class OracleState:
    """Host state tables with the same layout as the device tables."""

    def __init__(self, zones, nodes, proc_slots, ctr_slots, vm_slots, pod_slots):
        self.zones = zones
        per = {"node": nodes, "proc": proc_slots, "ctr": ctr_slots, "vm": vm_slots, "pod": pod_slots}
        zoned = {"energy", "power", "energy_total", "active_energy", "active_total", "idle_total",
                 "active_power", "idle_power"}
        self.t = {}
        for name, dt in TABLES:
            kind, rest = name.split("_", 1)
            n = per[kind] * (zones if rest in zoned else 1)
            self.t[name] = np.zeros(max(n, 1), dtype=dt)[:n] if n else np.zeros(0, dtype=dt)
        self.c = KorState(zones, 0, nodes, proc_slots, ctr_slots, vm_slots, pod_slots,
                          *[self.t[name].ctypes.data for name, _ in TABLES])

    def __getitem__(self, name):
        return self.t[name]

    def copy_tables(self):
        return {k: v.copy() for k, v in self.t.items()}


class Oracle:
    def __init__(self, zones, nodes, proc_slots, ctr_slots, vm_slots, pod_slots, sum_mode=KOR_SUM_TREE256):
        self.lib = load()
        self.state = OracleState(zones, nodes, proc_slots, ctr_slots, vm_slots, pod_slots)
        self.sum_mode = sum_mode

    def interval(self, arrays: dict, sizes: dict, flags: int = 0) -> None:
        it = make_interval(arrays, sizes, flags)
        rc = self.lib.kor_interval(ctypes.byref(self.state.c), ctypes.byref(it), self.sum_mode)
        if rc != 0:
            raise RuntimeError(f"kor_interval failed: {rc}")

    def interval_mt(self, arrays: dict, sizes: dict, threads: int, flags: int = 0) -> None:
        """kor_interval over `threads` host threads (the multi-core CPU baseline)."""
        it = make_interval(arrays, sizes, flags)
        rc = self.lib.kor_interval_mt(ctypes.byref(self.state.c), ctypes.byref(it), self.sum_mode, threads)
        if rc != 0:
            raise RuntimeError(f"kor_interval_mt failed: {rc}")

    def namespace_totals(self, ns_off: np.ndarray, ns_slot: np.ndarray):
        n_ns = len(ns_off) - 1
        e = np.zeros(n_ns * self.state.zones, dtype=np.uint64)
        p = np.zeros(n_ns * self.state.zones, dtype=np.float64)
        ns_off = np.ascontiguousarray(ns_off, dtype=np.uint32)
        ns_slot = np.ascontiguousarray(ns_slot, dtype=np.uint32)
        self.lib.kor_namespace_totals(ctypes.byref(self.state.c), n_ns, ns_off.ctypes.data,
                                      ns_slot.ctypes.data, e.ctypes.data, p.ctypes.data)
        return e, p


class GoFaithful:
    """The Go-data-structure baseline (string-keyed maps, per-object zone maps)."""

    def __init__(self, zones, nodes, proc_slots, ctr_slots, vm_slots, pod_slots):
        self.lib = load()
        self.state = OracleState(zones, nodes, proc_slots, ctr_slots, vm_slots, pod_slots)
        self.h = self.lib.kor_gf_create(zones)

    def interval(self, arrays: dict, sizes: dict, flags: int = 0) -> None:
        it = make_interval(arrays, sizes, flags)
        rc = self.lib.kor_gf_interval(self.h, ctypes.byref(self.state.c), ctypes.byref(it))
        if rc != 0:
            raise RuntimeError(f"kor_gf_interval failed: {rc}")

    def close(self):
        if self.h:
            self.lib.kor_gf_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


class AggregatedZone:
    """device/energy_zone.go:97-148 over n sub-zones (KAT helper)."""

    def __init__(self, sub_max):
        self.lib = load()
        self.sub_max = np.ascontiguousarray(sub_max, dtype=np.uint64)
        self.n = len(self.sub_max)
        self.last = np.zeros(self.n, dtype=np.uint64)
        self.seen = np.zeros(self.n, dtype=np.uint8)
        self.current = np.zeros(1, dtype=np.uint64)
        self.max = int(self.lib.kor_aggregated_max(self.n, self.sub_max.ctypes.data))

    def energy(self, readings) -> int:
        r = np.ascontiguousarray(readings, dtype=np.uint64)
        return int(self.lib.kor_aggregated_energy(self.n, r.ctypes.data, self.sub_max.ctypes.data,
                                                  self.last.ctypes.data, self.seen.ctypes.data,
                                                  self.current.ctypes.data, self.max))


class OracleZoneAgg:
    """AggregatedZone for every (node, zone) of a fleet: sub-zones [N*Z*S] (oracle)."""

    def __init__(self, n_nodes: int, zones: int, sockets: int, sub_max):
        self.nz, self.S = n_nodes * zones, sockets
        self.Z = zones
        m = np.ascontiguousarray(sub_max, dtype=np.uint64).reshape(self.nz, sockets)
        self.zones = [AggregatedZone(m[i]) for i in range(self.nz)]

    def read(self, readings, sub_status=None):
        """Returns (energy [N*Z], max [N*Z], node_status [N] with read errors)."""
        lib = load()
        r = np.ascontiguousarray(readings, dtype=np.uint64).reshape(self.nz, self.S)
        st = None if sub_status is None else np.ascontiguousarray(sub_status, dtype=np.uint32).reshape(self.nz, self.S)
        e = np.zeros(self.nz, np.uint64)
        mx = np.array([z.max for z in self.zones], dtype=np.uint64)
        ns = np.zeros(self.nz // self.Z, np.uint32)
        for i, z in enumerate(self.zones):
            out = np.zeros(1, np.uint64)
            ri = np.ascontiguousarray(r[i])
            si = None if st is None else np.ascontiguousarray(st[i])
            rc = lib.kor_aggregated_energy_st(self.S, ri.ctypes.data, None if si is None else si.ctypes.data,
                                              z.sub_max.ctypes.data, z.last.ctypes.data, z.seen.ctypes.data,
                                              z.current.ctypes.data, z.max, out.ctypes.data)
            if rc != 0:
                ns[i // self.Z] |= 1
            else:
                e[i] = out[0]
        return e, mx, ns


class OracleSlotMap:
    """CPU restatement of kacc_slot_join (oracle/kor_join.cpp)."""

    def __init__(self, slot_off: np.ndarray, policy: int = 0):
        self.lib = load()
        self.off = np.ascontiguousarray(slot_off, dtype=np.uint32)
        self.h = self.lib.kor_slotmap_create(self.off.size - 1, self.off.ctypes.data)
        if policy:  # KACC_JOIN_REUSE_TERMINATED
            self.lib.kor_slotmap_set_policy(self.h, policy)

    def join(self, row_off, keys, node_status=None):
        """Returns (rc, out_slot, term_key, term_slot, term_count) on host arrays;
        node n's terminated IDs are term_*[slot_off[n] : slot_off[n] + term_count[n]]."""
        row_off = np.ascontiguousarray(row_off, dtype=np.uint32)
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        n_rows = int(row_off[-1])
        out = np.zeros(max(n_rows, 1), dtype=np.uint32)
        cap = max(int(self.off[-1]), 1)
        tk = np.zeros(cap, dtype=np.uint64)
        ts = np.zeros(cap, dtype=np.uint32)
        cnt = np.zeros(max(self.off.size - 1, 1), dtype=np.uint32)
        st = None if node_status is None else np.ascontiguousarray(node_status, dtype=np.uint32)
        rc = self.lib.kor_slot_join(self.h, n_rows, row_off.ctypes.data, keys.ctypes.data if keys.size else None,
                                    None if st is None else st.ctypes.data, out.ctypes.data, tk.ctypes.data,
                                    ts.ctypes.data, cnt.ctypes.data)
        return rc, out[:n_rows], tk, ts, cnt[: self.off.size - 1]

    def terminated(self, tk, ts, cnt):
        """Flatten the per-node segments to a list of (key, slot)."""
        out = []
        for n, c in enumerate(cnt.tolist()):
            s0 = int(self.off[n])
            out += list(zip(tk[s0:s0 + c].tolist(), ts[s0:s0 + c].tolist()))
        return out

    def __del__(self):  # pragma: no cover
        try:
            self.lib.kor_slotmap_destroy(self.h)
        except Exception:
            pass


class OracleTracker:
    """TerminatedResourceTracker with Go's container/heap (oracle/kor_tracker.cpp)."""

    def __init__(self, max_size: int, min_energy: int, zones: int, zone: int = 0):
        self.lib = load()
        self.zones = zones
        self.h = self.lib.kor_tracker_create(max_size, min_energy, zones, zone)

    def clear(self, nodes=None):
        """Clear every node's tracker, or those of `nodes`."""
        if nodes is None:
            self.lib.kor_tracker_clear(self.h)
        else:
            for n in nodes:
                self.lib.kor_tracker_clear_node(self.h, int(n))

    def add_one(self, node: int, key: int, energy, power=None):
        e = np.ascontiguousarray(energy, dtype=np.uint64)
        p = np.zeros(self.zones) if power is None else np.ascontiguousarray(power, dtype=np.float64)
        self.lib.kor_tracker_add_one(self.h, node, key, e.ctypes.data, p.ctypes.data)

    def add_batch(self, node, key, slot, tab_e, tab_p):
        node = np.ascontiguousarray(node, dtype=np.uint32)
        key = np.ascontiguousarray(key, dtype=np.uint64)
        slot = np.ascontiguousarray(slot, dtype=np.uint32)
        tab_e = np.ascontiguousarray(tab_e, dtype=np.uint64)
        tab_p = np.ascontiguousarray(tab_p, dtype=np.float64)
        if node.size:
            self.lib.kor_tracker_add_batch(self.h, node.size, node.ctypes.data, key.ctypes.data, slot.ctypes.data,
                                           tab_e.ctypes.data, tab_p.ctypes.data)

    def items(self):
        """(key, node, energy [n, Z], power [n, Z]) sorted by (node, key)."""
        n = self.lib.kor_tracker_items(self.h, None, None, None, None)
        k = np.zeros(max(n, 1), np.uint64)
        nd = np.zeros(max(n, 1), np.uint32)
        e = np.zeros((max(n, 1), self.zones), np.uint64)
        p = np.zeros((max(n, 1), self.zones), np.float64)
        self.lib.kor_tracker_items(self.h, k.ctypes.data, nd.ctypes.data, e.ctypes.data, p.ctypes.data)
        return k[:n], nd[:n], e[:n], p[:n]

    def __del__(self):  # pragma: no cover
        try:
            self.lib.kor_tracker_destroy(self.h)
        except Exception:
            pass
