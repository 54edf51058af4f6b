"""ctypes binding of the C ABI in include/kepler_accel.h (libkepler_accel.so).

This is the Python twin of the cgo shim described in INTEGRATION.md: the same
entry points a Go `internal/accel` package binds, used here by the tests and
the benchmark.  There is no CPU fallback: if the HIP library is missing the
import of :func:`load` raises, so a GPU run can never pass on a silent
substitute.
"""

from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_int, c_uint32, c_uint64, c_void_p
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KACC_LIB", os.path.join(_HERE, "lib", "libkepler_accel.so"))  # KACC_LIB: A/B builds

KACC_ABI_VERSION = 5
KACC_MAX_ZONES = 8
KACC_OK = 0
KACC_EINVAL = -1
KACC_EHIP = -2
KACC_ENOMEM = -3
KACC_ERANGE = -4
KACC_ESTATE = -5
KACC_SLOT_NEW = 0x80000000
KACC_SLOT_MASK = 0x7FFFFFFF
KACC_NODE_READ_ERROR = 0x1
KACC_NODE_OK = 0
KACC_NODE_FIRST_READ = 1
KACC_NODE_SKIPPED = 2
KACC_F_NODE_CPU_DELTA_GIVEN = 0x1
KACC_FMT_WIDTH = 24
KACC_KIND_PROC, KACC_KIND_CTR, KACC_KIND_VM, KACC_KIND_POD = 0, 1, 2, 3
KACC_JOIN_REUSE_TERMINATED = 1  # kacc_slotmap_set_policy
KACC_KEY_EMPTY = 0xFFFFFFFFFFFFFFFF
KACC_F_FAST_NODES = 0x2
KACC_F_TRUSTED_LAYOUT = 0x4
KACC_FAST_MAX_PROCS = 2048
KACC_FAST_MAX_AGGREGATES = 512
KACC_F_SMALL_NODES = 0x8
KACC_F_NODE_SLOT_RANGES = 0x10
KACC_SMALL_MAX_PROCS = 512
KACC_SMALL_MAX_AGGREGATES = 128
KACC_F_MEDIUM_NODES = 0x20
KACC_F_STABLE_SLOT_NODES = 0x40  # a slot never changes node except through a NEW row (slot join ranges)
KACC_MEDIUM_MAX_PROCS = 1024
KACC_MEDIUM_MAX_AGGREGATES = 256
KACC_UNIQUE_ID_BYTES = 128
KACC_PROC_REGULAR, KACC_PROC_CONTAINER, KACC_PROC_VM = 0, 1, 2
KACC_KEY_TOMB = 0xFFFFFFFFFFFFFFFE

# kacc_table enum, in header order: (name, numpy dtype)
TABLES = [
    ("node_energy_total", np.uint64),
    ("node_active_energy", np.uint64),
    ("node_active_total", np.uint64),
    ("node_idle_total", np.uint64),
    ("node_power", np.float64),
    ("node_active_power", np.float64),
    ("node_idle_power", np.float64),
    ("node_ts", np.int64),
    ("node_has_prev", np.uint32),
    ("node_usage_ratio", np.float64),
    ("node_cpu_delta", np.float64),
    ("node_status", np.uint32),
    ("proc_energy", np.uint64),
    ("proc_power", np.float64),
    ("ctr_energy", np.uint64),
    ("ctr_power", np.float64),
    ("ctr_cpu_delta", np.float64),
    ("ctr_cpu_total", np.float64),
    ("vm_energy", np.uint64),
    ("vm_power", np.float64),
    ("vm_cpu_delta", np.float64),
    ("pod_energy", np.uint64),
    ("pod_power", np.float64),
    ("pod_cpu_delta", np.float64),
    ("pod_cpu_total", np.float64),
    ("proc_ratio", np.float64),
    ("proc_node", np.uint32),
    ("ctr_ratio", np.float64),
    ("ctr_node", np.uint32),
    ("vm_ratio", np.float64),
    ("vm_node", np.uint32),
]
# derived on read (no device storage, no upload / device pointer): a process's (container's,
# VM's) power is cpuTimeRatio x its node's ActivePower (process.go:124-142; kacc_derive.hpp)
DERIVED_TABLES = {"proc_power", "ctr_power", "vm_power"}
# engine storage behind a derived table (not a Go quantity): the CPU restatements keep them
# only to check the engine's layout
ENGINE_TABLES = {"proc_ratio", "proc_node", "ctr_ratio", "ctr_node", "vm_ratio", "vm_node"}
# tables holding node indices (a subset / shard of a fleet renumbers its nodes)
NODE_INDEX_TABLES = {"proc_node", "ctr_node", "vm_node"}
TABLE_INDEX = {name: i for i, (name, _) in enumerate(TABLES)}

# exported symbols, in header order (checked by tests/test_abi.py)
EXPORTS = [
    "kacc_format_values",
    "kacc_format_lines",
    "kacc_zone_agg_create",
    "kacc_zone_agg_destroy",
    "kacc_zone_agg_read",
    "kacc_tracker_create",
    "kacc_tracker_destroy",
    "kacc_tracker_clear",
    "kacc_tracker_add",
    "kacc_tracker_items",
    "kacc_pack",
    "kacc_unpack",
    "kacc_slotmap_create",
    "kacc_slotmap_destroy",
    "kacc_slotmap_reset",
    "kacc_slotmap_set_policy",
    "kacc_slot_join",
    "kacc_tickmap_create",
    "kacc_tickmap_destroy",
    "kacc_tickmap_reset",
    "kacc_ticks_delta",
    "kacc_tickmap_download",
    "kacc_abi_version",
    "kacc_create",
    "kacc_destroy",
    "kacc_last_error",
    "kacc_get_config",
    "kacc_reset",
    "kacc_run_interval",
    "kacc_run_intervals",
    "kacc_sync",
    "kacc_time_next_launch",
    "kacc_validate_host",
    "kacc_batch_alloc",
    "kacc_batch_submit",
    "kacc_batch_wait",
    "kacc_batch_free",
    "kacc_table_info",
    "kacc_table_device_ptr",
    "kacc_table_row_stride",
    "kacc_table_download",
    "kacc_table_upload",
    "kacc_table_read",
    "kacc_namespace_totals",
    "kacc_create_multi",
    "kacc_cluster_unique_id",
    "kacc_cluster_join",
    "kacc_cluster_destroy",
    "kacc_cluster_rccl",
    "kacc_cluster_info",
    "kacc_allreduce_namespaces",
    "kacc_cluster_partials",
    "kacc_allreduce_sums",
    "kacc_allreduce_exports",
    "kacc_run_interval_sums",
    "kacc_run_export_sums",
    "kacc_gather_pods",
    "kacc_last_error_copy",
    "kacc_intervals_bytes",
    "kacc_interval_bytes",
]


class KaccConfig(ctypes.Structure):
    _fields_ = [
        ("zones", c_uint32),
        ("reserved0", c_uint32),
        ("nodes", c_uint64),
        ("proc_slots", c_uint64),
        ("ctr_slots", c_uint64),
        ("vm_slots", c_uint64),
        ("pod_slots", c_uint64),
    ]


# pointer fields of kacc_interval, in header order
INTERVAL_ARRAYS = [
    "node_ts_ns",
    "node_usage_ratio",
    "node_status",
    "node_cpu_delta",
    "node_order",
    "node_proc_span",
    "zone_energy",
    "zone_max",
    "proc_off",
    "ctr_off",
    "vm_off",
    "pod_off",
    "proc_cpu_delta",
    "proc_slot",
    "ctr_proc_end",
    "ctr_slot",
    "vm_proc_end",
    "vm_slot",
    "pod_ctr_end",
    "pod_slot",
]
# the optional ones may be NULL
OPTIONAL_ARRAYS = {"node_status", "node_cpu_delta", "node_order", "node_proc_span"}
ARRAY_DTYPES = {
    "node_ts_ns": np.int64,
    "node_usage_ratio": np.float64,
    "node_status": np.uint32,
    "node_cpu_delta": np.float64,
    "node_order": np.uint32,
    "node_proc_span": np.uint32,
    "zone_energy": np.uint64,
    "zone_max": np.uint64,
    "proc_off": np.uint32,
    "ctr_off": np.uint32,
    "vm_off": np.uint32,
    "pod_off": np.uint32,
    "proc_cpu_delta": np.float64,
    "proc_slot": np.uint32,
    "ctr_proc_end": np.uint32,
    "ctr_slot": np.uint32,
    "vm_proc_end": np.uint32,
    "vm_slot": np.uint32,
    "pod_ctr_end": np.uint32,
    "pod_slot": np.uint32,
}


class KaccRecords(ctypes.Structure):
    _fields_ = [("n_nodes", c_uint32), ("reserved0", c_uint32)] + [
        (n, c_void_p) for n in ("rec_off", "pid", "cpu_delta", "type", "ctr_key", "vm_key", "pod_key", "pod_ns")]


PACKED_ARRAYS = [("proc_off", np.uint32), ("ctr_off", np.uint32), ("vm_off", np.uint32), ("pod_off", np.uint32),
                 ("proc_cpu_delta", np.float64), ("proc_key", np.uint32), ("row_record", np.uint32),
                 ("ctr_proc_end", np.uint32), ("ctr_key", np.uint64), ("vm_proc_end", np.uint32),
                 ("vm_key", np.uint64), ("pod_ctr_end", np.uint32), ("pod_key", np.uint64), ("pod_ns", np.uint32)]


class KaccPacked(ctypes.Structure):
    _fields_ = [(n, c_uint32) for n in ("n_procs", "n_ctrs", "n_vms", "n_pods")] + [
        (n, c_void_p) for n, _ in PACKED_ARRAYS]


class KaccShape(ctypes.Structure):
    _fields_ = [(n, c_uint32) for n in ("n_nodes", "n_procs", "n_ctrs", "n_vms", "n_pods", "intervals")]


# optional per-interval OUTPUT arrays (device): the cluster-total exports, and (ABI 5) the
# export row of each batch pod (an input: namespace order)
INTERVAL_OUTPUTS = ["pod_export", "node_export", "pod_export_pos"]


class KaccInterval(ctypes.Structure):
    _fields_ = [
        ("n_nodes", c_uint32),
        ("n_procs", c_uint32),
        ("n_ctrs", c_uint32),
        ("n_vms", c_uint32),
        ("n_pods", c_uint32),
        ("flags", c_uint32),
    ] + [(name, c_void_p) for name in INTERVAL_ARRAYS + INTERVAL_OUTPUTS]


class KaccExportSums(ctypes.Structure):
    """kacc_export_sums: partial sums of an earlier interval's exports (kacc_run_interval_sums)."""
    _fields_ = [(n, c_uint32) for n in ("n_ns", "n_pods", "n_nodes", "ns_ordered")] + [
        (n, c_void_p) for n in ("ns_pod_off", "ns_pod_row", "pod_export", "node_export", "out_energy", "out_power",
                                "out_node_energy", "out_node_power")]


KACC_TICKS_ESCAPED = 0xFFFF
KACC_USER_HZ = 100


class KaccTicks(ctypes.Structure):
    """kacc_ticks: one interval's CPU-tick increments (kacc_ticks_delta)."""
    _fields_ = [(n, c_uint32) for n in ("n_nodes", "n_procs", "n_escapes", "reserved0")] + [
        (n, c_void_p) for n in ("proc_off", "node_status", "proc_slot", "dticks", "esc_off", "esc_row", "esc_ticks",
                                "proc_cpu_delta")]


def encode_ticks(proc_off, ticks_now, ticks_prev):
    """Host side of the tick format: per row the increment ticks_now - ticks_prev (u64 modular;
    ticks_prev = 0 for a NEW row) as u16, or KACC_TICKS_ESCAPED with an int64 escape when it is
    outside 0 .. 0xfffe.  Returns dticks [P] u16, esc_off [N+1] u32, esc_row [E] u32 (ascending
    within each node), esc_ticks [E] i64."""
    proc_off = np.asarray(proc_off, dtype=np.int64)
    inc = (np.asarray(ticks_now, dtype=np.uint64) - np.asarray(ticks_prev, dtype=np.uint64)).view(np.int64)
    esc = (inc < 0) | (inc >= KACC_TICKS_ESCAPED)
    dticks = np.where(esc, KACC_TICKS_ESCAPED, inc).astype(np.uint16)
    esc_row = np.flatnonzero(esc).astype(np.uint32)
    esc_off = np.searchsorted(esc_row, proc_off).astype(np.uint32)
    return dticks, esc_off, esc_row, inc[esc_row.astype(np.int64)].astype(np.int64)


class AccelError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"kacc error {code}: {msg}")
        self.code = code


_lib: Optional[ctypes.CDLL] = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libkepler_accel.so (raises if it was not built — no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(
            f"{path} not found: build it with `make -C kepler_amd/csrc` "
            "(or __graft_entry__.build()); there is no CPU fallback"
        )
    lib = ctypes.CDLL(path)
    lib.kacc_abi_version.restype = c_uint32
    lib.kacc_create.argtypes = [c_int, POINTER(KaccConfig), POINTER(c_void_p)]
    lib.kacc_destroy.argtypes = [c_void_p]
    lib.kacc_destroy.restype = None
    lib.kacc_last_error.argtypes = [c_void_p]
    lib.kacc_last_error.restype = c_char_p
    lib.kacc_get_config.argtypes = [c_void_p, POINTER(KaccConfig)]
    lib.kacc_reset.argtypes = [c_void_p]
    lib.kacc_run_interval.argtypes = [c_void_p, POINTER(KaccInterval), c_void_p]
    lib.kacc_format_lines.argtypes = [c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, c_char_p,
                                      POINTER(c_char_p), POINTER(ctypes.c_uint32), ctypes.c_uint32,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_uint64,
                                      POINTER(ctypes.c_uint64), c_void_p]
    lib.kacc_run_intervals.argtypes = [c_void_p, POINTER(KaccInterval), ctypes.c_uint32, c_void_p]
    lib.kacc_sync.argtypes = [c_void_p, c_void_p]
    lib.kacc_time_next_launch.argtypes = [c_void_p, c_void_p, c_void_p]
    lib.kacc_validate_host.argtypes = [c_void_p, POINTER(KaccInterval)]
    lib.kacc_batch_alloc.argtypes = [c_void_p, POINTER(KaccShape), POINTER(c_void_p), POINTER(POINTER(KaccInterval))]
    lib.kacc_pack.argtypes = [POINTER(KaccRecords), POINTER(KaccPacked), c_uint32]
    lib.kacc_unpack.argtypes = [c_void_p, c_int, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
    lib.kacc_last_error_copy.argtypes = [c_void_p, c_char_p, ctypes.c_size_t]
    lib.kacc_last_error_copy.restype = ctypes.c_size_t
    lib.kacc_create_multi.argtypes = [POINTER(c_int), c_int, POINTER(KaccConfig), POINTER(c_void_p),
                                      POINTER(c_void_p)]
    lib.kacc_cluster_unique_id.argtypes = [c_char_p]
    lib.kacc_cluster_join.argtypes = [c_void_p, c_char_p, c_int, c_int, POINTER(c_void_p)]
    lib.kacc_cluster_destroy.argtypes = [c_void_p]
    lib.kacc_cluster_destroy.restype = None
    lib.kacc_cluster_info.argtypes = [c_void_p, POINTER(c_int), POINTER(c_int), POINTER(c_int)]
    lib.kacc_cluster_rccl.argtypes = [POINTER(c_int), c_char_p, ctypes.c_size_t]
    lib.kacc_allreduce_namespaces.argtypes = [c_void_p, c_uint32] + [POINTER(c_void_p)] * 8
    lib.kacc_cluster_partials.argtypes = [c_void_p, c_uint32] + [POINTER(c_void_p)] * 7
    lib.kacc_allreduce_sums.argtypes = [c_void_p, POINTER(c_void_p), c_uint64, POINTER(c_void_p), c_uint64,
                                        POINTER(c_void_p), POINTER(c_void_p)]
    lib.kacc_allreduce_exports.argtypes = [c_void_p, c_uint32, POINTER(c_void_p), POINTER(c_void_p), POINTER(c_uint32),
                                           POINTER(c_void_p), POINTER(c_uint32)] + [POINTER(c_void_p)] * 7
    lib.kacc_tickmap_create.argtypes = [c_void_p, POINTER(c_void_p)]
    lib.kacc_tickmap_destroy.argtypes = [c_void_p]
    lib.kacc_tickmap_destroy.restype = None
    lib.kacc_tickmap_reset.argtypes = [c_void_p]
    lib.kacc_ticks_delta.argtypes = [c_void_p, POINTER(KaccTicks), c_void_p]
    lib.kacc_tickmap_download.argtypes = [c_void_p, c_uint64, c_uint64, c_void_p]
    lib.kacc_run_interval_sums.argtypes = [c_void_p, POINTER(KaccInterval), POINTER(KaccExportSums), c_void_p]
    lib.kacc_run_export_sums.argtypes = [c_void_p, POINTER(KaccExportSums), c_void_p]
    lib.kacc_gather_pods.argtypes = [c_void_p, POINTER(c_uint32), POINTER(c_void_p), c_uint64, POINTER(c_void_p),
                                     POINTER(c_void_p), POINTER(c_uint64), POINTER(c_uint64), POINTER(c_void_p)]
    lib.kacc_batch_submit.argtypes = [c_void_p, c_void_p]
    lib.kacc_batch_wait.argtypes = [c_void_p, c_void_p]
    lib.kacc_batch_free.argtypes = [c_void_p, c_void_p]
    lib.kacc_batch_free.restype = None
    lib.kacc_table_info.argtypes = [c_void_p, c_int, POINTER(c_uint64), POINTER(c_uint64)]
    lib.kacc_table_device_ptr.argtypes = [c_void_p, c_int, POINTER(c_void_p)]
    lib.kacc_table_row_stride.argtypes = [c_void_p, c_int, POINTER(c_uint64)]
    lib.kacc_table_download.argtypes = [c_void_p, c_int, c_uint64, c_uint64, c_void_p]
    lib.kacc_table_upload.argtypes = [c_void_p, c_int, c_uint64, c_uint64, c_void_p]
    if hasattr(lib, "kacc_table_read"):  # KACC_LIB A/B builds of earlier sources lack it
        lib.kacc_table_read.argtypes = [c_void_p, c_int, c_uint64, c_uint64, c_void_p, c_void_p]
    lib.kacc_namespace_totals.argtypes = [
        c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
    ]
    lib.kacc_interval_bytes.argtypes = [c_uint32, c_uint64, c_uint64, c_uint64, c_uint64, c_uint64, c_uint32]
    lib.kacc_interval_bytes.restype = c_uint64
    lib.kacc_intervals_bytes.argtypes = [c_uint32, c_uint64, c_uint64, c_uint64, c_uint64, c_uint64, c_uint32, c_int,
                                         c_uint32]
    lib.kacc_intervals_bytes.restype = c_uint64
    lib.kacc_debug_run_variant.argtypes = [c_void_p, POINTER(KaccInterval), c_void_p, c_int]
    lib.kacc_debug_run_intervals_variant.argtypes = [c_void_p, POINTER(KaccInterval), c_uint32, c_void_p, c_int]
    lib.kacc_debug_carry_stamps.argtypes = [c_void_p, POINTER(KaccInterval), c_uint32, c_void_p, c_int, c_void_p]
    lib.kacc_format_values.argtypes = [c_void_p, c_int, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p]
    lib.kacc_zone_agg_create.argtypes = [c_void_p, c_uint32, c_uint32, c_void_p, POINTER(c_void_p)]
    lib.kacc_zone_agg_destroy.argtypes = [c_void_p]
    lib.kacc_zone_agg_destroy.restype = None
    lib.kacc_zone_agg_read.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
    lib.kacc_tracker_create.argtypes = [c_void_p, c_int, ctypes.c_int64, c_uint32, c_uint32, c_uint64,
                                        POINTER(c_void_p)]
    lib.kacc_tracker_destroy.argtypes = [c_void_p]
    lib.kacc_tracker_destroy.restype = None
    lib.kacc_tracker_clear.argtypes = [c_void_p, c_void_p, c_void_p]
    lib.kacc_tracker_add.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
    lib.kacc_tracker_items.argtypes = [c_void_p, POINTER(c_uint32), c_void_p, c_void_p, c_void_p, c_void_p]
    lib.kacc_slotmap_create.argtypes = [c_void_p, c_int, c_uint32, c_void_p, POINTER(c_void_p)]
    lib.kacc_slotmap_destroy.argtypes = [c_void_p]
    lib.kacc_slotmap_destroy.restype = None
    lib.kacc_slotmap_reset.argtypes = [c_void_p]
    lib.kacc_slotmap_set_policy.argtypes = [c_void_p, c_uint32]
    lib.kacc_slot_join.argtypes = [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
    if lib.kacc_abi_version() != KACC_ABI_VERSION:
        raise ImportError("libkepler_accel ABI version mismatch")
    _lib = lib
    return lib


def last_error(ctx=None) -> str:
    """kacc_last_error_copy: the message of the last failed call (ctx None: without a context)."""
    lib = load()
    buf = ctypes.create_string_buffer(1024)
    lib.kacc_last_error_copy(ctx, buf, len(buf))
    return buf.value.decode()


def pack(rec_off, pid, cpu_delta, ptype, ctr_key, vm_key, pod_key=None, pod_ns=None, threads: int = 1,
         out: Optional[dict] = None) -> dict:
    """kacc_pack over host arrays: informer records (per node, /proc listing order) -> the
    interval CSR + slot-join keys + row_record.  ``out``: preallocated arrays (e.g. views of a
    pinned batch) to write into; by default arrays sized for the worst case are allocated and
    trimmed to the counts.  Returns the arrays and the counts (n_procs, ...)."""
    lib = load()
    rec_off = np.ascontiguousarray(rec_off, dtype=np.uint32)
    n_nodes = rec_off.size - 1
    R = int(rec_off[-1])
    arrs = dict(pid=np.ascontiguousarray(pid, dtype=np.uint32), cpu_delta=np.ascontiguousarray(cpu_delta, np.float64),
                type=np.ascontiguousarray(ptype, dtype=np.uint8), ctr_key=np.ascontiguousarray(ctr_key, np.uint64),
                vm_key=np.ascontiguousarray(vm_key, np.uint64))
    if pod_key is not None:
        arrs["pod_key"] = np.ascontiguousarray(pod_key, np.uint64)
    if pod_ns is not None:
        arrs["pod_ns"] = np.ascontiguousarray(pod_ns, np.uint32)
    for k, a in arrs.items():
        if a.size != R:
            raise ValueError(f"{k}: {a.size} records, rec_off says {R}")
    rec = KaccRecords(n_nodes, 0, rec_off.ctypes.data,
                      *[arrs[k].ctypes.data if k in arrs else None
                        for k in ("pid", "cpu_delta", "type", "ctr_key", "vm_key", "pod_key", "pod_ns")])
    if out is None:
        sizes = dict(proc_off=n_nodes + 1, ctr_off=n_nodes + 1, vm_off=n_nodes + 1, pod_off=n_nodes + 1)
        out = {n: np.zeros(max(sizes.get(n, R), 1), dtype=dt) for n, dt in PACKED_ARRAYS}
        caps = (R, R, R, R)
    else:
        caps = (out["proc_cpu_delta"].size, out["ctr_key"].size, out["vm_key"].size, out["pod_key"].size)
    pk = KaccPacked(*caps, *[out[n].ctypes.data if out.get(n) is not None else None for n, _ in PACKED_ARRAYS])
    rc = lib.kacc_pack(ctypes.byref(rec), ctypes.byref(pk), threads)
    if rc != KACC_OK:
        raise AccelError(rc, last_error(None))
    counts = dict(n_nodes=n_nodes, n_procs=pk.n_procs, n_ctrs=pk.n_ctrs, n_vms=pk.n_vms, n_pods=pk.n_pods)
    per = dict(proc=pk.n_procs, row=pk.n_procs, ctr=pk.n_ctrs, vm=pk.n_vms, pod=pk.n_pods)
    res = {}
    for n, _ in PACKED_ARRAYS:
        if out.get(n) is None:
            continue
        res[n] = out[n] if n.endswith("_off") else out[n][:per[n.split("_")[0]]]
    res.update(counts)
    return res


def interval_bytes(zones: int, n_nodes: int, n_procs: int, n_ctrs: int, n_vms: int, n_pods: int, flags: int = 0) -> int:
    return int(load().kacc_interval_bytes(zones, n_nodes, n_procs, n_ctrs, n_vms, n_pods, flags))


def intervals_bytes(zones: int, n_nodes: int, n_procs: int, n_ctrs: int, n_vms: int, n_pods: int, intervals: int,
                    carried: bool, flags: int = 0) -> int:
    return int(load().kacc_intervals_bytes(zones, n_nodes, n_procs, n_ctrs, n_vms, n_pods, intervals, int(carried),
                                           flags))


KACC_CARRY_MAX_ZONES = 2


def fused_intervals(flags: int, intervals: int, node_order: bool = False, zones: int = 2,
                    exports: bool = False) -> bool:
    """Whether kacc_run_intervals runs these K intervals as one carried-state launch (never with
    pod / node exports: those take the per-interval kernels)."""
    return (intervals > 1 and zones <= KACC_CARRY_MAX_ZONES and bool(flags & KACC_F_FAST_NODES)
            and bool(flags & KACC_F_NODE_SLOT_RANGES) and not flags & KACC_F_SMALL_NODES and not node_order
            and not exports)


def make_interval(arrays: dict, sizes: dict, flags: int = 0, ptr=None) -> KaccInterval:
    """Build a kacc_interval from a dict of arrays.

    `ptr(array) -> int` returns the address (numpy: ctypes.data, torch:
    data_ptr()).  Missing optional arrays become NULL.  The caller keeps the
    arrays alive while the descriptor is in use.
    """
    if ptr is None:
        ptr = lambda a: a.ctypes.data  # noqa: E731
    it = KaccInterval()
    it.n_nodes = sizes["n_nodes"]
    it.n_procs = sizes["n_procs"]
    it.n_ctrs = sizes["n_ctrs"]
    it.n_vms = sizes["n_vms"]
    it.n_pods = sizes["n_pods"]
    it.flags = flags
    for name in INTERVAL_ARRAYS:
        a = arrays.get(name)
        if a is None:
            if name not in OPTIONAL_ARRAYS:
                raise ValueError(f"missing array {name}")
            setattr(it, name, None)
        else:
            setattr(it, name, ptr(a) or None)  # empty torch tensors give 0 -> NULL
    for name in INTERVAL_OUTPUTS:
        a = arrays.get(name)
        setattr(it, name, (ptr(a) or None) if a is not None else None)
    return it


class Accel:
    """One engine context on one GPU (kacc_ctx)."""

    def __init__(self, zones: int, nodes: int, proc_slots: int, ctr_slots: int, vm_slots: int,
                 pod_slots: int, device: int = 0):
        self.lib = load()
        self.cfg = KaccConfig(zones, 0, nodes, proc_slots, ctr_slots, vm_slots, pod_slots)
        h = c_void_p()
        rc = self.lib.kacc_create(device, ctypes.byref(self.cfg), ctypes.byref(h))
        if rc != KACC_OK:
            raise AccelError(rc, last_error(None))
        self.ctx = h
        self.zones = zones
        self.device = device
        self.owned = True

    @classmethod
    def _wrap(cls, handle: int, zones: int, device: int, cfg: "KaccConfig") -> "Accel":
        """A context owned by a Cluster (kacc_create_multi): never kacc_destroy'ed here."""
        self = cls.__new__(cls)
        self.lib = load()
        self.cfg = cfg
        self.ctx = c_void_p(handle)
        self.zones = zones
        self.device = device
        self.owned = False
        return self

    # -- plumbing ---------------------------------------------------------
    def _check(self, rc: int) -> None:
        if rc != KACC_OK:
            raise AccelError(rc, self.lib.kacc_last_error(self.ctx).decode())

    def close(self) -> None:
        if self.ctx:
            if self.owned:
                self.lib.kacc_destroy(self.ctx)
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # -- hot path ----------------------------------------------------------
    def reset(self) -> None:
        self._check(self.lib.kacc_reset(self.ctx))

    def run_interval(self, dev_interval: KaccInterval, stream: int = 0) -> None:
        self._check(self.lib.kacc_run_interval(self.ctx, ctypes.byref(dev_interval), c_void_p(stream or None)))

    def run_interval_sums(self, dev_interval: KaccInterval, sums: Optional[KaccExportSums], stream: int = 0) -> None:
        """kacc_run_interval_sums: the interval and, in its launch, the partial sums of an earlier
        interval's exports (``sums``; None: a plain interval)."""
        self._check(self.lib.kacc_run_interval_sums(self.ctx, ctypes.byref(dev_interval),
                                                    ctypes.byref(sums) if sums is not None else None, stream))

    def export_sums(self, sums: KaccExportSums, stream: int = 0) -> None:
        """kacc_run_export_sums: the partial sums of an interval's exports as one launch."""
        self._check(self.lib.kacc_run_export_sums(self.ctx, ctypes.byref(sums), stream))

    def run_intervals(self, dev_intervals, stream: int = 0) -> None:
        """kacc_run_intervals: consecutive intervals issued back to back from C."""
        arr = (KaccInterval * len(dev_intervals))(*dev_intervals)
        self._check(self.lib.kacc_run_intervals(self.ctx, arr, len(dev_intervals), c_void_p(stream or None)))

    def run_variant(self, dev_interval: KaccInterval, stream: int, variant: int) -> None:
        """Timing ablation (kacc_debug.h); variant != 0 is not the reference semantics."""
        self._check(self.lib.kacc_debug_run_variant(self.ctx, ctypes.byref(dev_interval),
                                                    c_void_p(stream or None), variant))

    def run_intervals_variant(self, dev_intervals, stream: int, variant: int) -> None:
        """Timing ablation of the one-launch K-interval kernel (kacc_debug.h); variant != 0 is not
        the reference semantics."""
        arr = (KaccInterval * len(dev_intervals))(*dev_intervals)
        self._check(self.lib.kacc_debug_run_intervals_variant(self.ctx, arr, len(dev_intervals),
                                                              c_void_p(stream or None), variant))

    def carry_stamps(self, dev_intervals, stream: int, variant: int, d_out: int) -> None:
        """Per-wave phase cycle totals of the carry kernel into d_out (kacc_debug.h; diagnostic)."""
        arr = (KaccInterval * len(dev_intervals))(*dev_intervals)
        self._check(self.lib.kacc_debug_carry_stamps(self.ctx, arr, len(dev_intervals), c_void_p(stream or None),
                                                     variant, c_void_p(d_out)))

    def time_next_launch(self, start_event: int, stop_event: int) -> None:
        """kacc_time_next_launch: the next launching call records these hipEvent_t handles on its
        first kernel's start and its last kernel's end (dispatch packets, no marker packets)."""
        self._check(self.lib.kacc_time_next_launch(self.ctx, c_void_p(start_event or None),
                                                   c_void_p(stop_event or None)))

    def sync(self, stream: int = 0) -> None:
        self._check(self.lib.kacc_sync(self.ctx, c_void_p(stream or None)))

    def validate_host(self, host_interval: KaccInterval) -> int:
        return self.lib.kacc_validate_host(self.ctx, ctypes.byref(host_interval))

    def last_error(self) -> str:
        return self.lib.kacc_last_error(self.ctx).decode()

    # -- tables --------------------------------------------------------------
    def table_info(self, name: str):
        eb, cnt = c_uint64(), c_uint64()
        self._check(self.lib.kacc_table_info(self.ctx, TABLE_INDEX[name], ctypes.byref(eb), ctypes.byref(cnt)))
        return eb.value, cnt.value

    def download(self, name: str, first: int = 0, count: Optional[int] = None) -> np.ndarray:
        _, total = self.table_info(name)
        if count is None:
            count = total - first
        out = np.empty(count, dtype=TABLES[TABLE_INDEX[name]][1])
        self._check(self.lib.kacc_table_download(self.ctx, TABLE_INDEX[name], first, count, out.ctypes.data))
        return out

    def upload(self, name: str, values: np.ndarray, first: int = 0) -> None:
        v = np.ascontiguousarray(values, dtype=TABLES[TABLE_INDEX[name]][1])
        self._check(self.lib.kacc_table_upload(self.ctx, TABLE_INDEX[name], first, v.size, v.ctypes.data))

    def read(self, name: str, dev_dst: int, first: int = 0, count: Optional[int] = None, stream=None) -> None:
        """kacc_table_read: the logical range into device memory at dev_dst, on `stream` (derived
        tables derived, pod tables gathered out of their records)."""
        _, total = self.table_info(name)
        if count is None:
            count = total - first
        self._check(self.lib.kacc_table_read(self.ctx, TABLE_INDEX[name], first, count, dev_dst, stream))

    def row_stride(self, name: str) -> int:
        """kacc_table_row_stride: elements between two slots' rows (2Z for the pod tables' records)."""
        s = c_uint64()
        self._check(self.lib.kacc_table_row_stride(self.ctx, TABLE_INDEX[name], ctypes.byref(s)))
        return s.value

    def device_ptr(self, name: str) -> int:
        p = c_void_p()
        self._check(self.lib.kacc_table_device_ptr(self.ctx, TABLE_INDEX[name], ctypes.byref(p)))
        return p.value

    def state(self) -> dict:
        return {name: self.download(name) for name, _ in TABLES}

    def format_values(self, name: str, first: int, count: int, out_ptr: int, len_ptr: int, stream: int = 0) -> None:
        """kacc_format_values: exposition text of table elements (KACC_FMT_WIDTH-byte fields)."""
        self._check(self.lib.kacc_format_values(self.ctx, TABLE_INDEX[name], first, count, c_void_p(out_ptr),
                                                c_void_p(len_ptr), c_void_p(stream or None)))

    def format_lines(self, name: str, metric: str, first: int, count: int, zone_names, labels_ptr: int,
                     label_off_ptr: int, line_off_ptr: int, out_ptr: int = 0, out_cap: int = 0,
                     zone_order=None, row_order_ptr: int = 0, stream: int = 0) -> int:
        """kacc_format_lines: sample lines of table `name` (device pointers); returns the text size."""
        t = TABLE_INDEX[name]
        zn = (c_char_p * len(zone_names))(*[z.encode() for z in zone_names])
        zo = (ctypes.c_uint32 * len(zone_names))(*zone_order) if zone_order is not None else None
        total = ctypes.c_uint64(0)
        self._check(self.lib.kacc_format_lines(self.ctx, t, first, count, metric.encode(), zn, zo, len(zone_names),
                                               c_void_p(labels_ptr or None), c_void_p(label_off_ptr or None),
                                               c_void_p(row_order_ptr or None), c_void_p(line_off_ptr or None),
                                               c_void_p(out_ptr or None), out_cap, ctypes.byref(total),
                                               c_void_p(stream or None)))
        return total.value

    def unpack(self, kind: int, n: int, slot_words_ptr: int, dest_ptr: int, out_energy_ptr: int,
               out_power_ptr: int, stream: int = 0) -> None:
        """kacc_unpack: per-workload energy / power rows out of the state tables (device pointers)."""
        self._check(self.lib.kacc_unpack(self.ctx, kind, n, c_void_p(slot_words_ptr), c_void_p(dest_ptr or None),
                                         c_void_p(out_energy_ptr), c_void_p(out_power_ptr), c_void_p(stream or None)))

    def namespace_totals(self, n_ns: int, ns_pod_off_ptr: int, ns_pod_slot_ptr: int,
                         out_energy_ptr: int, out_power_ptr: int, stream: int = 0) -> None:
        self._check(self.lib.kacc_namespace_totals(
            self.ctx, n_ns, c_void_p(ns_pod_off_ptr), c_void_p(ns_pod_slot_ptr),
            c_void_p(out_energy_ptr), c_void_p(out_power_ptr), c_void_p(stream or None)))


class SlotMap:
    """Device slot join of one workload kind (kacc_slotmap, kacc_slot_join).

    Node n owns slots [slot_off[n], slot_off[n+1]) of the kind's state tables.
    ``join`` takes device pointers (torch ``data_ptr()``) and runs on ``stream``.
    """

    def __init__(self, accel: Accel, kind: int, slot_off: np.ndarray):
        self.accel = accel
        self.lib = accel.lib
        off = np.ascontiguousarray(slot_off, dtype=np.uint32)
        h = c_void_p()
        accel._check(self.lib.kacc_slotmap_create(accel.ctx, kind, off.size - 1, off.ctypes.data, ctypes.byref(h)))
        self.handle = h
        self.n_nodes = off.size - 1

    def reset(self) -> None:
        self.accel._check(self.lib.kacc_slotmap_reset(self.handle))

    def set_policy(self, policy: int) -> None:
        """KACC_JOIN_REUSE_TERMINATED: new rows take this call's terminated slots first."""
        self.accel._check(self.lib.kacc_slotmap_set_policy(self.handle, policy))

    def join(self, n_rows: int, row_off_ptr: int, keys_ptr: int, node_status_ptr: int, out_slot_ptr: int,
             term_key_ptr: int, term_slot_ptr: int, term_count_ptr: int, stream: int = 0,
             out_span_ptr: int = 0) -> None:
        """term_key / term_slot: [slot_off[-1]], term_count: [n_nodes] (per-node segments);
        out_span: optional [2*n_nodes] {min, max} slot per node (kacc_interval.node_proc_span)."""
        self.accel._check(self.lib.kacc_slot_join(
            self.handle, n_rows, c_void_p(row_off_ptr), c_void_p(keys_ptr or None),
            c_void_p(node_status_ptr or None), c_void_p(out_slot_ptr), c_void_p(term_key_ptr),
            c_void_p(term_slot_ptr), c_void_p(term_count_ptr), c_void_p(out_span_ptr or None),
            c_void_p(stream or None)))

    def close(self) -> None:
        if self.handle:
            self.lib.kacc_slotmap_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class TickMap:
    """kacc_tickmap: per process slot, the ticks (STime+UTime) of its last reading; kacc_ticks_delta
    turns a batch's tick increments into Go's CPUTimeDelta on the device."""

    def __init__(self, accel: Accel):
        self.accel = accel
        self.lib = accel.lib
        h = c_void_p()
        accel._check(self.lib.kacc_tickmap_create(accel.ctx, ctypes.byref(h)))
        self.h = h

    def reset(self) -> None:
        self.accel._check(self.lib.kacc_tickmap_reset(self.h))

    def delta(self, t: KaccTicks, stream: int = 0) -> None:
        self.accel._check(self.lib.kacc_ticks_delta(self.h, ctypes.byref(t), stream))

    def download(self, first: int = 0, count: Optional[int] = None) -> np.ndarray:
        if count is None:
            count = self.accel.cfg.proc_slots - first
        out = np.zeros(count, dtype=np.uint64)
        self.accel._check(self.lib.kacc_tickmap_download(self.h, first, count, out.ctypes.data))
        return out

    def close(self) -> None:
        if self.h:
            self.lib.kacc_tickmap_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class ZoneAgg:
    """Device AggregatedZone for every (node, zone) of a fleet (kacc_zone_agg_*)."""

    def __init__(self, accel: Accel, n_nodes: int, sockets: int, sub_max: np.ndarray):
        self.accel = accel
        self.lib = accel.lib
        m = np.ascontiguousarray(sub_max, dtype=np.uint64)
        h = c_void_p()
        accel._check(self.lib.kacc_zone_agg_create(accel.ctx, n_nodes, sockets, m.ctypes.data, ctypes.byref(h)))
        self.handle = h

    def read(self, readings_ptr: int, sub_status_ptr: int, out_energy_ptr: int, out_max_ptr: int,
             node_status_ptr: int, stream: int = 0) -> None:
        self.accel._check(self.lib.kacc_zone_agg_read(
            self.handle, c_void_p(readings_ptr), c_void_p(sub_status_ptr or None), c_void_p(out_energy_ptr),
            c_void_p(out_max_ptr), c_void_p(node_status_ptr), c_void_p(stream or None)))

    def close(self) -> None:
        if self.handle:
            self.lib.kacc_zone_agg_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class Tracker:
    """Device TerminatedResourceTracker of one kind (kacc_tracker_*)."""

    def __init__(self, accel: Accel, kind: int, max_size: int, zone: int, min_energy: int, capacity: int = 0):
        self.accel = accel
        self.lib = accel.lib
        self.zones = accel.zones
        h = c_void_p()
        accel._check(self.lib.kacc_tracker_create(accel.ctx, kind, max_size, capacity, zone, min_energy,
                                                  ctypes.byref(h)))
        self.handle = h

    def clear(self, stream: int = 0, node_mask_ptr: int = 0) -> None:
        """Clear every node's tracker, or the nodes whose (device) mask entry is nonzero."""
        self.accel._check(self.lib.kacc_tracker_clear(self.handle, c_void_p(node_mask_ptr or None),
                                                      c_void_p(stream or None)))

    def add(self, slotmap: "SlotMap", term_key_ptr: int, term_slot_ptr: int, term_count_ptr: int,
            stream: int = 0) -> None:
        self.accel._check(self.lib.kacc_tracker_add(self.handle, slotmap.handle, c_void_p(term_key_ptr),
                                                    c_void_p(term_slot_ptr), c_void_p(term_count_ptr),
                                                    c_void_p(stream or None)))

    def items(self):
        """(key u64[n], node u32[n], energy u64[n, Z], power f64[n, Z]): node by node, each node's
        items highest energy first."""
        n = c_uint32()
        self.accel._check(self.lib.kacc_tracker_items(self.handle, ctypes.byref(n), None, None, None, None))
        k = np.zeros(max(n.value, 1), np.uint64)
        nd = np.zeros(max(n.value, 1), np.uint32)
        e = np.zeros((max(n.value, 1), self.zones), np.uint64)
        p = np.zeros((max(n.value, 1), self.zones), np.float64)
        m = c_uint32()
        self.accel._check(self.lib.kacc_tracker_items(self.handle, ctypes.byref(m), k.ctypes.data, nd.ctypes.data,
                                                      e.ctypes.data, p.ctypes.data))
        c = m.value
        return k[:c], nd[:c], e[:c], p[:c]

    def close(self) -> None:
        if self.handle:
            self.lib.kacc_tracker_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def _field_count(name: str, n_nodes: int, n_procs: int, n_ctrs: int, n_vms: int, n_pods: int, zones: int) -> int:
    """Elements of kacc_interval array `name` for these sizes (kacc_engine.hip kBatchFields)."""
    if name in ("zone_energy", "zone_max"):
        return n_nodes * zones
    if name == "node_proc_span":
        return 2 * n_nodes
    if name.endswith("_off"):
        return n_nodes + 1
    if name.startswith("node_"):
        return n_nodes
    return {"proc": n_procs, "ctr": n_ctrs, "vm": n_vms, "pod": n_pods}[name.split("_", 1)[0]]


class HostBatch:
    """A pinned-host batch of `intervals` consecutive intervals (kacc_batch_*): the cgo path."""

    def __init__(self, accel: Accel, handle: c_void_p, views, shape: KaccShape):
        self.accel = accel
        self.handle = handle
        self.views = views
        self.shape = shape
        self.intervals = shape.intervals
        self.orig = [{name: getattr(views[k], name) for name in INTERVAL_ARRAYS} for k in range(shape.intervals)]

    @property
    def view(self):  # interval 0's descriptor (single-interval batches)
        return ctypes.pointer(self.views[0])

    @classmethod
    def alloc(cls, accel: Accel, n_nodes: int, n_procs: int, n_ctrs: int, n_vms: int, n_pods: int,
              intervals: int = 1):
        h = c_void_p()
        v = POINTER(KaccInterval)()
        shape = KaccShape(n_nodes, n_procs, n_ctrs, n_vms, n_pods, intervals)
        accel._check(accel.lib.kacc_batch_alloc(accel.ctx, ctypes.byref(shape), ctypes.byref(h), ctypes.byref(v)))
        return cls(accel, h, v, shape)

    def capacity(self, name: str) -> int:
        sh = self.shape
        return _field_count(name, sh.n_nodes, sh.n_procs, sh.n_ctrs, sh.n_vms, sh.n_pods, self.accel.zones)

    def array(self, name: str, count: int, k: int = 0) -> np.ndarray:
        if count > self.capacity(name):
            raise ValueError(f"{name}: {count} elements exceed the batch capacity {self.capacity(name)}")
        addr = self.orig[k][name]
        dt = np.dtype(ARRAY_DTYPES[name])
        buf = (ctypes.c_char * max(count * dt.itemsize, 1)).from_address(addr)
        return np.frombuffer(buf, dtype=dt, count=count)

    def fill(self, arrays: dict, flags: int = 0, k: int = 0, sizes: Optional[dict] = None) -> None:
        """Copy `arrays` into interval k's pinned views; `sizes` (default: the shape) sets the view's
        row counts, which may be below the shape's capacities."""
        v = self.views[k]
        sh = self.shape
        sz = sizes or dict(n_nodes=sh.n_nodes, n_procs=sh.n_procs, n_ctrs=sh.n_ctrs, n_vms=sh.n_vms,
                           n_pods=sh.n_pods)
        for key in ("n_nodes", "n_procs", "n_ctrs", "n_vms", "n_pods"):
            if sz[key] > getattr(sh, key):
                raise ValueError(f"{key}={sz[key]} exceeds the batch shape {getattr(sh, key)}")
            setattr(v, key, sz[key])
        v.flags = flags
        for name in INTERVAL_ARRAYS:
            setattr(v, name, self.orig[k][name])
            a = arrays.get(name)
            if a is None:
                if name in OPTIONAL_ARRAYS:
                    setattr(v, name, None)
                    continue
                raise ValueError(name)
            a = np.asarray(a)
            need = _field_count(name, sz["n_nodes"], sz["n_procs"], sz["n_ctrs"], sz["n_vms"], sz["n_pods"],
                                self.accel.zones)
            if a.size != need:
                raise ValueError(f"{name}: {a.size} elements, the view's sizes need {need}")
            self.array(name, a.size, k)[:] = a

    def submit(self) -> None:
        self.accel._check(self.accel.lib.kacc_batch_submit(self.accel.ctx, self.handle))

    def wait(self) -> None:
        self.accel._check(self.accel.lib.kacc_batch_wait(self.accel.ctx, self.handle))

    def free(self) -> None:
        if self.handle:
            self.accel.lib.kacc_batch_free(self.accel.ctx, self.handle)
            self.handle = None


def _ptrs(values) -> "ctypes.Array":
    return (c_void_p * len(values))(*[c_void_p(v or None) for v in values])


class Cluster:
    """Cluster totals over RCCL (kacc_create_multi / kacc_cluster_join, kacc_allreduce_namespaces,
    kacc_gather_pods).  ``shards`` are the local Accel contexts, in shard order."""

    def __init__(self, handle: c_void_p, shards, owns: bool):
        self.lib = load()
        self.handle = handle
        self.shards = list(shards)
        self.owns = owns

    @classmethod
    def create_multi(cls, devices, zones: int, capacities) -> "Cluster":
        """One process, one shard per entry of ``devices`` (capacities: per-shard dicts of Accel's
        nodes / proc_slots / ctr_slots / vm_slots / pod_slots)."""
        lib = load()
        n = len(devices)
        devs = (c_int * n)(*devices)
        cfgs = (KaccConfig * n)(*[KaccConfig(zones, 0, c["nodes"], c["proc_slots"], c["ctr_slots"], c["vm_slots"],
                                             c["pod_slots"]) for c in capacities])
        h = c_void_p()
        ctxs = (c_void_p * n)()
        rc = lib.kacc_create_multi(devs, n, cfgs, ctypes.byref(h), ctxs)
        if rc != KACC_OK:
            raise AccelError(rc, last_error(None))
        shards = [Accel._wrap(ctxs[i], zones, devices[i], cfgs[i]) for i in range(n)]
        return cls(h, shards, True)

    @staticmethod
    def unique_id() -> bytes:
        lib = load()
        buf = ctypes.create_string_buffer(KACC_UNIQUE_ID_BYTES)
        rc = lib.kacc_cluster_unique_id(buf)
        if rc != KACC_OK:
            raise AccelError(rc, last_error(None))
        return buf.raw

    @staticmethod
    def rccl():
        """kacc_cluster_rccl: (ncclGetVersion(), path of the loaded librccl) the library's
        collectives run with (raises AccelError when no usable RCCL is found)."""
        lib = load()
        v = c_int(0)
        buf = ctypes.create_string_buffer(4096)
        rc = lib.kacc_cluster_rccl(ctypes.byref(v), buf, len(buf))
        if rc != KACC_OK:
            raise AccelError(rc, last_error(None))
        return v.value, buf.value.decode()

    @classmethod
    def join(cls, accel: Accel, uid: bytes, nranks: int, rank: int) -> "Cluster":
        """One process per GPU: this rank's context joins the cluster named by ``uid``."""
        h = c_void_p()
        accel._check(accel.lib.kacc_cluster_join(accel.ctx, ctypes.create_string_buffer(uid, KACC_UNIQUE_ID_BYTES),
                                                 nranks, rank, ctypes.byref(h)))
        return cls(h, [accel], False)

    def info(self):
        a, b, c = c_int(), c_int(), c_int()
        self.lib.kacc_cluster_info(self.handle, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        return a.value, b.value, c.value

    def _check(self, rc: int) -> None:
        if rc != KACC_OK:
            raise AccelError(rc, self.shards[0].last_error())

    def allreduce_namespaces(self, n_ns: int, ns_pod_off, ns_pod_slot, out_energy, out_power,
                             out_node_energy=None, out_node_power=None, streams=None, comm_streams=None) -> None:
        """Per-shard lists of device pointers; node totals when out_node_* are given."""
        n = len(self.shards)
        if n_ns and not (len(ns_pod_off) == len(ns_pod_slot) == len(out_energy) == len(out_power) == n):
            raise ValueError("one namespace CSR and output pair per local shard")
        node = out_node_energy is not None
        self._check(self.lib.kacc_allreduce_namespaces(
            self.handle, n_ns, _ptrs(ns_pod_off) if n_ns else None, _ptrs(ns_pod_slot) if n_ns else None,
            _ptrs(out_energy) if n_ns else None, _ptrs(out_power) if n_ns else None,
            _ptrs(out_node_energy) if node else None, _ptrs(out_node_power) if node else None,
            _ptrs(streams) if streams else None, _ptrs(comm_streams) if comm_streams else None))

    def partials(self, n_ns: int, ns_pod_off, ns_pod_slot, out_energy, out_power, out_node_energy=None,
                 out_node_power=None, streams=None) -> None:
        """kacc_cluster_partials: each shard's partial sums only (no collective)."""
        n = len(self.shards)
        if n_ns and not (len(ns_pod_off) == len(ns_pod_slot) == len(out_energy) == len(out_power) == n):
            raise ValueError("one namespace CSR and output pair per local shard")
        node = out_node_energy is not None
        self._check(self.lib.kacc_cluster_partials(
            self.handle, n_ns, _ptrs(ns_pod_off) if n_ns else None, _ptrs(ns_pod_slot) if n_ns else None,
            _ptrs(out_energy) if n_ns else None, _ptrs(out_power) if n_ns else None,
            _ptrs(out_node_energy) if node else None, _ptrs(out_node_power) if node else None,
            _ptrs(streams) if streams else None))

    def allreduce_sums(self, energy, n_e: int, power, n_p: int, streams=None, comm_streams=None) -> None:
        """kacc_allreduce_sums: in-place sum over shards and ranks of per-shard u64 [n_e] / f64 [n_p]
        device vectors (several intervals' partials back to back: one collective for all)."""
        n = len(self.shards)
        if (n_e and len(energy) != n) or (n_p and len(power) != n):
            raise ValueError("one vector pair per local shard")
        self._check(self.lib.kacc_allreduce_sums(
            self.handle, _ptrs(energy) if n_e else None, n_e, _ptrs(power) if n_p else None, n_p,
            _ptrs(streams) if streams else None, _ptrs(comm_streams) if comm_streams else None))

    def allreduce_exports(self, n_ns: int, ns_pod_off, ns_pod_row, n_pods, pod_export, out_energy, out_power,
                          n_nodes=None, node_export=None, out_node_energy=None, out_node_power=None, streams=None,
                          comm_streams=None) -> None:
        """kacc_allreduce_exports: per-shard lists of device pointers (n_pods / n_nodes: ints);
        everything runs on comm_streams after the work queued on streams."""
        n = len(self.shards)
        node = out_node_energy is not None
        u32 = lambda v: (c_uint32 * n)(*v)  # noqa: E731
        self._check(self.lib.kacc_allreduce_exports(
            self.handle, n_ns, _ptrs(ns_pod_off) if n_ns else None, _ptrs(ns_pod_row) if n_ns else None,
            u32(n_pods) if n_ns else None, _ptrs(pod_export) if n_ns else None,
            u32(n_nodes) if node else None, _ptrs(node_export) if node else None,
            _ptrs(out_energy) if n_ns else None, _ptrs(out_power) if n_ns else None,
            _ptrs(out_node_energy) if node else None, _ptrs(out_node_power) if node else None,
            _ptrs(streams) if streams else None, _ptrs(comm_streams) if comm_streams else None))

    def gather_pods(self, n_pods, pod_slot, out_cap: int, out_energy, out_power, streams=None):
        """Returns (total pods, first global pod index of each local shard)."""
        n = len(self.shards)
        cnt = (c_uint32 * n)(*n_pods)
        total = c_uint64()
        first = (c_uint64 * n)()
        self._check(self.lib.kacc_gather_pods(self.handle, cnt, _ptrs(pod_slot), out_cap, _ptrs(out_energy),
                                              _ptrs(out_power), ctypes.byref(total), first,
                                              _ptrs(streams) if streams else None))
        return total.value, list(first)

    def close(self) -> None:
        if self.handle:
            self.lib.kacc_cluster_destroy(self.handle)
            self.handle = None
            if self.owns:
                for s in self.shards:
                    s.ctx = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
