/*
 * kepler_accel.h — C ABI of the MI355X power-attribution engine.
 *
 * This is the drop-in boundary for Kepler's attribution hot path.  In the
 * reference the computation is private to PowerMonitor:
 *
 *   internal/monitor/monitor.go:399-431  PowerMonitor.calculatePower
 *     -> node.go:10-84      calculateNodePower   (+ node.go:87-98 calculateEnergyDelta,
 *                                                   node.go:101-131 firstNodeRead)
 *     -> resource/informer.go:349-410 Refresh    (segmented CPU-time sums:
 *                                                   informer.go:223-249/469-489 containers,
 *                                                   informer.go:275-326/491-510 pods,
 *                                                   informer.go:251-273/433-449 VMs,
 *                                                   informer.go:328-345 node total)
 *     -> process.go:79-161  calculateProcessPower
 *     -> container.go:71-153 calculateContainerPower
 *     -> vm.go:46-121       calculateVMPower
 *     -> pod.go:46-131      calculatePodPower
 *
 * The Go side (device zone readers, procfs informer, PowerMonitor snapshot
 * orchestration, exporters) is kept.  A cgo package internal/accel (see
 * INTEGRATION.md) packs one interval for a whole fleet of nodes into the
 * structure-of-arrays batch below and calls kacc_run_interval(); the results
 * land in device-resident state tables indexed by node and by workload slot,
 * which the shim reads back into monitor.Snapshot.
 *
 * Units follow internal/device/energy.go: energy is uint64 micro-joules
 * (energy.go:14), power is float64 micro-watts (energy.go:41).  Arithmetic
 * follows Go on amd64 exactly: uint64 modular add/sub, float64 IEEE with no
 * FMA contraction, float64->uint64 conversion with Go's amd64 semantics,
 * time.Duration.Seconds() for the interval length.
 *
 * All functions return 0 on success and a negative KACC_E* code on failure;
 * kacc_last_error() gives the message.  Every entry point calls
 * hipSetDevice(ctx device) first, so calls may come from any OS thread (cgo);
 * calls on one context must be serialised by the caller (the reference
 * serialises calculatePower with singleflight, monitor.go:265-302).
 */
#ifndef KEPLER_ACCEL_H
#define KEPLER_ACCEL_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KACC_ABI_VERSION 5u
#define KACC_MAX_ZONES 8u

/* Status codes. */
#define KACC_OK 0
#define KACC_EINVAL (-1)  /* bad argument / shape */
#define KACC_EHIP (-2)    /* HIP runtime error */
#define KACC_ENOMEM (-3)  /* device or pinned allocation failed */
#define KACC_ERANGE (-4)  /* device detected an out-of-range index in a batch */
#define KACC_ESTATE (-5)  /* call not valid in the current state */

/* Slot words: bits 0..30 index a workload slot table, bit 31 marks a workload
 * that has no previous snapshot entry (first time its ID is seen; the Go code
 * then uses the interval energy alone, process.go:133-138).                   */
#define KACC_SLOT_NEW 0x80000000u
#define KACC_SLOT_MASK 0x7fffffffu

/* node_status bits (input). */
#define KACC_NODE_READ_ERROR 0x1u /* a zone read failed: node.go:39-44 -> the whole
                                      interval fails and the previous snapshot is
                                      kept (monitor.go:328-335)                   */
/* node_status_out values (state table). */
#define KACC_NODE_OK 0u
#define KACC_NODE_FIRST_READ 1u /* firstReading path, monitor.go:366-397 */
#define KACC_NODE_SKIPPED 2u    /* read error: state left untouched      */

/* kacc_interval.flags */
#define KACC_F_NODE_CPU_DELTA_GIVEN 0x1u /* use node_cpu_delta[] instead of the
                                             on-device sum (mock informers)     */
#define KACC_F_FAST_NODES 0x2u /* caller guarantees every node has at most
                                   KACC_FAST_MAX_PROCS process rows and at most
                                   KACC_FAST_MAX_AGGREGATES containers+VMs+pods:
                                   the big-node (chunk / deferred-pod) launches
                                   are skipped.  A node that does not fit is not
                                   computed and raises KACC_ERANGE (bit 32).
                                   kacc_batch_submit sets it by itself.       */
#define KACC_F_TRUSTED_LAYOUT 0x4u /* kacc_batch_submit skips the host layout
                                       check (kacc_validate_host): for packers
                                       whose slots come from kacc_slot_join.  The
                                       device still clamps every index and raises
                                       KACC_ERANGE; only duplicate slots go
                                       unchecked (they would race, not fault). */
#define KACC_F_SMALL_NODES 0x8u /* caller guarantees every node has at most
                                    KACC_SMALL_MAX_PROCS process rows and at most
                                    KACC_SMALL_MAX_AGGREGATES containers+VMs+pods:
                                    one wavefront per node (4 nodes per
                                    workgroup), bit-identical results; implies
                                    KACC_F_FAST_NODES.  A node that does not fit
                                    is not computed and raises KACC_ERANGE (bit
                                    32).  kacc_batch_submit sets it by itself. */
#define KACC_F_NODE_SLOT_RANGES 0x10u /* caller guarantees every workload slot the
                                          batch's rows and aggregates use belongs to
                                          one node only for the whole call (the
                                          per-node slot ranges of kacc_slot_join).
                                          With KACC_F_FAST_NODES on every batch of a
                                          kacc_run_intervals call, the K intervals
                                          run as ONE launch (each node carried
                                          through K intervals by one workgroup);
                                          results are bit-identical.            */
#define KACC_F_MEDIUM_NODES 0x20u /* caller guarantees every node has at most
                                     KACC_MEDIUM_MAX_PROCS process rows and at
                                     most KACC_MEDIUM_MAX_AGGREGATES containers+
                                     VMs+pods; implies KACC_F_FAST_NODES.  The
                                     one-launch K-interval path then runs 256-
                                     thread workgroups (four per CU: a 1k-node
                                     shard resident at once).  A node that does
                                     not fit is not computed and raises
                                     KACC_ERANGE (bit 32).  kacc_batch_submit
                                     sets it by itself.                      */
#define KACC_F_STABLE_SLOT_NODES 0x40u /* caller guarantees that a process
                                          slot's node never changes while this
                                          context lives, except through a row
                                          whose slot word carries KACC_SLOT_NEW
                                          (a slot stays in one node's range:
                                          kacc_slot_join's fixed per-node
                                          ranges).  KACC_T_PROC_NODE then already
                                          holds the node of every other row, so
                                          the interval writes it only for NEW
                                          rows and on a node's first read: 4 B
                                          per process row less HBM traffic (the
                                          one-wavefront-per-node kernel of
                                          KACC_F_SMALL_NODES ignores it: faster
                                          without the per-lane predicate).
                                          Results are bit-identical.           */
#define KACC_FAST_MAX_PROCS 2048u
#define KACC_FAST_MAX_AGGREGATES 512u
#define KACC_SMALL_MAX_PROCS 512u
#define KACC_SMALL_MAX_AGGREGATES 128u
#define KACC_MEDIUM_MAX_PROCS 1024u
#define KACC_MEDIUM_MAX_AGGREGATES 256u

typedef struct kacc_ctx kacc_ctx;

typedef struct kacc_config {
  uint32_t zones;       /* Z: RAPL zones per node, 1..KACC_MAX_ZONES         */
  uint32_t reserved0;
  uint64_t nodes;       /* node state capacity; node i of a batch is node i  */
  uint64_t proc_slots;  /* workload slot-table capacities                    */
  uint64_t ctr_slots;
  uint64_t vm_slots;
  uint64_t pod_slots;
} kacc_config;

/* One collection interval for the whole fleet.  Layout rules (checked by
 * kacc_validate_host; the kernel additionally clamps every index so a bad
 * batch cannot fault the GPU, it raises KACC_ERANGE instead):
 *
 *  - node n owns process rows [proc_off[n], proc_off[n+1]), containers
 *    [ctr_off[n], ctr_off[n+1]), VMs [vm_off[n], vm_off[n+1]) and pods
 *    [pod_off[n], pod_off[n+1]);
 *  - inside a node the rows are ordered: container processes grouped by
 *    container (in /proc listing order inside each container), then VM
 *    processes grouped by VM, then every other process;
 *  - container c owns rows [begin, ctr_proc_end[c]) where begin is
 *    proc_off[n] for the node's first container, else ctr_proc_end[c-1];
 *  - VM v owns rows [begin, vm_proc_end[v]) where begin is the end of the
 *    node's container rows for its first VM, else vm_proc_end[v-1];
 *  - containers are grouped by pod; pod q owns containers
 *    [begin, pod_ctr_end[q]) with begin = ctr_off[n] for the node's first pod,
 *    else pod_ctr_end[q-1]; containers without a pod follow the pods.
 *
 * In kacc_run_interval every pointer is a DEVICE pointer; in the host batch
 * path (kacc_batch_*) they are pinned host pointers owned by the library.  */
typedef struct kacc_interval {
  uint32_t n_nodes, n_procs, n_ctrs, n_vms, n_pods;
  uint32_t flags;
  /* nodes [n_nodes] */
  const int64_t *node_ts_ns;      /* clock.Now() of this read, monotonic ns (node.go:15) */
  const double *node_usage_ratio; /* resources.Node().CPUUsageRatio as read before
                                     Refresh (node.go:25): the lagged ratio          */
  const uint32_t *node_status;    /* KACC_NODE_* bits, may be NULL                    */
  const double *node_cpu_delta;   /* ProcessTotalCPUTimeDelta override (flags)        */
  const uint32_t *node_order;     /* optional launch order (heaviest first), NULL=id  */
  const uint32_t *node_proc_span; /* optional [2*n_nodes]: {min, max} process slot of
                                     each node's rows (kacc_slot_join's out_span).
                                     When max - min < KACC_FAST_MAX_PROCS the node's
                                     rows are moved in slot order (1 KiB-contiguous
                                     wave accesses however fragmented the slots are);
                                     a row outside its node's span raises ERANGE.   */
  /* zones [n_nodes * Z], node-major */
  const uint64_t *zone_energy;    /* EnergyZone.Energy()   (cpu_power_meter.go:22) */
  const uint64_t *zone_max;       /* EnergyZone.MaxEnergy() (cpu_power_meter.go:26) */
  /* per-node CSR offsets [n_nodes + 1] */
  const uint32_t *proc_off;
  const uint32_t *ctr_off;
  const uint32_t *vm_off;
  const uint32_t *pod_off;
  /* processes [n_procs] */
  const double *proc_cpu_delta;   /* resource.Process.CPUTimeDelta (informer.go:518) */
  const uint32_t *proc_slot;      /* slot word                                        */
  /* containers [n_ctrs] */
  const uint32_t *ctr_proc_end;
  const uint32_t *ctr_slot;
  /* virtual machines [n_vms] */
  const uint32_t *vm_proc_end;
  const uint32_t *vm_slot;
  /* pods [n_pods] */
  const uint32_t *pod_ctr_end;
  const uint32_t *pod_slot;
  /* Optional OUTPUTS (device pointers, NULL = off): this interval's values for
   * the cluster totals, written in batch order by the interval's own kernels
   * (coalesced), so kacc_allreduce_exports reduces them on another stream
   * while the next interval runs (double-buffer them across intervals):
   *   pod_export  [n_pods * 2Z] u64 words: batch pod q's EnergyTotal[Z], then
   *               the bits of its Power[Z] (zeros for a pod whose slot is out
   *               of range);
   *   node_export [n_nodes * 5Z] u64 words: node n's ActiveEnergyTotal[Z],
   *               IdleEnergyTotal[Z], then the bits of Power[Z], ActivePower[Z],
   *               IdlePower[Z] (monitor/types.go:27-40).
   * Every node of the batch is exported, a skipped node (read error) with its
   * unchanged values.  The pinned batch path passes the view's pointers
   * through as device pointers.                                             */
  uint64_t *pod_export;
  uint64_t *node_export;
  /* Optional INPUT (ABI 5, NULL = identity; a device pointer in every path,
   * passed through by kacc_batch_submit like the exports): [n_pods] the
   * pod_export row of batch pod q, each < n_pods and no row given twice (a row
   * given twice is not detected: two pods would write one record).  With the rows of a namespace CSR (pod q of namespace k at its place in
   * ns_pod_off[k] .. ns_pod_off[k+1]) the export is in NAMESPACE order and its
   * partial sums stream contiguous records (kacc_export_sums.ns_ordered)
   * instead of gathering one record per pod (Pod.Namespace,
   * resource/types.go:109).  Exports written through pod_export_pos are in
   * namespace order: only kacc_run_export_sums / kacc_run_interval_sums with
   * kacc_export_sums.ns_ordered = 1 may sum them (kacc_allreduce_exports and
   * the cluster export partials read pod exports in batch order).  A row
   * >= n_pods raises KACC_ERANGE and is not written.                         */
  const uint32_t *pod_export_pos;
} kacc_interval;

/* Device-resident state / result tables.  [n*Z+z] tables are node-major or
 * slot-major with the zone innermost.  After kacc_run_interval they hold the
 * new snapshot: node zones = monitor.NodeUsage (types.go:27-40), workload
 * zones = monitor.Usage (types.go:44-47).
 *
 * KACC_T_PROC_POWER, KACC_T_CTR_POWER and KACC_T_VM_POWER are DERIVED, not
 * stored (ABI 3): a process's (container's, VM's) power is
 * cpuTimeRatio · NodeUsage.ActivePower for a zone that passed the guard
 * (process.go:124, 142; container.go:114, 134; vm.go:84, 103), and 0 otherwise,
 * so the engine keeps per slot the ratio (KACC_T_*_RATIO) and the node
 * (KACC_T_*_NODE) of the slot's last attribution and multiplies on read,
 * bit-identical to a stored value (8Z - 12 bytes less per row and interval).
 * Pod power stays stored (its guard is the node's Power, pod.go:96, and the
 * namespace totals gather it).  kacc_table_download,
 * kacc_unpack, kacc_format_*, and the trackers' frozen copies derive it; it
 * has no device pointer (kacc_table_device_ptr: KACC_EINVAL) and cannot be
 * uploaded.  The derived value is Usage.Power for every slot its node
 * attributed in the node's LAST processed interval (the snapshot's running
 * processes); for a slot that left its node's batch it is defined only until
 * that node's next interval (a terminated process's final power is read by
 * kacc_tracker_add before then).                                             */
typedef enum kacc_table {
  KACC_T_NODE_ENERGY_TOTAL = 0, /* u64 [N*Z] NodeUsage.EnergyTotal          */
  KACC_T_NODE_ACTIVE_ENERGY,    /* u64 [N*Z] NodeUsage.activeEnergy (interval) */
  KACC_T_NODE_ACTIVE_TOTAL,     /* u64 [N*Z] NodeUsage.ActiveEnergyTotal    */
  KACC_T_NODE_IDLE_TOTAL,       /* u64 [N*Z] NodeUsage.IdleEnergyTotal      */
  KACC_T_NODE_POWER,            /* f64 [N*Z] NodeUsage.Power                */
  KACC_T_NODE_ACTIVE_POWER,     /* f64 [N*Z] NodeUsage.ActivePower          */
  KACC_T_NODE_IDLE_POWER,       /* f64 [N*Z] NodeUsage.IdlePower            */
  KACC_T_NODE_TS,               /* i64 [N]   Node.Timestamp (last good read) */
  KACC_T_NODE_HAS_PREV,         /* u32 [N]   1 once a snapshot exists        */
  KACC_T_NODE_USAGE_RATIO,      /* f64 [N]   Node.UsageRatio                 */
  KACC_T_NODE_CPU_DELTA,        /* f64 [N]   ProcessTotalCPUTimeDelta used   */
  KACC_T_NODE_STATUS,           /* u32 [N]   KACC_NODE_OK/FIRST_READ/SKIPPED */
  KACC_T_PROC_ENERGY,           /* u64 [Sp*Z] Process Usage.EnergyTotal      */
  KACC_T_PROC_POWER,            /* f64 [Sp*Z] Process Usage.Power (DERIVED)  */
  KACC_T_CTR_ENERGY,            /* u64 [Sc*Z]                                */
  KACC_T_CTR_POWER,             /* f64 [Sc*Z] (DERIVED)                      */
  KACC_T_CTR_CPU_DELTA,         /* f64 [Sc]  resource.Container.CPUTimeDelta */
  KACC_T_CTR_CPU_TOTAL,         /* f64 [Sc]  resource.Container.CPUTotalTime */
  KACC_T_VM_ENERGY,             /* u64 [Sv*Z]                                */
  KACC_T_VM_POWER,              /* f64 [Sv*Z] (DERIVED)                      */
  KACC_T_VM_CPU_DELTA,          /* f64 [Sv]  resource.VirtualMachine.CPUTimeDelta */
  KACC_T_POD_ENERGY,            /* u64 [Sq*Z] (stored in pod records, below) */
  KACC_T_POD_POWER,             /* f64 [Sq*Z] (stored in pod records, below) */
  KACC_T_POD_CPU_DELTA,         /* f64 [Sq]  resource.Pod.CPUTimeDelta       */
  KACC_T_POD_CPU_TOTAL,         /* f64 [Sq]  resource.Pod.CPUTotalTime       */
  KACC_T_PROC_RATIO,            /* f64 [Sp]  cpuTimeRatio of the slot's last attribution
                                              (process.go:128; Δ / ProcessTotalCPUTimeDelta) */
  KACC_T_PROC_NODE,             /* u32 [Sp]  the node of that attribution     */
  KACC_T_CTR_RATIO,             /* f64 [Sc]  container cpuTimeRatio (container.go:118) */
  KACC_T_CTR_NODE,              /* u32 [Sc]                                   */
  KACC_T_VM_RATIO,              /* f64 [Sv]  VM cpuTimeRatio (vm.go:89)       */
  KACC_T_VM_NODE,               /* u32 [Sv]                                   */
  KACC_T_COUNT
} kacc_table;

/* ---- context ------------------------------------------------------------ */
uint32_t kacc_abi_version(void);
int kacc_create(int device, const kacc_config *cfg, kacc_ctx **out);
void kacc_destroy(kacc_ctx *ctx);
/* Message of the last failed call on ctx, or (ctx NULL) of the last failed
 * call made without a context (kacc_create, kacc_create_multi, ...) on ANY
 * thread of the process: a cgo caller needs no runtime.LockOSThread between
 * the failing call and this one.  The pointer stays valid until the next
 * failing call; kacc_last_error_copy() copies the message into buf (len
 * bytes incl. the NUL, truncated) under the library's lock and returns the
 * full message length — the form to use from cgo.                           */
const char *kacc_last_error(const kacc_ctx *ctx);
size_t kacc_last_error_copy(const kacc_ctx *ctx, char *buf, size_t len);
int kacc_get_config(const kacc_ctx *ctx, kacc_config *out);

/* Zero every state table (fresh PowerMonitor, snapshot == nil). */
int kacc_reset(kacc_ctx *ctx);

/* ---- the hot path ------------------------------------------------------- */
/* Run one interval (device pointers) on `stream` (a hipStream_t; NULL = the
 * context's own stream).  Asynchronous: call kacc_sync() to wait and to
 * collect device-detected range errors.                                      */
int kacc_run_interval(kacc_ctx *ctx, const kacc_interval *dev_batch, void *stream);
/* `count` consecutive intervals (host array of device-pointer descriptors) in
 * order on `stream`: interval k+1 sees the state interval k wrote, exactly as
 * `count` kacc_run_interval calls, but issued back to back from C (fleet
 * replay; BASELINE config 5: 60 batched intervals with counter wraparound).
 * Every descriptor's shape is checked before the first launch.  When every
 * descriptor has KACC_F_FAST_NODES | KACC_F_NODE_SLOT_RANGES (not
 * KACC_F_SMALL_NODES), the same n_nodes and no node_order, the K intervals
 * are one kernel launch (bit-identical to K launches).                      */
int kacc_run_intervals(kacc_ctx *ctx, const kacc_interval *dev_batches, uint32_t count, void *stream);
int kacc_sync(kacc_ctx *ctx, void *stream);
/* Measurement hook (no reference counterpart; bench.py and profiling): the
 * NEXT call on ctx that launches kernels (kacc_run_interval, kacc_run_intervals,
 * or this context's cluster partial sums in kacc_allreduce_namespaces /
 * kacc_allreduce_exports) records `start_event` (a hipEvent_t) when its first
 * kernel starts and `stop_event` when its last kernel ends.  The events ride on
 * the kernels' own dispatch packets (hipExtLaunchKernelGGL): no marker packet
 * is queued between two kernels, so timing every step costs no stream gap.
 * Either event may be NULL; the hook is consumed by that one call.           */
int kacc_time_next_launch(kacc_ctx *ctx, void *start_event, void *stop_event);

/* Host-side layout check of a batch held in host memory (O(N+C+V+Q+P)). */
int kacc_validate_host(const kacc_ctx *ctx, const kacc_interval *host_batch);

/* ---- pinned host batch path (what the cgo shim uses) -------------------- */
typedef struct kacc_batch kacc_batch;
/* Shape of a pinned batch (SURVEY §8(b) kacc_shape): row capacities of each
 * interval and the number of consecutive intervals one submit runs (a replay
 * of `intervals` collection intervals, as kacc_run_intervals; 1 = live).     */
typedef struct kacc_shape {
  uint32_t n_nodes, n_procs, n_ctrs, n_vms, n_pods;
  uint32_t intervals;
} kacc_shape;
/* Allocates pinned host arrays (and their device twins) for shape->intervals
 * intervals of the given capacities.  *views points at the batch's own
 * descriptors, views[0 .. intervals-1]: their arrays are writable pinned host
 * memory (cast away const) that the caller fills.  Per view the caller may
 * set `flags`, lower n_nodes / n_procs / n_ctrs / n_vms / n_pods (never above
 * the shape: only the used prefix of each array is copied) and set the
 * optional node_status / node_cpu_delta / node_order / node_proc_span to
 * NULL; every other pointer is fixed (submit rejects a moved pointer).      */
int kacc_batch_alloc(kacc_ctx *ctx, const kacc_shape *shape, kacc_batch **out, kacc_interval **views);
/* Validate (host, multi-threaded), copy H2D on the context's copy stream and
 * launch the batch's intervals in order on the context stream (asynchronous).
 * With two batches the copies of one overlap the kernels of the other (fill
 * B, submit B, wait A, ...).                                                 */
int kacc_batch_submit(kacc_ctx *ctx, kacc_batch *batch);
/* Wait for this batch's interval; afterwards it may be refilled and
 * resubmitted.  Reports device range errors raised up to this interval.    */
int kacc_batch_wait(kacc_ctx *ctx, kacc_batch *batch);
void kacc_batch_free(kacc_ctx *ctx, kacc_batch *batch);

/* ---- state access -------------------------------------------------------- */
/* Element size in bytes and element count of a table. */
int kacc_table_info(const kacc_ctx *ctx, kacc_table t, uint64_t *elem_bytes, uint64_t *count);
/* Device pointer of a table's first element (for zero-copy readers on the same
 * device).  Slot s's row starts row_stride elements after slot s-1's: Z for a
 * zoned table, 1 for a scalar one, and 2Z for the two pod tables, which are
 * stored as one record per pod slot — its Z energy words, then its Z power
 * words (KACC_T_POD_POWER's pointer is KACC_T_POD_ENERGY's + Z elements) — so
 * that the namespace totals gather ONE 64-B record per pod at Z = 4.
 * kacc_table_download / upload / format take logical [slot*Z + z] ranges.     */
int kacc_table_device_ptr(kacc_ctx *ctx, kacc_table t, void **dev_ptr);
int kacc_table_row_stride(const kacc_ctx *ctx, kacc_table t, uint64_t *stride);
/* Synchronous copies of `count` elements starting at element `first`. */
int kacc_table_download(kacc_ctx *ctx, kacc_table t, uint64_t first, uint64_t count, void *host_dst);
int kacc_table_upload(kacc_ctx *ctx, kacc_table t, uint64_t first, uint64_t count, const void *host_src);
/* Asynchronous device-side read of the same logical range into dev_dst
 * (device, count elements, dense): the scrape of a snapshot without the PCIe
 * hop — a derived table (KACC_T_PROC_POWER, ...) is derived into it
 * (ratio x its node's ActivePower, the guard of process.go:124-142), a pod
 * table is gathered out of its records, any other table is copied.  Ordered
 * on `stream` (NULL: the context's) after the intervals launched before it. */
int kacc_table_read(kacc_ctx *ctx, kacc_table t, uint64_t first, uint64_t count, void *dev_dst, void *stream);

/* ---- cluster namespace totals (north star: only these cross GPUs) -------- */
/* Per-namespace sums over pods of this context: ns k owns pod slots
 * ns_pod_slot[ns_pod_off[k] .. ns_pod_off[k+1]) summed in that order.
 * out_energy: u64 [n_ns*Z] (modular, exact), out_power: f64 [n_ns*Z].
 * All pointers are device pointers; asynchronous on `stream`.  The caller
 * all-reduces the two vectors across GPUs (RCCL sum).                        */
int kacc_namespace_totals(kacc_ctx *ctx, uint32_t n_ns, const uint32_t *ns_pod_off,
                          const uint32_t *ns_pod_slot, uint64_t *out_energy, double *out_power,
                          void *stream);

/* ---- multi-GPU cluster: node shards on several GPUs, totals over RCCL ------
 * SURVEY §8(b)/(e).  Kepler itself has no collectives (each node exports its
 * own metrics; cluster sums are PromQL's `sum by (namespace)`); here a fleet
 * is cut into contiguous node shards (one engine context each, no data-path
 * traffic between them) and only these cross GPUs, over RCCL (xGMI):
 *   - per-namespace totals over pods (Pod.Namespace, resource/types.go:106-110):
 *     u64 energy per zone (modular sum: exact, order independent) and f64
 *     power per zone (sum order fixed per shard; across shards RCCL's order,
 *     <= 1e-12 relative to any other order);
 *   - cluster node totals per zone (monitor/types.go:27-40):
 *     node energy u64 [2*Z] = { Σ ActiveEnergyTotal[z] }, { Σ IdleEnergyTotal[z] }
 *     node power  f64 [3*Z] = { Σ Power[z] }, { Σ ActivePower[z] }, { Σ IdlePower[z] }
 *     over nodes [0, n_nodes) of the last interval run on each shard (a node
 *     that left the batch stops exporting, so PromQL's sum no longer counts
 *     it; a context with no interval run yet contributes zeros);
 *   - the pods themselves (a pod lives on one node: a gather, not a sum).
 * RCCL ranks are GPUs.  A process may hold several shards of one GPU (their
 * partial vectors are added on that GPU in shard order before the collective)
 * and several GPUs (ncclCommInitAll), or one shard per process
 * (ncclCommInitRank: the one-process-per-GPU launch of torchrun / MPI).
 * Per-shard arguments are arrays indexed by local shard; every collective is
 * enqueued on the shard's stream (streams[s], or the context's stream when
 * `streams` or streams[s] is NULL) after the work already queued there.
 * Errors: details via kacc_last_error(first local shard's context).         */
typedef struct kacc_cluster kacc_cluster;
#define KACC_UNIQUE_ID_BYTES 128
/* One process, n shards: shard i = a new context on devices[i] with
 * capacities cfgs[i] (equal zones); shards of one device must be contiguous
 * in `devices`.  ctxs[i] receives shard i's context, owned by the cluster
 * (destroyed by kacc_cluster_destroy, never by kacc_destroy).               */
int kacc_create_multi(const int *devices, int n, const kacc_config *cfgs, kacc_cluster **out,
                      kacc_ctx **ctxs);
/* One process per GPU: rank 0 creates the id and hands it to every rank
 * (any side channel: torch.distributed, MPI, a file); each rank then joins
 * with its own context (not owned by the cluster).                          */
int kacc_cluster_unique_id(uint8_t id[KACC_UNIQUE_ID_BYTES]);
int kacc_cluster_join(kacc_ctx *ctx, const uint8_t id[KACC_UNIQUE_ID_BYTES], int nranks, int rank,
                      kacc_cluster **out);
void kacc_cluster_destroy(kacc_cluster *c);
/* The RCCL the library runs its collectives with.  RCCL is loaded on first
 * use (dlopen, not a link-time dependency): the copy the process already
 * holds under the soname librccl.so.1 (e.g. a framework's), else the first one
 * on the search path (/opt/rocm/lib), or the file named by KACC_RCCL_PATH.  A
 * major version other than the headers' the library was built with (NCCL_MAJOR
 * 2) is refused.  version: ncclGetVersion(); path: the loaded file (len bytes
 * incl. the NUL, truncated).  KACC_EHIP (message via kacc_last_error(NULL))
 * when no usable RCCL is found; the cluster entry points then fail the same. */
int kacc_cluster_rccl(int *version, char *path, size_t len);
/* nranks: GPUs in the cluster; rank: this process's first GPU; n_shards: local shards. */
int kacc_cluster_info(const kacc_cluster *c, int *nranks, int *rank, int *n_shards);
/* Cluster namespace totals (and, when out_node_* are non-NULL, cluster node
 * totals): each shard sums its own pods (kacc_namespace_totals over
 * ns_pod_off[s] / ns_pod_slot[s]: the shard's pod slots grouped by the global
 * namespace index, n_ns the same on every shard), then the sums are
 * all-reduced; every local shard receives the cluster result in its own
 * out_energy[s] / out_power[s] [n_ns*Z] and out_node_energy[s] [2*Z] /
 * out_node_power[s] [3*Z] (device pointers on the shard's GPU).  Async: the
 * partial sums run on streams[s]; the collective runs on comm_streams[s] when
 * given (after the partial sums), so the next interval can be queued on
 * streams[s] at once and overlap it — the outputs are complete when
 * comm_streams[s] (else streams[s]) reaches this point.                    */
int kacc_allreduce_namespaces(kacc_cluster *c, uint32_t n_ns, const uint32_t *const *ns_pod_off,
                              const uint32_t *const *ns_pod_slot, uint64_t *const *out_energy,
                              double *const *out_power, uint64_t *const *out_node_energy,
                              double *const *out_node_power, void *const *streams,
                              void *const *comm_streams);
/* The two halves of kacc_allreduce_namespaces, for a caller that reduces the
 * totals of several intervals with ONE collective (one all-reduce
 * per K intervals; the cluster sum is PromQL's in the reference,
 * internal/resource/types.go:106-110, so no reference call is replaced).
 * kacc_cluster_partials: step 1 only — each shard's partial sums into its own
 * out_* on streams[s] (arguments as kacc_allreduce_namespaces).
 * kacc_allreduce_sums: the rest, in place, over any vectors: energy[s] u64
 * [n_e] and power[s] f64 [n_p] of every local shard are summed over the
 * shards (shard order) and the ranks, and every shard receives the sum.  Lay
 * K intervals' partials out back to back ([K][n_ns*Z + 2Z] u64, [K][n_ns*Z +
 * 3Z] f64) and one call reduces all of them: one compute-to-comm stream
 * handoff (an event packet on streams[s]) and one RCCL group per K
 * intervals instead of per interval.  The collective runs on comm_streams[s]
 * when given.  One rank with one shard: nothing to do.                     */
int kacc_cluster_partials(kacc_cluster *c, uint32_t n_ns, const uint32_t *const *ns_pod_off,
                          const uint32_t *const *ns_pod_slot, uint64_t *const *out_energy,
                          double *const *out_power, uint64_t *const *out_node_energy,
                          double *const *out_node_power, void *const *streams);
int kacc_allreduce_sums(kacc_cluster *c, uint64_t *const *energy, uint64_t n_e, double *const *power,
                        uint64_t n_p, void *const *streams, void *const *comm_streams);
/* The same cluster totals from the interval's exports (kacc_interval.pod_export
 * / node_export) instead of the state tables: nothing runs on streams[s]
 * except an event record — the partial sums run on comm_streams[s] after the
 * work queued on streams[s] so far (the interval that wrote the exports),
 * then the all-reduce, so the next interval on streams[s] overlaps all of it.
 * ns_pod_off[s] / ns_pod_row[s]: namespace k owns the shard's batch pod ROWS
 * ns_pod_row[ns_pod_off[k] .. ns_pod_off[k+1]) (the CSR of
 * kacc_namespace_totals with pod rows for slots: the same sum order, so the
 * results are bit-identical to kacc_allreduce_namespaces); n_pods[s] / n_nodes[s]
 * (HOST): rows of the exports.  The exports must stay untouched until
 * comm_streams[s] has passed this call (kacc_allreduce_exports reads them
 * asynchronously): a caller alternates two export buffers.                  */
int kacc_allreduce_exports(kacc_cluster *c, uint32_t n_ns, const uint32_t *const *ns_pod_off,
                           const uint32_t *const *ns_pod_row, const uint32_t *n_pods,
                           const uint64_t *const *pod_export, const uint32_t *n_nodes,
                           const uint64_t *const *node_export, uint64_t *const *out_energy,
                           double *const *out_power, uint64_t *const *out_node_energy,
                           double *const *out_node_power, void *const *streams, void *const *comm_streams);
/* ---- cluster partial sums of an earlier interval, in the next one's launch --
 * The per-shard partial sums of kacc_cluster_partials (namespace sums and the
 * cluster node totals) computed from an interval's EXPORTS, so that they can run
 * inside the NEXT interval's kernel launch: its sums workgroups are dispatched
 * behind the node workgroups and fill the launch's tail, and a collection step is
 * ONE launch instead of two (each kernel boundary on a stream costs several us:
 * DESIGN §7).  Results are bit-identical to kacc_cluster_partials over the tables
 * that interval left (the same per-lane order; namespace-ordered exports give
 * the same sums as the slot CSR they were ordered by).  No reference call is
 * replaced: the cluster sums are PromQL's in the reference
 * (internal/resource/types.go:106-110).                                     */
typedef struct kacc_export_sums {
  uint32_t n_ns;               /* namespaces (0: no namespace sums)                  */
  uint32_t n_pods;             /* rows of pod_export (the exporting batch's n_pods)  */
  uint32_t n_nodes;            /* rows of node_export (its n_nodes)                  */
  uint32_t ns_ordered;         /* 1: pod_export is in namespace order (written through
                                  kacc_interval.pod_export_pos): namespace k owns rows
                                  [ns_pod_off[k], ns_pod_off[k+1]) and ns_pod_row is
                                  not read; 0: it owns rows ns_pod_row[ns_pod_off[k] ..] */
  const uint32_t *ns_pod_off;  /* [n_ns + 1] (device)                                */
  const uint32_t *ns_pod_row;  /* [ns_pod_off[n_ns]] batch pod rows (device)         */
  const uint64_t *pod_export;  /* [n_pods][2Z] (device)                              */
  const uint64_t *node_export; /* [n_nodes][5Z] (device); NULL: no node totals       */
  uint64_t *out_energy;        /* [n_ns * Z] u64 namespace energy (device)           */
  double *out_power;           /* [n_ns * Z] f64 namespace power                     */
  uint64_t *out_node_energy;   /* [2Z]: Σ ActiveEnergyTotal, Σ IdleEnergyTotal       */
  double *out_node_power;      /* [3Z]: Σ Power, Σ ActivePower, Σ IdlePower          */
} kacc_export_sums;
/* One interval (as kacc_run_interval) plus, in the same launch, the partial sums
 * `prev` of an earlier interval's exports (NULL: none).  The exports `prev` reads
 * must not be the ones dev_batch writes (double-buffer them: KACC_EINVAL on
 * overlap); they were complete when this call's work starts on `stream` (the
 * interval that wrote them was queued there before).  The outputs are complete
 * when this call's work is.  Batches of KACC_F_SMALL_NODES, and node totals over
 * more than 16384 nodes, run the sums as a launch of their own (same results).
 * Past 16384 nodes the node-total columns are split over node blocks whose
 * partials meet in per-CONTEXT arrival counters: the launches of one context
 * that compute node totals (this call, kacc_run_export_sums,
 * kacc_cluster_partials) must be serialized — one stream, or ordered by events.
 * The outputs may not alias any export read or written by the launch
 * (KACC_EINVAL).                                                              */
int kacc_run_interval_sums(kacc_ctx *ctx, const kacc_interval *dev_batch, const kacc_export_sums *prev,
                           void *stream);
/* The same partial sums alone, as one launch on `stream` (the last interval's). */
int kacc_run_export_sums(kacc_ctx *ctx, const kacc_export_sums *sums, void *stream);

/* Cluster pod gather: shard s contributes n_pods[s] (HOST) pods, its slots
 * pod_slot[s] (device), in that order; every local shard receives all pods of
 * the cluster in (rank, shard) order — energy u64 / power f64 [total*Z] into
 * out_energy[s] / out_power[s] (device, capacity out_cap pods).  *total
 * (HOST) = pods in the cluster; first (HOST [n_shards], optional) = the
 * global index of each local shard's first pod.  Blocks on the count
 * exchange; KACC_ERANGE when total > out_cap.                               */
int kacc_gather_pods(kacc_cluster *c, const uint32_t *n_pods, const uint32_t *const *pod_slot,
                     uint64_t out_cap, uint64_t *const *out_energy, double *const *out_power,
                     uint64_t *total, uint64_t *first, void *const *streams);

/* ---- slot join: workload IDs -> slot words on the device ------------------
 * SURVEY §8f row 1, the step before the path.  Replaces, for a whole fleet,
 * the per-row string-keyed lookups of the previous snapshot that decide
 * "new workload or running total" (process.go:132-138 prev.Processes[pid],
 * container.go:126, vm.go:96, pod.go:106) and the informer's terminated sets
 * (informer.go:206-212 processes, :236-246 containers, :260-270 VMs,
 * :311-322 pods) whose prev entries feed the terminated trackers
 * (process.go:87-99, container.go:80-90, vm.go:55-65, pod.go:56-66).
 *
 * One slot map per workload kind.  Node n owns the slot range
 * [slot_off[n], slot_off[n+1]) of that kind's state tables and a private
 * device hash table (load <= 2/3) of its live IDs.  kacc_slot_join() takes
 * the IDs of the node's rows in batch order and, per node:
 *   - a live ID keeps its slot (slot word without KACC_SLOT_NEW);
 *   - an ID that was not live at the node's previous processed interval gets
 *     the lowest slot of its range that was free at the start of this call,
 *     new rows taking slots in row order (KACC_SLOT_NEW set) — deterministic;
 *   - an ID live before but absent now is terminated: (key, slot) goes to the
 *     node's segment of the term_* arrays, in slot order, and its slot is NOT
 *     reused before the next call, so the tracker can still read its final
 *     values (the reference reads them from prev, process.go:90-99);
 *   - a node with KACC_NODE_READ_ERROR is skipped (map unchanged), as the
 *     reference skips Refresh when calculateNodePower fails (monitor.go:399-410).
 * Keys: KACC_KIND_PROC takes uint32_t PIDs (resource.Process.PID, a Linux
 * pid <= pid_max = 2^22; 0xfffffffe/0xffffffff reserved); the other kinds take
 * uint64_t IDs (the packer's 64-bit IDs of the container / VM / pod ID
 * strings; the two top values reserved).  Errors (duplicate ID in a node, a
 * reserved key, more live IDs than the node's range) are raised as
 * KACC_ERANGE at kacc_sync; the affected rows get slot word 0xffffffff (of
 * two rows carrying one ID, which one keeps a slot is unspecified: the whole
 * call is reported as failed).  A PID node with <= 2730 slots given more than
 * 3072 rows fails whole: every row 0xffffffff, its map unchanged.            */
typedef enum kacc_kind {
  KACC_KIND_PROC = 0, /* key: uint32_t PID — process.go:120 StringID        */
  KACC_KIND_CTR = 1,  /* key: uint64_t ID of the container ID string        */
  KACC_KIND_VM = 2,   /* key: uint64_t ID of the VM ID string               */
  KACC_KIND_POD = 3   /* key: uint64_t ID of the pod UID                    */
} kacc_kind;
#define KACC_KEY_EMPTY 0xffffffffffffffffull /* reserved (u32 keys: 0xffffffff) */
#define KACC_KEY_TOMB 0xfffffffffffffffeull  /* reserved (u32 keys: 0xfffffffe) */

typedef struct kacc_slotmap kacc_slotmap;
/* slot_off: HOST [n_nodes + 1], monotonic, slot_off[n_nodes] <= the kind's
 * slot capacity in kacc_config, each range <= 131072 slots.  Starts empty.   */
int kacc_slotmap_create(kacc_ctx *ctx, kacc_kind kind, uint32_t n_nodes, const uint32_t *slot_off,
                        kacc_slotmap **out);
void kacc_slotmap_destroy(kacc_slotmap *m); /* safe before or after kacc_destroy(ctx); other
                                               calls need the context alive */
int kacc_slotmap_reset(kacc_slotmap *m); /* forget every ID (PowerMonitor restart) */
/* Slot numbering policy of later kacc_slot_join calls (default 0: the rules
 * below).  KACC_JOIN_REUSE_TERMINATED: the new rows of a node take, in row
 * order, first the slots of the IDs this same call finds terminated (ascending
 * by slot), then the lowest free slots — so a node whose processes exit and
 * start at the same rate keeps exactly its live rows' slots and, when /proc
 * lists a newcomer where an exited process was, its slot order.  The caller
 * must read the terminated slots' final values (kacc_tracker_add, or its own
 * copy) BEFORE the next interval kernel writes those slots.                  */
#define KACC_JOIN_REUSE_TERMINATED 1u
int kacc_slotmap_set_policy(kacc_slotmap *m, uint32_t policy);
/* Device pointers, asynchronous on `stream` (NULL = the context's stream).
 * n_rows = row_off[n_nodes] (the batch's n_procs / n_ctrs / n_vms / n_pods);
 * row_off [n_nodes+1]: the batch's proc_off / ctr_off / vm_off / pod_off;
 * keys [n_rows] (uint32_t for KACC_KIND_PROC, else uint64_t); node_status
 * [n_nodes] or NULL; out_slot [n_rows] (may be the batch's *_slot array).
 * Terminated IDs, per node: term_count[n] of them, at positions
 * [slot_off[n], slot_off[n] + term_count[n]) of term_key (uint64_t) and
 * term_slot (both sized slot_off[n_nodes]), ascending by slot.  term_count of
 * a skipped node is set to 0.  out_span (optional, [2*n_nodes]): {min, max}
 * slot word & KACC_SLOT_MASK over the node's rows ({1, 0} for a node without
 * rows; untouched for a skipped node) — kacc_interval.node_proc_span.        */
int kacc_slot_join(kacc_slotmap *m, uint32_t n_rows, const uint32_t *row_off, const void *keys,
                   const uint32_t *node_status, uint32_t *out_slot, uint64_t *term_key,
                   uint32_t *term_slot, uint32_t *term_count, uint32_t *out_span, void *stream);

/* ---- CPU-tick input format: CPUTimeDelta on the device (ABI 5) -------------
 * A leaner PCIe format for the host path.  The reference computes every
 * process's CPUTimeDelta on the host (populateProcessFields,
 * internal/resource/informer.go:512-524) from its cumulative CPU ticks
 * (procWrapper.CPUTime, procfs_reader.go:75-82: float64(STime+UTime) / 100):
 *     cpuTotalTime = float64(ticks) / 100;  CPUTimeDelta = cpuTotalTime - p.CPUTotalTime
 * where p.CPUTotalTime is the same expression of the ticks the informer saw at the
 * PID's previous reading (0 for a new process).  A tick map keeps, per process
 * slot, the ticks of its last reading (u64, on the device), so the caller sends
 * only each row's tick INCREMENT — 2 bytes for almost every row instead of the
 * 8-byte float64 Δ — and kacc_ticks_delta writes Go's float64 CPUTimeDelta into
 * the interval batch's proc_cpu_delta, bit-exact (float64(uint64) correctly
 * rounded, one IEEE division by 100, one subtraction).  With the slot words from
 * kacc_slot_join on the device as well, a process row crosses PCIe as its PID
 * (4 B) plus its increment (2 B): 6 bytes instead of 12.
 *
 * Per row r of node n (rows of a KACC_NODE_READ_ERROR node are skipped: the
 * reference skips Refresh for that node, monitor.go:399-410, so neither its
 * informer cache nor the tick map moves):
 *   prev  = proc_slot[r] has KACC_SLOT_NEW ? 0 : map[slot]      (new process)
 *   inc   = dticks[r] != KACC_TICKS_ESCAPED ? dticks[r] : the escape of row r
 *   now   = prev + inc (mod 2^64: a negative increment — a reused PID whose
 *           new process has fewer ticks, informer.go:518 — is an escape)
 *   proc_cpu_delta[r] = float64(now)/100 - float64(prev)/100;  map[slot] = now
 * Escapes: increments outside 0 .. 0xfffe (big first readings of new
 * processes, negative ones), per node n at [esc_off[n], esc_off[n+1]) of
 * esc_row (absolute row numbers inside the node's rows) / esc_ticks (int64).
 * The map starts at 0 (every process's first reading must be a NEW row, as
 * the slot join makes it).  Errors (a slot past the capacity, an escape row
 * outside its node, an escaped row without an escape) raise KACC_ERANGE at
 * kacc_sync; such rows get Δ 0.                                              */
#define KACC_TICKS_ESCAPED 0xffffu
#define KACC_USER_HZ 100u /* procfs_reader.go:73 userHZ */
typedef struct kacc_tickmap kacc_tickmap;
typedef struct kacc_ticks {
  uint32_t n_nodes, n_procs, n_escapes, reserved0;
  const uint32_t *proc_off;   /* [n_nodes + 1] the batch's (device)                  */
  const uint32_t *node_status;/* [n_nodes] or NULL                                   */
  const uint32_t *proc_slot;  /* [n_procs] slot words (kacc_slot_join's out_slot)    */
  const uint16_t *dticks;     /* [n_procs] tick increments, KACC_TICKS_ESCAPED = escape */
  const uint32_t *esc_off;    /* [n_nodes + 1] (may be NULL when n_escapes == 0)     */
  const uint32_t *esc_row;    /* [n_escapes]                                         */
  const int64_t *esc_ticks;   /* [n_escapes]                                         */
  double *proc_cpu_delta;     /* [n_procs] OUT: CPUTimeDelta (the batch's array)     */
} kacc_ticks;
/* A tick map over the context's process slots (all zero). */
int kacc_tickmap_create(kacc_ctx *ctx, kacc_tickmap **out);
void kacc_tickmap_destroy(kacc_tickmap *m);
int kacc_tickmap_reset(kacc_tickmap *m);
/* Device pointers, asynchronous on `stream` (NULL = the context's stream). */
int kacc_ticks_delta(kacc_tickmap *m, const kacc_ticks *t, void *stream);
/* Synchronous copy of count ticks from slot `first` (tests, checkpoints). */
int kacc_tickmap_download(kacc_tickmap *m, uint64_t first, uint64_t count, uint64_t *host_dst);

/* ---- host packer: informer records -> interval CSR -----
 * The step before the path: what resource.Informer.Refresh
 * (internal/resource/informer.go:167-326) leaves per node — the running
 * processes in /proc listing order with PID, CPUTimeDelta, Type and their
 * container / VM / pod — packed into kacc_interval's layout, on host threads:
 * container processes grouped by container (containers grouped by pod, pods
 * in order of their containers' first appearance, ContainersNoPod last; a
 * container's rows in listing order: its CPU-time sum order, :229-233), then
 * VM processes grouped by VM (listing order: the last row is the writer,
 * :445), then the others.  Container / VM / pod IDs are the caller's 64-bit
 * keys of the ID strings (KACC_KEY_EMPTY / KACC_KEY_TOMB reserved).  The
 * packer emits the keys kacc_slot_join takes (PIDs per row, IDs per
 * aggregate) and row_record (the input record of every row) for kacc_unpack.
 * Outputs may point into a pinned batch view (kacc_batch_alloc).             */
#define KACC_PROC_REGULAR 0u   /* resource.RegularProcess   */
#define KACC_PROC_CONTAINER 1u /* resource.ContainerProcess */
#define KACC_PROC_VM 2u        /* resource.VMProcess        */
typedef struct kacc_records {
  uint32_t n_nodes;
  uint32_t reserved0;
  const uint32_t *rec_off;   /* [n_nodes + 1] node n's records [rec_off[n], rec_off[n+1])   */
  const uint32_t *pid;       /* [R] Process.PID                                              */
  const double *cpu_delta;   /* [R] Process.CPUTimeDelta (informer.go:518)                   */
  const uint8_t *type;       /* [R] KACC_PROC_*  (Process.Type)                              */
  const uint64_t *ctr_key;   /* [R] key of Process.Container.ID (type CONTAINER)             */
  const uint64_t *vm_key;    /* [R] key of Process.VirtualMachine.ID (type VM)               */
  const uint64_t *pod_key;   /* [R] key of the container's Pod.ID per LookupByContainerID
                                    (pod.go:209-239), KACC_KEY_EMPTY = not found (the container
                                    goes to ContainersNoPod), KACC_KEY_TOMB rejected; or NULL */
  const uint32_t *pod_ns;    /* [R] the pod's namespace index (namespace totals); or NULL    */
} kacc_records;
typedef struct kacc_packed {
  /* in: array capacities; out: the counts (also on KACC_ERANGE: the sizes needed) */
  uint32_t n_procs, n_ctrs, n_vms, n_pods;
  uint32_t *proc_off, *ctr_off, *vm_off, *pod_off; /* [n_nodes + 1]                    */
  double *proc_cpu_delta;                          /* [P] rows                          */
  uint32_t *proc_key;                              /* [P] PID of each row               */
  uint32_t *row_record;                            /* [P] input record of each row, or NULL */
  uint32_t *ctr_proc_end;                          /* [C]                               */
  uint64_t *ctr_key;                               /* [C]                               */
  uint32_t *vm_proc_end;                           /* [V]                               */
  uint64_t *vm_key;                                /* [V]                               */
  uint32_t *pod_ctr_end;                           /* [Q]                               */
  uint64_t *pod_key;                               /* [Q]                               */
  uint32_t *pod_ns;                                /* [Q]                               */
} kacc_packed;
/* HOST arrays; `threads` host threads (0 = 1).  KACC_ERANGE when a capacity
 * is short (out->n_* then hold the sizes needed; nothing was written).     */
int kacc_pack(const kacc_records *in, kacc_packed *out, uint32_t threads);
/* The unpack (device, async on `stream`): for i < n, the kind's state-table
 * row of slot word slot_words[i] (energy u64 / power f64, Z each) goes to
 * out row dest[i] (dest = the packer's row_record: results in input-record
 * order) or row i (dest NULL: in batch order, the order of the packer's
 * keys) — what the cgo shim turns into Snapshot entries (types.go:75-193). */
int kacc_unpack(kacc_ctx *ctx, kacc_kind kind, uint32_t n, const uint32_t *slot_words, const uint32_t *dest,
                uint64_t *out_energy, double *out_power, void *stream);

/* ---- terminated-workload trackers ---------------------
 * TerminatedResourceTracker (internal/monitor/terminated_resource_tracker.go)
 * for one workload kind, on the device — ONE TRACKER PER NODE, as every
 * node's PowerMonitor owns its own (monitor.go:123-144): per node, the top
 * max_size terminated workloads of that node by their final energy in the
 * target zone (the meter's primary zone): max_size 0 disables (:82), an ID
 * already tracked is ignored (:90), energy below min_energy is dropped
 * (:102), below capacity an item is pushed (:116), at capacity it must beat
 * the node's minimum (:124); Clear() after an export (process.go:80-84), for
 * every node or for the nodes of a mask (each node exports on its own).
 *
 * kacc_tracker_add() takes one interval's terminated workloads — the per-node
 * segments of kacc_slot_join — and reads their final values from the kind's
 * state tables (the slots are not reused before the next join).  A node's
 * batch is added as Go's loop over procs.Terminated (process.go:89-99) would
 * add it in the map order "descending target-zone energy, then slot"; Go's
 * map order is unspecified, and for any batch whose energies differ at the
 * retention boundary the retained set is the same for every order.  Ties at
 * the boundary keep items already tracked first (Go's heap requires a strictly
 * higher energy to evict), then the batch order.  Tracked items are frozen
 * copies (energy and power per zone), as Add(prev.Clone()) keeps.  Nodes are
 * those of the context (kacc_config.nodes): the device holds, PER NODE,
 * max_size items (capacity for an unlimited tracker), i.e.
 * kacc_config.nodes x items x (8 + 16Z) bytes — 10k nodes x 500 x Z=4 is
 * 360 MB; KACC_ENOMEM, with that figure in the message, when it does not fit. */
typedef struct kacc_tracker kacc_tracker;
#define KACC_TRACKER_MAX_BOUNDED 8192u /* largest max_size > 0 supported */
/* max_size: > 0 top-N per node (<= KACC_TRACKER_MAX_BOUNDED), 0 disabled,
 * < 0 unlimited (at most `capacity` items PER NODE, more raise ERANGE).
 * zone: target zone index in the kind's [slot*Z + z] tables.  min_energy:
 * minEnergyThreshold in µJ.                                                 */
int kacc_tracker_create(kacc_ctx *ctx, kacc_kind kind, int64_t max_size, uint32_t capacity,
                        uint32_t zone, uint64_t min_energy, kacc_tracker **out);
void kacc_tracker_destroy(kacc_tracker *t); /* safe before or after kacc_destroy(ctx) */
/* node_mask: DEVICE [nodes], nonzero = clear that node's tracker; NULL = all. */
int kacc_tracker_clear(kacc_tracker *t, const uint32_t *node_mask, void *stream);
/* m: the slot map whose kacc_slot_join produced term_key / term_slot /
 * term_count (device pointers); asynchronous on `stream`.
 * ORDERING: call it after that join and BEFORE the next kacc_run_interval (or
 * kacc_run_intervals / kacc_batch_submit) of the same context, on the same
 * stream or with an event the interval's stream waits for.  The frozen power
 * of a terminated process / container / VM is derived (its stored ratio x its
 * node's ActivePower, see kacc_table), and the next interval rewrites the
 * node's ActivePower (and, under KACC_JOIN_REUSE_TERMINATED, the slots): a
 * tracker that runs beside or after that interval freezes a wrong power.
 * This is Go's own order: calculateProcessPower adds procs.Terminated
 * (process.go:87-99) before it attributes the interval (:118-148).           */
int kacc_tracker_add(kacc_tracker *t, const kacc_slotmap *m, const uint64_t *term_key,
                     const uint32_t *term_slot, const uint32_t *term_count, void *stream);
/* Items(): synchronous.  *count = tracked items of all nodes; when the arrays
 * are non-NULL (HOST, sized >= *count; energy/power [*count * Z]) they receive
 * key, node and the frozen per-zone energy (µJ) and power (µW): node by node
 * in node order, each node's items highest energy first.                    */
int kacc_tracker_items(kacc_tracker *t, uint32_t *count, uint64_t *key, uint32_t *node,
                       uint64_t *energy, double *power);

/* ---- multi-socket aggregated zones ---------------------
 * device.AggregatedZone (internal/device/energy_zone.go:47-148) for every
 * (node, zone) of the fleet, each made of `sockets` sub-zones (package-0,
 * package-1, ... of a multi-socket node).  sub_max: HOST [n_nodes*Z*sockets]
 * MaxEnergy() of each sub-zone, summed (saturating) at creation as
 * NewAggregatedZone caches it (:55-67).                                      */
typedef struct kacc_zone_agg kacc_zone_agg;
int kacc_zone_agg_create(kacc_ctx *ctx, uint32_t n_nodes, uint32_t sockets, const uint64_t *sub_max,
                         kacc_zone_agg **out);
void kacc_zone_agg_destroy(kacc_zone_agg *z); /* safe before or after kacc_destroy(ctx) */
/* One Energy() per aggregated zone (device pointers, async on `stream`):
 * readings [n_nodes*Z*sockets] sub-zone counters, [node][zone][socket];
 * sub_status (optional, same shape) nonzero = that sub-zone's read failed:
 * the zone's Energy() returns the error there (:104-108), the node's interval
 * fails.  node_status [n_nodes]: the KACC_NODE_READ_ERROR bit of every node is
 * written — set when one of its zones failed, cleared otherwise (other bits
 * are kept), so the same array can be passed every interval.  Outputs
 * out_energy / out_max [n_nodes*Z] = the batch's zone_energy / zone_max.      */
int kacc_zone_agg_read(kacc_zone_agg *z, const uint64_t *readings, const uint32_t *sub_status,
                       uint64_t *out_energy, uint64_t *out_max, uint32_t *node_status, void *stream);

/* ---- exposition values ---------------------------------
 * The numbers of the Prometheus exposition (power_collector.go:306-436):
 * every element of an energy table as Energy.Joules() (device/energy.go:30-32)
 * or of a power table as Power.Watts() (:57-59), written as the text format
 * writes floats (expfmt writeFloat, prometheus/common v0.62.0: 1/0/-1/NaN/
 * +Inf/-Inf spelled out, else Go strconv.AppendFloat(f, 'g', -1, 64)).
 * out: device [count * KACC_FMT_WIDTH] bytes, element i's text left-aligned in
 * its field (zero-padded); len: device [count] text lengths.  Labels are the
 * Go side's strings; it joins them with these fields into sample lines.
 * KACC_T_NODE_USAGE_RATIO is written as the float64 it is
 * (kepler_node_cpu_usage_ratio, power_collector.go:250-255).                 */
#define KACC_FMT_WIDTH 24
int kacc_format_values(kacc_ctx *ctx, kacc_table t, uint64_t first, uint64_t count, char *out,
                       uint8_t *len, void *stream);

/* ---- exposition lines (the text around the values) -----
 * The sample lines of one workload metric family, as Kepler's collector
 * (power_collector.go:306-436: MustNewConstMetric, whose label pairs
 * client_golang sorts by name) is written by expfmt's text format:
 *     NAME{LABELS,zone="ZONE"} VALUE\n
 * "zone" sorts after every other label name of Kepler's process / container /
 * VM / pod metrics (power_collector.go:128-139, and the node_name const label
 * of :63-95), so LABELS is the row's other label pairs incl. node_name,
 * name-sorted and escaped by the caller (`comm="bash",...`); VALUE is written
 * as kacc_format_values writes it.  Lines are row-major: for i in [0, count)
 * row first + (row_order ? row_order[i] : i), for j in [0, n_zones) the table
 * zone zone_order ? zone_order[j] : j named zone_names[j].
 *   name, zone_names, zone_order: HOST; labels, label_off [count + 1] (u64
 *   offsets into labels, indexed by i's row - first), row_order [count]: DEVICE
 *   line_off: DEVICE [count * n_zones + 1] byte offset of every line (+ total)
 *   out: DEVICE buffer of out_cap bytes, or NULL to size only
 *   *total: HOST, bytes of the whole text.
 * t is a workload energy / power table (rows = slots) or one of the node x
 * zone energy / power tables (rows = nodes; the node families carry a
 * per-zone `path` label that sorts before zone, so a caller writes them one
 * zone per call, power_collector.go:257-298).
 * Synchronous (the total is read back).  KACC_ERANGE when out_cap < *total.   */
int kacc_format_lines(kacc_ctx *ctx, kacc_table t, uint64_t first, uint64_t count, const char *name,
                      const char *const *zone_names, const uint32_t *zone_order, uint32_t n_zones,
                      const char *labels, const uint64_t *label_off, const uint32_t *row_order,
                      uint64_t *line_off, char *out, uint64_t out_cap, uint64_t *total, void *stream);

/* Algorithmic HBM bytes of K consecutive intervals of these sizes: K times
 * kacc_interval_bytes, or (carried != 0: kacc_run_intervals' one-launch path,
 * which reads the engine state a node / row / aggregate needs once and carries
 * it on chip while the slots stay put) that minus K-1 state reads.          */
uint64_t kacc_intervals_bytes(uint32_t zones, uint64_t n_nodes, uint64_t n_procs, uint64_t n_ctrs,
                              uint64_t n_vms, uint64_t n_pods, uint32_t intervals, int carried, uint32_t flags);
/* Algorithmic HBM bytes one kacc_run_interval moves for a batch of these
 * sizes and flags (the roofline numerator): with
 * KACC_F_STABLE_SLOT_NODES a process row does not write its node (4 B; the
 * few NEW rows of an interval that do are not counted).                      */
uint64_t kacc_interval_bytes(uint32_t zones, uint64_t n_nodes, uint64_t n_procs, uint64_t n_ctrs,
                             uint64_t n_vms, uint64_t n_pods, uint32_t flags);

#ifdef __cplusplus
}
#endif
#endif /* KEPLER_ACCEL_H */
