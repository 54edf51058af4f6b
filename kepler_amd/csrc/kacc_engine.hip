// MI355X (gfx950) power-attribution engine: kernels + C ABI (kepler_accel.h).
//
// One kacc_run_interval() = one collection interval of Kepler's
// PowerMonitor.calculatePower (internal/monitor/monitor.go:399-431) for every
// node of a fleet, as ONE kernel launch: one workgroup per node snapshot
// (node snapshots are independent, node.go / process.go only read the node's
// own zones and totals).  Inside a workgroup:
//
//   A  node zones       node.go:10-84 / node.go:101-131 (threads z < Z)
//   B  node CPU total   informer.go:328-345, canonical 256-lane tree order
//   C  container / VM   informer.go:223-249 + 469-489, 251-273 + 433-449
//                        (segmented sums, one lane per segment, listing order)
//   D  pods             informer.go:275-326 + 491-510 (one lane per pod)
//   E  attribution      process.go:118-148, container.go:106-140,
//                        vm.go:78-109, pod.go:87-118 (coalesced row pass)
//
// Everything is HBM-bandwidth bound (≈0.1 flop/B); no MFMA.  Workload
// energy/power live in device-resident slot tables that are updated in place,
// so the per-row traffic is Δcpu 8 B + slot 4 B + prev total 8Z B in and
// total 8Z B + power 8Z B out.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <type_traits>
#include <cstdarg>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/kepler_accel.h"
#include "kacc_debug.h"
#include "kacc_derive.hpp"
#include "kacc_device.hpp"
#include "kacc_internal.hpp"

namespace kacc {

constexpr int kTree = 256;                   // lanes of the canonical node-total tree
constexpr int kRowsLds = 2048;               // Δcpu rows staged in LDS per node (16 KiB)
constexpr int kBlock = 256;                  // namespace kernel workgroup
template <int Z>
constexpr bool kTransposed = (Z % 2 == 0) && Z >= 4;  // 32-B+ rows: transpose 64-row groups
// KACC_NS_LANES / KACC_NS_UNROLL: namespace-sum geometry (the lane count fixes
// the f64 summation order, mirrored by oracle/kor_namespace_totals)
#ifndef KACC_NS_LANES
#define KACC_NS_LANES 16
#endif
#ifndef KACC_NS_UNROLL
#define KACC_NS_UNROLL 2  // 2: 17.9 us at config 3, 4: 19.4, 8: 18.8 (profiles/r03/sq ns_*)
#endif
constexpr int kNsLanes = KACC_NS_LANES;      // lanes per namespace (namespace_kernel)
constexpr int kNsUnroll = KACC_NS_UNROLL;    // pods in flight per namespace lane

// Debug variants (kacc_debug_run_variant, timing ablations only; results of a
// variant != 0 are NOT the reference semantics).
constexpr int kVarSkipAggregates = 1;  // skip containers / VMs / pods
constexpr int kVarSkipProcs = 2;       // skip the process attribution pass
constexpr int kVarUnstaged = 4;        // never stage Δ in LDS
constexpr int kVarTemporalStores = 8;  // plain (temporal) stores for the row outputs
constexpr int kVarNoTranspose = 32;    // per-row scatter only (no 64-row group transpose)
constexpr int kVarLateAgg = 128;       // flips kLateAgg below (timing ablation)
constexpr int kVarNoSweep = 2048;      // never sweep the node's slot span (row order only)
constexpr int kVarNtAgg = 4096;        // non-temporal stores for the aggregate rows too (round 2)
constexpr int kVarNtScatter = 8192;    // non-temporal per-row scattered process stores (round 2)
constexpr int kVarTemporalLoads = 16384;  // plain loads of the streamed inputs and prev totals
// per-workgroup real-time stamps into DevState::stamps (diagnostic; results are
// the reference's): [blk][8] = start, rows staged (first barrier), attribution
// start, end (after a final barrier), XCC_ID, HW_ID, node, 0 — in s_memrealtime
// ticks (100 MHz, one clock for the whole device)
constexpr int kVarStamps = 131072;
// KACC_LATE_AGG: interval_kernel loads the aggregates' previous totals and stores
// their rows AFTER the process pass (1, round 3) or before it (0, rounds 1-2).
// Early aggregate rows sit dirty in L2 through the whole process stream and
// leave it as ~80 MB of extra write traffic per config-3 launch (WRITE_SIZE
// 1.083 GB early vs 1.002 GB late = the algorithmic writes; profiles/r03/pmcvar2);
// same-box bench A/B 363 -> 347 us (profiles/r03/late)
#ifndef KACC_LATE_AGG
#define KACC_LATE_AGG 1  // 347 vs 363 us at config 3, same box (profiles/r03/late)
#endif
// small_kernel (one wavefront per node): the same late aggregate stores, and it
// ignores KACC_F_STABLE_SLOT_NODES — the per-lane node-store predicate cost it
// more than the 4 B (config-1 fleet, same box: 312.6 / 289.2 us with the flag
// honoured and early aggregates, 289.2 / 265.7 us like this; profiles/r03/small2)
#ifndef KACC_SMALL_LATE_AGG
#define KACC_SMALL_LATE_AGG 1
#endif
#ifndef KACC_SMALL_STABLE
#define KACC_SMALL_STABLE 0
#endif
template <int V>
constexpr bool kLateAgg = (KACC_LATE_AGG != 0) != ((V & kVarLateAgg) != 0);
constexpr int kVarBigNoTotal = 256;    // big nodes: no node CPU-total pass
constexpr int kVarBigNoScan = 512;     // big nodes: no segment-owner scan
constexpr int kVarBigNoAtomic = 1024;  // big nodes: no item-list atomic (chunk kernel idles)

// interval_kernel stores the aggregate rows (containers / VMs / pods: 32 B
// energy + 32 B power per row, at slots scattered over the tables) through L2,
// unlike the process row streams: a non-temporal 32 B store goes to HBM as a
// partial line, while L2 merges the rows of one line written by different
// nodes' blocks.  Measured 2-9 % of interval_kernel<4,0> at config 3 in three
// in-process A/Bs (profiles/r02/aggab); the hint on the process rows stays
// (5 %, profiles/r01/ablations).  The carry kernel (1.4 %, config 2 x 60) and
// small_kernel (1.1 %, config 1, three process pairs, profiles/r02/aggrest) do
// the same; chunk_kernel / pod_kernel keep non-temporal aggregate stores (1.5 %
// slower plain at config 5, where a big node's aggregates are long runs).
// KACC_NT_AGG=1 builds the earlier behaviour for A/B.
#ifndef KACC_NT_AGG
#define KACC_NT_AGG 0
#endif
constexpr bool kNtAggStores = KACC_NT_AGG != 0;
// Process rows that take the per-row fallback (a node's slots neither sweepable
// nor in contiguous 64-slot groups: fragmented ranges, the held join policy)
// are stored through L2 too: one 32 B row per lane at scattered slots is the
// aggregate case again, and non-temporal partial lines made that fallback 3.2x
// slower at config 3 with 10 % slot fragmentation (profiles/r02/fragst).
// KACC_NT_SCATTER=1 builds the earlier behaviour.
#ifndef KACC_NT_SCATTER
#define KACC_NT_SCATTER 0
#endif
constexpr bool kNtScatterStores = KACC_NT_SCATTER != 0;
constexpr uint32_t kPodGrid = 256;     // deferred-pod kernel workgroups (kBlock threads)
constexpr int kTotLoads = 16;          // Δ loads in flight per lane (big-node CPU total)
// KACC_CHUNK_THREADS: chunk kernel workgroup (4 rows per lane: 512 -> 2048-row
// chunks); KACC_CHUNK_WAVES: waves per SIMD it is compiled for at Z <= 4
// (512 threads: 4 = two workgroups per CU, 119 VGPRs; 6 = three, 80 VGPRs with
// spills; 256 threads: a workgroup is one wave per SIMD)
#ifndef KACC_CHUNK_THREADS
#define KACC_CHUNK_THREADS 512
#endif
#ifndef KACC_CHUNK_WAVES
#define KACC_CHUNK_WAVES 4
#endif
constexpr int kChunkThreads = KACC_CHUNK_THREADS;
constexpr int kChunkRpt = 4;
constexpr int kChunkRows = kChunkRpt * kChunkThreads;  // big-node rows per chunk item
static_assert(kChunkRows <= kRowsLds, "a chunk's rows are staged like a fast node's");
// persistent chunk-kernel workgroups: all resident (256 CUs)
constexpr uint32_t kChunkGrid = 256u * 4u * KACC_CHUNK_WAVES / (kChunkThreads / 64);

template <int V>
constexpr int kTpb = 512;  // threads per workgroup (fast path)
template <int V>
constexpr int kRpt = kRowsLds / kTpb<V>;            // fast-path rows per lane

// device error bits (KACC_ERANGE)
constexpr uint32_t kErrNode = 1u << 0;
constexpr uint32_t kErrOffsets = 1u << 1;
constexpr uint32_t kErrSlot = 1u << 2;
constexpr uint32_t kErrNs = 1u << 3;
constexpr uint32_t kErrCapacity = 1u << 4;
constexpr uint32_t kErrBigNode = 1u << 5;  // oversized node under KACC_F_FAST_NODES
static_assert(kRowsLds == KACC_FAST_MAX_PROCS && kTpb<0> == KACC_FAST_MAX_AGGREGATES,
              "KACC_FAST_* must match the fast path's capacity");

// One big-node chunk (see big_node_prepare).  ctr_begin / vm_begin / pod_begin:
// the first container / VM / pod the chunk owns; it owns them up to the next
// chunk's begin (or the node's end for the last chunk).
struct ChunkItem {
  uint32_t node, chunk, nchunks, ctr_begin, vm_begin, pod_begin, pad[2];
};

// Cluster node totals (kacc_allreduce_namespaces, kacc_cluster_partials): one
// block per output value — block c sums column c (node table c / Z of the five,
// zone c % Z) over every node: lane l < kBlock adds nodes l, l + kBlock, ... in
// order (kColLoads loads in flight), then the wave tree and the four waves in
// order — and writes it.  No cross-block combine up to kColSplitFrom nodes
// (config 3: 40 loads per lane, hidden under the namespace blocks of the same
// launch; the 1/8 shard: 5 per lane, one round trip).
// Past kColSplitFrom nodes (config 1: 40k) ONE column is more than one CU
// streams in time (a CU takes in ~11 B per clock: 40k x 16 B of strided column
// ~ 24 us), so each column is split over ceil(N / kColSplitNodes) blocks: block
// (c, k) sums nodes [k R, (k+1) R) in the per-lane order above, publishes its
// partial (an agent-scope store, then an acq_rel agent-scope add to the column's
// arrival count), and the block that arrives last adds the partials in k order
// and re-arms the count for the next launch.  The per-column order is fixed by N
// alone, so every launch (and the fused path, which never splits) gives the same
// bits for the same inputs.  Round 4's wide instance (32 loads in flight per lane,
// 166 VGPRs: 27.8 us at 40k nodes) is gone.
constexpr int kColLoads = 8;
#ifndef KACC_COL_SPLIT_FROM
#define KACC_COL_SPLIT_FROM 16384  // from 4096 with 2048-node blocks: config 3 16.6 -> 19.2 us,
#endif                             // config 1 23.1 -> 28.5 us (profiles/r05/r05l)
#ifndef KACC_COL_SPLIT_NODES
#define KACC_COL_SPLIT_NODES 4096
#endif
constexpr uint64_t kColSplitFrom = KACC_COL_SPLIT_FROM, kColSplitNodes = KACC_COL_SPLIT_NODES;
struct NodeTotalsArgs {
  uint64_t n_nodes;
  const uint64_t *active_total, *idle_total;
  const double *power, *active_power, *idle_power;
  const uint64_t *node_export;  // else the five tables: an interval's node export [n_nodes][5Z]
  uint64_t *out_e;              // [2Z]: Σ ActiveEnergyTotal, Σ IdleEnergyTotal (u64, modular)
  double *out_p;                // [3Z]: Σ Power, Σ ActivePower, Σ IdlePower (f64)
  uint32_t split;               // blocks per column (1: no combine)
  uint64_t *part;               // [5Z][split] the column blocks' partials (split > 1)
  uint32_t *arrived;            // [5Z] arrival counts, 0 between launches
};

struct DevState {
  uint64_t *node_energy_total, *node_active_energy, *node_active_total, *node_idle_total;
  double *node_power, *node_active_power, *node_idle_power;
  int64_t *node_ts;
  uint32_t *node_has_prev;
  double *node_usage_ratio, *node_cpu_delta;
  uint32_t *node_status;
  uint64_t *proc_energy;
  double *proc_ratio;   // [Sp] cpuTimeRatio of the slot's last attribution (power is derived)
  uint32_t *proc_node;  // [Sp] the node that attribution belonged to
  uint64_t *ctr_energy;
  double *ctr_ratio, *ctr_cpu_delta, *ctr_cpu_total;  // container / VM power is derived (as processes')
  uint32_t *ctr_node;
  uint64_t *vm_energy;
  double *vm_ratio, *vm_cpu_delta;
  uint32_t *vm_node;
  uint64_t *pod_energy;
  double *pod_power, *pod_cpu_delta, *pod_cpu_total;
  uint64_t proc_slots, ctr_slots, vm_slots, pod_slots;
  uint32_t *err;
  uint2 *defer;        // [defer_cap] (node, pod) pods left to pod_kernel
  uint32_t *defer_ctr;  // [0] length; re-armed by interval_kernel
  uint32_t defer_cap;
  ChunkItem *items;    // [item_cap] big-node chunks this launch
  uint32_t *item_ctr;  // [0] length, [1] dequeue head; cleared by pod_kernel
  uint32_t item_cap;
  // kacc_run_intervals over intervals of ONE layout (the same offset arrays):
  // the chunk items are generated once (items_kernel) and reused, so the node
  // phase skips them; pod_kernel keeps the list for the next interval
  uint32_t items_given, keep_items;
  uint64_t *stamps;  // kVarStamps only
};

struct NodeShared {
  uint64_t active_energy[KACC_MAX_ZONES];
  double power[KACC_MAX_ZONES];
  double active_power[KACC_MAX_ZONES];
  double node_delta;
  uint32_t first;
};

__device__ __forceinline__ void raise_err(uint32_t *err, uint32_t bit) { atomicOr(err, bit); }

// Block-uniform values live in SGPRs (saves VGPRs for rows in flight).
__device__ __forceinline__ uint64_t uniform_u64(uint64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(x));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(x >> 32));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}
__device__ __forceinline__ double uniform_f64(double x) {
  return __longlong_as_double(static_cast<long long>(uniform_u64(static_cast<uint64_t>(__double_as_longlong(x)))));
}
__device__ __forceinline__ uint32_t uniform_u32(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// Experiments (timing A/B only; results are identical): KACC_WT_PROC writes the
// non-temporal row stores through the L2 (sc0 sc1 nt: no dirty line is left for
// the end-of-kernel write-back), KACC_WT_AGG the aggregate rows likewise.
// Experiment: extra dynamic LDS per interval_kernel workgroup (fewer resident
// workgroups per CU, each with a larger share of the bandwidth: shorter lifetimes)
#ifndef KACC_FAST_EXTRA_LDS
#define KACC_FAST_EXTRA_LDS 0
#endif
#ifndef KACC_WT_PROC
#define KACC_WT_PROC 0
#endif
#ifndef KACC_WT_AGG
#define KACC_WT_AGG 0
#endif
template <typename T>
__device__ __forceinline__ void wt_store(T v, T *p) {
  if constexpr (sizeof(T) == 16)
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
  else if constexpr (sizeof(T) == 8)
    asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
  else
    asm volatile("global_store_dword %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
}
template <typename T>
__device__ __forceinline__ void nt_store(T v, T *p) {
  if constexpr (KACC_WT_PROC != 0)
    wt_store(v, p);
  else
    __builtin_nontemporal_store(v, p);
}

template <int Z>
__device__ __forceinline__ void load_row(const uint64_t *__restrict__ base, uint64_t s,
                                         uint64_t (&out)[Z]) {
  if constexpr (Z % 2 == 0) {
    using u64x2 = __attribute__((ext_vector_type(2))) unsigned long long;
    const u64x2 *p = reinterpret_cast<const u64x2 *>(base + s * Z);
#pragma unroll
    for (int k = 0; k < Z / 2; ++k) {
      const u64x2 x = p[k];
      out[2 * k] = x.x;
      out[2 * k + 1] = x.y;
    }
  } else {
#pragma unroll
    for (int z = 0; z < Z; ++z) out[z] = base[s * Z + z];
  }
}

template <int Z>
__device__ __forceinline__ void load_row_f64(const double *__restrict__ base, uint64_t s,
                                             double (&out)[Z]) {
  if constexpr (Z % 2 == 0) {
    using f64x2 = __attribute__((ext_vector_type(2))) double;
    const f64x2 *p = reinterpret_cast<const f64x2 *>(base + s * Z);
#pragma unroll
    for (int k = 0; k < Z / 2; ++k) {
      const f64x2 x = p[k];
      out[2 * k] = x.x;
      out[2 * k + 1] = x.y;
    }
  } else {
#pragma unroll
    for (int z = 0; z < Z; ++z) out[z] = base[s * Z + z];
  }
}

template <int Z, bool NT, typename T>
__device__ __forceinline__ void store_row(T *__restrict__ base, uint64_t s, const T (&in)[Z]) {
  if constexpr (Z % 2 == 0) {
    using v2 = __attribute__((ext_vector_type(2))) T;
    v2 *p = reinterpret_cast<v2 *>(base + s * Z);
#pragma unroll
    for (int k = 0; k < Z / 2; ++k) {
      v2 x;
      x.x = in[2 * k];
      x.y = in[2 * k + 1];
      if constexpr (NT)
        nt_store(x, p + k);
      else
        p[k] = x;
    }
  } else {
#pragma unroll
    for (int z = 0; z < Z; ++z) {
      if constexpr (NT)
        nt_store(in[z], base + s * Z + z);
      else
        base[s * Z + z] = in[z];
    }
  }
}

// Pod rows are stored as one record per slot: the Z energy words then the Z
// power words (KACC_T_POD_POWER's base is KACC_T_POD_ENERGY's + Z words), so a
// pod's row is ONE 64-B gather at Z = 4 for the namespace totals (two 32-B rows
// of two tables before: cluster partials 31.5 -> 22.0 us at config 3,
// profiles/r03/abns).  load_row / store_row address base + s*Z, so a pod slot s
// is passed as row 2s.
constexpr uint64_t kPodRowScale = 2;
__device__ __forceinline__ uint64_t pod_row(uint64_t s) { return s * kPodRowScale; }
// the row index of aggregate slot s in its role's tables (1 container, 2 VM, 3 pod)
__device__ __forceinline__ uint64_t agg_row(uint32_t role, uint64_t s) { return role == 3 ? pod_row(s) : s; }

// Node-uniform attribution parameters (SGPRs) for the row passes.
template <int Z>
struct Attr {
  uint64_t aE[Z];  // NodeUsage.activeEnergy
  double aP[Z];    // NodeUsage.ActivePower
  uint32_t live;   // bit z: zone passes the guard (ActivePower, activeEnergy, ΔcpuNode)
  uint32_t live_pod;  // pod.go:96 guards on Power instead of ActivePower
  double nd;       // ProcessTotalCPUTimeDelta
  uint32_t first;  // first*Read variant: EnergyTotal = interval energy, Power 0
  // KACC_F_STABLE_SLOT_NODES on a node past its first read: a row's slot already
  // holds this node in KACC_T_PROC_NODE unless the row is NEW, so only NEW rows
  // store it (4 B per process row less HBM traffic)
  uint32_t keep_node;
};

// Attr from the node phase's LDS results (block-uniform -> SGPRs).
template <int Z>
__device__ __forceinline__ Attr<Z> make_attr(const NodeShared &sh, uint32_t flags) {
  Attr<Z> a;
  a.nd = uniform_f64(sh.node_delta);
  a.first = uniform_u32(sh.first);
  a.keep_node = (flags & KACC_F_STABLE_SLOT_NODES) && !a.first ? 1u : 0u;
  a.live = 0;
  a.live_pod = 0;
#pragma unroll
  for (int z = 0; z < Z; ++z) {
    a.aE[z] = uniform_u64(sh.active_energy[z]);
    a.aP[z] = uniform_f64(sh.active_power[z]);
    const double pw = uniform_f64(sh.power[z]);
    const bool ok = a.aE[z] != 0 && a.nd != 0;
    if (ok && a.aP[z] != 0) a.live |= 1u << z;                       // process.go:124
    if (ok && (a.first ? a.aP[z] : pw) != 0) a.live_pod |= 1u << z;  // pod.go:96 / :23
  }
  return a;
}

// process.go:118-148 (and its container/VM/pod twins) for one row.
template <int Z>
__device__ __forceinline__ double attribute_row(const Attr<Z> &a, uint32_t live, double delta,
                                                bool is_new, const uint64_t (&prev)[Z],
                                                uint64_t (&E)[Z], double (&P)[Z]) {
  const double ratio = delta / a.nd;  // one IEEE division per row, never a reciprocal
#pragma unroll
  for (int z = 0; z < Z; ++z) {
    if (live & (1u << z)) {
      const uint64_t e = go_f64_to_u64(ratio * u2f(a.aE[z]));
      E[z] = a.first ? e : e + (is_new ? 0ull : prev[z]);
      P[z] = a.first ? 0.0 : ratio * a.aP[z];
    } else {  // skipped zone keeps the zero Usage of newProcess (process.go:58-63)
      E[z] = 0;
      P[z] = 0.0;
    }
  }
  return ratio;
}

// process.go:118-148 for one process row: the energy totals, and the row's
// cpuTimeRatio (returned), which the state keeps INSTEAD of the Z powers: a
// process's Power is ratio · the node's ActivePower when the zone passes the
// guard (process.go:124, 142) — a function of the node's own tables of the same
// interval (kacc_derive.hpp), derived wherever it is read.  8 + 4 bytes per row
// (ratio, node) instead of 8Z.
template <int Z>
__device__ __forceinline__ double attribute_proc(const Attr<Z> &a, double delta, bool is_new,
                                                 const uint64_t (&prev)[Z], uint64_t (&E)[Z]) {
  const double ratio = delta / a.nd;  // one IEEE division per row, never a reciprocal
#pragma unroll
  for (int z = 0; z < Z; ++z) {
    if (a.live & (1u << z)) {
      const uint64_t e = go_f64_to_u64(ratio * u2f(a.aE[z]));
      E[z] = a.first ? e : e + (is_new ? 0ull : prev[z]);
    } else {  // skipped zone keeps the zero Usage of newProcess (process.go:58-63)
      E[z] = 0;
    }
  }
  return ratio;
}

// A process row's outputs at slot s: energy totals, ratio and node.
template <int Z, bool NT>
__device__ __forceinline__ void store_proc(const DevState &st, uint64_t s, const uint64_t (&E)[Z], double ratio,
                                           uint32_t node, bool wnode) {
  store_row<Z, NT, uint64_t>(st.proc_energy, s, E);
  if constexpr (NT) {
    nt_store(ratio, st.proc_ratio + s);
    if (wnode) nt_store(node, st.proc_node + s);
  } else {
    st.proc_ratio[s] = ratio;
    if (wnode) st.proc_node[s] = node;
  }
}

// Cluster-total exports (kacc_interval.pod_export / node_export): what a pod /
// node contributes to the cluster totals, in batch order, written by the
// interval's own kernels so that kacc_allreduce_exports reduces them on
// another stream while the next interval runs.  Pod row q: EnergyTotal[Z] then
// the bits of Power[Z] (zeros for a pod whose slot is out of range).
// Plain stores: a lane's record leaves as Z/2 + Z/2 16-B pieces, so each wave
// instruction writes every 2Z-th 16 B of the wave's span; L2 merges the pieces
// into full lines (non-temporal, each piece would reach HBM as a partial line).
// The export row of batch pod q (kacc_interval.pod_export_pos: namespace order),
// or ~0u when it is out of range (raised; nothing is written).
__device__ __forceinline__ uint32_t export_row(const kacc_interval &b, uint32_t q, uint32_t *err) {
  if (!b.pod_export_pos) return q;
  const uint32_t r = b.pod_export_pos[q];
  if (r >= b.n_pods) {
    atomicOr(err, 1u << 1);  // kErrOffsets
    return ~0u;
  }
  return r;
}
template <int Z>
__device__ __forceinline__ void export_pod_at(const kacc_interval &b, uint32_t row, const uint64_t (&E)[Z],
                                              const double (&P)[Z]) {
  if (!b.pod_export || row == ~0u) return;
  uint64_t *o = b.pod_export + static_cast<uint64_t>(row) * (2 * Z);
  store_row<Z, false, uint64_t>(o, 0, E);
  store_row<Z, false, double>(reinterpret_cast<double *>(o), 1, P);
}
template <int Z>
__device__ __forceinline__ void export_pod(const kacc_interval &b, uint32_t q, const uint64_t (&E)[Z],
                                           const double (&P)[Z], uint32_t *err) {
  if (!b.pod_export) return;
  export_pod_at<Z>(b, export_row(b, q, err), E, P);
}
template <int Z>
__device__ __forceinline__ void export_pod_zero(const kacc_interval &b, uint32_t q, uint32_t *err) {
  uint64_t E[Z];
  double P[Z];
#pragma unroll
  for (int z = 0; z < Z; ++z) {
    E[z] = 0;
    P[z] = 0.0;
  }
  export_pod<Z>(b, q, E, P, err);
}
// Node n, zone z: ActiveEnergyTotal, IdleEnergyTotal, Power, ActivePower, IdlePower.
template <int Z>
__device__ __forceinline__ void export_node_zone(const kacc_interval &b, uint32_t n, uint32_t z, uint64_t at,
                                                 uint64_t it, double p, double ap, double ip) {
  if (!b.node_export) return;
  uint64_t *o = b.node_export + static_cast<uint64_t>(n) * (5 * Z) + z;
  o[0] = at;
  o[Z] = it;
  o[2 * Z] = static_cast<uint64_t>(__double_as_longlong(p));
  o[3 * Z] = static_cast<uint64_t>(__double_as_longlong(ap));
  o[4 * Z] = static_cast<uint64_t>(__double_as_longlong(ip));
}

// An aggregate row's outputs at slot s: energy totals; for a pod its powers,
// for a container / VM its ratio and node (their power is derived on read as
// a process's: the same guard, container.go:106-140, vm.go:78-109).
template <int Z, typename T>
__device__ __forceinline__ void wt_row(T *__restrict__ base, uint64_t s, const T (&in)[Z]) {
  if constexpr (Z % 2 == 0) {
    using v2 = __attribute__((ext_vector_type(2))) T;
    v2 *p = reinterpret_cast<v2 *>(base + s * Z);
#pragma unroll
    for (int k = 0; k < Z / 2; ++k) {
      v2 x;
      x.x = in[2 * k];
      x.y = in[2 * k + 1];
      wt_store(x, p + k);
    }
  } else {
#pragma unroll
    for (int z = 0; z < Z; ++z) wt_store(in[z], base + s * Z + z);
  }
}

template <int Z, bool NT>
__device__ __forceinline__ void store_agg(const DevState &st, uint32_t role, uint64_t s, const uint64_t (&E)[Z],
                                          const double (&P)[Z], double ratio, uint32_t node) {
  if constexpr (KACC_WT_AGG != 0 && !NT) {
    if (role == 3) {
      wt_row<Z, uint64_t>(st.pod_energy, pod_row(s), E);
      wt_row<Z, double>(st.pod_power, pod_row(s), P);
      return;
    }
    wt_row<Z, uint64_t>(role == 1 ? st.ctr_energy : st.vm_energy, s, E);
    wt_store(ratio, (role == 1 ? st.ctr_ratio : st.vm_ratio) + s);
    wt_store(node, (role == 1 ? st.ctr_node : st.vm_node) + s);
    return;
  }
  if (role == 3) {
    store_row<Z, NT, uint64_t>(st.pod_energy, pod_row(s), E);
    store_row<Z, NT, double>(st.pod_power, pod_row(s), P);
    return;
  }
  store_row<Z, NT, uint64_t>(role == 1 ? st.ctr_energy : st.vm_energy, s, E);
  double *r = role == 1 ? st.ctr_ratio : st.vm_ratio;
  uint32_t *nd = role == 1 ? st.ctr_node : st.vm_node;
  if constexpr (NT) {
    nt_store(ratio, r + s);
    nt_store(node, nd + s);
  } else {
    r[s] = ratio;
    nd[s] = node;
  }
}

// A container's CPU time (informer.go:229-233, 481-486): delta and total summed
// over rows [i, e) of s_d in listing order — Go's order, so one lane adds them
// one after the other.  kB reads are issued together per step; a tail step adds
// +0.0 for rows past e, an identity on sums that start at +0.0 (neither sum can
// ever be -0.0), and reads a clamped in-bounds row.
template <int kB>
__device__ __forceinline__ void segment_load(const double *s_d, uint32_t i, uint32_t e, double (&v)[kB]) {
#pragma unroll
  for (int u = 0; u < kB; ++u) v[u] = s_d[min(i + u, e - 1)];  // e > i: in bounds
}
template <int kB>
__device__ __forceinline__ void segment_add(const double (&v)[kB], uint32_t i, uint32_t e, double &delta,
                                            double &total) {
#pragma unroll
  for (int u = 0; u < kB; ++u) {
    const double x = i + u < e ? v[u] : 0.0;
    delta = delta + x;
    total = total + x;
  }
}
// One batch at a time (kernels short of registers).
template <int kB>
__device__ __forceinline__ void segment_sum(const double *s_d, uint32_t i, uint32_t e, double &delta,
                                            double &total) {
  for (; i < e; i += kB) {
    double v[kB];
    segment_load<kB>(s_d, i, e, v);
    segment_add<kB>(v, i, e, delta, total);
  }
}
// Slot sweep: a node whose rows' slots span at most kRowsLds slots (the slot
// join keeps each node in its own slot range) is attributed in SLOT order:
// 64-slot groups [smin + pos0, +64) moved with 1 KiB-contiguous wave
// instructions, each slot's row found through the LDS inverse map s_inv
// (0xffff = no row: a free slot, skipped).  The same two functions move a
// 64-row group whose slots are consecutive (row = row0 + index, no map).
// Piece p = lane + 64j of a group holds zones 2(p mod Z/2), +1 of the group's
// slot p div (Z/2); pieces past len or the table end are masked.
// Loads are unconditional (a masked piece reads slot `safe`, a valid slot,
// and is zeroed): no exec-mask branches, so every group's loads stay in flight.
template <int Z, bool kMasked, bool kNtLoad = false>
__device__ __forceinline__ void load_group_masked(const uint64_t *__restrict__ base, uint64_t s0,
                                                  uint32_t len, uint64_t safe, uint64_t (&out)[Z]) {
  using u64x2 = __attribute__((ext_vector_type(2))) unsigned long long;
  constexpr int kHalf = Z / 2;
  const uint32_t lane = threadIdx.x & 63u;
  const u64x2 *p = reinterpret_cast<const u64x2 *>(base + s0 * Z);
  const u64x2 *q = reinterpret_cast<const u64x2 *>(base + safe * Z);
#pragma unroll
  for (int j = 0; j < kHalf; ++j) {
    const uint32_t piece = lane + 64u * j;
    if constexpr (!kMasked) {  // a full group of consecutive slots
      const u64x2 x = kNtLoad ? __builtin_nontemporal_load(p + piece) : p[piece];
      out[2 * j] = x.x;
      out[2 * j + 1] = x.y;
      continue;
    }
    const bool ok = piece / kHalf < len;
    const u64x2 *src = ok ? p + piece : q;
    const u64x2 x = kNtLoad ? __builtin_nontemporal_load(src) : *src;
    out[2 * j] = ok ? x.x : 0ull;
    out[2 * j + 1] = ok ? x.y : 0ull;
  }
}

template <int Z, bool NT, bool kInv>
__device__ __forceinline__ void attribute_group_masked(const Attr<Z> &a, const NodeShared &sh,
                                                       const double *s_d, const uint32_t *s_w,
                                                       const uint16_t *s_inv,
                                                       uint32_t row0, uint64_t s0, uint32_t len,
                                                       const uint64_t (&prev)[Z],
                                                       uint64_t *__restrict__ energy,
                                                       double *__restrict__ ratio_tab,
                                                       uint32_t *__restrict__ node_tab, uint32_t node) {
  using u64x2 = __attribute__((ext_vector_type(2))) unsigned long long;
  constexpr int kHalf = Z / 2;
  const uint32_t lane = threadIdx.x & 63u;
  u64x2 *pe = reinterpret_cast<u64x2 *>(energy + s0 * Z);
#pragma unroll
  for (int j = 0; j < kHalf; ++j) {
    const uint32_t piece = lane + 64u * j;
    const uint32_t idx = piece / kHalf;
    const uint32_t zp = piece % kHalf;
    uint32_t row = row0 + idx;
    if constexpr (kInv) {
      if (idx >= len) continue;
      row = s_inv[row];
      if (row == 0xffffu) continue;  // free slot of the node's range
    }
    const uint32_t wr = s_w[row];
    const bool is_new = (wr & KACC_SLOT_NEW) != 0;
    const double ratio = s_d[row] / a.nd;  // the row's own IEEE division
    uint64_t E[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      // zone 2*zp+h: lane-dependent, so read from LDS (a register array
      // indexed by a lane value would be demoted to scratch)
      const uint32_t z = 2 * zp + h;
      const uint64_t aE = sh.active_energy[z];
      if (a.live & (1u << z)) {
        const uint64_t e = go_f64_to_u64(ratio * u2f(aE));
        E[h] = a.first ? e : e + (is_new ? 0ull : prev[2 * j + h]);
      } else {
        E[h] = 0;
      }
    }
    u64x2 ev;
    ev.x = E[0];
    ev.y = E[1];
    if constexpr (NT)
      nt_store(ev, pe + piece);
    else
      pe[piece] = ev;
    if (zp == 0) {  // the slot's ratio and node: contiguous across the group's lanes
      const bool wnode = !a.keep_node || is_new;
      if constexpr (NT) {
        nt_store(ratio, ratio_tab + s0 + idx);
        if (wnode) nt_store(node, node_tab + s0 + idx);
      } else {
        ratio_tab[s0 + idx] = ratio;
        if (wnode) node_tab[s0 + idx] = node;
      }
    }
  }
}

// Phase A for one zone (thread z < Z): node.go:10-84 / node.go:101-131.
template <int Z>
__device__ __forceinline__ void node_zone(const kacc_interval &b, const DevState &st, uint32_t n,
                                          int z, NodeShared &sh) {
  const bool first = st.node_has_prev[n] == 0u;
  const uint64_t i = static_cast<uint64_t>(n) * Z + z;
  const double ratio = b.node_usage_ratio[n];
  const uint64_t abs_e = b.zone_energy[i];
  uint64_t active;
  double p = 0.0, ap = 0.0, ip = 0.0;
  uint64_t at, it;
  if (first) {  // firstNodeRead, node.go:111-128
    active = go_f64_to_u64(u2f(abs_e) * ratio);
    at = active;
    it = abs_e - active;
  } else {  // calculateNodePower, node.go:50-68
    const double dt = go_duration_seconds(go_sub_mono(b.node_ts_ns[n], st.node_ts[n]));
    const uint64_t delta = energy_delta(abs_e, st.node_energy_total[i], b.zone_max[i]);
    active = go_f64_to_u64(u2f(delta) * ratio);
    at = st.node_active_total[i] + active;
    it = st.node_idle_total[i] + (delta - active);
    p = u2f(delta) / dt;
    ap = p * ratio;
    ip = p - ap;
  }
  st.node_active_total[i] = at;
  st.node_idle_total[i] = it;
  export_node_zone<Z>(b, n, static_cast<uint32_t>(z), at, it, p, ap, ip);
  st.node_energy_total[i] = abs_e;
  st.node_active_energy[i] = active;
  st.node_power[i] = p;
  st.node_active_power[i] = ap;
  st.node_idle_power[i] = ip;
  sh.active_energy[z] = active;
  sh.power[z] = p;
  sh.active_power[z] = ap;
  if (z == 0) sh.first = first ? 1u : 0u;
}

struct NodeRanges {
  uint32_t p0, p1, c0, c1, v0, v1, q0, q1;
};

// A skipped node (read error) keeps its snapshot (node.go:39-44): its exports
// are its unchanged table values, lanes [lane, +nlanes) of the node's workers.
template <int Z>
__device__ __forceinline__ void export_skipped(const kacc_interval &b, const DevState &st, uint32_t n,
                                               const NodeRanges &r, uint32_t lane, uint32_t nlanes) {
  if (b.node_export) {
    for (uint32_t z = lane; z < static_cast<uint32_t>(Z); z += nlanes) {
      const uint64_t i = static_cast<uint64_t>(n) * Z + z;
      export_node_zone<Z>(b, n, z, st.node_active_total[i], st.node_idle_total[i], st.node_power[i],
                          st.node_active_power[i], st.node_idle_power[i]);
    }
  }
  if (b.pod_export) {
    for (uint32_t q = r.q0 + lane; q < r.q1; q += nlanes) {
      const uint64_t sl = b.pod_slot[q] & KACC_SLOT_MASK;
      if (sl >= st.pod_slots) {
        export_pod_zero<Z>(b, q, st.err);
        continue;
      }
      uint64_t E[Z];
      double P[Z];
      load_row<Z>(st.pod_energy, pod_row(sl), E);
      load_row_f64<Z>(st.pod_power, pod_row(sl), P);
      export_pod<Z>(b, q, E, P, st.err);
    }
  }
}

// Row ranges of node n, clamped so a malformed batch cannot fault.
__device__ __forceinline__ NodeRanges clamp_ranges(const kacc_interval &b, const DevState &st, NodeRanges r,
                                                   int tid);
__device__ __forceinline__ NodeRanges node_ranges(const kacc_interval &b, const DevState &st,
                                                  uint32_t n, int tid) {
  return clamp_ranges(b, st,
                      NodeRanges{b.proc_off[n], b.proc_off[n + 1], b.ctr_off[n], b.ctr_off[n + 1], b.vm_off[n],
                                 b.vm_off[n + 1], b.pod_off[n], b.pod_off[n + 1]},
                      tid);
}

// Status and row ranges of node n as ONE batch of vector loads through an index
// the compiler must treat as per-lane, waited for once, then made uniform: as
// scalar loads they took two dependent round trips (the offsets behind the
// status branch) before a workgroup could issue its row loads.
__device__ __forceinline__ void node_words(const kacc_interval &b, uint32_t n, uint32_t &status, NodeRanges &r) {
  uint32_t ni = n;
  asm volatile("" : "+v"(ni));
  const uint32_t *sp = b.node_status ? b.node_status : b.proc_off;  // a stand-in address: no branch
  const uint32_t s = sp[ni];
  uint32_t w[8] = {b.proc_off[ni], b.proc_off[ni + 1], b.ctr_off[ni], b.ctr_off[ni + 1],
                   b.vm_off[ni],   b.vm_off[ni + 1],   b.pod_off[ni], b.pod_off[ni + 1]};
  asm volatile("" ::"v"(s), "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]), "v"(w[6]),
               "v"(w[7]));  // the one wait
  status = b.node_status ? __builtin_amdgcn_readfirstlane(s) : 0u;
  auto u = [](uint32_t x) { return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(x)); };
  r = NodeRanges{u(w[0]), u(w[1]), u(w[2]), u(w[3]), u(w[4]), u(w[5]), u(w[6]), u(w[7])};
}

__device__ __forceinline__ NodeRanges clamp_ranges(const kacc_interval &b, const DevState &st, NodeRanges r,
                                                   int tid) {
  if (r.p1 > b.n_procs || r.p0 > r.p1 || r.c1 > b.n_ctrs || r.c0 > r.c1 || r.v1 > b.n_vms ||
      r.v0 > r.v1 || r.q1 > b.n_pods || r.q0 > r.q1) {
    if (tid == 0) raise_err(st.err, kErrOffsets);
    r.p1 = min(r.p1, b.n_procs);
    r.p0 = min(r.p0, r.p1);
    r.c1 = min(r.c1, b.n_ctrs);
    r.c0 = min(r.c0, r.c1);
    r.v1 = min(r.v1, b.n_vms);
    r.v0 = min(r.v0, r.v1);
    r.q1 = min(r.q1, b.n_pods);
    r.q0 = min(r.q0, r.q1);
  }
  return r;
}

template <int Z, int V>
__device__ void big_node_prepare(const kacc_interval &b, const DevState &st, uint32_t n,
                                 const NodeRanges &rg, double *red, NodeShared &sh,
                                 uint32_t &s_base);

template <int V>
__device__ __forceinline__ bool fits_fast(const NodeRanges &r) {
  return (V & kVarUnstaged) == 0 && r.p1 - r.p0 <= static_cast<uint32_t>(kRowsLds) &&
         (r.c1 - r.c0) + (r.v1 - r.v0) + (r.q1 - r.q0) <= static_cast<uint32_t>(kTpb<V>);
}

// Namespace totals: kNsLanes lanes per namespace (4 namespaces per wave);
// lane l sums pods l, l+16, ... of its namespace in CSR order (loads issued
// kNsUnroll at a time, adds in order), then the 16 lane sums are halved
// pairwise (l += l+s, s = 8..1).  u64 energy sums are order independent;
// f64 power follows this fixed order (mirrored by oracle/kor_namespace_totals).
// kW: 8-byte words between consecutive rows — 2Z both for the state tables
// (rows = pod slots: one [energy Z | power Z] record per slot, pod_row) and for
// an interval's pod export (rows = batch pod rows, the same record).
// kIdentity: the rows are the CSR positions themselves (an export written in namespace
// order, kacc_interval.pod_export_pos): each namespace is a run of contiguous records.
template <int Z, int kW = 2 * Z, int kThreads = kBlock, bool kIdentity = false>
__device__ __forceinline__ void namespace_block(uint32_t blk, uint32_t n_ns, const uint32_t *__restrict__ off,
                                                const uint32_t *__restrict__ slots, const uint64_t *__restrict__ pe,
                                                const double *__restrict__ pp, uint64_t pod_slots, uint64_t *out_e,
                                                double *out_p, uint32_t *err) {
  const uint32_t k = (blk * kThreads + threadIdx.x) / kNsLanes;
  const uint32_t lane = threadIdx.x % kNsLanes;
  const bool active = k < n_ns;  // inactive lanes still join the shuffles
  unsigned long long e[Z];
  double p[Z];
#pragma unroll
  for (int z = 0; z < Z; ++z) {
    e[z] = 0;
    p[z] = 0.0;
  }
  const uint32_t beg = active ? off[k] : 0u;
  uint32_t end = active ? off[k + 1] : 0u;
  if (pod_slots == 0 && end > beg) {  // no rows to gather from (an empty export): nothing is read
    raise_err(err, kErrNs);
    end = beg;
  }
  // loads unconditional from clamped indices (a predicated load makes the
  // compiler branch around it and wait per element); the adds are masked
  for (uint32_t j0 = beg + lane; j0 < end; j0 += kNsLanes * kNsUnroll) {
    uint32_t sl[kNsUnroll];
#pragma unroll
    for (int u = 0; u < kNsUnroll; ++u) {
      const uint32_t j = min(j0 + u * kNsLanes, end - 1);
      sl[u] = kIdentity ? j : slots[j] & KACC_SLOT_MASK;
    }
    uint64_t er[kNsUnroll][Z];
    double pr[kNsUnroll][Z];
#pragma unroll
    for (int u = 0; u < kNsUnroll; ++u) {
      uint64_t at = sl[u] < pod_slots ? sl[u] : 0u;
      load_row<Z>(pe + at * kW, 0, er[u]);
      load_row_f64<Z>(pp + at * kW, 0, pr[u]);
    }
#pragma unroll
    for (int u = 0; u < kNsUnroll; ++u) {
      const bool in = j0 + u * kNsLanes < end;
      if (in && sl[u] >= pod_slots) raise_err(err, kErrNs);
      const bool use = in && sl[u] < pod_slots;
#pragma unroll
      for (int z = 0; z < Z; ++z) {
        e[z] += use ? er[u][z] : 0ull;
        if (use) p[z] = p[z] + pr[u][z];
      }
    }
  }
#pragma unroll
  for (int z = 0; z < Z; ++z) {
#pragma unroll
    for (int sft = kNsLanes / 2; sft >= 1; sft >>= 1) {
      e[z] += __shfl_down(e[z], sft, kNsLanes);
      p[z] = p[z] + __shfl_down(p[z], sft, kNsLanes);
    }
  }
  if (active && lane == 0) {
    store_row<Z, false, unsigned long long>(reinterpret_cast<unsigned long long *>(out_e), k, e);
    store_row<Z, false, double>(out_p, k, p);
  }
}

template <int Z>
__global__ __launch_bounds__(kBlock) void namespace_kernel(uint32_t n_ns, const uint32_t *__restrict__ off,
                                                           const uint32_t *__restrict__ slots,
                                                           const uint64_t *__restrict__ pe,
                                                           const double *__restrict__ pp, uint64_t pod_slots,
                                                           uint64_t *out_e, double *out_p, uint32_t *err) {
  namespace_block<Z>(blockIdx.x, n_ns, off, slots, pe, pp, pod_slots, out_e, out_p, err);
}

// Cluster partial sums of one context in ONE launch (kacc_allreduce_namespaces):
// the first 5Z blocks are the node-total columns (NodeTotalsArgs), the last
// ns_blocks blocks are namespace_kernel's.
// Column mode of the cluster node totals (see NodeTotalsArgs): block b owns output
// value b / split — column (b / split) / Z of the five node tables, zone (b / split) % Z —
// and, split > 1, its node range b % split; lanes tid < kBlock sum it (the same order
// whatever the caller's block size); s_w: kBlock / 64 words.  kSplit: the instance
// that may split (cluster_partials_kernel past kColSplitFrom nodes).
template <int Z, bool kSplit = false>
__device__ __forceinline__ void node_column_block(const NodeTotalsArgs na, uint32_t b, uint64_t *s_w) {
  const uint32_t tid = threadIdx.x;
  if (tid >= static_cast<uint32_t>(kBlock)) return;  // no barrier below: the idle lanes leave
  const uint32_t split = kSplit ? na.split : 1u;
  const uint32_t o = b / split, part = b % split;
  const uint32_t t = o / Z, z = o % Z;
  const bool is_u64 = t < 2;
  const uint64_t *col = na.node_export ? na.node_export + t * Z + z
                        : t == 0 ? na.active_total + z
                        : t == 1 ? na.idle_total + z
                        : reinterpret_cast<const uint64_t *>(t == 2 ? na.power : t == 3 ? na.active_power
                                                                                        : na.idle_power) + z;
  const uint64_t stride = na.node_export ? 5ull * Z : static_cast<uint64_t>(Z);
  const uint64_t lo = kSplit ? min(static_cast<uint64_t>(part) * kColSplitNodes, na.n_nodes) : 0ull;
  const uint64_t hi = kSplit && split > 1 ? min(lo + kColSplitNodes, na.n_nodes) : na.n_nodes;
  unsigned long long e = 0;
  double p = 0.0;
  // lane tid adds nodes lo + tid, lo + tid + kBlock, ... in that order
  for (uint64_t n0 = lo + tid; n0 < hi; n0 += static_cast<uint64_t>(kBlock) * kColLoads) {
    uint64_t v[kColLoads];
#pragma unroll
    for (int u = 0; u < kColLoads; ++u) {  // unconditional from clamped nodes: all in flight
      const uint64_t n = min(n0 + static_cast<uint64_t>(u) * kBlock, hi - 1);
      v[u] = col[n * stride];
    }
#pragma unroll
    for (int u = 0; u < kColLoads; ++u) {
      if (n0 + static_cast<uint64_t>(u) * kBlock >= hi) continue;
      if (is_u64)
        e += v[u];
      else
        p = p + __longlong_as_double(static_cast<long long>(v[u]));
    }
  }
#pragma unroll
  for (int sft = 32; sft >= 1; sft >>= 1) {
    e += __shfl_down(e, sft, 64);
    p = p + __shfl_down(p, sft, 64);
  }
  if ((tid & 63u) == 0) s_w[tid >> 6] = is_u64 ? e : static_cast<uint64_t>(__double_as_longlong(p));
  __syncthreads();
  if (tid != 0) return;
  auto add = [&](uint64_t a, uint64_t x) -> uint64_t {  // u64 (modular) or f64 bits
    if (is_u64) return a + x;
    const double f = __longlong_as_double(static_cast<long long>(a)) + __longlong_as_double(static_cast<long long>(x));
    return static_cast<uint64_t>(__double_as_longlong(f));
  };
  uint64_t r = s_w[0];  // the block's value
  for (int w = 1; w < kBlock / 64; ++w) r = add(r, s_w[w]);
  if (kSplit && split > 1) {  // publish; the last block of the column adds the partials in order
    __hip_atomic_store(na.part + static_cast<uint64_t>(o) * split + part, r, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    if (__hip_atomic_fetch_add(na.arrived + o, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) != split - 1) return;
    r = __hip_atomic_load(na.part + static_cast<uint64_t>(o) * split, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t k = 1; k < split; ++k) {
      const uint64_t x =
          __hip_atomic_load(na.part + static_cast<uint64_t>(o) * split + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      r = add(r, x);
    }
    __hip_atomic_store(na.arrived + o, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // the next launch's
  }
  if (is_u64)
    na.out_e[t * Z + z] = r;
  else
    na.out_p[(t - 2) * Z + z] = __longlong_as_double(static_cast<long long>(r));
}

// Partial sums of an earlier interval's exports inside an interval launch
// (kacc_run_interval_sums): node_blocks node-total columns before the n_nodes node
// workgroups and ns_blocks namespace-sum blocks of kTpb threads after them — the
// same per-lane orders as cluster_partials_kernel (node_column_block sums with
// its first kBlock lanes whatever the block size; a namespace is kNsLanes lanes
// wherever its block starts), so the same bits.  The namespace blocks run in the
// launch's tail, when the last residency round leaves compute units free; every sums
// block reads only the earlier interval's exports (never a table this launch writes):
// no wait, no second launch.
struct SumsArgs {
  uint32_t node_blocks, ns_blocks, n_ns, ordered;
  const uint32_t *off, *rows;
  const uint64_t *pe;
  const double *pp;
  uint64_t n_pods;
  uint64_t *out_e;
  double *out_p;
  NodeTotalsArgs na;
};

template <int Z, int kThreads>
__device__ __forceinline__ void sums_block(const SumsArgs &sa, uint32_t sb, uint32_t *err) {
  if (sb < sa.node_blocks) {
    __shared__ uint64_t s_w[kBlock / 64];
    node_column_block<Z>(sa.na, sb, s_w);
    return;
  }
  sb -= sa.node_blocks;
  if (sa.ordered)
    namespace_block<Z, 2 * Z, kThreads, true>(sb, sa.n_ns, sa.off, sa.rows, sa.pe, sa.pp, sa.n_pods, sa.out_e,
                                              sa.out_p, err);
  else
    namespace_block<Z, 2 * Z, kThreads, false>(sb, sa.n_ns, sa.off, sa.rows, sa.pe, sa.pp, sa.n_pods, sa.out_e,
                                               sa.out_p, err);
}

// One node snapshot of one interval on workgroup `blk` (interval_kernel).
template <int Z, int V>
__device__ __forceinline__ void interval_node(const kacc_interval &b, const DevState &st, const uint32_t blk) {
  constexpr int kThreads = kTpb<V>;
  constexpr int kRowsPerThread = kRpt<V>;
  // non-temporal hints on the row streams (read once / written once per
  // interval, 2.5 GB at config 3: nothing to keep in L2 or the Infinity
  // Cache): loads + stores together measured 5 % faster (profiles/r01/ablations)
  constexpr bool kNT = (V & kVarTemporalStores) == 0;
  constexpr bool kNtLd = (V & kVarTemporalLoads) == 0;
  constexpr bool kNtAgg = kNT && (kNtAggStores || (V & kVarNtAgg) != 0);
  constexpr bool kNtScat = kNT && (kNtScatterStores || (V & kVarNtScatter) != 0);
  __shared__ double s_d[kRowsLds];   // this node's Δcpu rows
  __shared__ uint32_t s_w[kRowsLds];  // and their slot words (frees VGPRs across barriers)
  __shared__ double s_cd[kThreads];  // container Δ of this interval
  __shared__ double s_ct[kThreads];  // container running CPU total
  __shared__ double red[kTree];
  __shared__ NodeShared sh;
  __shared__ uint16_t s_inv[kRowsLds];  // slot sweep: slot - smin -> row (0xffff: none)

  const int tid = threadIdx.x;
  constexpr bool kStamp = (V & kVarStamps) != 0;
  uint64_t *stamp = kStamp ? st.stamps + static_cast<uint64_t>(blk) * 8 : nullptr;
  if constexpr (kStamp) {
    if (tid == 0) {
      stamp[0] = __builtin_amdgcn_s_memrealtime();
      stamp[4] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
      stamp[5] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
      stamp[6] = blk;
    }
  }
  // the previous interval's pod_kernel has drained the deferred list; this
  // interval's chunk_kernel refills it after this kernel
  if (blk == 0 && tid == 0) st.defer_ctr[0] = 0u;
  uint32_t n = blk;
  if (b.node_order) n = b.node_order[blk];
  if (n >= b.n_nodes) {
    if (tid == 0) raise_err(st.err, kErrNode);
    return;
  }
  uint32_t status;
  NodeRanges raw;
  node_words(b, n, status, raw);
  if (status & KACC_NODE_READ_ERROR) {
    // node.go:39-44 -> calculatePower fails, previous snapshot kept.
    if (tid == 0) st.node_status[n] = KACC_NODE_SKIPPED;
    if (b.pod_export || b.node_export)
      export_skipped<Z>(b, st, n, clamp_ranges(b, st, raw, tid), static_cast<uint32_t>(tid), kThreads);
    return;
  }
  const NodeRanges rg = clamp_ranges(b, st, raw, tid);
  if (!fits_fast<V>(rg)) {  // node phase here, the rest in chunk_kernel (+ pod_kernel)
    if (b.flags & KACC_F_FAST_NODES) {  // the caller promised no such node: no launch follows
      if (tid == 0) raise_err(st.err, kErrBigNode);
      return;
    }
    __shared__ uint32_t s_base;
    big_node_prepare<Z, V>(b, st, n, rg, red, sh, s_base);
    return;
  }
  const uint32_t p0 = rg.p0, p1 = rg.p1, c0 = rg.c0, c1 = rg.c1, v0 = rg.v0, v1 = rg.v1,
                 q0 = rg.q0, q1 = rg.q1;
  const uint32_t rows = p1 - p0, nc = c1 - c0, nv = v1 - v0, nq = q1 - q0;

  // ---- A: node zones (threads z < Z) ------------------------------------------
  if (tid < Z) node_zone<Z>(b, st, n, tid, sh);

  // ======================= fast path: one node fits the block ===================
  // Every global load the node needs is issued here, before the first barrier:
  // the rows' Δ and slot words, then (dependent) their previous totals; one
  // aggregate per lane (containers, then VMs, then pods) with its range,
  // slot, previous totals and running CPU total.
  const double *__restrict__ dcpu = b.proc_cpu_delta + p0;
  const uint32_t *__restrict__ pslot = b.proc_slot + p0;
  double d[kRowsPerThread];
  uint32_t w[kRowsPerThread];
#pragma unroll
  for (int k = 0; k < kRowsPerThread; ++k) {
    const uint32_t r = tid + k * kThreads;
    const bool in = r < rows;
    if constexpr (kNtLd) {
      d[k] = in ? __builtin_nontemporal_load(dcpu + r) : 0.0;
      w[k] = in ? __builtin_nontemporal_load(pslot + r) : 0xffffffffu;
    } else {
      d[k] = in ? dcpu[r] : 0.0;
      w[k] = in ? pslot[r] : 0xffffffffu;
    }
  }
  // aggregate role of this lane: 1 container, 2 VM, 3 pod
  // role/index/validity are recomputed from tid and the node's (SGPR) counts
  // wherever needed instead of being held in VGPRs across the barriers.
  const uint32_t utid = static_cast<uint32_t>(tid);
  auto role_of = [&]() -> uint32_t {
    if ((V & kVarSkipAggregates) != 0) return 0u;
    return utid < nc ? 1u : utid < nc + nv ? 2u : utid < nc + nv + nq ? 3u : 0u;
  };
  auto index_of = [&]() -> uint32_t {  // position inside the role's range
    return utid < nc ? utid : utid < nc + nv ? utid - nc : utid - nc - nv;
  };
  uint32_t a_beg = 0, a_end = 0, a_w = 0xffffffffu;
  {
    const uint32_t role = role_of(), j = index_of();
    if (role == 1) {
      a_beg = j == 0 ? p0 : b.ctr_proc_end[c0 + j - 1];
      a_end = b.ctr_proc_end[c0 + j];
      a_w = b.ctr_slot[c0 + j];
    } else if (role == 2) {
      a_beg = j == 0 ? (nc ? b.ctr_proc_end[c1 - 1] : p0) : b.vm_proc_end[v0 + j - 1];
      a_end = b.vm_proc_end[v0 + j];
      a_w = b.vm_slot[v0 + j];
    } else if (role == 3) {
      a_beg = j == 0 ? c0 : b.pod_ctr_end[q0 + j - 1];
      a_end = b.pod_ctr_end[q0 + j];
      a_w = b.pod_slot[q0 + j];
    }
  }
  auto a_cap = [&]() -> uint64_t {
    const uint32_t role = role_of();
    return role == 1 ? st.ctr_slots : role == 2 ? st.vm_slots : role == 3 ? st.pod_slots : 0;
  };
  const uint32_t a_s = a_w & KACC_SLOT_MASK;
  auto a_ok_f = [&]() -> bool { return role_of() != 0 && a_s < a_cap(); };
  const bool a_ok = a_ok_f();
  const uint32_t role = role_of();
  const uint32_t j = index_of();
  // per-role tables, re-derived at each use (keeps 8 VGPRs of pointers dead)
  auto a_energy = [&]() { return role == 1 ? st.ctr_energy : role == 2 ? st.vm_energy : st.pod_energy; };
  auto a_cpu_total = [&]() { return role == 1 ? st.ctr_cpu_total : st.pod_cpu_total; };
  auto a_cpu_delta = [&]() {
    return role == 1 ? st.ctr_cpu_delta : role == 2 ? st.vm_cpu_delta : st.pod_cpu_delta;
  };
  // second-level gathers (depend on the slot words).  A 64-row group with
  // consecutive slots is loaded 1 KiB-contiguous per wave instruction; a node
  // whose slots are not consecutive but span <= kRowsLds slots is swept in
  // slot order instead (see load_span_group).
  uint64_t prev[kRowsPerThread][Z];
  uint32_t contig = 0;  // bit k: group k of this wave is transposed (wave-uniform)
  constexpr bool kSweepable =
      kTransposed<Z> && (V & (kVarNoTranspose | kVarNoSweep | kVarSkipProcs)) == 0;
  // Z without the transposed paths: the same sweep, one slot position per lane
  constexpr bool kRowSweep = !kTransposed<Z> && (V & (kVarNoSweep | kVarSkipProcs)) == 0;
  // slot sweep when the caller gives the node's slot span (kacc_slot_join's
  // out_span) and it fits the LDS inverse map; node-uniform -> SGPRs
  uint32_t smin = 0, span = 0;
  bool sweep = false;
  if constexpr (kSweepable || kRowSweep) {
    if (b.node_proc_span) {
      const uint32_t lo = uniform_u32(b.node_proc_span[2 * n]);
      const uint32_t hi = uniform_u32(b.node_proc_span[2 * n + 1]);
      sweep = rows > 0 && hi >= lo && hi - lo < static_cast<uint32_t>(kRowsLds) && hi < st.proc_slots;
      smin = lo;
      span = hi - lo + 1;
      if (sweep) {
#pragma unroll
        for (int k = 0; k < kRowsPerThread; ++k) s_inv[tid + k * kThreads] = 0xffffu;
      }
    }
  }
  const bool swept = (kSweepable || kRowSweep) && sweep;
  if constexpr ((V & kVarSkipProcs) == 0) {
    if (swept) {  // prev totals of the span's 64-slot groups (free slots read too)
      if constexpr (kRowSweep) {  // slot smin + position (clamped: loads stay unconditional)
#pragma unroll
        for (int k = 0; k < kRowsPerThread; ++k)
          load_row<Z>(st.proc_energy, static_cast<uint64_t>(smin) + min(tid + k * kThreads, span - 1), prev[k]);
      }
      if constexpr (kSweepable) {
#pragma unroll
        for (int k = 0; k < kRowsPerThread; ++k) {
          const uint32_t pos0 = static_cast<uint32_t>(tid & ~63) + k * kThreads;
          const uint32_t len = pos0 < span ? min(span - pos0, 64u) : 0u;
          load_group_masked<Z, true, kNtLd>(st.proc_energy, static_cast<uint64_t>(smin) + pos0, len, smin,
                                     prev[k]);
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < kRowsPerThread; ++k) {
        const uint64_t sl = w[k] & KACC_SLOT_MASK;
        if constexpr (kTransposed<Z> && (V & kVarNoTranspose) == 0) {
          const uint64_t g0 = uniform_u32(static_cast<uint32_t>(sl));  // lane 0's slot
          if (__all((tid + k * kThreads) < rows && sl == g0 + (tid & 63) && g0 + 64 <= st.proc_slots)) {
            contig |= 1u << k;
            load_group_masked<Z, false, kNtLd>(st.proc_energy, g0, 64u, g0, prev[k]);
            continue;
          }
        }
        if (sl < st.proc_slots) {
          load_row<Z>(st.proc_energy, sl, prev[k]);
        } else {
#pragma unroll
          for (int z = 0; z < Z; ++z) prev[k][z] = 0;
        }
      }
    }
  }
  uint64_t a_prev[Z];
  double a_total = 0.0;
  if (a_ok) {
    if constexpr (!kLateAgg<V>) load_row<Z>(a_energy(), agg_row(role, a_s), a_prev);
    if (role != 2 && !(a_w & KACC_SLOT_NEW)) a_total = a_cpu_total()[a_s];
  } else {
#pragma unroll
    for (int z = 0; z < Z; ++z) a_prev[z] = 0;
  }
  if (role != 0 && !a_ok) raise_err(st.err, kErrSlot);

  // ---- B: stage Δ, ProcessTotalCPUTimeDelta (informer.go:330-333) ------------
#pragma unroll
  for (int k = 0; k < kRowsPerThread; ++k) {
    const uint32_t r = tid + k * kThreads;
    if (r < rows) {
      s_d[r] = d[k];
      s_w[r] = w[k];
    }
  }
  __syncthreads();
  if constexpr (kStamp) {
    if (tid == 0) stamp[1] = __builtin_amdgcn_s_memrealtime();
  }
  if (swept) {  // inverse map (s_inv was reset before the barrier; read at E, >= 1 barrier later)
#pragma unroll
    for (int k = 0; k < kRowsPerThread; ++k) {
      const uint32_t r = tid + k * kThreads;
      if (r >= rows) continue;
      const uint32_t sl = s_w[r] & KACC_SLOT_MASK;
      if (sl - smin < span && sl < st.proc_slots)
        s_inv[sl - smin] = static_cast<uint16_t>(r);
      else  // outside the node's span / the table: not attributed
        raise_err(st.err, kErrSlot);
    }
  }
  if (b.flags & KACC_F_NODE_CPU_DELTA_GIVEN) {
    if (tid == 0) sh.node_delta = b.node_cpu_delta[n];
  } else {
    // lane l < 256 sums rows l, l+256, l+512, ... in order; then the halving tree
    if (tid < kTree) {  // all reads in flight; +0.0 past the node's end is an identity
      double v[kRowsLds / kTree];
#pragma unroll
      for (int u = 0; u < kRowsLds / kTree; ++u) v[u] = s_d[tid + kTree * u];
      double s = 0.0;
#pragma unroll
      for (int u = 0; u < kRowsLds / kTree; ++u) s = s + (tid + kTree * u < rows ? v[u] : 0.0);
      red[tid] = s;
    }
    __syncthreads();
    if (tid < 128) red[tid] = red[tid] + red[tid + 128];
    __syncthreads();
    if (tid < 64) {
      double x = red[tid] + red[tid + 64];
#pragma unroll
      for (int k = 32; k >= 1; k >>= 1) x = x + __shfl_down(x, k, 64);
      if (tid == 0) sh.node_delta = x;
    }
  }

  // ---- C: containers and VMs (segmented sums, one lane per segment) ----------
  double a_delta = 0.0;
  if (role == 1 || role == 2) {
    uint32_t beg = a_beg, end = a_end;
    if (beg < p0 || end < beg || end > p1) {
      raise_err(st.err, kErrOffsets);
      beg = max(min(beg, p1), p0);
      end = max(min(end, p1), beg);
    }
    if (role == 1) {
      // resetCPUTime on the first process (informer.go:229-233, 481-486)
      segment_sum<8>(s_d, beg - p0, end - p0, a_delta, a_total);
      s_cd[j] = a_ok ? a_delta : 0.0;
      s_ct[j] = a_ok ? a_total : 0.0;
    } else {
      // updateVMCache (informer.go:445): the last process in listing order wins
      a_delta = end > beg ? s_d[end - 1 - p0] : 0.0;
    }
    if (a_ok) {
      a_cpu_delta()[a_s] = a_delta;
      if (role == 1) a_cpu_total()[a_s] = a_total;
    }
  }
  __syncthreads();

  // ---- D: pods (informer.go:305-309, 502-507) ----------------------------------
  if (role == 3) {
    uint32_t beg = a_beg, end = a_end;
    if (beg < c0 || end < beg || end > c1) {
      raise_err(st.err, kErrOffsets);
      beg = max(min(beg, c1), c0);
      end = max(min(end, c1), beg);
    }
    for (uint32_t c = beg - c0; c < end - c0; ++c) {
      a_delta = a_delta + s_cd[c];
      a_total = a_total + s_ct[c];  // quirk: the container's running total
    }
    if (a_ok) {
      a_cpu_delta()[a_s] = a_delta;
      a_cpu_total()[a_s] = a_total;
    }
  }

  // ---- E: attribution ------------------------------------------------------------
  const Attr<Z> a = make_attr<Z>(sh, b.flags);
  if constexpr (kStamp) {
    if (tid == 0) stamp[2] = __builtin_amdgcn_s_memrealtime();
  }
  if (tid == 0) {  // node scalars of the new snapshot
    st.node_ts[n] = b.node_ts_ns[n];
    st.node_has_prev[n] = 1u;
    st.node_usage_ratio[n] = a.first ? 0.0 : b.node_usage_ratio[n];  // firstNodeRead leaves 0
    st.node_cpu_delta[n] = a.nd;
    st.node_status[n] = a.first ? KACC_NODE_FIRST_READ : KACC_NODE_OK;
  }
  // A batch-order pod export (no pod_export_pos) leaves through LDS: the node's pods are
  // export rows [q0, q1), so after the process pass (s_d free) each pod lane puts its
  // record in s_d and the workgroup writes the node's records as one contiguous run of
  // non-temporal 16-B stores — 1 KiB per wave instruction instead of 16-B pieces at a
  // 16Z-B stride per lane (block-uniform; the late-aggregate order only)
  constexpr uint32_t kStageWords = kRowsLds;  // s_d as u64 words
  const bool stage = kLateAgg<V> && (V & kVarSkipAggregates) == 0 && b.pod_export && !b.pod_export_pos &&
                     nq * 2u * Z <= kStageWords;
  uint64_t *s_stage = reinterpret_cast<uint64_t *>(s_d);
  auto aggregate_out = [&]() {  // container.go:106-140 / vm.go:78-109 / pod.go:87-118
    if (!a_ok) {
      if (role == 3) {
        if (stage) {
#pragma unroll
          for (int z = 0; z < 2 * Z; ++z) s_stage[j * 2 * Z + z] = 0;
        } else {
          export_pod_zero<Z>(b, q0 + j, st.err);
        }
      }
      return;
    }
    if constexpr (kLateAgg<V>) load_row<Z>(a_energy(), agg_row(role, a_s), a_prev);
    // a pod's export row (namespace order) loads beside its previous totals: no extra round trip
    const uint32_t xrow = role == 3 && b.pod_export && !stage ? export_row(b, q0 + j, st.err) : ~0u;
    uint64_t E[Z];
    double P[Z];
    const double ratio = attribute_row<Z>(a, role == 3 ? a.live_pod : a.live, a_delta,
                                          (a_w & KACC_SLOT_NEW) != 0, a_prev, E, P);
    store_agg<Z, kNtAgg>(st, role, a_s, E, P, ratio, n);
    if (role == 3) {
      if (stage) {
#pragma unroll
        for (int z = 0; z < Z; ++z) {
          s_stage[j * 2 * Z + z] = E[z];
          s_stage[j * 2 * Z + Z + z] = static_cast<uint64_t>(__double_as_longlong(P[z]));
        }
      } else {
        export_pod_at<Z>(b, xrow, E, P);
      }
    }
  };
  if constexpr (!kLateAgg<V>) aggregate_out();
  if (swept) {  // process.go:118-148 in slot order: slot smin + pos0 + i holds row s_inv[pos0 + i]
    if constexpr (kRowSweep) {
#pragma unroll
      for (int k = 0; k < kRowsPerThread; ++k) {
        const uint32_t pos = tid + k * kThreads;
        if (pos >= span) continue;
        const uint32_t r = s_inv[pos];
        if (r == 0xffffu) continue;  // a free slot of the node's range
        const uint32_t wk = s_w[r];
        uint64_t E[Z];
        const double ratio = attribute_proc<Z>(a, s_d[r], (wk & KACC_SLOT_NEW) != 0, prev[k], E);
        store_proc<Z, kNT>(st, static_cast<uint64_t>(smin) + pos, E, ratio, n, !a.keep_node || (wk & KACC_SLOT_NEW));
      }
    }
    if constexpr (kSweepable) {
#pragma unroll
      for (int k = 0; k < kRowsPerThread; ++k) {
        const uint32_t pos0 = static_cast<uint32_t>(tid & ~63) + k * kThreads;
        const uint32_t len = pos0 < span ? min(span - pos0, 64u) : 0u;
        attribute_group_masked<Z, kNT, true>(a, sh, s_d, s_w, s_inv, pos0,
                                             static_cast<uint64_t>(smin) + pos0, len, prev[k],
                                             st.proc_energy, st.proc_ratio, st.proc_node, n);
      }
    }
  } else if constexpr ((V & kVarSkipProcs) == 0) {  // process.go:118-148
#pragma unroll
    for (int k = 0; k < kRowsPerThread; ++k) {
      const uint32_t r = tid + k * kThreads;
      if constexpr (kTransposed<Z> && (V & kVarNoTranspose) == 0) {
        if (contig & (1u << k)) {  // rows pos0 + i hold slots s0 + i
          const uint32_t pos0 = r - (tid & 63);
          attribute_group_masked<Z, kNT, false>(a, sh, s_d, s_w, s_inv, pos0,
                                                uniform_u32(s_w[pos0] & KACC_SLOT_MASK), 64u, prev[k],
                                                st.proc_energy, st.proc_ratio, st.proc_node, n);
          continue;
        }
      }
      if (r >= rows) continue;
      const uint32_t wk = s_w[r];
      const uint64_t sl = wk & KACC_SLOT_MASK;
      if (sl >= st.proc_slots) {
        raise_err(st.err, kErrSlot);
        continue;
      }
      uint64_t E[Z];
      const double ratio = attribute_proc<Z>(a, s_d[r], (wk & KACC_SLOT_NEW) != 0, prev[k], E);
      store_proc<Z, kNtScat>(st, sl, E, ratio, n, !a.keep_node || (wk & KACC_SLOT_NEW));
    }
  }
  if (stage) __syncthreads();  // every wave is past the process pass: s_d is free
  if constexpr (kLateAgg<V>) aggregate_out();
  if (stage) {  // the node's pod records, rows [q0, q1) of the export: one contiguous run
    __syncthreads();
    using u64x2 = __attribute__((ext_vector_type(2))) unsigned long long;
    const u64x2 *src = reinterpret_cast<const u64x2 *>(s_stage);
    u64x2 *dst = reinterpret_cast<u64x2 *>(b.pod_export + static_cast<uint64_t>(q0) * (2 * Z));
    for (uint32_t i = utid; i < nq * Z; i += kThreads) nt_store(src[i], dst + i);
  }
  if constexpr (kStamp) {
    __syncthreads();
    if (tid == 0) stamp[3] = __builtin_amdgcn_s_memrealtime();
  }
}

template <int Z, int V>
#ifndef KACC_FAST_WAVES
#define KACC_FAST_WAVES 6  // interval_kernel: waves per SIMD it is compiled for at Z <= 4
#endif
__global__ __launch_bounds__(kTpb<V>, Z > 4 ? 2 : KACC_FAST_WAVES)
void interval_kernel(const kacc_interval b, const DevState st) {
  interval_node<Z, V>(b, st, blockIdx.x);
}

// interval_kernel + the partial sums of an earlier interval's exports in its tail
// blocks (kacc_run_interval_sums; SumsArgs below)
template <int Z, int V>
__global__ __launch_bounds__(kTpb<V>, Z > 4 ? 2 : KACC_FAST_WAVES)
void interval_sums_kernel(const kacc_interval b, const DevState st, const SumsArgs sa) {
  // the node-total columns FIRST (latency chains of 8-B loads: dispatched last they
  // lengthened the launch's tail), then the nodes, then the namespace blocks in the tail
  if (blockIdx.x < sa.node_blocks) {
    sums_block<Z, kTpb<V>>(sa, blockIdx.x, st.err);
    return;
  }
  const uint32_t x = blockIdx.x - sa.node_blocks;
  if (x >= b.n_nodes) {
    sums_block<Z, kTpb<V>>(sa, sa.node_blocks + (x - b.n_nodes), st.err);
    return;
  }
  interval_node<Z, V>(b, st, x);
}

// ============ K intervals in one launch, state carried on chip ====================
// intervals_carry_kernel: the same node snapshot (fast path, per-row slot
// accesses) for K consecutive intervals, one workgroup per node, with
//   * the node's state (has_prev, last timestamp, zone counters and active /
//     idle totals) carried in registers;
//   * every row's last written totals carried in LDS (s_cw / s_cE, keyed by
//     the row position and its slot word) and every aggregate's in registers:
//     when interval k+1 gives a position the slot it had in interval k (the
//     steady state: the slot join keeps a running workload's slot), its
//     previous total is on chip — no 8Z-byte reload per row;
//   * interval k+1's inputs (offsets, Δ, slot words, aggregate descriptors,
//     node readings) loaded into registers during interval k (staged into LDS
//     at the top of k+1), and LDS-only barriers inside an interval, so neither
//     the prefetch nor interval k's stores are waited on before use.
// A position whose slot changed (churn moved rows, aggregates appeared)
// makes the workgroup take one full barrier (its earlier stores complete and
// become visible) and reload those previous totals from the tables.
// Arithmetic, order and outputs are interval_node's, bit for bit.  Z <= 2 (the
// carried totals take 16Z KiB of LDS: two workgroups per CU at Z = 2).
constexpr int kCarryMaxZ = 2;

__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Descriptors read from memory hold generic pointers: flat loads, which also
// count on lgkmcnt, so every LDS wait would drain the prefetch.  Every array of
// a batch is global memory: say so.
#define KACC_GLOBAL __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ const T KACC_GLOBAL *gbl(const T *p) {
  return (const T KACC_GLOBAL *)p;
}

// An index the compiler must treat as per-lane: loads through it are vector
// loads (vmcnt, waited for at the first use of the value) rather than scalar
// loads (lgkmcnt, which every LDS wait drains).
__device__ __forceinline__ uint32_t lane_index(uint32_t x) {
  asm volatile("" : "+v"(x));
  return x;
}
// The wait for a prefetched register happens here (ahead of the interval's
// stores, so that it never waits on them).
template <typename T>
__device__ __forceinline__ void land(const T &x) {
  asm volatile("" ::"v"(x));
}
// What an empty array or an absent optional input reads (never written).
__device__ const uint64_t kacc_zero_words[2] = {0ull, 0ull};
__device__ __forceinline__ const uint32_t *zero_u32() { return reinterpret_cast<const uint32_t *>(kacc_zero_words); }
__device__ __forceinline__ const double *zero_f64() { return reinterpret_cast<const double *>(kacc_zero_words); }

// Node inputs of up to kCarryChunk + 1 consecutive intervals, staged in LDS
// once per chunk (one memory round trip per kCarryChunk intervals): the row
// offsets, readings and status of node n.  Entry e is interval c + e (the last
// interval repeated past K).
// Two shapes: T = 512 threads for KACC_F_FAST_NODES (2048 rows, 512 aggregates)
// and T = 256 for KACC_F_MEDIUM_NODES (1024 rows, 256 aggregates: four
// workgroups per CU, so a 1k-node shard is resident in one round).
constexpr int kCarryRpt = 4;  // row positions per lane
template <int T>
constexpr int kCarryEntries = T / 8;  // one offset word per lane
template <int T>
constexpr int kCarryChunk = kCarryEntries<T> - 1;  // + the lookahead entry the row prefetch reads
template <int Z, int T>
struct CarryTables {
  uint32_t off[kCarryEntries<T> * 8];
  uint32_t status[kCarryEntries<T>];
  int64_t ts[kCarryEntries<T>];
  double ratio[kCarryEntries<T>], nd_given[kCarryEntries<T>];
  uint64_t ze[kCarryEntries<T> * Z], zm[kCarryEntries<T> * Z];
  uint32_t span_lo[kCarryEntries<T>], span_hi[kCarryEntries<T>];  // node_proc_span (lo > hi: none)
};
// A node's rows and this lane's aggregate descriptor (raw; loaded an interval
// ahead): resolved at use, so that no instruction reads them right after the load.
template <int Z>
struct CarryRows {
  double d[kCarryRpt];
  uint32_t w[kCarryRpt];
  uint32_t ce, cb, cw, ve, vb, vw, qe, qb, qw, cre;
};

template <int Z, int T>
__device__ __forceinline__ void fill_tables(const kacc_interval *bs, uint32_t K, uint32_t c, uint32_t n,
                                            CarryTables<Z, T> &t) {
  const uint32_t tid = threadIdx.x;
  {
    const uint32_t e = tid >> 3, f = tid & 7u;
    const kacc_interval &b = bs[lane_index(min(c + e, K - 1))];
    const uint32_t *arr = f < 2 ? b.proc_off : f < 4 ? b.ctr_off : f < 6 ? b.vm_off : b.pod_off;
    t.off[tid] = gbl(arr)[n + (f & 1u)];
  }
  if (tid < static_cast<uint32_t>(kCarryEntries<T>)) {
    const kacc_interval &b = bs[lane_index(min(c + tid, K - 1))];
    t.status[tid] = b.node_status ? gbl(b.node_status)[n] : 0u;
    t.ts[tid] = gbl(b.node_ts_ns)[n];
    t.ratio[tid] = gbl(b.node_usage_ratio)[n];
    t.nd_given[tid] = (b.flags & KACC_F_NODE_CPU_DELTA_GIVEN) ? gbl(b.node_cpu_delta)[n] : 0.0;
    t.span_lo[tid] = b.node_proc_span ? gbl(b.node_proc_span)[2 * static_cast<uint64_t>(n)] : 1u;
    t.span_hi[tid] = b.node_proc_span ? gbl(b.node_proc_span)[2 * static_cast<uint64_t>(n) + 1] : 0u;
#pragma unroll
    for (int z = 0; z < Z; ++z) {
      t.ze[tid * Z + z] = gbl(b.zone_energy)[static_cast<uint64_t>(n) * Z + z];
      t.zm[tid * Z + z] = gbl(b.zone_max)[static_cast<uint64_t>(n) * Z + z];
    }
  }
}

// Row ranges from raw offsets (uniform), clamped as node_ranges() does; a
// malformed batch is reported at use.
__device__ __forceinline__ NodeRanges carry_ranges(const kacc_interval &b, const uint32_t *o, uint32_t &bad) {
  NodeRanges r{uniform_u32(o[0]), uniform_u32(o[1]), uniform_u32(o[2]), uniform_u32(o[3]),
               uniform_u32(o[4]), uniform_u32(o[5]), uniform_u32(o[6]), uniform_u32(o[7])};
  bad = 0u;
  if (r.p1 > b.n_procs || r.p0 > r.p1 || r.c1 > b.n_ctrs || r.c0 > r.c1 || r.v1 > b.n_vms || r.v0 > r.v1 ||
      r.q1 > b.n_pods || r.q0 > r.q1) {
    bad = 1u;
    r.p1 = min(r.p1, b.n_procs);
    r.p0 = min(r.p0, r.p1);
    r.c1 = min(r.c1, b.n_ctrs);
    r.c0 = min(r.c0, r.c1);
    r.v1 = min(r.v1, b.n_vms);
    r.v0 = min(r.v0, r.v1);
    r.q1 = min(r.q1, b.n_pods);
    r.q0 = min(r.q0, r.q1);
  }
  return r;
}

// Every load unconditional from a clamped index into the node's own rows (lanes
// past the node's end re-read its last row: one cache line), empty arrays read
// the zero words: no branch, and no instruction touches a loaded value here.
template <int Z, int T>
__device__ __forceinline__ void load_rows(const kacc_interval &b, const NodeRanges &r, CarryRows<Z> &o) {
  constexpr int kThreads = T, kR = kCarryRpt;
  const uint32_t tid = threadIdx.x;
  const uint32_t rows = r.p1 - r.p0, nc = r.c1 - r.c0, nv = r.v1 - r.v0, nq = r.q1 - r.q0;
  {
    const bool has = b.n_procs != 0;
    const double *pd = has ? b.proc_cpu_delta : zero_f64();
    const uint32_t *pw = has ? b.proc_slot : zero_u32();
    const uint32_t hi = !has ? 0u : rows ? r.p1 - 1 : min(r.p0, b.n_procs - 1);
#pragma unroll
    for (int k = 0; k < kR; ++k) {
      const uint32_t at = lane_index(min(r.p0 + tid + k * kThreads, hi));
      o.d[k] = __builtin_nontemporal_load(gbl(pd) + at);
      o.w[k] = __builtin_nontemporal_load(gbl(pw) + at);
    }
  }
  {  // containers: lanes [0, nc)
    const bool has = b.n_ctrs != 0;
    const uint32_t *pe = has ? b.ctr_proc_end : zero_u32();
    const uint32_t *ps = has ? b.ctr_slot : zero_u32();
    const uint32_t last = has ? b.n_ctrs - 1 : 0u;
    const uint32_t at = lane_index(min(r.c0 + min(tid, nc ? nc - 1 : 0u), last));
    o.ce = gbl(pe)[at];
    o.cb = gbl(pe)[at ? at - 1 : 0u];
    o.cw = gbl(ps)[at];
    o.cre = gbl(pe)[lane_index(nc ? min(r.c1 - 1, last) : 0u)];  // the VM rows' start when nc > 0
  }
  {  // VMs: lanes [nc, nc + nv)
    const bool has = b.n_vms != 0;
    const uint32_t *pe = has ? b.vm_proc_end : zero_u32();
    const uint32_t *ps = has ? b.vm_slot : zero_u32();
    const uint32_t last = has ? b.n_vms - 1 : 0u;
    const uint32_t j = tid >= nc ? min(tid - nc, nv ? nv - 1 : 0u) : 0u;
    const uint32_t at = lane_index(min(r.v0 + j, last));
    o.ve = gbl(pe)[at];
    o.vb = gbl(pe)[at ? at - 1 : 0u];
    o.vw = gbl(ps)[at];
  }
  {  // pods: lanes [nc + nv, nc + nv + nq)
    const bool has = b.n_pods != 0;
    const uint32_t *pe = has ? b.pod_ctr_end : zero_u32();
    const uint32_t *ps = has ? b.pod_slot : zero_u32();
    const uint32_t last = has ? b.n_pods - 1 : 0u;
    const uint32_t j = tid >= nc + nv ? min(tid - nc - nv, nq ? nq - 1 : 0u) : 0u;
    const uint32_t at = lane_index(min(r.q0 + j, last));
    o.qe = gbl(pe)[at];
    o.qb = gbl(pe)[at ? at - 1 : 0u];
    o.qw = gbl(ps)[at];
  }
}

template <int Z>
__device__ __forceinline__ void land_rows(const CarryRows<Z> &o) {
#pragma unroll
  for (int k = 0; k < kCarryRpt; ++k) {
    land(o.d[k]);
    land(o.w[k]);
  }
  land(o.ce), land(o.cb), land(o.cw), land(o.ve), land(o.vb), land(o.vw), land(o.qe), land(o.qb), land(o.qw);
  land(o.cre);
}

// Timing ablations of intervals_carry_kernel (kacc_debug_run_intervals_variant; a
// variant != 0 does NOT compute the reference results).
constexpr int kCarryNoRowStores = 1;   // no process-row stores
constexpr int kCarryPrefetch = 2;      // rows loaded an interval ahead into registers (measured
                                       // slower at four workgroups per CU: profiles/r02/carry_*)
constexpr int kCarryNoAggregates = 4;  // containers / VMs / pods skipped
constexpr int kCarryNeverMoved = 8;    // never take the moved path (no barrier, no reload)
constexpr int kCarryStamps = 16;       // per-wave s_memtime phase totals into st.items (diagnostic)
constexpr int kCarryNtAgg = 32;        // aggregate rows stored non-temporal (round 2; production
                                       // stores them through L2: 1.4 %, profiles/r02/aggab/carry_c2.log)
constexpr int kCarryPhases = 8;

template <int Z, int V = 0, int T = 512>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(4, 4))) void intervals_carry_kernel(const kacc_interval *__restrict__ bs,
                                                                        const uint32_t K, const DevState st) {
  static_assert(Z <= kCarryMaxZ, "carried totals are sized for Z <= kCarryMaxZ");
  static_assert(T == 512 || T == 256, "carry shapes: FAST (512) and MEDIUM (256)");
  constexpr int kThreads = T, kR = kCarryRpt, kRows = kR * T;
  constexpr bool kPrefetch = (V & kCarryPrefetch) != 0;
  __shared__ double s_d[kRows];        // this interval's Δ
  __shared__ uint32_t s_w[kRows];      // and slot words
  __shared__ uint32_t s_cw[kRows];     // carried: the slot word last written at each position
  __shared__ uint64_t s_cE[kRows * Z]; // carried: the totals written there
  __shared__ double s_cd[kThreads];
  __shared__ double s_ct[kThreads];
  __shared__ NodeShared sh;
  __shared__ uint32_t s_moved;
  const uint32_t tid = threadIdx.x, n = blockIdx.x;
  if (n == 0 && tid == 0) st.defer_ctr[0] = 0u;
  uint64_t t_acc[kCarryPhases] = {};
  uint64_t t_last = (V & kCarryStamps) ? __builtin_amdgcn_s_memtime() : 0;
  auto mark = [&](int ph) {
    if constexpr ((V & kCarryStamps) != 0) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      t_acc[ph] += t - t_last;
      t_last = t;
    }
  };
  // carried node state: zone tid (< Z) and the node scalars (every lane)
  const uint64_t zi = static_cast<uint64_t>(n) * Z + (tid < static_cast<uint32_t>(Z) ? tid : 0u);
  uint32_t c_has_prev = st.node_has_prev[n];
  int64_t c_ts = st.node_ts[n];
  // the zone totals (lanes < Z) are carried in LDS, each lane its own entries: out of
  // the registers live across the interval loop (a spill at Z = 2, 256 threads)
  __shared__ uint64_t s_zc[3 * kCarryMaxZ];  // [etot | atot | itot] per zone
  if (tid < static_cast<uint32_t>(Z)) {
    s_zc[tid] = st.node_energy_total[zi];
    s_zc[Z + tid] = st.node_active_total[zi];
    s_zc[2 * Z + tid] = st.node_idle_total[zi];
  }
  // carried aggregate (one per lane)
  uint32_t c_role = 0, c_aw = 0xffffffffu;
  uint64_t c_aE[Z];
  double c_atotal = 0.0;
#pragma unroll
  for (int z = 0; z < Z; ++z) c_aE[z] = 0;
#pragma unroll
  for (int j = 0; j < kR; ++j) s_cw[tid + j * kThreads] = 0xffffffffu;
  if (tid == 0) s_moved = 0;
  // Process-row totals are carried either by ROW position (s_cw: the slot word
  // last written there; a changed slot means "moved") or, when the interval
  // gives the node's slot span (node_proc_span, hi - lo < kRows), by SLOT
  // position in a window [c_sbase, c_sbase + kRows) of the node's own slots:
  // rows are then attributed in slot order through an LDS inverse map (s_inv,
  // in s_cw's memory), so every wave instruction writes contiguous slots even
  // when the join left the node's slots in random row order.  The window is
  // loaded once (the node's slots are private for the whole call) and stays
  // valid across intervals while lo is unchanged.
  constexpr uint32_t kNoWindow = 0xffffffffu, kWindowPending = 0xfffffffeu;
  uint32_t c_sbase = kNoWindow;
  uint16_t *s_inv = reinterpret_cast<uint16_t *>(s_cw);

  // node inputs staged in LDS per chunk of intervals; the rows one interval ahead
  __shared__ CarryTables<Z, T> tab;
  CarryRows<Z> rw;
  fill_tables<Z, T>(bs, K, 0u, n, tab);
  lds_barrier();
  if constexpr (kPrefetch) {  // otherwise every interval loads its own rows at its top: rw
    uint32_t bad;             // is then dead across the loop's back edge (no carried VGPRs)
    load_rows<Z, T>(bs[0], carry_ranges(bs[0], tab.off, bad), rw);
  }
  for (uint32_t k = 0, c = 0; k < K; ++k) {
    if (k - c == static_cast<uint32_t>(kCarryChunk<T>)) {  // block-uniform: the next chunk's inputs
      c = k;
      fill_tables<Z, T>(bs, K, c, n, tab);
      lds_barrier();
    }
    mark(7);
    const uint32_t e = k - c;
    const kacc_interval &b = bs[k];
    if constexpr (!kPrefetch) {
      uint32_t bad;
      load_rows<Z, T>(b, carry_ranges(b, tab.off + e * 8, bad), rw);
    }
    uint32_t bad_offsets;
    const NodeRanges rg = carry_ranges(b, tab.off + e * 8, bad_offsets);
    const uint32_t p0 = rg.p0, p1 = rg.p1, c0 = rg.c0, c1 = rg.c1, q0 = rg.q0, q1 = rg.q1;
    const uint32_t rows = p1 - p0, nc = c1 - c0, nv = rg.v1 - rg.v0, nq = q1 - q0;
    const bool fits = rows <= static_cast<uint32_t>(kRows) && nc + nv + nq <= static_cast<uint32_t>(kThreads);
    // this interval's node inputs (uniform ones to SGPRs) and this lane's aggregate
    const uint32_t status = uniform_u32(tab.status[e]);
    const int64_t ts = static_cast<int64_t>(uniform_u64(static_cast<uint64_t>(tab.ts[e])));
    const double ratio = uniform_f64(tab.ratio[e]), nd_given = uniform_f64(tab.nd_given[e]);
    const uint32_t zl = tid < static_cast<uint32_t>(Z) ? tid : 0u;
    const uint64_t ze = tab.ze[e * Z + zl], zm = tab.zm[e * Z + zl];
    const bool is_c = tid < nc, is_v = !is_c && tid < nc + nv, is_q = !is_c && !is_v && tid < nc + nv + nq;
    const uint32_t a_beg0 = is_c   ? (tid == 0 ? p0 : rw.cb)
                            : is_v ? (tid == nc ? (nc ? rw.cre : p0) : rw.vb)
                            : is_q ? (tid == nc + nv ? c0 : rw.qb)
                                   : 0u;
    const uint32_t a_end0 = is_c ? rw.ce : is_v ? rw.ve : is_q ? rw.qe : 0u;
    const uint32_t a_w = is_c ? rw.cw : is_v ? rw.vw : is_q ? rw.qw : 0xffffffffu;
    // slot sweep this interval? (block-uniform)
    const uint32_t s_lo = uniform_u32(tab.span_lo[e]), s_hi = uniform_u32(tab.span_hi[e]);
    const bool sweep = rows > 0 && s_hi >= s_lo && s_hi - s_lo < static_cast<uint32_t>(kRows) && s_hi < st.proc_slots;
    const uint32_t span = sweep ? s_hi - s_lo + 1 : 0u;
    if (sweep != (c_sbase != kNoWindow)) {  // layout change: drop the row keys / start an empty map
#pragma unroll
      for (int j = 0; j < kR; ++j) s_cw[tid + j * kThreads] = 0xffffffffu;  // s_inv: all 0xffff
      c_sbase = sweep ? kWindowPending : kNoWindow;
      lds_barrier();
    }
    const bool process = !(status & KACC_NODE_READ_ERROR) && fits;
    bool moved = false, outside = false;
#pragma unroll
    for (int j = 0; j < kR; ++j) {  // stage the rows (LDS of interval k-1 is free: barrier at its end)
      const uint32_t r = tid + j * kThreads;
      if (r < rows && fits) {
        s_d[r] = rw.d[j];
        s_w[r] = rw.w[j];
        if (sweep) {
          const uint32_t pos = (rw.w[j] & KACC_SLOT_MASK) - s_lo;
          if (process && pos < span)
            s_inv[pos] = static_cast<uint16_t>(r);
          else
            outside = process;  // a row outside its node's span: not computed
        } else {
          moved |= (rw.w[j] & KACC_SLOT_MASK) != (s_cw[r] & KACC_SLOT_MASK);
        }
      }
    }
    if (outside) raise_err(st.err, kErrSlot);
    const uint32_t flags = b.flags;
    // in flight during interval k: rows and node inputs of k+1, offsets of k+2
    // (a past-the-end interval re-reads the last one: no branch)
    if constexpr (kPrefetch) {
      const uint32_t k1 = min(k + 1, K - 1);
      uint32_t bad;
      load_rows<Z, T>(bs[k1], carry_ranges(bs[k1], tab.off + (k1 - c) * 8, bad), rw);
    }
    if (bad_offsets) {
      if (tid == 0) raise_err(st.err, kErrOffsets);
    }
    if (status & KACC_NODE_READ_ERROR) {  // node.go:39-44: previous snapshot kept
      if (tid == 0) st.node_status[n] = KACC_NODE_SKIPPED;
    } else if (!fits) {  // the caller's KACC_F_FAST_NODES promise was wrong
      if (tid == 0) raise_err(st.err, kErrBigNode);
    } else {
      // ---- this lane's aggregate; did any position move? ---------------------------------
      const uint32_t role = (V & kCarryNoAggregates) ? 0u : is_c ? 1u : is_v ? 2u : is_q ? 3u : 0u;
      const uint32_t a_s = a_w & KACC_SLOT_MASK;
      const uint64_t a_cap = role == 1 ? st.ctr_slots : role == 2 ? st.vm_slots : role == 3 ? st.pod_slots : 0;
      const bool a_ok = role != 0 && a_s < a_cap;
      if (role != 0 && !a_ok) raise_err(st.err, kErrSlot);
      const bool a_moved = a_ok && (role != c_role || a_s != (c_aw & KACC_SLOT_MASK));
      moved |= a_moved;
      if (__any(moved) && (tid & 63) == 0) s_moved = 1u;
      const bool load_window = sweep && c_sbase != s_lo;  // block-uniform
      mark(0);
      lds_barrier();  // s_d / s_w / s_inv staged, s_moved set
      mark(1);
      if (((V & kCarryNeverMoved) == 0 && s_moved) || load_window) {  // block-uniform: the rare path
        __syncthreads();  // this workgroup's earlier stores complete and visible (and ordered)
        if (load_window) {  // the table rows of slots [lo, lo + kRows) (those in the table)
#pragma unroll
          for (int j = 0; j < kR; ++j) {
            const uint32_t pos = tid + j * kThreads;
            const uint64_t sl = static_cast<uint64_t>(s_lo) + pos;
            uint64_t pv[Z];
            if (sl < st.proc_slots) {
              load_row<Z>(st.proc_energy, sl, pv);
#pragma unroll
              for (int z = 0; z < Z; ++z) s_cE[pos * Z + z] = pv[z];
            }
          }
          c_sbase = s_lo;
        } else if (!sweep) {
#pragma unroll
          for (int j = 0; j < kR; ++j) {
            const uint32_t r = tid + j * kThreads;
            if (r >= rows) continue;
            const uint32_t sw = s_w[r];
            const uint64_t sl = sw & KACC_SLOT_MASK;
            if (sl == (s_cw[r] & KACC_SLOT_MASK)) continue;
            uint64_t pv[Z];
            if (sl < st.proc_slots) {
              load_row<Z>(st.proc_energy, sl, pv);
            } else {
#pragma unroll
              for (int z = 0; z < Z; ++z) pv[z] = 0;
            }
#pragma unroll
            for (int z = 0; z < Z; ++z) s_cE[r * Z + z] = pv[z];
          }
        }
        if (a_moved) {
          load_row<Z>(role == 1 ? st.ctr_energy : role == 2 ? st.vm_energy : st.pod_energy, agg_row(role, a_s), c_aE);
          c_atotal = role == 1 ? st.ctr_cpu_total[a_s] : role == 3 ? st.pod_cpu_total[a_s] : 0.0;
        }
        lds_barrier();
        if (tid == 0) s_moved = 0;
      }
      double a_total = (role != 2 && a_ok && !(a_w & KACC_SLOT_NEW)) ? c_atotal : 0.0;

      // ---- A: node zones (node.go:10-84 / 101-131) from the carried state ------------------
      const bool first = c_has_prev == 0u;
      uint64_t z_active = 0;
      double z_p = 0.0, z_ap = 0.0, z_ip = 0.0;
      if (tid < static_cast<uint32_t>(Z)) {
        const uint64_t c_etot = s_zc[tid];
        uint64_t c_atot = s_zc[Z + tid], c_itot = s_zc[2 * Z + tid];
        if (first) {
          z_active = go_f64_to_u64(u2f(ze) * ratio);
          c_atot = z_active;
          c_itot = ze - z_active;
        } else {
          const double dt = go_duration_seconds(go_sub_mono(ts, c_ts));
          const uint64_t delta = energy_delta(ze, c_etot, zm);
          z_active = go_f64_to_u64(u2f(delta) * ratio);
          c_atot = c_atot + z_active;
          c_itot = c_itot + (delta - z_active);
          z_p = u2f(delta) / dt;
          z_ap = z_p * ratio;
          z_ip = z_p - z_ap;
        }
        s_zc[tid] = ze;
        s_zc[Z + tid] = c_atot;
        s_zc[2 * Z + tid] = c_itot;
        sh.active_energy[tid] = z_active;
        sh.power[tid] = z_p;
        sh.active_power[tid] = z_ap;
        if (tid == 0) sh.first = first ? 1u : 0u;
      }
      // ---- B: ProcessTotalCPUTimeDelta (informer.go:330-333) by the last wave, while the
      //      others sum containers: interval_kernel's canonical 256-leaf tree evaluated by
      //      64 lanes as small_kernel does (lane t: leaves t, t+64, t+128, t+192, each the
      //      in-order sum of rows l, l+256, ...) — the same additions in the same order
      if (flags & KACC_F_NODE_CPU_DELTA_GIVEN) {
        if (tid == 0) sh.node_delta = nd_given;
      } else if (tid >= static_cast<uint32_t>(kThreads - 64)) {
        const uint32_t t = tid - (kThreads - 64);
        // a leaf's LDS reads issued together (r < kRows: in bounds); a row past the
        // node's end adds +0.0, an identity on a sum that starts at +0.0
        constexpr int kU = kRows / kTree, kB = kU < 4 ? kU : 4;  // reads in flight
        double leaf[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          double sum = 0.0;
#pragma unroll
          for (int u0 = 0; u0 < kU; u0 += kB) {
            double v[kB];
#pragma unroll
            for (int u = 0; u < kB; ++u) v[u] = s_d[t + 64u * q + static_cast<uint32_t>(kTree) * (u0 + u)];
#pragma unroll
            for (int u = 0; u < kB; ++u) {
              const uint32_t r = t + 64u * q + static_cast<uint32_t>(kTree) * (u0 + u);
              sum = sum + (r < rows ? v[u] : 0.0);
            }
          }
          leaf[q] = sum;
        }
        double x = (leaf[0] + leaf[2]) + (leaf[1] + leaf[3]);
#pragma unroll
        for (int s2 = 32; s2 >= 1; s2 >>= 1) x = x + __shfl_down(x, s2, 64);
        if (t == 0) sh.node_delta = x;
      }
      // ---- C: containers and VMs (one lane per segment, listing order) -------------------
      double a_delta = 0.0;
      if (role == 1 || role == 2) {
        uint32_t beg = a_beg0, end = a_end0;
        if (beg < p0 || end < beg || end > p1) {
          raise_err(st.err, kErrOffsets);
          beg = max(min(beg, p1), p0);
          end = max(min(end, p1), beg);
        }
        if (role == 1) {  // informer.go:229-233, 481-486: in order, 4 LDS reads in flight
          segment_sum<4>(s_d, beg - p0, end - p0, a_delta, a_total);
          s_cd[tid] = a_ok ? a_delta : 0.0;
          s_ct[tid] = a_ok ? a_total : 0.0;
        } else {  // informer.go:445: the last process in listing order wins
          a_delta = end > beg ? s_d[end - 1 - p0] : 0.0;
        }
      }
      mark(2);
      lds_barrier();
      mark(3);
      // ---- D: pods (informer.go:305-309, 502-507) -----------------------------------------
      if (role == 3) {
        uint32_t beg = a_beg0, end = a_end0;
        if (beg < c0 || end < beg || end > c1) {
          raise_err(st.err, kErrOffsets);
          beg = max(min(beg, c1), c0);
          end = max(min(end, c1), beg);
        }
        for (uint32_t c = beg - c0; c < end - c0; ++c) {
          a_delta = a_delta + s_cd[c];
          a_total = a_total + s_ct[c];  // quirk: the container's running total
        }
      }
      // ---- E: attribution; the prefetch lands before the first store -----------------------
      if constexpr (kPrefetch) {
        land_rows<Z>(rw);
      }
      mark(4);
      if (tid < static_cast<uint32_t>(Z)) {
        st.node_active_total[zi] = s_zc[Z + tid];
        st.node_idle_total[zi] = s_zc[2 * Z + tid];
        st.node_energy_total[zi] = ze;
        st.node_active_energy[zi] = z_active;
        st.node_power[zi] = z_p;
        st.node_active_power[zi] = z_ap;
        st.node_idle_power[zi] = z_ip;
      }
      const Attr<Z> a = make_attr<Z>(sh, b.flags);
      if (tid == 0) {
        st.node_ts[n] = ts;
        st.node_has_prev[n] = 1u;
        st.node_usage_ratio[n] = a.first ? 0.0 : ratio;
        st.node_cpu_delta[n] = a.nd;
        st.node_status[n] = a.first ? KACC_NODE_FIRST_READ : KACC_NODE_OK;
      }
      if (a_ok) {  // container.go:106-140 / vm.go:78-109 / pod.go:87-118
        if (role == 1) {
          st.ctr_cpu_delta[a_s] = a_delta;
          st.ctr_cpu_total[a_s] = a_total;
        } else if (role == 2) {
          st.vm_cpu_delta[a_s] = a_delta;
        } else {
          st.pod_cpu_delta[a_s] = a_delta;
          st.pod_cpu_total[a_s] = a_total;
        }
        uint64_t E[Z];
        double P[Z];
        const double ratio =
            attribute_row<Z>(a, role == 3 ? a.live_pod : a.live, a_delta, (a_w & KACC_SLOT_NEW) != 0, c_aE, E, P);
        store_agg<Z, kNtAggStores || (V & kCarryNtAgg) != 0>(st, role, a_s, E, P, ratio, n);
#pragma unroll
        for (int z = 0; z < Z; ++z) c_aE[z] = E[z];
        c_atotal = a_total;
      }
      c_role = a_ok ? role : 0u;
      c_aw = a_ok ? a_w : 0xffffffffu;
      if (sweep) {  // process.go:118-148 in slot order: slot lo + pos holds row s_inv[pos]
#pragma unroll
        for (int j = 0; j < kR; ++j) {
          const uint32_t pos = tid + j * kThreads;
          if (pos >= span) continue;
          const uint32_t r = s_inv[pos];
          if (r == 0xffffu) continue;  // a free slot of the node's range
          s_inv[pos] = 0xffffu;        // the map starts empty next interval (this lane's entry)
          const uint32_t wk = s_w[r];
          uint64_t pv[Z], E[Z];
#pragma unroll
          for (int z = 0; z < Z; ++z) pv[z] = s_cE[pos * Z + z];
          const double ratio = attribute_proc<Z>(a, s_d[r], (wk & KACC_SLOT_NEW) != 0, pv, E);
          if constexpr ((V & kCarryNoRowStores) == 0) {
            store_proc<Z, true>(st, static_cast<uint64_t>(s_lo) + pos, E, ratio, n, !a.keep_node || (wk & KACC_SLOT_NEW));
          }
#pragma unroll
          for (int z = 0; z < Z; ++z) s_cE[pos * Z + z] = E[z];
        }
      } else {
#pragma unroll
      for (int j = 0; j < kR; ++j) {  // process.go:118-148
        const uint32_t r = tid + j * kThreads;
        if (r >= rows) {
          s_cw[r] = 0xffffffffu;
          continue;
        }
        const uint32_t wk = s_w[r];
        const uint64_t sl = wk & KACC_SLOT_MASK;
        if (sl >= st.proc_slots) {
          raise_err(st.err, kErrSlot);
          s_cw[r] = 0xffffffffu;
          continue;
        }
        uint64_t pv[Z], E[Z];
#pragma unroll
        for (int z = 0; z < Z; ++z) pv[z] = s_cE[r * Z + z];
        const double ratio = attribute_proc<Z>(a, s_d[r], (wk & KACC_SLOT_NEW) != 0, pv, E);
        if constexpr ((V & kCarryNoRowStores) == 0) {
          store_proc<Z, kNtScatterStores>(st, sl, E, ratio, n, !a.keep_node || (wk & KACC_SLOT_NEW));
        }
#pragma unroll
        for (int z = 0; z < Z; ++z) s_cE[r * Z + z] = E[z];
        s_cw[r] = wk;  // read back only by this lane (same position) next interval
      }
      }
      c_has_prev = 1u;
      c_ts = ts;
    }
    mark(5);
    lds_barrier();  // LDS of interval k read by every wave before interval k+1 writes it
    mark(6);
  }
  if constexpr ((V & kCarryStamps) != 0) {
    if ((tid & 63u) == 0) {
      uint64_t *out = reinterpret_cast<uint64_t *>(st.items) + (static_cast<uint64_t>(n) * 8 + tid / 64) * kCarryPhases;
#pragma unroll
      for (int ph = 0; ph < kCarryPhases; ++ph) out[ph] = t_acc[ph];
    }
  }
}

// ======================= small nodes: one wavefront per node ======================
// Real nodes run a few hundred processes (the reference's own single-node case
// is 500 procs -> 50 containers -> 20 pods).  A 512-lane workgroup per such
// node leaves most lanes idle and caps residency at 3 nodes per CU (measured:
// 250 procs/node 1.7 TB/s, 500 procs/node 2.9 TB/s against 5.5 TB/s at 2000).
// Under KACC_F_SMALL_NODES every node has <= kSmallRows rows and
// <= kSmallAgg aggregates, and one WAVEFRONT owns a node: the same phases
// A-E as interval_kernel with wave-level LDS ordering instead of workgroup
// barriers, the canonical 256-lane CPU-total tree evaluated by 64 lanes (4
// partial sums per lane, the same additions in the same order), two
// aggregates per lane, and the rows moved as 64-row groups in two batches of
// four (the first batch's previous totals are in flight with the Δ loads).
// Results are bit-identical to interval_kernel's.
constexpr int kSmallRows = 512;
constexpr int kSmallAgg = 128;
constexpr int kSmallWaves = 4;                   // nodes per workgroup
constexpr int kSmallGroups = kSmallRows / 64;    // 64-row groups per node
constexpr int kSmallBatch = 4;                   // groups whose prev totals are in flight together
static_assert(kSmallRows == KACC_SMALL_MAX_PROCS && kSmallAgg == KACC_SMALL_MAX_AGGREGATES,
              "KACC_SMALL_* must match the small-node kernel's capacity");
static_assert(kSmallRows <= 2 * kTree && kSmallGroups == 2 * kSmallBatch && kSmallAgg == 128,
              "small-node tree / batch / aggregate loops assume these sizes");

// LDS writes of one lane made visible to the other lanes of the same wave.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Waves per SIMD small_kernel is compiled for: what its LDS allows (a workgroup is four waves,
// one per SIMD; 160 KiB per CU): 25.4 KiB -> six workgroups at Z <= 3 without the
// slot-order buffer (SW false), 29.5 KiB -> five with it (Z <= 3), 37.7 KiB -> four
// at Z = 4.  Asking for more only failed the target (build warnings, round 3).
template <int Z, bool SW>
constexpr int kSmallWavesPerEu = Z <= 3 ? (SW || Z == 3 ? 5 : 6) : Z == 4 ? 4 : 1;
template <int Z, bool SW>
__global__ __launch_bounds__(64 * kSmallWaves) __attribute__((amdgpu_waves_per_eu(kSmallWavesPerEu<Z, SW>))) void small_kernel(
    const kacc_interval b, const DevState st) {
  constexpr bool kNT = true, kNtLd = true;  // as interval_kernel's production variant
  __shared__ double s_d_all[kSmallWaves][kSmallRows];
  // slot words are read across lanes only by the transposed (sweep / contiguous
  // group) paths; otherwise each lane keeps its own in w[] and the LDS per node
  // drops from 8.4 KB to 6.4 KB (Z = 2: 6 nodes' workgroups per CU, not 4)
  constexpr bool kSweepable = kTransposed<Z>;
  // Z without the transposed paths: with node_proc_span (SW) the rows are moved
  // in slot order too, one slot position per lane, through an inverse map whose
  // entries carry the row's NEW bit (the slot words stay in their lanes' registers)
  constexpr bool kRowSweep = SW && !kTransposed<Z>;
  __shared__ uint32_t s_w_all[kSmallWaves][kSweepable ? kSmallRows : 1];
  __shared__ double s_cd_all[kSmallWaves][kSmallAgg];
  __shared__ double s_ct_all[kSmallWaves][kSmallAgg];
  __shared__ uint16_t s_inv_all[kSmallWaves][kSmallRows];
  __shared__ NodeShared sh_all[kSmallWaves];

  const uint32_t wv = uniform_u32(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63u;
  double *s_d = s_d_all[wv];
  uint32_t *s_w = s_w_all[wv];
  double *s_cd = s_cd_all[wv];
  double *s_ct = s_ct_all[wv];
  uint16_t *s_inv = s_inv_all[wv];
  NodeShared &sh = sh_all[wv];

  if (blockIdx.x == 0 && threadIdx.x == 0) st.defer_ctr[0] = 0u;  // as interval_kernel
  const uint32_t idx = blockIdx.x * kSmallWaves + wv;
  if (idx >= b.n_nodes) return;  // wave-uniform: no workgroup barrier below
  const uint32_t n = b.node_order ? uniform_u32(b.node_order[idx]) : idx;
  if (n >= b.n_nodes) {
    if (lane == 0) raise_err(st.err, kErrNode);
    return;
  }
  uint32_t status;
  NodeRanges raw;
  node_words(b, n, status, raw);
  if (status & KACC_NODE_READ_ERROR) {  // node.go:39-44
    if (lane == 0) st.node_status[n] = KACC_NODE_SKIPPED;
    if (b.pod_export || b.node_export)
      export_skipped<Z>(b, st, n, clamp_ranges(b, st, raw, static_cast<int>(lane)), lane, 64u);
    return;
  }
  const NodeRanges rg = clamp_ranges(b, st, raw, static_cast<int>(lane));
  const uint32_t p0 = rg.p0, p1 = rg.p1, c0 = rg.c0, c1 = rg.c1, q0 = rg.q0, q1 = rg.q1;
  const uint32_t rows = p1 - p0, nc = c1 - c0, nv = rg.v1 - rg.v0, nq = q1 - q0;
  if (rows > static_cast<uint32_t>(kSmallRows) || nc + nv + nq > static_cast<uint32_t>(kSmallAgg)) {
    if (lane == 0) raise_err(st.err, kErrBigNode);  // the caller's promise was wrong
    return;
  }

  // ---- A: node zones ---------------------------------------------------------------
  if (lane < static_cast<uint32_t>(Z)) node_zone<Z>(b, st, n, static_cast<int>(lane), sh);

  // ---- loads: Δ and slot words of every row, then the first batch's prev totals ----
  const double *__restrict__ dcpu = b.proc_cpu_delta + p0;
  const uint32_t *__restrict__ pslot = b.proc_slot + p0;
  double d[kSmallGroups];
  uint32_t w[kSmallGroups];
#pragma unroll
  for (int k = 0; k < kSmallGroups; ++k) {
    const uint32_t r = lane + 64u * k;
    const bool in = r < rows;
    d[k] = in ? __builtin_nontemporal_load(dcpu + r) : 0.0;
    w[k] = in ? __builtin_nontemporal_load(pslot + r) : 0xffffffffu;
  }
  uint32_t smin = 0, span = 0;
  bool swept = false;
  if constexpr (kSweepable || kRowSweep) {
    if (b.node_proc_span) {
      const uint32_t lo = uniform_u32(b.node_proc_span[2 * n]);
      const uint32_t hi = uniform_u32(b.node_proc_span[2 * n + 1]);
      swept = rows > 0 && hi >= lo && hi - lo < static_cast<uint32_t>(kSmallRows) && hi < st.proc_slots;
      smin = lo;
      span = hi - lo + 1;
      if (swept) {
#pragma unroll
        for (int k = 0; k < kSmallGroups; ++k) s_inv[lane + 64u * k] = 0xffffu;
      }
    }
  }
  // batch kb (groups 4kb .. 4kb+3): previous totals into prev; bit g of contig:
  // group 4kb+g is a full group of consecutive slots (wave-uniform)
  uint64_t prev[kSmallBatch][Z];
  uint32_t contig = 0;
  auto load_batch = [&](int kb, bool from_regs) {
    contig = 0;
#pragma unroll
    for (int g = 0; g < kSmallBatch; ++g) {
      const int k = kb * kSmallBatch + g;
      const uint32_t pos0 = 64u * k;
      if constexpr (kRowSweep) {
        if (swept) {  // slot smin + pos0 + lane (clamped: the load stays unconditional)
          load_row<Z>(st.proc_energy, static_cast<uint64_t>(smin) + min(pos0 + lane, span - 1), prev[g]);
          continue;
        }
      }
      if constexpr (kSweepable) {
        if (swept) {
          const uint32_t len = pos0 < span ? min(span - pos0, 64u) : 0u;
          load_group_masked<Z, true, kNtLd>(st.proc_energy, static_cast<uint64_t>(smin) + pos0, len, smin,
                                            prev[g]);
          continue;
        }
      }
      const uint32_t r = pos0 + lane;
      const uint32_t wk = (from_regs || !kSweepable) ? w[k] : (r < rows ? s_w[r] : 0xffffffffu);
      const uint64_t sl = wk & KACC_SLOT_MASK;
      if constexpr (kTransposed<Z>) {
        const uint64_t g0 = uniform_u32(static_cast<uint32_t>(sl));
        if (__all(r < rows && sl == g0 + lane && g0 + 64 <= st.proc_slots)) {
          contig |= 1u << g;
          load_group_masked<Z, false, kNtLd>(st.proc_energy, g0, 64u, g0, prev[g]);
          continue;
        }
      }
      if (r < rows && sl < st.proc_slots) {
        load_row<Z>(st.proc_energy, sl, prev[g]);
      } else {
#pragma unroll
        for (int z = 0; z < Z; ++z) prev[g][z] = 0;
      }
    }
  };
  load_batch(0, true);

  // aggregates: lane handles aggregate i = lane + 64h (containers, VMs, pods)
  auto role_of = [&](uint32_t i) -> uint32_t {
    return i < nc ? 1u : i < nc + nv ? 2u : i < nc + nv + nq ? 3u : 0u;
  };
  auto index_of = [&](uint32_t i) -> uint32_t { return i < nc ? i : i < nc + nv ? i - nc : i - nc - nv; };
  auto cap_of = [&](uint32_t role) -> uint64_t {
    return role == 1 ? st.ctr_slots : role == 2 ? st.vm_slots : role == 3 ? st.pod_slots : 0;
  };
  auto energy_of = [&](uint32_t role) { return role == 1 ? st.ctr_energy : role == 2 ? st.vm_energy : st.pod_energy; };
  auto cpu_total_of = [&](uint32_t role) { return role == 1 ? st.ctr_cpu_total : st.pod_cpu_total; };
  auto cpu_delta_of = [&](uint32_t role) {
    return role == 1 ? st.ctr_cpu_delta : role == 2 ? st.vm_cpu_delta : st.pod_cpu_delta;
  };
  uint32_t a_beg[2], a_end[2], a_w[2];
  uint64_t a_prev[2][Z];
  double a_total[2], a_delta[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t i = lane + 64u * h, role = role_of(i), j = index_of(i);
    a_beg[h] = a_end[h] = 0;
    a_w[h] = 0xffffffffu;
    if (role == 1) {
      a_beg[h] = j == 0 ? p0 : b.ctr_proc_end[c0 + j - 1];
      a_end[h] = b.ctr_proc_end[c0 + j];
      a_w[h] = b.ctr_slot[c0 + j];
    } else if (role == 2) {
      a_beg[h] = j == 0 ? (nc ? b.ctr_proc_end[c1 - 1] : p0) : b.vm_proc_end[rg.v0 + j - 1];
      a_end[h] = b.vm_proc_end[rg.v0 + j];
      a_w[h] = b.vm_slot[rg.v0 + j];
    } else if (role == 3) {
      a_beg[h] = j == 0 ? c0 : b.pod_ctr_end[q0 + j - 1];
      a_end[h] = b.pod_ctr_end[q0 + j];
      a_w[h] = b.pod_slot[q0 + j];
    }
    const uint32_t a_s = a_w[h] & KACC_SLOT_MASK;
    const bool a_ok = role != 0 && a_s < cap_of(role);
    a_total[h] = 0.0;
    a_delta[h] = 0.0;
    if (a_ok) {
      load_row<Z>(energy_of(role), agg_row(role, a_s), a_prev[h]);
      if (role != 2 && !(a_w[h] & KACC_SLOT_NEW)) a_total[h] = cpu_total_of(role)[a_s];
    } else {
#pragma unroll
      for (int z = 0; z < Z; ++z) a_prev[h][z] = 0;
    }
    if (role != 0 && !a_ok) raise_err(st.err, kErrSlot);
  }

  // ---- B: stage Δ / slot words; ProcessTotalCPUTimeDelta (informer.go:330-333) ------
#pragma unroll
  for (int k = 0; k < kSmallGroups; ++k) {
    const uint32_t r = lane + 64u * k;
    if (r < rows) {
      s_d[r] = d[k];
      if constexpr (kSweepable) s_w[r] = w[k];
    }
  }
  wave_sync();  // s_inv reset and the staged rows visible to every lane
  if (kRowSweep && swept) {  // position -> row | NEW bit << 15 (rows < 512)
#pragma unroll
    for (int k = 0; k < kSmallGroups; ++k) {
      const uint32_t r = lane + 64u * k;
      if (r >= rows) continue;
      const uint32_t sl = w[k] & KACC_SLOT_MASK;
      if (sl - smin < span && sl < st.proc_slots)
        s_inv[sl - smin] = static_cast<uint16_t>(r | ((w[k] & KACC_SLOT_NEW) ? 0x8000u : 0u));
      else
        raise_err(st.err, kErrSlot);
    }
  }
  if (kSweepable && swept) {
#pragma unroll
    for (int k = 0; k < kSmallGroups; ++k) {
      const uint32_t r = lane + 64u * k;
      if (r >= rows) continue;
      const uint32_t sl = s_w[r] & KACC_SLOT_MASK;
      if (sl - smin < span && sl < st.proc_slots)
        s_inv[sl - smin] = static_cast<uint16_t>(r);
      else
        raise_err(st.err, kErrSlot);
    }
  }
  if (b.flags & KACC_F_NODE_CPU_DELTA_GIVEN) {
    if (lane == 0) sh.node_delta = b.node_cpu_delta[n];
  } else {
    // the 256 tree leaves of interval_kernel: leaf l sums rows l, l+256 in order;
    // lane t holds leaves t, t+64, t+128, t+192; then red[l] + red[l+128],
    // red[t] + red[t+64] and the shuffle tree, exactly as there
    double leaf[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t r0 = lane + 64u * q, r1 = r0 + kTree;  // both < kSmallRows: in bounds
      const double v0 = s_d[r0], v1 = s_d[r1];
      double s = 0.0;
      s = s + (r0 < rows ? v0 : 0.0);  // +0.0 past the node's end: an identity
      s = s + (r1 < rows ? v1 : 0.0);
      leaf[q] = s;
    }
    const double t0 = leaf[0] + leaf[2];
    const double t1 = leaf[1] + leaf[3];
    double x = t0 + t1;
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) x = x + __shfl_down(x, k, 64);
    if (lane == 0) sh.node_delta = x;
  }

  // ---- C: containers and VMs ---------------------------------------------------------
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t i = lane + 64u * h, role = role_of(i), j = index_of(i);
    if (role != 1 && role != 2) continue;
    const uint32_t a_s = a_w[h] & KACC_SLOT_MASK;
    const bool a_ok = a_s < cap_of(role);
    uint32_t beg = a_beg[h], end = a_end[h];
    if (beg < p0 || end < beg || end > p1) {
      raise_err(st.err, kErrOffsets);
      beg = max(min(beg, p1), p0);
      end = max(min(end, p1), beg);
    }
    double ad = 0.0;
    if (role == 1) {  // informer.go:229-233, 481-486
      double at = a_total[h];
      segment_sum<4>(s_d, beg - p0, end - p0, ad, at);
      a_total[h] = at;
      s_cd[j] = a_ok ? ad : 0.0;
      s_ct[j] = a_ok ? at : 0.0;
    } else {  // informer.go:445: the last process in listing order wins
      ad = end > beg ? s_d[end - 1 - p0] : 0.0;
    }
    a_delta[h] = ad;
    if (a_ok) {
      cpu_delta_of(role)[a_s] = ad;
      if (role == 1) cpu_total_of(role)[a_s] = a_total[h];
    }
  }
  wave_sync();

  // ---- D: pods (informer.go:305-309, 502-507) ---------------------------------------
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t i = lane + 64u * h;
    if (role_of(i) != 3) continue;
    const uint32_t a_s = a_w[h] & KACC_SLOT_MASK;
    uint32_t beg = a_beg[h], end = a_end[h];
    if (beg < c0 || end < beg || end > c1) {
      raise_err(st.err, kErrOffsets);
      beg = max(min(beg, c1), c0);
      end = max(min(end, c1), beg);
    }
    double ad = 0.0, at = a_total[h];
    for (uint32_t c = beg - c0; c < end - c0; ++c) {
      ad = ad + s_cd[c];
      at = at + s_ct[c];  // quirk: the container's running total
    }
    a_delta[h] = ad;
    a_total[h] = at;
    if (a_s < st.pod_slots) {
      st.pod_cpu_delta[a_s] = ad;
      st.pod_cpu_total[a_s] = at;
    }
  }

  // ---- E: attribution ------------------------------------------------------------------
  const Attr<Z> a = make_attr<Z>(sh, KACC_SMALL_STABLE ? b.flags : (b.flags & ~KACC_F_STABLE_SLOT_NODES));
  if (lane == 0) {
    st.node_ts[n] = b.node_ts_ns[n];
    st.node_has_prev[n] = 1u;
    st.node_usage_ratio[n] = a.first ? 0.0 : b.node_usage_ratio[n];
    st.node_cpu_delta[n] = a.nd;
    st.node_status[n] = a.first ? KACC_NODE_FIRST_READ : KACC_NODE_OK;
  }
  // aggregate rows: stored after the process rows when KACC_SMALL_LATE_AGG (as
  // interval_kernel's KACC_LATE_AGG: early rows sit dirty in L2 through the stream)
  auto aggregate_out = [&]() {
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // container.go:106-140 / vm.go:78-109 / pod.go:87-118
      const uint32_t i = lane + 64u * h, role = role_of(i);
      const uint32_t a_s = a_w[h] & KACC_SLOT_MASK;
      if (role == 0) continue;
      if (a_s >= cap_of(role)) {
        if (role == 3) export_pod_zero<Z>(b, q0 + index_of(i), st.err);
        continue;
      }
      uint64_t E[Z];
      double P[Z];
      const double ratio = attribute_row<Z>(a, role == 3 ? a.live_pod : a.live, a_delta[h],
                                            (a_w[h] & KACC_SLOT_NEW) != 0, a_prev[h], E, P);
      store_agg<Z, kNT && kNtAggStores>(st, role, a_s, E, P, ratio, n);
      if (role == 3) export_pod<Z>(b, q0 + index_of(i), E, P, st.err);
    }
  };
  if constexpr (KACC_SMALL_LATE_AGG == 0) aggregate_out();
  auto attr_batch = [&](int kb) {  // process.go:118-148
#pragma unroll
    for (int g = 0; g < kSmallBatch; ++g) {
      const uint32_t pos0 = 64u * (kb * kSmallBatch + g);
      if constexpr (kRowSweep) {
        if (swept) {  // slot smin + pos: row s_inv[pos] (0xffff: a free slot)
          const uint32_t pos = pos0 + lane;
          if (pos >= span) continue;
          const uint32_t e = s_inv[pos];
          if (e == 0xffffu) continue;
          uint64_t E[Z];
          const double ratio = attribute_proc<Z>(a, s_d[e & 0x7fffu], (e & 0x8000u) != 0, prev[g], E);
          store_proc<Z, kNT>(st, static_cast<uint64_t>(smin) + pos, E, ratio, n, !a.keep_node || (e & 0x8000u));
          continue;
        }
      }
      if constexpr (kSweepable) {
        if (swept) {
          const uint32_t len = pos0 < span ? min(span - pos0, 64u) : 0u;
          attribute_group_masked<Z, kNT, true>(a, sh, s_d, s_w, s_inv, pos0, static_cast<uint64_t>(smin) + pos0,
                                               len, prev[g], st.proc_energy, st.proc_ratio, st.proc_node, n);
          continue;
        }
        if (contig & (1u << g)) {
          attribute_group_masked<Z, kNT, false>(a, sh, s_d, s_w, s_inv, pos0,
                                                uniform_u32(s_w[pos0] & KACC_SLOT_MASK), 64u, prev[g],
                                                st.proc_energy, st.proc_ratio, st.proc_node, n);
          continue;
        }
      }
      const uint32_t r = pos0 + lane;
      if (r >= rows) continue;
      uint32_t wk;
      if constexpr (kSweepable)
        wk = s_w[r];
      else
        wk = kb == 0 ? w[g] : w[kSmallBatch + g];  // this lane's own row
      const uint64_t sl = wk & KACC_SLOT_MASK;
      if (sl >= st.proc_slots) {
        raise_err(st.err, kErrSlot);
        continue;
      }
      uint64_t E[Z];
      const double ratio = attribute_proc<Z>(a, s_d[r], (wk & KACC_SLOT_NEW) != 0, prev[g], E);
      store_proc<Z, kNT && kNtScatterStores>(st, sl, E, ratio, n, !a.keep_node || (wk & KACC_SLOT_NEW));
    }
  };
  attr_batch(0);
  const uint32_t extent = swept ? span : rows;  // wave-uniform
  if (extent > 64u * kSmallBatch) {
    load_batch(1, false);
    attr_batch(1);
  }
  if constexpr (KACC_SMALL_LATE_AGG != 0) aggregate_out();
}

// ======================= big nodes: chunked row passes ==========================
// A node that does not fit one fast workgroup (> kRowsLds rows or > kTpb
// aggregates, e.g. BASELINE config 5's 10-50k-process nodes) is cut into
// kChunkRows-row chunks so that no single node bounds the launch:
//   interval_kernel  node zones, the canonical node CPU total and the node
//                    scalars (big_node_prepare), then one ChunkItem per chunk
//                    naming the first container / VM / pod the chunk owns.  A
//                    container or VM belongs to the chunk holding its first
//                    row, a pod to the chunk owning its first container;
//   chunk_kernel     per chunk, the fast path's phases C-E on the chunk: the
//                    process rows, the owned containers / VMs (sequential sums;
//                    rows past the chunk come from global memory) and the owned
//                    pods whose containers all lie in the chunk (LDS sums).  A
//                    pod reaching past its chunk goes on the deferred list;
//   pod_kernel       the deferred pods, one lane each, from the container
//                    sums chunk_kernel stored (the kernel boundary makes them
//                    visible across XCDs: no cross-workgroup wait anywhere).
// Every sum keeps its sequential / canonical-tree order, so results are
// bit-identical to one workgroup handling the whole node.
// Chunk items of big node n (see big_node_prepare): items [base, base + nch)
// with the first container / VM / pod each chunk owns.  A segment belongs to
// the chunk holding its first row (rows are [containers][VMs][rest]); a pod to
// the chunk owning its first container.  Segment i is the first one owned by
// chunks (key(i-1), key(i)].  Lanes g < kGen of the caller generate.
template <int V, uint32_t kGen>
__device__ __forceinline__ void gen_items(const kacc_interval &b, const DevState &st, uint32_t n,
                                          const NodeRanges &rg, uint32_t base, uint32_t nch, uint32_t g) {
  constexpr int kScan = 4;  // segments per generating lane per step
  const uint32_t p0 = rg.p0, p1 = rg.p1;
  ChunkItem *__restrict__ items = st.items + base;
  const uint32_t c0 = rg.c0, c1 = rg.c1, v0 = rg.v0, v1 = rg.v1, q0 = rg.q0, q1 = rg.q1;
  auto clampr = [&](uint32_t x) { return min(max(x, p0), p1); };
  auto clampc = [&](uint32_t x) { return min(max(x, c0), c1); };
  auto chunk_of = [&](uint32_t start) -> int {
    return static_cast<int>(min((start - p0) / kChunkRows, nch - 1));
  };
  // first row of container c given ctr_proc_end[c - 1] (p0 for c0)
  const uint32_t ctr_rows_end = c1 > c0 ? clampr(b.ctr_proc_end[c1 - 1]) : p0;
  // segment i (owner chunk kc, its predecessor's kp) begins chunks kp+1..kc
  auto mark = [&](uint32_t i, int kc, int kp, uint32_t ChunkItem::*field) {
    if (kc < kp) raise_err(st.err, kErrOffsets);
    for (int k = kp + 1; k <= kc; ++k) items[k].*field = i;
  };
  // containers: start(c) = c == c0 ? p0 : end[c-1]
  for (uint32_t cb = c0 + g; cb < ((V & kVarBigNoScan) ? c0 : c1); cb += kGen * kScan) {
    uint32_t e1[kScan], e2[kScan];
#pragma unroll
    for (int u = 0; u < kScan; ++u) {
      const uint32_t c = cb + u * kGen;
      e1[u] = (c < c1 && c > c0) ? b.ctr_proc_end[c - 1] : p0;
      e2[u] = (c < c1 && c > c0 + 1) ? b.ctr_proc_end[c - 2] : p0;
    }
#pragma unroll
    for (int u = 0; u < kScan; ++u) {
      const uint32_t c = cb + u * kGen;
      if (c >= c1) continue;
      mark(c, chunk_of(clampr(e1[u])), c > c0 ? chunk_of(clampr(e2[u])) : -1,
           &ChunkItem::ctr_begin);
    }
  }
  // VMs: start(v) = v == v0 ? ctr_rows_end : vm_end[v-1]
  for (uint32_t vb = v0 + g; vb < ((V & kVarBigNoScan) ? v0 : v1); vb += kGen * kScan) {
    uint32_t e1[kScan], e2[kScan];
#pragma unroll
    for (int u = 0; u < kScan; ++u) {
      const uint32_t v = vb + u * kGen;
      e1[u] = (v < v1 && v > v0) ? b.vm_proc_end[v - 1] : ctr_rows_end;
      e2[u] = (v < v1 && v > v0 + 1) ? b.vm_proc_end[v - 2] : ctr_rows_end;
    }
#pragma unroll
    for (int u = 0; u < kScan; ++u) {
      const uint32_t v = vb + u * kGen;
      if (v >= v1) continue;
      mark(v, chunk_of(clampr(e1[u])), v > v0 ? chunk_of(clampr(e2[u])) : -1,
           &ChunkItem::vm_begin);
    }
  }
  // pods: first container f(q) = q == q0 ? c0 : pod_end[q-1]; key = key of
  // container f(q), or the last chunk when the pod starts past the containers
  if constexpr ((V & (kVarSkipAggregates | kVarBigNoScan)) == 0) {
    for (uint32_t qb = q0 + g; qb < q1; qb += kGen * kScan) {
      uint32_t f1[kScan], f2[kScan], s1[kScan], s2[kScan];
#pragma unroll
      for (int u = 0; u < kScan; ++u) {
        const uint32_t q = qb + u * kGen;
        f1[u] = (q < q1 && q > q0) ? clampc(b.pod_ctr_end[q - 1]) : c0;
        f2[u] = (q < q1 && q > q0 + 1) ? clampc(b.pod_ctr_end[q - 2]) : c0;
      }
#pragma unroll
      for (int u = 0; u < kScan; ++u) {
        s1[u] = (f1[u] > c0 && f1[u] < c1) ? b.ctr_proc_end[f1[u] - 1] : p0;
        s2[u] = (f2[u] > c0 && f2[u] < c1) ? b.ctr_proc_end[f2[u] - 1] : p0;
      }
#pragma unroll
      for (int u = 0; u < kScan; ++u) {
        const uint32_t q = qb + u * kGen;
        if (q >= q1) continue;
        const int kc = f1[u] < c1 ? chunk_of(clampr(s1[u])) : static_cast<int>(nch - 1);
        const int kp = q == q0 ? -1 : f2[u] < c1 ? chunk_of(clampr(s2[u])) : static_cast<int>(nch - 1);
        mark(q, kc, kp, &ChunkItem::pod_begin);
      }
    }
  }
  // chunks after the last segment's owner own none of that kind
  const int kl_ctr = c1 > c0 ? chunk_of(c1 - 1 > c0 ? clampr(b.ctr_proc_end[c1 - 2]) : p0) : -1;
  const int kl_vm = v1 > v0 ? chunk_of(v1 - 1 > v0 ? clampr(b.vm_proc_end[v1 - 2]) : ctr_rows_end) : -1;
  int kl_pod = -1;
  if (q1 > q0) {
    const uint32_t f = q1 - 1 > q0 ? clampc(b.pod_ctr_end[q1 - 2]) : c0;
    kl_pod = f < c1 ? chunk_of(f > c0 ? clampr(b.ctr_proc_end[f - 1]) : p0) : static_cast<int>(nch - 1);
  }
  for (uint32_t k = g; k < nch; k += kGen) {
    items[k].node = n;
    items[k].chunk = k;
    items[k].nchunks = nch;
    if (static_cast<int>(k) > kl_ctr) items[k].ctr_begin = c1;
    if (static_cast<int>(k) > kl_vm) items[k].vm_begin = v1;
    if (static_cast<int>(k) > kl_pod) items[k].pod_begin = q1;
  }
}

template <int Z, int V>
__device__ void big_node_prepare(const kacc_interval &b, const DevState &st, const uint32_t n,
                                 const NodeRanges &rg, double *red, NodeShared &sh,
                                 uint32_t &s_base) {
  constexpr int kThreads = kTpb<V>;
  constexpr uint32_t kGen = kThreads - kTree;  // lanes generating chunk items
  const int tid = threadIdx.x;
  const uint32_t p0 = rg.p0, p1 = rg.p1, rows = p1 - p0;
  const uint32_t nch = rows ? (rows + kChunkRows - 1) / kChunkRows : 1u;
  if (tid == 0 && !st.items_given)
    s_base = (V & kVarBigNoAtomic) ? n + p0 / kChunkRows : atomicAdd(st.item_ctr, nch);
  if (tid < Z) node_zone<Z>(b, st, n, tid, sh);
  __syncthreads();
  const uint32_t base = st.items_given ? 0u : s_base;
  const bool fits = st.items_given || (base + nch <= st.item_cap && base + nch >= base);  // host sizes the list
  if (!fits && tid == 0) raise_err(st.err, kErrCapacity);
  const bool given = (b.flags & KACC_F_NODE_CPU_DELTA_GIVEN) != 0;
  if (tid < kTree) {
    // ---- B: ProcessTotalCPUTimeDelta; lane l sums rows l, l+256, ... ---------
    // software-pipelined: the next kTotLoads rows are in flight while the
    // current ones are added (latency, not bandwidth, bounds one node's sum)
    if (!given && (V & kVarBigNoTotal) == 0) {
      const double *__restrict__ dcpu = b.proc_cpu_delta + p0;
      double s = 0.0;
      double v[kTotLoads];
#pragma unroll
      for (int k = 0; k < kTotLoads; ++k) {
        const uint32_t i = tid + k * kTree;
        v[k] = i < rows ? dcpu[i] : 0.0;
      }
      for (uint32_t r0 = 0; r0 < rows; r0 += kTree * kTotLoads) {
        double nx[kTotLoads];
#pragma unroll
        for (int k = 0; k < kTotLoads; ++k) {
          const uint32_t i = r0 + kTree * kTotLoads + tid + k * kTree;
          nx[k] = i < rows ? dcpu[i] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < kTotLoads; ++k)
          if (r0 + tid + k * kTree < rows) s = s + v[k];
#pragma unroll
        for (int k = 0; k < kTotLoads; ++k) v[k] = nx[k];
      }
      red[tid] = s;
    }
  } else if (fits && !st.items_given) {
    // ---- chunk items, concurrently with the sum (the other kGen lanes) --------
    gen_items<V, kGen>(b, st, n, rg, base, nch, static_cast<uint32_t>(tid) - kTree);
  }
  __syncthreads();
  if (given) {
    if (tid == 0) sh.node_delta = b.node_cpu_delta[n];
  } else {
    if (tid < 128) red[tid] = red[tid] + red[tid + 128];
    __syncthreads();
    if (tid < 64) {
      double x = red[tid] + red[tid + 64];
#pragma unroll
      for (int k = 32; k >= 1; k >>= 1) x = x + __shfl_down(x, k, 64);
      if (tid == 0) sh.node_delta = x;
    }
  }
  __syncthreads();
  if (tid == 0) {  // node scalars of the new snapshot (as the fast path)
    const bool first = sh.first != 0;
    st.node_ts[n] = b.node_ts_ns[n];
    st.node_has_prev[n] = 1u;
    st.node_usage_ratio[n] = first ? 0.0 : b.node_usage_ratio[n];
    st.node_cpu_delta[n] = sh.node_delta;
    st.node_status[n] = first ? KACC_NODE_FIRST_READ : KACC_NODE_OK;
  }
}

// The chunk items of every big node of a layout, once for all the intervals of a
// kacc_run_intervals call over that layout (every descriptor the same offset
// arrays): one workgroup per node, all lanes generating.  Items exist for
// every big node whatever its status; chunk_kernel skips the items of a node
// that is skipped in its interval.
template <int V>
__global__ __launch_bounds__(kTpb<V>) void items_kernel(const kacc_interval b, const DevState st) {
  constexpr int kThreads = kTpb<V>;
  __shared__ uint32_t s_base;
  const uint32_t n = blockIdx.x;
  if (n >= b.n_nodes) return;
  uint32_t status_unused;
  NodeRanges raw;
  node_words(b, n, status_unused, raw);
  const NodeRanges rg = clamp_ranges(b, st, raw, threadIdx.x);
  if (fits_fast<V>(rg)) return;  // block-uniform: the fast path takes this node
  const uint32_t rows = rg.p1 - rg.p0;
  const uint32_t nch = rows ? (rows + kChunkRows - 1) / kChunkRows : 1u;
  if (threadIdx.x == 0) s_base = atomicAdd(st.item_ctr, nch);
  __syncthreads();
  const uint32_t base = s_base;
  if (base + nch > st.item_cap || base + nch < base) {
    if (threadIdx.x == 0) raise_err(st.err, kErrCapacity);
    return;
  }
  gen_items<V, kThreads>(b, st, n, rg, base, nch, threadIdx.x);
}

// Node-uniform attribution parameters written by the node phase, back into LDS.
template <int Z>
__device__ __forceinline__ void node_params_to_lds(const DevState &st, uint32_t n, int tid,
                                                   NodeShared &sh) {
  if (tid < Z) {
    const uint64_t i = static_cast<uint64_t>(n) * Z + tid;
    sh.active_energy[tid] = st.node_active_energy[i];
    sh.active_power[tid] = st.node_active_power[i];
    sh.power[tid] = st.node_power[i];
  }
  if (tid == 0) {
    sh.node_delta = st.node_cpu_delta[n];
    sh.first = st.node_status[n] == KACC_NODE_FIRST_READ ? 1u : 0u;
  }
}

template <int Z, int V>
__global__ __launch_bounds__(kChunkThreads, (Z > 4 ? 2 : KACC_CHUNK_WAVES)) void chunk_kernel(const kacc_interval b,
                                                                           const DevState st) {
  constexpr int kThreads = kChunkThreads;
  constexpr int kR = kChunkRpt;
  // non-temporal hints on the row streams (read once / written once per
  // interval, 2.5 GB at config 3: nothing to keep in L2 or the Infinity
  // Cache): loads + stores together measured 5 % faster (profiles/r01/ablations)
  constexpr bool kNT = (V & kVarTemporalStores) == 0;
  constexpr bool kNtLd = (V & kVarTemporalLoads) == 0;
  constexpr bool kT = kTransposed<Z> && (V & kVarNoTranspose) == 0;
  constexpr bool kAgg = (V & kVarSkipAggregates) == 0;
  __shared__ double s_d[kChunkRows];
  __shared__ uint32_t s_w[kChunkRows];
  __shared__ double s_cd[kThreads];  // owned containers' Δ (first kThreads of them)
  __shared__ double s_ct[kThreads];  // and running CPU totals
  __shared__ NodeShared sh;
  __shared__ uint32_t s_next[2];
  const int tid = threadIdx.x;
  const uint32_t utid = static_cast<uint32_t>(tid);
  const uint32_t count =
      min(__hip_atomic_load(st.item_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), st.item_cap);
  uint32_t idx = blockIdx.x;  // first item static, the rest dequeued
  for (uint32_t parity = 0; idx < count; parity ^= 1u) {
    if (tid == 0) s_next[parity] = atomicAdd(st.item_ctr + 1, 1u) + gridDim.x;
    // the item's words and its successor's begins as ONE batch of vector loads
    // (waited for once), then the node's ranges as another: as scalar loads
    // behind the `last` selects they took nine dependent round trips per chunk
    uint32_t f[9];
    {
      uint32_t ii = idx;
      asm volatile("" : "+v"(ii));
      const uint32_t *w0 = reinterpret_cast<const uint32_t *>(st.items + ii);
      const uint32_t *w1 = reinterpret_cast<const uint32_t *>(st.items + min(ii + 1, st.item_cap - 1));
      f[0] = w0[0];
      f[1] = w0[1];
      f[2] = w0[2];
      f[3] = w0[3];
      f[4] = w0[4];
      f[5] = w0[5];
      f[6] = w1[3];
      f[7] = w1[4];
      f[8] = w1[5];
      asm volatile("" ::"v"(f[0]), "v"(f[1]), "v"(f[2]), "v"(f[3]), "v"(f[4]), "v"(f[5]), "v"(f[6]), "v"(f[7]),
                   "v"(f[8]));
#pragma unroll
      for (int q = 0; q < 9; ++q) f[q] = uniform_u32(f[q]);
    }
    const uint32_t n = f[0], k = f[1], nch = f[2];
    if (n >= b.n_nodes) {  // corrupt item: cannot happen unless the list overflowed
      if (tid == 0) raise_err(st.err, kErrCapacity);
      __syncthreads();
      idx = uniform_u32(s_next[parity]);
      continue;
    }
    uint32_t status;
    NodeRanges raw;
    node_words(b, n, status, raw);
    if (status & KACC_NODE_READ_ERROR) {  // reused items (items_given) of a node skipped now
      __syncthreads();
      idx = uniform_u32(s_next[parity]);
      continue;
    }
    const NodeRanges rg = clamp_ranges(b, st, raw, tid);
    const bool last = k + 1 >= nch;
    const uint32_t lo = min(rg.p0 + min(k, nch) * static_cast<uint32_t>(kChunkRows), rg.p1);
    const uint32_t hi = last ? rg.p1 : min(lo + static_cast<uint32_t>(kChunkRows), rg.p1);
    const uint32_t rows = hi - lo;
    const uint32_t cb = min(max(f[3], rg.c0), rg.c1);
    const uint32_t ce = max(min(last ? rg.c1 : f[6], rg.c1), cb);
    const uint32_t vb = min(max(f[4], rg.v0), rg.v1);
    const uint32_t ve = max(min(last ? rg.v1 : f[7], rg.v1), vb);
    const uint32_t qb = min(max(f[5], rg.q0), rg.q1);
    const uint32_t qe = max(min(last ? rg.q1 : f[8], rg.q1), qb);
    const uint32_t nca = kAgg ? ce - cb : 0u;
    const uint32_t ncv = kAgg ? nca + (ve - vb) : 0u;  // containers + VMs
    const uint32_t nagg = kAgg ? ncv + (qe - qb) : 0u;  // + pods

    // ---- loads: rows, their previous totals, one owned aggregate per lane -----
    const double *__restrict__ dcpu = b.proc_cpu_delta + lo;
    const uint32_t *__restrict__ pslot = b.proc_slot + lo;
    double d[kR];
    uint32_t w[kR];
#pragma unroll
    for (int u = 0; u < kR; ++u) {
      const uint32_t r = utid + u * kThreads;
      const bool in = r < rows;
      d[u] = in ? (kNtLd ? __builtin_nontemporal_load(dcpu + r) : dcpu[r]) : 0.0;
      w[u] = in ? (kNtLd ? __builtin_nontemporal_load(pslot + r) : pslot[r]) : 0xffffffffu;
    }
    uint64_t prev[kR][Z];
    uint32_t contig = 0;
    if constexpr ((V & kVarSkipProcs) == 0) {
#pragma unroll
      for (int u = 0; u < kR; ++u) {
        const uint64_t sl = w[u] & KACC_SLOT_MASK;
        if constexpr (kT) {
          const uint64_t s0 = uniform_u32(static_cast<uint32_t>(sl));
          const bool mine = (utid + u * kThreads) < rows && sl == s0 + (tid & 63) &&
                            s0 + 64 <= st.proc_slots;
          if (__all(mine)) {
            contig |= 1u << u;
            load_group_masked<Z, false, kNtLd>(st.proc_energy, s0, 64u, s0, prev[u]);
            continue;
          }
        }
        if (sl < st.proc_slots) {
          load_row<Z>(st.proc_energy, sl, prev[u]);
        } else {
#pragma unroll
          for (int z = 0; z < Z; ++z) prev[u][z] = 0;
        }
      }
    }
    // aggregate j of this chunk: containers [cb, ce), VMs [vb, ve), pods [qb, qe)
    const uint32_t ctr_rows_end = rg.c1 > rg.c0 ? b.ctr_proc_end[rg.c1 - 1] : rg.p0;
    auto agg = [&](uint32_t j, uint32_t &beg, uint32_t &end, uint32_t &wd) -> uint32_t {
      if (j < nca) {
        const uint32_t c = cb + j;
        beg = c == rg.c0 ? rg.p0 : b.ctr_proc_end[c - 1];
        end = b.ctr_proc_end[c];
        wd = b.ctr_slot[c];
        return 1u;
      }
      if (j < ncv) {
        const uint32_t v = vb + (j - nca);
        beg = v == rg.v0 ? ctr_rows_end : b.vm_proc_end[v - 1];
        end = b.vm_proc_end[v];
        wd = b.vm_slot[v];
        return 2u;
      }
      const uint32_t q = qb + (j - ncv);
      beg = q == rg.q0 ? rg.c0 : b.pod_ctr_end[q - 1];
      end = b.pod_ctr_end[q];
      wd = b.pod_slot[q];
      return 3u;
    };
    auto cap_of = [&](uint32_t role) {
      return role == 1 ? st.ctr_slots : role == 2 ? st.vm_slots : st.pod_slots;
    };
    auto energy_of = [&](uint32_t role) {
      return role == 1 ? st.ctr_energy : role == 2 ? st.vm_energy : st.pod_energy;
    };
    uint32_t a_role = 0, a_beg = 0, a_end = 0, a_w = 0xffffffffu;
    if (utid < nagg) a_role = agg(utid, a_beg, a_end, a_w);
    const uint32_t a_s = a_w & KACC_SLOT_MASK;
    const bool a_ok = a_role != 0 && a_s < cap_of(a_role);
    uint64_t a_prev[Z];
    double a_total = 0.0;
    if (a_ok) {
      load_row<Z>(energy_of(a_role), agg_row(a_role, a_s), a_prev);
      if (a_role != 2 && !(a_w & KACC_SLOT_NEW))
        a_total = (a_role == 1 ? st.ctr_cpu_total : st.pod_cpu_total)[a_s];
    } else {
#pragma unroll
      for (int z = 0; z < Z; ++z) a_prev[z] = 0;
    }
    if (a_role != 0 && !a_ok) raise_err(st.err, kErrSlot);
    node_params_to_lds<Z>(st, n, tid, sh);
#pragma unroll
    for (int u = 0; u < kR; ++u) {
      const uint32_t r = utid + u * kThreads;
      if (r < rows) {
        s_d[r] = d[u];
        s_w[r] = w[u];
      }
    }
    __syncthreads();
    const Attr<Z> a = make_attr<Z>(sh, b.flags);

    auto agg_out = [&](uint32_t role, uint32_t wd, double delta, const uint64_t (&pv)[Z]) {
      const uint64_t s = wd & KACC_SLOT_MASK;
      uint64_t E[Z];
      double P[Z];
      const double ratio =
          attribute_row<Z>(a, role == 3 ? a.live_pod : a.live, delta, (wd & KACC_SLOT_NEW) != 0, pv, E, P);
      store_agg<Z, kNT>(st, role, s, E, P, ratio, n);
    };
    // ---- C: owned containers / VMs (informer.go:223-273) ------------------------
    auto segment = [&](uint32_t role, uint32_t beg, uint32_t end, uint32_t wd, bool ok,
                       double &total) -> double {
      if (beg < rg.p0 || end < beg || end > rg.p1) {
        raise_err(st.err, kErrOffsets);
        beg = max(min(beg, rg.p1), rg.p0);
        end = max(min(end, rg.p1), beg);
      }
      auto delta_at = [&](uint32_t i) -> double {
        return (i >= lo && i < hi) ? s_d[i - lo] : b.proc_cpu_delta[i];
      };
      double delta = 0.0;
      if (role == 1) {
        for (uint32_t i = beg; i < end; ++i) {
          const double di = delta_at(i);
          delta = delta + di;
          total = total + di;
        }
      } else {
        delta = end > beg ? delta_at(end - 1) : 0.0;  // informer.go:445, last one wins
      }
      if (ok) {
        const uint64_t s = wd & KACC_SLOT_MASK;
        if (role == 1) {
          st.ctr_cpu_delta[s] = delta;
          st.ctr_cpu_total[s] = total;
        } else {
          st.vm_cpu_delta[s] = delta;
        }
      }
      return delta;
    };
    double a_delta = 0.0;
    if (a_role == 1 || a_role == 2) {
      a_delta = segment(a_role, a_beg, a_end, a_w, a_ok, a_total);
      if (a_role == 1) {
        s_cd[utid] = a_ok ? a_delta : 0.0;
        s_ct[utid] = a_ok ? a_total : 0.0;
      }
    }
    __syncthreads();
    // ---- D: owned pods whose containers are all in s_cd / s_ct ---------------
    bool defer = false;
    if (a_role == 3) {
      uint32_t beg = a_beg, end = a_end;
      if (beg < rg.c0 || end < beg || end > rg.c1) {
        raise_err(st.err, kErrOffsets);
        beg = max(min(beg, rg.c1), rg.c0);
        end = max(min(end, rg.c1), beg);
      }
      if (end <= ce && end - cb <= static_cast<uint32_t>(kThreads) && beg >= cb) {
        for (uint32_t c = beg - cb; c < end - cb; ++c) {
          a_delta = a_delta + s_cd[c];
          a_total = a_total + s_ct[c];  // quirk: the container's running total
        }
        if (a_ok) {
          st.pod_cpu_delta[a_s] = a_delta;
          st.pod_cpu_total[a_s] = a_total;
        }
      } else {
        defer = true;  // pod_kernel, after every chunk's containers are stored
      }
    }
    // ---- E: aggregates, then process rows (process.go:118-148) ------------------
    if (a_ok && !defer) {
      const uint64_t s = a_w & KACC_SLOT_MASK;
      uint64_t E[Z];
      double P[Z];
      const double ratio =
          attribute_row<Z>(a, a_role == 3 ? a.live_pod : a.live, a_delta, (a_w & KACC_SLOT_NEW) != 0, a_prev, E, P);
      store_agg<Z, kNT>(st, a_role, s, E, P, ratio, n);
      if (a_role == 3) export_pod<Z>(b, qb + (utid - ncv), E, P, st.err);
    } else if (a_role == 3 && !a_ok) {
      export_pod_zero<Z>(b, qb + (utid - ncv), st.err);
    }
    if (defer && a_ok) {
      const uint32_t i = atomicAdd(st.defer_ctr, 1u);
      if (i < st.defer_cap)
        st.defer[i] = make_uint2(n, qb + (utid - ncv));
      else
        raise_err(st.err, kErrCapacity);
    }
    if constexpr ((V & kVarSkipProcs) == 0) {
#pragma unroll
      for (int u = 0; u < kR; ++u) {
        const uint32_t r = utid + u * kThreads;
        if constexpr (kT) {
          if (contig & (1u << u)) {
            const uint32_t g = r - (tid & 63);
            attribute_group_masked<Z, kNT, false>(a, sh, s_d, s_w, nullptr, g,
                                           uniform_u32(s_w[g] & KACC_SLOT_MASK), 64u, prev[u],
                                           st.proc_energy, st.proc_ratio, st.proc_node, n);
            continue;
          }
        }
        if (r >= rows) continue;
        const uint32_t wk = s_w[r];
        const uint64_t sl = wk & KACC_SLOT_MASK;
        if (sl >= st.proc_slots) {
          raise_err(st.err, kErrSlot);
          continue;
        }
        uint64_t E[Z];
        const double ratio = attribute_proc<Z>(a, s_d[r], (wk & KACC_SLOT_NEW) != 0, prev[u], E);
        store_proc<Z, kNT && kNtScatterStores>(st, sl, E, ratio, n, !a.keep_node || (wk & KACC_SLOT_NEW));
      }
    }
    // aggregates beyond one per lane (chunks of mostly empty containers):
    // containers / VMs here, their pods always deferred
    for (uint32_t j = kThreads + utid; j < nagg; j += kThreads) {
      uint32_t beg, end, wd;
      const uint32_t role = agg(j, beg, end, wd);
      const uint64_t s = wd & KACC_SLOT_MASK;
      const bool ok = s < cap_of(role);
      if (!ok) {
        raise_err(st.err, kErrSlot);
        if (role == 3) export_pod_zero<Z>(b, qb + (j - ncv), st.err);
        continue;
      }
      if (role == 3) {
        const uint32_t i = atomicAdd(st.defer_ctr, 1u);
        if (i < st.defer_cap)
          st.defer[i] = make_uint2(n, qb + (j - ncv));
        else
          raise_err(st.err, kErrCapacity);
        continue;
      }
      uint64_t pv[Z];
      load_row<Z>(energy_of(role), agg_row(role, s), pv);
      double total = (role == 1 && !(wd & KACC_SLOT_NEW)) ? st.ctr_cpu_total[s] : 0.0;
      const double delta = segment(role, beg, end, wd, true, total);
      agg_out(role, wd, delta, pv);
    }
    __syncthreads();  // LDS reused by the next item; s_next[parity] written
    idx = uniform_u32(s_next[parity]);
  }
}

// Deferred pods (informer.go:275-326 + pod.go:46-131), one lane each: ΔCPU and
// the running-total quirk summed over the pod's containers in batch order from
// the tables chunk_kernel wrote, then attribution (pod.go:96 guards on Power).
// Also re-arms the chunk list for the next interval (chunk_kernel has ended);
// the deferred list itself is re-armed by the next interval_kernel.
template <int Z, int V>
__global__ __launch_bounds__(kBlock) void pod_kernel(const kacc_interval b, const DevState st) {
  constexpr bool kNT = (V & kVarTemporalStores) == 0;  // as interval_kernel
  const int tid = threadIdx.x;
  if (blockIdx.x == 0 && tid == 0) {
    if (!st.keep_items) st.item_ctr[0] = 0u;  // the list stays for the next interval of one layout
    st.item_ctr[1] = 0u;
  }
  const uint32_t count = min(st.defer_ctr[0], st.defer_cap);
  for (uint32_t i = blockIdx.x * kBlock + tid; i < count; i += gridDim.x * kBlock) {
    const uint2 e = st.defer[i];
    const uint32_t n = e.x, q = e.y;
    if (n >= b.n_nodes || q >= b.n_pods) {
      raise_err(st.err, kErrCapacity);
      continue;
    }
    const NodeRanges rg = node_ranges(b, st, n, 1);
    uint32_t beg = q == rg.q0 ? rg.c0 : b.pod_ctr_end[q - 1];
    uint32_t end = b.pod_ctr_end[q];
    beg = max(min(beg, rg.c1), rg.c0);  // offsets were checked by chunk_kernel
    end = max(min(end, rg.c1), beg);
    const uint32_t w = b.pod_slot[q];
    const uint64_t sl = w & KACC_SLOT_MASK;  // < pod_slots (checked before deferral)
    uint64_t prev[Z];
    load_row<Z>(st.pod_energy, pod_row(sl), prev);
    double total = (w & KACC_SLOT_NEW) ? 0.0 : st.pod_cpu_total[sl];
    double delta = 0.0;
    for (uint32_t c = beg; c < end; ++c) {
      const uint64_t cs = b.ctr_slot[c] & KACC_SLOT_MASK;
      if (cs >= st.ctr_slots) continue;  // contributes 0, as s_cd / s_ct
      delta = delta + st.ctr_cpu_delta[cs];
      total = total + st.ctr_cpu_total[cs];
    }
    st.pod_cpu_delta[sl] = delta;
    st.pod_cpu_total[sl] = total;
    // this lane's node parameters (per lane: deferred pods of many nodes)
    Attr<Z> a;
    a.nd = st.node_cpu_delta[n];
    a.first = st.node_status[n] == KACC_NODE_FIRST_READ ? 1u : 0u;
    a.keep_node = 0;  // pods only
    a.live = 0;
    a.live_pod = 0;
#pragma unroll
    for (int z = 0; z < Z; ++z) {
      const uint64_t iz = static_cast<uint64_t>(n) * Z + z;
      a.aE[z] = st.node_active_energy[iz];
      a.aP[z] = st.node_active_power[iz];
      const double pw = st.node_power[iz];
      const bool ok = a.aE[z] != 0 && a.nd != 0;
      if (ok && a.aP[z] != 0) a.live |= 1u << z;
      if (ok && (a.first ? a.aP[z] : pw) != 0) a.live_pod |= 1u << z;
    }
    uint64_t E[Z];
    double P[Z];
    attribute_row<Z>(a, a.live_pod, delta, (w & KACC_SLOT_NEW) != 0, prev, E, P);
    store_row<Z, kNT, uint64_t>(st.pod_energy, pod_row(sl), E);
    store_row<Z, kNT, double>(st.pod_power, pod_row(sl), P);
    export_pod<Z>(b, q, E, P, st.err);
  }
}

template <int Z, int kW = 2 * Z, bool kSplit = false, bool kIdentity = false>
__global__ __launch_bounds__(kBlock) void cluster_partials_kernel(uint32_t ns_blocks, uint32_t n_ns,
                                                                  const uint32_t *__restrict__ off,
                                                                  const uint32_t *__restrict__ slots,
                                                                  const uint64_t *__restrict__ pe,
                                                                  const double *__restrict__ pp, uint64_t pod_slots,
                                                                  uint64_t *out_e, double *out_p, uint32_t *err,
                                                                  const NodeTotalsArgs na) {
  // the first 5Z x split blocks are the cluster node totals in column mode: block b
  // owns output value b / split (column (b / split) / Z of the five node tables, zone
  // (b / split) % Z) and, split > 1 (kSplit instance), node range b % split, whose
  // partial the column's last-arriving block adds (node_column_block); they come first
  // because their per-lane chain of loads is the longer one (node blocks dispatched
  // last finished last: profiles/r03/tprobe2).  The remaining ns_blocks blocks are the
  // namespace sums.
  const uint32_t nb = gridDim.x - ns_blocks;
  if (blockIdx.x >= nb) {
    namespace_block<Z, kW, kBlock, kIdentity>(blockIdx.x - nb, n_ns, off, slots, pe, pp, pod_slots, out_e, out_p,
                                               err);
    return;
  }
  __shared__ uint64_t s_w[kBlock / 64];
  node_column_block<Z, kSplit>(na, blockIdx.x, s_w);  // column (b / split) / Z, zone (b / split) % Z
}


// Derived powers of elements [first, first + count) ([slot*Z + z]) into out: one lane per
// SLOT (round 6), a wave per 64 consecutive slots — the slots' ratio and node words load
// coalesced (768 B per wave, once per slot instead of once per element), the node's guard
// values from cache, the lane's Z powers through the wave's LDS so that every store is 64
// consecutive elements (512 B, non-temporal).  The arithmetic is process.go:124, 142's,
// one multiply per power.  Per slot: ratio 8 + node 4 in, 8Z out (bench.py scrape_powers).
constexpr int kPowWaves = kBlock / 64;
template <int Z>
__global__ __launch_bounds__(kBlock) void proc_power_kernel(const ProcDerive d, uint64_t first, uint64_t count,
                                                            double *out) {
  __shared__ double s_p[kPowWaves][64 * Z];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint64_t s_first = first / Z, s_last = (first + count - 1) / Z;  // count > 0
  const uint64_t S0 = s_first + (static_cast<uint64_t>(blockIdx.x) * kPowWaves + wv) * 64u;
  if (S0 > s_last) return;  // wave-uniform
  const uint64_t s = min(S0 + lane, s_last);  // (clamped: the loads stay unconditional)
  const uint32_t n = d.node[s];
  const double r = d.ratio[s];
  double *const sp = s_p[wv];
  if (n < d.nodes) {
    const bool busy = d.cpu_delta[n] != 0;
#pragma unroll
    for (int z = 0; z < Z; ++z) {
      const uint64_t k = static_cast<uint64_t>(n) * Z + z;
      const double aP = d.active_power[k];
      sp[lane * Z + z] = (d.active_energy[k] != 0 && busy && aP != 0) ? r * aP : 0.0;
    }
  } else {
#pragma unroll
    for (int z = 0; z < Z; ++z) sp[lane * Z + z] = 0.0;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint64_t e0 = S0 * Z, end = first + count;
#pragma unroll
  for (int z = 0; z < Z; ++z) {
    const uint64_t e = e0 + static_cast<uint64_t>(z) * 64u + lane;
    if (e >= first && e < end) __builtin_nontemporal_store(sp[z * 64 + lane], out + (e - first));
  }
}

// Elements [first, first + count) of a pod table (logical [slot*Z + z]) to / from
// a dense array: base is the table's first element inside the [Sq][2Z] records.
__global__ __launch_bounds__(kBlock) void pod_pair_copy_kernel(uint64_t *base, uint32_t Z, uint64_t first,
                                                               uint64_t count, uint64_t *dense, int to_table) {
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; i < count;
       i += static_cast<uint64_t>(gridDim.x) * kBlock) {
    const uint64_t e = first + i;
    uint64_t *p = base + (e / Z) * (2ull * Z) + e % Z;
    if (to_table)
      *p = dense[i];
    else
      dense[i] = *p;
  }
}

}  // namespace kacc

// =============================================================================
// C ABI
// =============================================================================
namespace {

// Errors of calls without a context (kacc_create, kacc_create_multi, ...):
// process-wide, not thread-local — a cgo caller's next C call may run on
// another OS thread (goroutines migrate).  kacc_last_error_copy() reads it
// under the lock.
std::mutex g_err_mu;
std::string g_create_error;

struct TableDesc {
  uint32_t elem;   // bytes
  int per;         // 0 = per node, 1 = per proc slot, 2 ctr, 3 vm, 4 pod
  bool zoned;      // × Z
  bool derived;    // no storage: computed on read (KACC_T_PROC_POWER, kacc_derive.hpp)
};

const TableDesc kTables[KACC_T_COUNT] = {
    {8, 0, true, false},  {8, 0, true, false},  {8, 0, true, false},  {8, 0, true, false},
    {8, 0, true, false},  {8, 0, true, false},  {8, 0, true, false},  {8, 0, false, false},
    {4, 0, false, false}, {8, 0, false, false}, {8, 0, false, false}, {4, 0, false, false},
    {8, 1, true, false},  {8, 1, true, true},   {8, 2, true, false},  {8, 2, true, true},
    {8, 2, false, false}, {8, 2, false, false}, {8, 3, true, false},  {8, 3, true, true},
    {8, 3, false, false}, {8, 4, true, false},  {8, 4, true, false},  {8, 4, false, false},
    {8, 4, false, false}, {8, 1, false, false}, {4, 1, false, false}, {8, 2, false, false},
    {4, 2, false, false}, {8, 3, false, false}, {4, 3, false, false},
};
static_assert(KACC_T_PROC_POWER == 13 && KACC_T_PROC_RATIO == 25 && KACC_T_PROC_NODE == 26 &&
                  KACC_T_CTR_RATIO == 27 && KACC_T_VM_NODE == 30 && KACC_T_COUNT == 31,
              "kTables rows follow the kacc_table enum");

}  // namespace

int kacc_fail(kacc_ctx *ctx, int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (ctx) {
    ctx->err = buf;
  } else {
    std::lock_guard<std::mutex> lk(g_err_mu);
    g_create_error = buf;
  }
  return code;
}

namespace {

#define fail kacc_fail

// KACC_T_POD_ENERGY's allocation holds the pod records [Sq][2Z] (energy Z words,
// then power Z words: kacc_table_row_stride 2Z); KACC_T_POD_POWER points Z words in.
bool pod_paired(int t) { return t == KACC_T_POD_ENERGY || t == KACC_T_POD_POWER; }

uint64_t table_count(const kacc_config &c, int t);
size_t table_alloc_bytes(const kacc_ctx *ctx, int t) {
  const size_t n = std::max<uint64_t>(ctx->counts[t], 1) * kTables[t].elem;
  return t == KACC_T_POD_ENERGY ? 2 * n : n;
}

uint64_t table_count(const kacc_config &c, int t) {
  const TableDesc &d = kTables[t];
  uint64_t base = 0;
  switch (d.per) {
    case 0: base = c.nodes; break;
    case 1: base = c.proc_slots; break;
    case 2: base = c.ctr_slots; break;
    case 3: base = c.vm_slots; break;
    default: base = c.pod_slots; break;
  }
  return d.zoned ? base * c.zones : base;
}

// the split cluster node totals' scratch (NodeTotalsArgs.part / arrived)
constexpr size_t kColArrivedBytes = 5 * KACC_MAX_ZONES * sizeof(uint32_t);
size_t col_part_bytes(uint64_t nodes) {
  const uint64_t split = std::max<uint64_t>((nodes + kacc::kColSplitNodes - 1) / kacc::kColSplitNodes, 1);
  return 5 * KACC_MAX_ZONES * split * sizeof(uint64_t);
}

kacc::DevState dev_state(const kacc_ctx *ctx) {
  kacc::DevState s;
  auto T = [ctx](int t) { return ctx->tables[t]; };
  s.node_energy_total = (uint64_t *)T(KACC_T_NODE_ENERGY_TOTAL);
  s.node_active_energy = (uint64_t *)T(KACC_T_NODE_ACTIVE_ENERGY);
  s.node_active_total = (uint64_t *)T(KACC_T_NODE_ACTIVE_TOTAL);
  s.node_idle_total = (uint64_t *)T(KACC_T_NODE_IDLE_TOTAL);
  s.node_power = (double *)T(KACC_T_NODE_POWER);
  s.node_active_power = (double *)T(KACC_T_NODE_ACTIVE_POWER);
  s.node_idle_power = (double *)T(KACC_T_NODE_IDLE_POWER);
  s.node_ts = (int64_t *)T(KACC_T_NODE_TS);
  s.node_has_prev = (uint32_t *)T(KACC_T_NODE_HAS_PREV);
  s.node_usage_ratio = (double *)T(KACC_T_NODE_USAGE_RATIO);
  s.node_cpu_delta = (double *)T(KACC_T_NODE_CPU_DELTA);
  s.node_status = (uint32_t *)T(KACC_T_NODE_STATUS);
  s.proc_energy = (uint64_t *)T(KACC_T_PROC_ENERGY);
  s.proc_ratio = (double *)T(KACC_T_PROC_RATIO);
  s.proc_node = (uint32_t *)T(KACC_T_PROC_NODE);
  s.ctr_energy = (uint64_t *)T(KACC_T_CTR_ENERGY);
  s.ctr_ratio = (double *)T(KACC_T_CTR_RATIO);
  s.ctr_node = (uint32_t *)T(KACC_T_CTR_NODE);
  s.ctr_cpu_delta = (double *)T(KACC_T_CTR_CPU_DELTA);
  s.ctr_cpu_total = (double *)T(KACC_T_CTR_CPU_TOTAL);
  s.vm_energy = (uint64_t *)T(KACC_T_VM_ENERGY);
  s.vm_ratio = (double *)T(KACC_T_VM_RATIO);
  s.vm_node = (uint32_t *)T(KACC_T_VM_NODE);
  s.vm_cpu_delta = (double *)T(KACC_T_VM_CPU_DELTA);
  s.pod_energy = (uint64_t *)T(KACC_T_POD_ENERGY);
  s.pod_power = (double *)T(KACC_T_POD_POWER);
  s.pod_cpu_delta = (double *)T(KACC_T_POD_CPU_DELTA);
  s.pod_cpu_total = (double *)T(KACC_T_POD_CPU_TOTAL);
  s.proc_slots = ctx->cfg.proc_slots;
  s.ctr_slots = ctx->cfg.ctr_slots;
  s.vm_slots = ctx->cfg.vm_slots;
  s.pod_slots = ctx->cfg.pod_slots;
  s.err = ctx->d_err;
  s.items = ctx->d_items;
  s.item_ctr = ctx->d_ctr;
  s.item_cap = ctx->item_cap;
  s.defer = ctx->d_defer;
  s.defer_ctr = ctx->d_ctr + 2;
  s.defer_cap = ctx->defer_cap;
  s.items_given = 0;
  s.keep_items = 0;
  s.stamps = nullptr;
  return s;
}

// One interval = the fast kernel (one workgroup per node; oversized nodes get
// their node phase there and are cut into chunk items), the chunk kernel and
// the deferred-pod kernel (both exit at once when no node was oversized; not
// launched at all under KACC_F_FAST_NODES).
template <int Z>
void launch_small(const kacc_interval &b, const kacc::DevState &s, hipStream_t st) {
  const uint32_t grid = (b.n_nodes + kacc::kSmallWaves - 1) / kacc::kSmallWaves;
  if (!kacc::kTransposed<Z> && b.node_proc_span)  // Z without the transposed paths: row-wise slot sweep
    KACC_LAUNCH((kacc::small_kernel<Z, true>), dim3(grid), dim3(64 * kacc::kSmallWaves), 0, st, b, s);
  else
    KACC_LAUNCH((kacc::small_kernel<Z, false>), dim3(grid), dim3(64 * kacc::kSmallWaves), 0, st, b, s);
}

template <int Z, int V>
void launch_zv(const kacc_interval &b, const kacc::DevState &s, hipStream_t st) {
  if (V == 0 && (b.flags & KACC_F_SMALL_NODES)) return launch_small<Z>(b, s, st);
  KACC_LAUNCH((kacc::interval_kernel<Z, V>), dim3(b.n_nodes), dim3(kacc::kTpb<V>),
              KACC_FAST_EXTRA_LDS, st, b, s);
  if (b.flags & (KACC_F_FAST_NODES | KACC_F_SMALL_NODES)) return;
  const uint32_t chunk_grid = std::min<uint32_t>(s.item_cap, kacc::kChunkGrid);
  KACC_LAUNCH((kacc::chunk_kernel<Z, V>), dim3(chunk_grid), dim3(kacc::kChunkThreads), 0, st,
                     b, s);
  KACC_LAUNCH((kacc::pod_kernel<Z, V>), dim3(kacc::kPodGrid), dim3(kacc::kBlock), 0, st, b, s);
}

void launch(uint32_t Z, const kacc_interval &b, const kacc::DevState &s, hipStream_t st) {
  switch (Z) {
    case 1: launch_zv<1, 0>(b, s, st); break;
    case 2: launch_zv<2, 0>(b, s, st); break;
    case 3: launch_zv<3, 0>(b, s, st); break;
    case 4: launch_zv<4, 0>(b, s, st); break;
    case 5: launch_zv<5, 0>(b, s, st); break;
    case 6: launch_zv<6, 0>(b, s, st); break;
    case 7: launch_zv<7, 0>(b, s, st); break;
    default: launch_zv<8, 0>(b, s, st); break;
  }
}

// timing ablations (Z = 4 only): see kacc::kVar*
bool launch_variant(uint32_t Z, int v, const kacc_interval &b, const kacc::DevState &s,
                    hipStream_t st) {
  if (Z != 4) return false;
  switch (v) {
    case 0: launch_zv<4, 0>(b, s, st); return true;
    case 1: launch_zv<4, 1>(b, s, st); return true;
    case 2: launch_zv<4, 2>(b, s, st); return true;
    case 3: launch_zv<4, 3>(b, s, st); return true;
    case 4: launch_zv<4, 4>(b, s, st); return true;
    case 8: launch_zv<4, 8>(b, s, st); return true;
    case 32: launch_zv<4, 32>(b, s, st); return true;
    case 128: launch_zv<4, 128>(b, s, st); return true;
    case 256: launch_zv<4, 256>(b, s, st); return true;
    case 512: launch_zv<4, 512>(b, s, st); return true;
    case 768: launch_zv<4, 768>(b, s, st); return true;
    case 1024: launch_zv<4, 1024>(b, s, st); return true;
    case 2048: launch_zv<4, 2048>(b, s, st); return true;
    case 4096: launch_zv<4, 4096>(b, s, st); return true;
    case 8192: launch_zv<4, 8192>(b, s, st); return true;
    case 16384: launch_zv<4, 16384>(b, s, st); return true;
    case 16392: launch_zv<4, 16392>(b, s, st); return true;
    case 65536: launch_small<4>(b, s, st); return true;  // one wavefront per node
    default: return false;
  }
}

template <int Z>
void launch_ns(uint32_t n_ns, const uint32_t *off, const uint32_t *slots, const kacc_ctx *ctx,
               uint64_t *out_e, double *out_p, hipStream_t st) {
  const uint32_t per_block = kacc::kBlock / kacc::kNsLanes;
  const uint32_t grid = (n_ns + per_block - 1) / per_block;
  hipLaunchKernelGGL((kacc::namespace_kernel<Z>), dim3(grid), dim3(kacc::kBlock), 0, st, n_ns, off,
                     slots, (const uint64_t *)ctx->tables[KACC_T_POD_ENERGY],
                     (const double *)ctx->tables[KACC_T_POD_POWER], ctx->cfg.pod_slots, out_e, out_p,
                     ctx->d_err);
}

// The node-total columns of the context's tables (node_export NULL) or of an export.
kacc::NodeTotalsArgs node_totals_args(const kacc_ctx *ctx, uint64_t live, const uint64_t *node_export,
                                      uint64_t *node_energy, double *node_power) {
  kacc::NodeTotalsArgs na{};
  na.n_nodes = live;
  na.active_total = (const uint64_t *)ctx->tables[KACC_T_NODE_ACTIVE_TOTAL];
  na.idle_total = (const uint64_t *)ctx->tables[KACC_T_NODE_IDLE_TOTAL];
  na.power = (const double *)ctx->tables[KACC_T_NODE_POWER];
  na.active_power = (const double *)ctx->tables[KACC_T_NODE_ACTIVE_POWER];
  na.idle_power = (const double *)ctx->tables[KACC_T_NODE_IDLE_POWER];
  na.out_e = node_energy;
  na.out_p = node_power;
  na.node_export = node_export;
  na.split = 1;
  return na;
}

// pod_export NULL: the namespace sums gather the state tables by pod slot;
// else the interval's pod export by batch pod row (n_pods rows)
template <int Z>
void launch_cluster_partials(uint32_t n_ns, const uint32_t *off, const uint32_t *slots, kacc_ctx *ctx,
                             uint64_t *out_e, double *out_p, const kacc::NodeTotalsArgs &na, uint32_t node_blocks,
                             hipStream_t st, const uint64_t *pod_export = nullptr, uint64_t n_pods = 0,
                             bool ordered = false) {
  const uint32_t per_block = kacc::kBlock / kacc::kNsLanes;
  const uint32_t ns_blocks = (n_ns + per_block - 1) / per_block;
  // pod_export NULL: the pod tables, one [energy | power] record per slot like an export row
  const uint64_t *pe = pod_export ? pod_export : (const uint64_t *)ctx->tables[KACC_T_POD_ENERGY];
  const double *pp = pod_export ? reinterpret_cast<const double *>(pod_export + Z)
                                : (const double *)ctx->tables[KACC_T_POD_POWER];
  const uint64_t rows = pod_export ? n_pods : ctx->cfg.pod_slots;
  const bool wide = na.n_nodes > kacc::kColSplitFrom && node_blocks;
  kacc::NodeTotalsArgs nas = na;
  if (wide) {  // each column over ceil(N / kColSplitNodes) blocks, combined by the last one
    nas.split = static_cast<uint32_t>((na.n_nodes + kacc::kColSplitNodes - 1) / kacc::kColSplitNodes);
    nas.part = ctx->d_colpart;
    nas.arrived = ctx->d_colarrived;
    node_blocks *= nas.split;
  }
  if (wide && ordered)
    KACC_LAUNCH((kacc::cluster_partials_kernel<Z, 2 * Z, true, true>), dim3(ns_blocks + node_blocks),
                dim3(kacc::kBlock), 0, st, ns_blocks, n_ns, off, slots, pe, pp, rows, out_e, out_p, ctx->d_err, nas);
  else if (wide)
    KACC_LAUNCH((kacc::cluster_partials_kernel<Z, 2 * Z, true>), dim3(ns_blocks + node_blocks), dim3(kacc::kBlock),
                0, st, ns_blocks, n_ns, off, slots, pe, pp, rows, out_e, out_p, ctx->d_err, nas);
  else if (ordered)
    KACC_LAUNCH((kacc::cluster_partials_kernel<Z, 2 * Z, false, true>), dim3(ns_blocks + node_blocks),
                dim3(kacc::kBlock), 0, st, ns_blocks, n_ns, off, slots, pe, pp, rows, out_e, out_p, ctx->d_err, nas);
  else
    KACC_LAUNCH((kacc::cluster_partials_kernel<Z>), dim3(ns_blocks + node_blocks), dim3(kacc::kBlock), 0, st,
                ns_blocks, n_ns, off, slots, pe, pp, rows, out_e, out_p, ctx->d_err, nas);
}

// An interval and the partial sums of an earlier interval's exports in ONE launch
// (kacc_run_interval_sums): interval_sums_kernel, then the big-node launches as
// launch_zv does.
template <int Z>
void launch_fused(const kacc_interval &b, const kacc::DevState &s, const kacc::SumsArgs &sa, hipStream_t st) {
  KACC_LAUNCH((kacc::interval_sums_kernel<Z, 0>), dim3(b.n_nodes + sa.node_blocks + sa.ns_blocks),
              dim3(kacc::kTpb<0>), KACC_FAST_EXTRA_LDS, st, b, s, sa);
  if (b.flags & (KACC_F_FAST_NODES | KACC_F_SMALL_NODES)) return;
  const uint32_t chunk_grid = std::min<uint32_t>(s.item_cap, kacc::kChunkGrid);
  KACC_LAUNCH((kacc::chunk_kernel<Z, 0>), dim3(chunk_grid), dim3(kacc::kChunkThreads), 0, st, b, s);
  KACC_LAUNCH((kacc::pod_kernel<Z, 0>), dim3(kacc::kPodGrid), dim3(kacc::kBlock), 0, st, b, s);
}

void launch_fused_z(uint32_t Z, const kacc_interval &b, const kacc::DevState &s, const kacc::SumsArgs &sa,
                    hipStream_t st) {
  switch (Z) {
    case 1: launch_fused<1>(b, s, sa, st); break;
    case 2: launch_fused<2>(b, s, sa, st); break;
    case 3: launch_fused<3>(b, s, sa, st); break;
    case 4: launch_fused<4>(b, s, sa, st); break;
    case 5: launch_fused<5>(b, s, sa, st); break;
    case 6: launch_fused<6>(b, s, sa, st); break;
    case 7: launch_fused<7>(b, s, sa, st); break;
    default: launch_fused<8>(b, s, sa, st); break;
  }
}

// [p, p + bytes) and [q, q + bytes2) share a byte
bool overlaps(const void *p, uint64_t bytes, const void *q, uint64_t bytes2) {
  if (!p || !q || !bytes || !bytes2) return false;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p), c = reinterpret_cast<uintptr_t>(q);
  return a < c + bytes2 && c < a + bytes;
}

// The checked device arguments of a kacc_export_sums, for namespace blocks of
// `threads` threads.
int sums_args(kacc_ctx *ctx, const kacc_export_sums *x, uint32_t threads, kacc::SumsArgs &sa) {
  if (!x) return fail(ctx, KACC_EINVAL, "export sums: NULL descriptor");
  const uint64_t Z = ctx->cfg.zones;
  const bool nodes = x->out_node_energy || x->out_node_power;
  if (nodes && (!x->out_node_energy || !x->out_node_power))
    return fail(ctx, KACC_EINVAL, "export sums: node totals need both output arrays");
  if (nodes && x->n_nodes && !x->node_export) return fail(ctx, KACC_EINVAL, "export sums: node_export is NULL");
  if (x->n_nodes > ctx->cfg.nodes)
    return fail(ctx, KACC_EINVAL, "export sums: n_nodes %u exceeds node capacity", x->n_nodes);
  if (x->n_ns && (!x->ns_pod_off || !x->out_energy || !x->out_power || (!x->ns_ordered && !x->ns_pod_row) ||
                  (x->n_pods && !x->pod_export)))
    return fail(ctx, KACC_EINVAL, "export sums: NULL namespace / pod export array");
  if (x->ns_ordered > 1) return fail(ctx, KACC_EINVAL, "export sums: ns_ordered must be 0 or 1");
  sa = kacc::SumsArgs{};
  sa.node_blocks = nodes ? static_cast<uint32_t>(5 * Z) : 0u;
  const uint32_t per_block = threads / kacc::kNsLanes;
  sa.ns_blocks = (x->n_ns + per_block - 1) / per_block;
  sa.n_ns = x->n_ns;
  sa.ordered = x->ns_ordered;
  sa.off = x->ns_pod_off;
  sa.rows = x->ns_pod_row;
  sa.pe = x->pod_export;
  sa.pp = x->pod_export ? reinterpret_cast<const double *>(x->pod_export + Z) : nullptr;
  sa.n_pods = x->pod_export ? x->n_pods : 0;  // no export: no row to read (a non-empty namespace raises)
  sa.out_e = x->out_energy;
  sa.out_p = x->out_power;
  sa.na = node_totals_args(ctx, nodes ? x->n_nodes : 0, x->node_export, x->out_node_energy, x->out_node_power);
  return KACC_OK;
}

// Chunk-item list sized for the worst case of a batch (every node oversized,
// plus one partial chunk per node) and the deferred-pod list for every pod.
// Grown (synchronously, between intervals) only when a batch is larger than
// the capacities suggested at kacc_create.
int ensure_items(kacc_ctx *ctx, uint64_t nodes, uint64_t procs, uint64_t pods) {
  const uint64_t need = nodes + (procs + kacc::kChunkRows - 1) / kacc::kChunkRows + 1;
  const uint64_t need_defer = std::max<uint64_t>(pods, 1);
  if (need > 0xffffffffull || need_defer > 0xffffffffull)
    return fail(ctx, KACC_EINVAL, "batch too large for the chunk lists");
  if (need > ctx->item_cap || need_defer > ctx->defer_cap) KACC_HIP(ctx, hipDeviceSynchronize());
  if (need > ctx->item_cap) {
    if (ctx->d_items) KACC_HIP(ctx, hipFree(ctx->d_items));
    ctx->d_items = nullptr;
    ctx->item_cap = 0;
    KACC_HIP(ctx, hipMalloc(&ctx->d_items, need * sizeof(kacc::ChunkItem)));
    ctx->item_cap = static_cast<uint32_t>(need);
  }
  if (need_defer > ctx->defer_cap) {
    if (ctx->d_defer) KACC_HIP(ctx, hipFree(ctx->d_defer));
    ctx->d_defer = nullptr;
    ctx->defer_cap = 0;
    KACC_HIP(ctx, hipMalloc(&ctx->d_defer, need_defer * sizeof(uint2)));
    ctx->defer_cap = static_cast<uint32_t>(need_defer);
  }
  return KACC_OK;
}

int check_shape(kacc_ctx *ctx, const kacc_interval *b) {
  if (!b) return fail(ctx, KACC_EINVAL, "batch is NULL");
  if (b->n_nodes > ctx->cfg.nodes)
    return fail(ctx, KACC_EINVAL, "n_nodes %u exceeds node capacity %llu", b->n_nodes,
                (unsigned long long)ctx->cfg.nodes);
  if (b->n_nodes == 0) return KACC_OK;
  if (!b->node_ts_ns || !b->node_usage_ratio || !b->zone_energy || !b->zone_max ||
      !b->proc_off || !b->ctr_off || !b->vm_off || !b->pod_off)
    return fail(ctx, KACC_EINVAL, "required node array is NULL");
  if ((b->n_procs && (!b->proc_cpu_delta || !b->proc_slot)) ||
      (b->n_ctrs && (!b->ctr_proc_end || !b->ctr_slot)) ||
      (b->n_vms && (!b->vm_proc_end || !b->vm_slot)) ||
      (b->n_pods && (!b->pod_ctr_end || !b->pod_slot)))
    return fail(ctx, KACC_EINVAL, "required row array is NULL");
  if ((b->flags & KACC_F_NODE_CPU_DELTA_GIVEN) && !b->node_cpu_delta)
    return fail(ctx, KACC_EINVAL, "KACC_F_NODE_CPU_DELTA_GIVEN without node_cpu_delta");
  if (b->flags & ~(KACC_F_NODE_CPU_DELTA_GIVEN | KACC_F_FAST_NODES | KACC_F_TRUSTED_LAYOUT |
                   KACC_F_SMALL_NODES | KACC_F_NODE_SLOT_RANGES | KACC_F_MEDIUM_NODES |
                   KACC_F_STABLE_SLOT_NODES))
    return fail(ctx, KACC_EINVAL, "unknown flags 0x%x", b->flags);
  return KACC_OK;
}

int check_offsets(kacc_ctx *ctx, const char *name, const uint32_t *off, uint32_t n, uint32_t count) {
  if (off[0] != 0) return fail(ctx, KACC_EINVAL, "%s[0] must be 0", name);
  for (uint32_t i = 0; i < n; ++i)
    if (off[i + 1] < off[i]) return fail(ctx, KACC_EINVAL, "%s not monotonic at %u", name, i);
  if (off[n] != count) return fail(ctx, KACC_EINVAL, "%s[n] != row count", name);
  return KACC_OK;
}

// Host checks of big batches run on up to kHostThreads threads (the Go caller
// blocks in cgo meanwhile; a 20M-row batch is ~10 ms on one core).
constexpr uint32_t kHostThreads = 16;
constexpr uint64_t kHostGrain = 1u << 18;  // rows per thread at least

// Runs fn(begin, end) over [0, n) in contiguous pieces; returns the smallest
// index any piece reported (fn returns n when its piece is clean).
template <typename F>
uint64_t par_first(uint64_t n, F fn) {
  const uint32_t hw = std::max(1u, std::thread::hardware_concurrency());
  const uint64_t t = std::min<uint64_t>({kHostThreads, hw, (n + kHostGrain - 1) / kHostGrain});
  if (t <= 1) return fn(0, n);
  std::vector<uint64_t> first(t, n);
  std::vector<std::thread> pool;
  const uint64_t piece = (n + t - 1) / t;
  for (uint64_t i = 0; i < t; ++i)
    pool.emplace_back([&, i] { first[i] = fn(std::min(n, i * piece), std::min(n, (i + 1) * piece)); });
  for (auto &th : pool) th.join();
  return *std::min_element(first.begin(), first.end());
}

// Range and duplicate check of a slot column.  Each thread takes a contiguous
// piece of rows and marks a private bitset over the piece's own slot range
// (slots are allocated per node, so pieces rarely overlap); overlapping word
// ranges of different pieces are then ANDed.  No atomics, no cap-sized clear.
int check_slots(kacc_ctx *ctx, const char *name, const uint32_t *w, uint32_t n, uint64_t cap) {
  if (n == 0) return KACC_OK;
  const uint32_t hw = std::max(1u, std::thread::hardware_concurrency());
  const uint64_t T = std::max<uint64_t>(1, std::min<uint64_t>({kHostThreads, hw, (n + kHostGrain - 1) / kHostGrain}));
  const uint64_t piece = (n + T - 1) / T;
  struct Piece {
    uint64_t b, e, lo, hi, bad = ~0ull, dup = ~0ull;  // rows [b, e); words [lo, hi]
    std::vector<uint64_t> bits;
  };
  std::vector<Piece> pc(T);
  auto mark = [&](uint64_t i) {
    Piece &p = pc[i];
    p.b = std::min<uint64_t>(n, i * piece);
    p.e = std::min<uint64_t>(n, (i + 1) * piece);
    uint64_t lo = ~0ull, hi = 0;
    for (uint64_t r = p.b; r < p.e; ++r) {
      const uint64_t s = w[r] & KACC_SLOT_MASK;
      if (s >= cap) {
        p.bad = r;
        return;
      }
      lo = std::min(lo, s);
      hi = std::max(hi, s);
    }
    if (p.b == p.e) return;
    p.lo = lo >> 6;
    p.hi = hi >> 6;
    p.bits.assign(p.hi - p.lo + 1, 0);
    for (uint64_t r = p.b; r < p.e; ++r) {
      const uint64_t s = w[r] & KACC_SLOT_MASK;
      uint64_t &word = p.bits[(s >> 6) - p.lo];
      const uint64_t bit = 1ull << (s & 63);
      if (word & bit) {
        p.dup = s;
        return;
      }
      word |= bit;
    }
  };
  if (T == 1) {
    mark(0);
  } else {
    std::vector<std::thread> pool;
    for (uint64_t i = 0; i < T; ++i) pool.emplace_back(mark, i);
    for (auto &th : pool) th.join();
  }
  for (const Piece &p : pc) {  // first bad row in row order
    if (p.bad != ~0ull)
      return fail(ctx, KACC_EINVAL, "%s[%llu]=%llu >= capacity", name, (unsigned long long)p.bad,
                  (unsigned long long)(w[p.bad] & KACC_SLOT_MASK));
    if (p.dup != ~0ull) return fail(ctx, KACC_EINVAL, "%s: slot %llu used twice", name, (unsigned long long)p.dup);
  }
  // pieces whose word ranges overlap: a bit set in two of them is a duplicate
  for (uint64_t i = 0; i < T; ++i)
    for (uint64_t j = i + 1; j < T; ++j) {
      const Piece &a = pc[i], &c = pc[j];
      if (a.bits.empty() || c.bits.empty()) continue;
      const uint64_t lo = std::max(a.lo, c.lo), hi = std::min(a.hi, c.hi);
      for (uint64_t x = lo; x <= hi && lo <= hi; ++x) {
        const uint64_t both = a.bits[x - a.lo] & c.bits[x - c.lo];
        if (both)
          return fail(ctx, KACC_EINVAL, "%s: slot %llu used twice", name,
                      (unsigned long long)(x * 64 + __builtin_ctzll(both)));
      }
    }
  return KACC_OK;
}

// KACC_F_FAST_NODES when every node fits the fast workgroup (| KACC_F_MEDIUM_NODES
// / KACC_F_SMALL_NODES when every node also fits those shapes), else 0 (host
// batch, offsets already validated).
uint32_t node_size_flags(const kacc_interval &b) {
  bool small = true, medium = true;
  for (uint32_t n = 0; n < b.n_nodes; ++n) {
    const uint32_t rows = b.proc_off[n + 1] - b.proc_off[n];
    const uint32_t agg = (b.ctr_off[n + 1] - b.ctr_off[n]) + (b.vm_off[n + 1] - b.vm_off[n]) +
                         (b.pod_off[n + 1] - b.pod_off[n]);
    if (rows > KACC_FAST_MAX_PROCS || agg > KACC_FAST_MAX_AGGREGATES) return 0u;
    small = small && rows <= KACC_SMALL_MAX_PROCS && agg <= KACC_SMALL_MAX_AGGREGATES;
    medium = medium && rows <= KACC_MEDIUM_MAX_PROCS && agg <= KACC_MEDIUM_MAX_AGGREGATES;
  }
  return KACC_F_FAST_NODES | (small ? KACC_F_SMALL_NODES : 0u) | (medium ? KACC_F_MEDIUM_NODES : 0u);
}

// The K descriptors of a fused kacc_run_intervals, copied to the device on
// `st` through a pinned staging buffer (reused once its last copy is done).
int stage_batches(kacc_ctx *ctx, const kacc_interval *b, uint32_t K, hipStream_t st) {
  if (K > ctx->batch_cap) {
    if (ctx->batch_copied) KACC_HIP(ctx, hipEventSynchronize(ctx->batch_copied));
    if (ctx->d_batches) KACC_HIP(ctx, hipFree(ctx->d_batches));
    if (ctx->h_batches) KACC_HIP(ctx, hipHostFree(ctx->h_batches));
    ctx->d_batches = nullptr;
    ctx->h_batches = nullptr;
    ctx->batch_cap = 0;
    KACC_HIP(ctx, hipMalloc(&ctx->d_batches, sizeof(kacc_interval) * K));
    KACC_HIP(ctx, hipHostMalloc(reinterpret_cast<void **>(&ctx->h_batches), sizeof(kacc_interval) * K,
                                hipHostMallocDefault));
    ctx->batch_cap = K;
  }
  if (!ctx->batch_copied) KACC_HIP(ctx, hipEventCreateWithFlags(&ctx->batch_copied, hipEventDisableTiming));
  KACC_HIP(ctx, hipEventSynchronize(ctx->batch_copied));  // the previous copy has read the staging buffer
  std::memcpy(ctx->h_batches, b, sizeof(kacc_interval) * K);
  KACC_HIP(ctx, hipMemcpyAsync(ctx->d_batches, ctx->h_batches, sizeof(kacc_interval) * K, hipMemcpyHostToDevice, st));
  KACC_HIP(ctx, hipEventRecord(ctx->batch_copied, st));
  return KACC_OK;
}

template <int V>
void launch_carry(uint32_t Z, bool medium, const kacc_interval *d_b, uint32_t K, uint32_t n_nodes,
                  const kacc::DevState &s, hipStream_t st) {
  if (medium) {
    if (Z == 1)
      KACC_LAUNCH((kacc::intervals_carry_kernel<1, V, 256>), dim3(n_nodes), dim3(256), 0, st, d_b, K, s);
    else
      KACC_LAUNCH((kacc::intervals_carry_kernel<2, V, 256>), dim3(n_nodes), dim3(256), 0, st, d_b, K, s);
  } else {
    if (Z == 1)
      KACC_LAUNCH((kacc::intervals_carry_kernel<1, V, 512>), dim3(n_nodes), dim3(512), 0, st, d_b, K, s);
    else
      KACC_LAUNCH((kacc::intervals_carry_kernel<2, V, 512>), dim3(n_nodes), dim3(512), 0, st, d_b, K, s);
  }
}

void launch_intervals(uint32_t Z, bool medium, const kacc_interval *d_b, uint32_t K, uint32_t n_nodes,
                      const kacc::DevState &s, hipStream_t st) {
  launch_carry<0>(Z, medium, d_b, K, n_nodes, s, st);
}

// every descriptor promises KACC_F_MEDIUM_NODES
bool all_medium(const kacc_interval *b, uint32_t count) {
  for (uint32_t k = 0; k < count; ++k)
    if (!(b[k].flags & KACC_F_MEDIUM_NODES)) return false;
  return true;
}

}  // namespace

extern "C" {

uint32_t kacc_abi_version(void) { return KACC_ABI_VERSION; }

const char *kacc_last_error(const kacc_ctx *ctx) {
  if (ctx) return ctx->err.c_str();
  std::lock_guard<std::mutex> lk(g_err_mu);
  return g_create_error.c_str();
}

size_t kacc_last_error_copy(const kacc_ctx *ctx, char *buf, size_t len) {
  std::string msg;
  if (ctx) {
    msg = ctx->err;
  } else {
    std::lock_guard<std::mutex> lk(g_err_mu);
    msg = g_create_error;
  }
  if (buf && len) {
    const size_t n = std::min(len - 1, msg.size());
    std::memcpy(buf, msg.data(), n);
    buf[n] = '\0';
  }
  return msg.size();
}

int kacc_create(int device, const kacc_config *cfg, kacc_ctx **out) {
  if (!cfg || !out) return fail(nullptr, KACC_EINVAL, "NULL argument");
  *out = nullptr;
  if (cfg->zones == 0 || cfg->zones > KACC_MAX_ZONES)
    return fail(nullptr, KACC_EINVAL, "zones must be 1..%u", KACC_MAX_ZONES);
  if (cfg->proc_slots > KACC_SLOT_MASK || cfg->ctr_slots > KACC_SLOT_MASK ||
      cfg->vm_slots > KACC_SLOT_MASK || cfg->pod_slots > KACC_SLOT_MASK || cfg->nodes > 0xffffffffu)
    return fail(nullptr, KACC_EINVAL, "capacity exceeds the 31-bit slot range");
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return fail(nullptr, KACC_EHIP, "hipSetDevice(%d): %s", device, hipGetErrorString(e));
  auto *ctx = new kacc_ctx;
  ctx->device = device;
  ctx->cfg = *cfg;
  int rc = KACC_OK;
  auto bail = [&](int code) {
    {
      std::lock_guard<std::mutex> lk(g_err_mu);
      g_create_error = ctx->err;
    }
    kacc_destroy(ctx);
    return code;
  };
  if ((e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking)) != hipSuccess) {
    fail(ctx, KACC_EHIP, "hipStreamCreate: %s", hipGetErrorString(e));
    return bail(KACC_EHIP);
  }
  for (int t = 0; t < KACC_T_COUNT; ++t) {
    ctx->counts[t] = table_count(ctx->cfg, t);
    if (kTables[t].derived || t == KACC_T_POD_POWER) continue;  // computed on read / inside the pod records
    const size_t bytes = table_alloc_bytes(ctx, t);
    if ((e = hipMalloc(&ctx->tables[t], bytes)) != hipSuccess) {
      fail(ctx, KACC_ENOMEM, "hipMalloc table %d (%zu B): %s", t, bytes, hipGetErrorString(e));
      return bail(KACC_ENOMEM);
    }
  }
  ctx->tables[KACC_T_POD_POWER] = static_cast<char *>(ctx->tables[KACC_T_POD_ENERGY]) + 8ull * ctx->cfg.zones;
  if ((e = hipMalloc(&ctx->d_err, sizeof(uint32_t))) != hipSuccess ||
      (e = hipMalloc(&ctx->d_ctr, 16)) != hipSuccess ||
      (e = hipMalloc(&ctx->d_colpart, col_part_bytes(cfg->nodes))) != hipSuccess ||
      (e = hipMalloc(&ctx->d_colarrived, kColArrivedBytes)) != hipSuccess) {
    fail(ctx, KACC_ENOMEM, "hipMalloc work words: %s", hipGetErrorString(e));
    return bail(KACC_ENOMEM);
  }
  if ((rc = ensure_items(ctx, cfg->nodes, cfg->proc_slots, cfg->pod_slots)) != KACC_OK) return bail(rc);
  if ((rc = kacc_reset(ctx)) != KACC_OK) return bail(rc);
  *out = ctx;
  return KACC_OK;
}

void kacc_destroy(kacc_ctx *ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  for (int t = 0; t < KACC_T_COUNT; ++t)
    if (ctx->tables[t] && t != KACC_T_POD_POWER) (void)hipFree(ctx->tables[t]);  // pod power: inside the records
  if (ctx->d_err) (void)hipFree(ctx->d_err);
  if (ctx->d_ctr) (void)hipFree(ctx->d_ctr);
  if (ctx->d_colpart) (void)hipFree(ctx->d_colpart);
  if (ctx->d_colarrived) (void)hipFree(ctx->d_colarrived);
  if (ctx->d_items) (void)hipFree(ctx->d_items);
  if (ctx->d_defer) (void)hipFree(ctx->d_defer);
  if (ctx->batch_copied) {
    (void)hipEventSynchronize(ctx->batch_copied);
    (void)hipEventDestroy(ctx->batch_copied);
  }
  if (ctx->d_batches) (void)hipFree(ctx->d_batches);
  if (ctx->h_batches) (void)hipHostFree(ctx->h_batches);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->copy_stream) {
    (void)hipStreamSynchronize(ctx->copy_stream);
    (void)hipStreamDestroy(ctx->copy_stream);
  }
  delete ctx;
}

int kacc_get_config(const kacc_ctx *ctx, kacc_config *out) {
  if (!ctx || !out) return KACC_EINVAL;
  *out = ctx->cfg;
  return KACC_OK;
}

int kacc_reset(kacc_ctx *ctx) {
  if (!ctx) return KACC_EINVAL;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  for (int t = 0; t < KACC_T_COUNT; ++t)
    if (!kTables[t].derived && t != KACC_T_POD_POWER)
      KACC_HIP(ctx, hipMemsetAsync(ctx->tables[t], 0, table_alloc_bytes(ctx, t), ctx->stream));
  KACC_HIP(ctx, hipMemsetAsync(ctx->d_err, 0, sizeof(uint32_t), ctx->stream));
  KACC_HIP(ctx, hipMemsetAsync(ctx->d_ctr, 0, 16, ctx->stream));
  KACC_HIP(ctx, hipMemsetAsync(ctx->d_colarrived, 0, kColArrivedBytes, ctx->stream));
  KACC_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->live_nodes = 0;
  return KACC_OK;
}

int kacc_time_next_launch(kacc_ctx *ctx, void *start_event, void *stop_event) {
  if (!ctx) return KACC_EINVAL;
  ctx->time_start = static_cast<hipEvent_t>(start_event);
  ctx->time_stop = static_cast<hipEvent_t>(stop_event);
  return KACC_OK;
}

static int run_one(kacc_ctx *ctx, const kacc_interval *b, void *stream);

int kacc_run_interval(kacc_ctx *ctx, const kacc_interval *b, void *stream) {
  if (!ctx) return KACC_EINVAL;
  const kacc::TimingScope timing(ctx);
  return run_one(ctx, b, stream);
}

// One interval (kacc_run_interval, kacc_run_intervals of one).
static int run_one(kacc_ctx *ctx, const kacc_interval *b, void *stream) {
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  int rc = check_shape(ctx, b);
  if (rc != KACC_OK) return rc;
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  if (b->n_nodes == 0) {  // an emptied batch: no node of it counts in the cluster totals
    ctx->live_nodes = 0;
    return KACC_OK;
  }
  if ((rc = ensure_items(ctx, b->n_nodes, b->n_procs, b->n_pods)) != KACC_OK) return rc;
  (void)hipGetLastError();  // clear a stale error of an earlier call
  launch(ctx->cfg.zones, *b, dev_state(ctx), st);
  KACC_HIP(ctx, hipGetLastError());
  ctx->live_nodes = b->n_nodes;
  return KACC_OK;
}


// K consecutive intervals in one call (fleet replay, BASELINE config 5's 60
// batched intervals): interval k+1 reads the state interval k wrote, so the
// launches are issued in order on one stream, back to back from C (no host
// round trip between intervals).  Every shape is checked before any launch.
int kacc_run_intervals(kacc_ctx *ctx, const kacc_interval *dev_batches, uint32_t count, void *stream) {
  if (!ctx) return KACC_EINVAL;
  const kacc::TimingScope timing(ctx);
  if (count && !dev_batches) return fail(ctx, KACC_EINVAL, "dev_batches is NULL");
  if (count == 1) return run_one(ctx, dev_batches, stream);
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  uint64_t max_nodes = 0, max_procs = 0, max_pods = 0;
  for (uint32_t k = 0; k < count; ++k) {
    const int rc = check_shape(ctx, &dev_batches[k]);
    if (rc != KACC_OK) return fail(ctx, rc, "interval %u: %s", k, std::string(ctx->err).c_str());
    max_nodes = std::max<uint64_t>(max_nodes, dev_batches[k].n_nodes);
    max_procs = std::max<uint64_t>(max_procs, dev_batches[k].n_procs);
    max_pods = std::max<uint64_t>(max_pods, dev_batches[k].n_pods);
  }
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  int rc = ensure_items(ctx, max_nodes, max_procs, max_pods);
  if (rc != KACC_OK) return rc;
  (void)hipGetLastError();  // clear a stale error of an earlier call
  const kacc::DevState ds = dev_state(ctx);
  // one launch for all K intervals when every node stays in one workgroup's
  // hands: fast nodes, node-private slots, one node set, launch order = node id
  bool fused = count > 1 && ctx->cfg.zones <= static_cast<uint32_t>(kacc::kCarryMaxZ);
  for (uint32_t k = 0; k < count && fused; ++k) {
    const kacc_interval &b = dev_batches[k];
    // exports (kacc_interval.pod_export / node_export) are written by the per-interval
    // kernels only: the carry kernel without them spills less (SGPR pressure, round 4)
    fused = (b.flags & KACC_F_FAST_NODES) && (b.flags & KACC_F_NODE_SLOT_RANGES) &&
            !(b.flags & KACC_F_SMALL_NODES) && !b.node_order && b.n_nodes == dev_batches[0].n_nodes &&
            b.n_nodes > 0 && !b.pod_export && !b.node_export;
  }
  if (fused) {
    if ((rc = stage_batches(ctx, dev_batches, count, st)) != KACC_OK) return rc;
    launch_intervals(ctx->cfg.zones, all_medium(dev_batches, count), ctx->d_batches, count, dev_batches[0].n_nodes,
                     ds, st);
    KACC_HIP(ctx, hipGetLastError());
    ctx->live_nodes = dev_batches[count - 1].n_nodes;
    return KACC_OK;
  }
  // intervals over ONE layout (every descriptor the same offset arrays and sizes)
  // that may hold big nodes: their chunk items are generated once and reused
  bool one_layout = count > 1;
  for (uint32_t k = 1; k < count && one_layout; ++k) {
    const kacc_interval &a = dev_batches[0], &b = dev_batches[k];
    one_layout = a.n_nodes == b.n_nodes && a.n_procs == b.n_procs && a.n_ctrs == b.n_ctrs && a.n_vms == b.n_vms &&
                 a.n_pods == b.n_pods && a.proc_off == b.proc_off && a.ctr_off == b.ctr_off && a.vm_off == b.vm_off &&
                 a.pod_off == b.pod_off && a.ctr_proc_end == b.ctr_proc_end && a.vm_proc_end == b.vm_proc_end &&
                 a.pod_ctr_end == b.pod_ctr_end && !(b.flags & (KACC_F_FAST_NODES | KACC_F_SMALL_NODES));
  }
  if (one_layout && dev_batches[0].n_nodes && !(dev_batches[0].flags & (KACC_F_FAST_NODES | KACC_F_SMALL_NODES))) {
    KACC_LAUNCH((kacc::items_kernel<0>), dim3(dev_batches[0].n_nodes), dim3(kacc::kTpb<0>), 0, st,
                       dev_batches[0], ds);
    kacc::DevState dk = ds;
    dk.items_given = 1;
    for (uint32_t k = 0; k < count; ++k) {
      dk.keep_items = k + 1 < count ? 1u : 0u;  // the last interval's pod_kernel clears the list
      launch(ctx->cfg.zones, dev_batches[k], dk, st);
    }
  } else {
    for (uint32_t k = 0; k < count; ++k)
      if (dev_batches[k].n_nodes) launch(ctx->cfg.zones, dev_batches[k], ds, st);
  }
  KACC_HIP(ctx, hipGetLastError());
  if (count) ctx->live_nodes = dev_batches[count - 1].n_nodes;
  return KACC_OK;
}

int kacc_sync(kacc_ctx *ctx, void *stream) {
  if (!ctx) return KACC_EINVAL;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  KACC_HIP(ctx, hipStreamSynchronize(st));
  uint32_t err = 0;
  KACC_HIP(ctx, hipMemcpy(&err, ctx->d_err, sizeof(err), hipMemcpyDeviceToHost));
  if (err) {
    KACC_HIP(ctx, hipMemset(ctx->d_err, 0, sizeof(uint32_t)));
    // every bit a library kernel raises (kacc_engine / join / format / tracker / ticks /
    // packer / cluster); any other bit has no writer in the library — a stray device
    // store into this word — and is named as such
    constexpr uint32_t kKnown = 0x1ffu | (1u << 10);
    if (err & ~kKnown)
      return fail(ctx, KACC_ERANGE, "device error word 0x%x holds bits no library kernel raises (0x%x): a stray "
                  "device store into the context's error word; known bits 0x%x", err, err & ~kKnown, err & kKnown);
    return fail(ctx, KACC_ERANGE, "device range check failed (bits 0x%x: 1=node 2=offsets 4=slot 8=namespace 16=work list 32=oversized node under KACC_F_FAST_NODES 64=join key 128=join range 256=format lines 1024=tracker capacity)", err);
  }
  return KACC_OK;
}

int kacc_validate_host(const kacc_ctx *cctx, const kacc_interval *b) {
  kacc_ctx *ctx = const_cast<kacc_ctx *>(cctx);
  if (!ctx) return KACC_EINVAL;
  int rc = check_shape(ctx, b);
  if (rc != KACC_OK || b->n_nodes == 0) return rc;
  const uint32_t N = b->n_nodes;
  if ((rc = check_offsets(ctx, "proc_off", b->proc_off, N, b->n_procs))) return rc;
  if ((rc = check_offsets(ctx, "ctr_off", b->ctr_off, N, b->n_ctrs))) return rc;
  if ((rc = check_offsets(ctx, "vm_off", b->vm_off, N, b->n_vms))) return rc;
  if ((rc = check_offsets(ctx, "pod_off", b->pod_off, N, b->n_pods))) return rc;
  // membership per node: containers then VMs tile the node's rows in order,
  // pods tile the node's containers (first bad node reported)
  enum { kOkNode, kBadCtr, kBadVm, kBadPod };
  std::vector<uint8_t> why(N, kOkNode);
  std::vector<uint32_t> where(N, 0);
  const uint64_t bad_node = par_first(N, [&](uint64_t nb, uint64_t ne) -> uint64_t {
    for (uint64_t n = nb; n < ne; ++n) {
      const uint32_t p0 = b->proc_off[n], p1 = b->proc_off[n + 1];
      uint32_t prev = p0;
      for (uint32_t c = b->ctr_off[n]; c < b->ctr_off[n + 1]; ++c) {
        if (b->ctr_proc_end[c] < prev || b->ctr_proc_end[c] > p1) {
          why[n] = kBadCtr, where[n] = c;
          return n;
        }
        prev = b->ctr_proc_end[c];
      }
      for (uint32_t v = b->vm_off[n]; v < b->vm_off[n + 1]; ++v) {
        if (b->vm_proc_end[v] < prev || b->vm_proc_end[v] > p1) {
          why[n] = kBadVm, where[n] = v;
          return n;
        }
        prev = b->vm_proc_end[v];
      }
      uint32_t cprev = b->ctr_off[n];
      for (uint32_t q = b->pod_off[n]; q < b->pod_off[n + 1]; ++q) {
        if (b->pod_ctr_end[q] < cprev || b->pod_ctr_end[q] > b->ctr_off[n + 1]) {
          why[n] = kBadPod, where[n] = q;
          return n;
        }
        cprev = b->pod_ctr_end[q];
      }
    }
    return N;
  });
  if (bad_node < N) {
    const unsigned i = where[bad_node], n = static_cast<unsigned>(bad_node);
    if (why[bad_node] == kBadCtr) return fail(ctx, KACC_EINVAL, "ctr_proc_end[%u] outside node %u rows", i, n);
    if (why[bad_node] == kBadVm) return fail(ctx, KACC_EINVAL, "vm_proc_end[%u] outside node %u rows", i, n);
    return fail(ctx, KACC_EINVAL, "pod_ctr_end[%u] outside node %u containers", i, n);
  }
  if ((rc = check_slots(ctx, "proc_slot", b->proc_slot, b->n_procs, ctx->cfg.proc_slots))) return rc;
  if ((rc = check_slots(ctx, "ctr_slot", b->ctr_slot, b->n_ctrs, ctx->cfg.ctr_slots))) return rc;
  if ((rc = check_slots(ctx, "vm_slot", b->vm_slot, b->n_vms, ctx->cfg.vm_slots))) return rc;
  if ((rc = check_slots(ctx, "pod_slot", b->pod_slot, b->n_pods, ctx->cfg.pod_slots))) return rc;
  if (b->node_proc_span) {
    const uint64_t bad = par_first(N, [&](uint64_t nb, uint64_t ne) -> uint64_t {
      for (uint64_t n = nb; n < ne; ++n)
        for (uint32_t r = b->proc_off[n]; r < b->proc_off[n + 1]; ++r) {
          const uint32_t sl = b->proc_slot[r] & KACC_SLOT_MASK;
          if (sl < b->node_proc_span[2 * n] || sl > b->node_proc_span[2 * n + 1]) return n;
        }
      return N;
    });
    if (bad < N)
      return fail(ctx, KACC_EINVAL, "a proc_slot of node %u lies outside its node_proc_span",
                  static_cast<unsigned>(bad));
  }
  if (b->node_order) {
    std::vector<uint8_t> seen(N, 0);
    for (uint32_t i = 0; i < N; ++i) {
      if (b->node_order[i] >= N || seen[b->node_order[i]])
        return fail(ctx, KACC_EINVAL, "node_order is not a permutation");
      seen[b->node_order[i]] = 1;
    }
  }
  return KACC_OK;
}

}  // extern "C"

namespace {

// Pointer fields of kacc_interval with their element size and count rule.
enum BatchDim { kDimN, kDimNZ, kDimN1, kDim2N, kDimP, kDimC, kDimV, kDimQ };
struct BatchField {
  size_t off;  // offsetof(kacc_interval, field)
  uint32_t elem;
  BatchDim dim;
  bool optional;
};
#define KACC_BF(f, e, d, o) BatchField{offsetof(kacc_interval, f), e, d, o}
const BatchField kBatchFields[] = {
    KACC_BF(node_ts_ns, 8, kDimN, false),       KACC_BF(node_usage_ratio, 8, kDimN, false),
    KACC_BF(node_status, 4, kDimN, true),       KACC_BF(node_cpu_delta, 8, kDimN, true),
    KACC_BF(node_order, 4, kDimN, true),        KACC_BF(node_proc_span, 4, kDim2N, true),
    KACC_BF(zone_energy, 8, kDimNZ, false),     KACC_BF(zone_max, 8, kDimNZ, false),
    KACC_BF(proc_off, 4, kDimN1, false),        KACC_BF(ctr_off, 4, kDimN1, false),
    KACC_BF(vm_off, 4, kDimN1, false),          KACC_BF(pod_off, 4, kDimN1, false),
    KACC_BF(proc_cpu_delta, 8, kDimP, false),   KACC_BF(proc_slot, 4, kDimP, false),
    KACC_BF(ctr_proc_end, 4, kDimC, false),     KACC_BF(ctr_slot, 4, kDimC, false),
    KACC_BF(vm_proc_end, 4, kDimV, false),      KACC_BF(vm_slot, 4, kDimV, false),
    KACC_BF(pod_ctr_end, 4, kDimQ, false),      KACC_BF(pod_slot, 4, kDimQ, false),
};
#undef KACC_BF

const void *&field_ptr(kacc_interval &b, const BatchField &f) {
  return *reinterpret_cast<const void **>(reinterpret_cast<char *>(&b) + f.off);
}

size_t field_bytes(const BatchField &f, uint64_t N, uint64_t P, uint64_t C, uint64_t V, uint64_t Q, uint64_t Z) {
  uint64_t n = 0;
  switch (f.dim) {
    case kDimN: n = N; break;
    case kDimNZ: n = N * Z; break;
    case kDimN1: n = N + 1; break;
    case kDim2N: n = 2 * N; break;
    case kDimP: n = P; break;
    case kDimC: n = C; break;
    case kDimV: n = V; break;
    case kDimQ: n = Q; break;
  }
  return static_cast<size_t>(n * f.elem);
}

}  // namespace

extern "C" {

int kacc_batch_alloc(kacc_ctx *ctx, const kacc_shape *shape, kacc_batch **out, kacc_interval **views) {
  if (!ctx || !shape || !out || !views) return KACC_EINVAL;
  *out = nullptr;
  *views = nullptr;
  if (shape->intervals == 0) return fail(ctx, KACC_EINVAL, "a batch needs >= 1 interval");
  if (shape->n_nodes > ctx->cfg.nodes) return fail(ctx, KACC_EINVAL, "n_nodes exceeds capacity");
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  auto *bt = new kacc_batch;
  bt->cap = *shape;
  const uint64_t Z = ctx->cfg.zones, K = shape->intervals;
  bt->host.assign(K, kacc_interval{});
  bt->dev.assign(K, kacc_interval{});
  hipError_t e = hipEventCreateWithFlags(&bt->copied, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&bt->done, hipEventDisableTiming);
  if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void **>(&bt->h_err), sizeof(uint32_t), hipHostMallocDefault);
  if (e != hipSuccess) {
    kacc_batch_free(ctx, bt);
    return fail(ctx, KACC_EHIP, "batch events: %s", hipGetErrorString(e));
  }
  *bt->h_err = 0;
  for (uint64_t k = 0; k < K; ++k) {
    kacc_interval &h = bt->host[k], &d = bt->dev[k];
    h.n_nodes = d.n_nodes = shape->n_nodes;
    h.n_procs = d.n_procs = shape->n_procs;
    h.n_ctrs = d.n_ctrs = shape->n_ctrs;
    h.n_vms = d.n_vms = shape->n_vms;
    h.n_pods = d.n_pods = shape->n_pods;
    for (const BatchField &f : kBatchFields) {
      const size_t bytes = std::max<size_t>(
          field_bytes(f, shape->n_nodes, shape->n_procs, shape->n_ctrs, shape->n_vms, shape->n_pods, Z), 8);
      void *hp = nullptr, *dp = nullptr;
      e = hipHostMalloc(&hp, bytes, hipHostMallocDefault);
      if (hp) bt->allocs.push_back(hp);
      if (e == hipSuccess) e = hipMalloc(&dp, bytes);
      if (dp) bt->dev_allocs.push_back(dp);
      if (e != hipSuccess) {
        kacc_batch_free(ctx, bt);
        return fail(ctx, KACC_ENOMEM, "batch allocation (%zu B): %s", bytes, hipGetErrorString(e));
      }
      std::memset(hp, 0, bytes);
      field_ptr(h, f) = hp;
      field_ptr(d, f) = dp;
    }
  }
  bt->orig = bt->host;
  *out = bt;
  *views = bt->host.data();
  return KACC_OK;
}

// Two (or more) batches pipeline: the H2D copies of a batch run on the copy
// stream while the previous batch's interval kernels run on the context
// stream; the kernels wait for their own copies (event), and a batch's device
// buffers are not overwritten before its previous kernels have read them.
int kacc_batch_submit(kacc_ctx *ctx, kacc_batch *bt) {
  if (!ctx || !bt) return KACC_EINVAL;
  const uint32_t K = bt->cap.intervals;
  const uint64_t Z = ctx->cfg.zones;
  std::vector<kacc_interval> dv(K);
  uint64_t max_nodes = 0, max_procs = 0, max_pods = 0;
  for (uint32_t k = 0; k < K; ++k) {
    kacc_interval &h = bt->host[k];
    // a view's sizes may shrink (only the used prefix is copied), never grow
    if (h.n_nodes > bt->cap.n_nodes || h.n_procs > bt->cap.n_procs || h.n_ctrs > bt->cap.n_ctrs ||
        h.n_vms > bt->cap.n_vms || h.n_pods > bt->cap.n_pods)
      return fail(ctx, KACC_EINVAL, "interval %u: view sizes exceed the batch shape", k);
    for (const BatchField &f : kBatchFields) {
      const void *p = field_ptr(h, f);
      if (p != field_ptr(bt->orig[k], f) && !(f.optional && p == nullptr))
        return fail(ctx, KACC_EINVAL, "interval %u: a view pointer was moved (views are fixed)", k);
    }
    int rc = (h.flags & KACC_F_TRUSTED_LAYOUT) ? check_shape(ctx, &h) : kacc_validate_host(ctx, &h);
    if (rc != KACC_OK) return K > 1 ? fail(ctx, rc, "interval %u: %s", k, std::string(ctx->err).c_str()) : rc;
    dv[k] = bt->dev[k];
    dv[k].n_nodes = h.n_nodes;
    dv[k].n_procs = h.n_procs;
    dv[k].n_ctrs = h.n_ctrs;
    dv[k].n_vms = h.n_vms;
    dv[k].n_pods = h.n_pods;
    dv[k].flags = (h.flags & ~KACC_F_TRUSTED_LAYOUT) | (h.n_nodes ? node_size_flags(h) : 0u);
    dv[k].pod_export = h.pod_export;  // device outputs the caller owns, passed through
    dv[k].node_export = h.node_export;
    dv[k].pod_export_pos = h.pod_export_pos;  // a device input, like the exports
    for (const BatchField &f : kBatchFields)  // honour optional arrays the caller switched off
      if (!field_ptr(h, f)) field_ptr(dv[k], f) = nullptr;
    max_nodes = std::max<uint64_t>(max_nodes, h.n_nodes);
    max_procs = std::max<uint64_t>(max_procs, h.n_procs);
    max_pods = std::max<uint64_t>(max_pods, h.n_pods);
  }
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  if (bt->submitted) KACC_HIP(ctx, hipStreamWaitEvent(ctx->copy_stream, bt->done, 0));
  for (uint32_t k = 0; k < K; ++k) {
    kacc_interval &h = bt->host[k];
    for (const BatchField &f : kBatchFields) {
      const void *hp = field_ptr(h, f);
      const size_t bytes = field_bytes(f, h.n_nodes, h.n_procs, h.n_ctrs, h.n_vms, h.n_pods, Z);
      if (!hp || !bytes || !h.n_nodes) continue;  // switched off, or empty
      KACC_HIP(ctx, hipMemcpyAsync(const_cast<void *>(field_ptr(bt->dev[k], f)), hp, bytes, hipMemcpyHostToDevice,
                                   ctx->copy_stream));
    }
  }
  KACC_HIP(ctx, hipEventRecord(bt->copied, ctx->copy_stream));
  int rc = ensure_items(ctx, max_nodes, max_procs, max_pods);
  if (rc != KACC_OK) return rc;
  KACC_HIP(ctx, hipStreamWaitEvent(ctx->stream, bt->copied, 0));
  (void)hipGetLastError();  // clear a stale error of an earlier call
  const kacc::DevState ds = dev_state(ctx);
  for (uint32_t k = 0; k < K; ++k)
    if (dv[k].n_nodes) launch(ctx->cfg.zones, dv[k], ds, ctx->stream);
  KACC_HIP(ctx, hipGetLastError());
  KACC_HIP(ctx, hipMemcpyAsync(bt->h_err, ctx->d_err, sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
  KACC_HIP(ctx, hipEventRecord(bt->done, ctx->stream));
  bt->submitted = true;
  ctx->live_nodes = bt->host[K - 1].n_nodes;
  return KACC_OK;
}

// Waits for this batch only (earlier work on the context stream is done too;
// later submits may still run).  The device error word is per context, so an
// error reported here may come from any interval up to this batch's.
int kacc_batch_wait(kacc_ctx *ctx, kacc_batch *bt) {
  if (!ctx || !bt) return KACC_EINVAL;
  if (!bt->submitted) return KACC_OK;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  KACC_HIP(ctx, hipEventSynchronize(bt->done));
  if (*bt->h_err) {
    *bt->h_err = 0;
    return kacc_sync(ctx, nullptr);  // drains the stream, reports and clears the word
  }
  return KACC_OK;
}

void kacc_batch_free(kacc_ctx *ctx, kacc_batch *bt) {
  if (!bt) return;
  if (ctx) (void)hipSetDevice(ctx->device);
  if (bt->done && bt->submitted) (void)hipEventSynchronize(bt->done);
  for (void *p : bt->allocs) (void)hipHostFree(p);
  for (void *p : bt->dev_allocs) (void)hipFree(p);
  if (bt->copied) (void)hipEventDestroy(bt->copied);
  if (bt->done) (void)hipEventDestroy(bt->done);
  if (bt->h_err) (void)hipHostFree(bt->h_err);
  delete bt;
}


int kacc_table_info(const kacc_ctx *ctx, kacc_table t, uint64_t *elem_bytes, uint64_t *count) {
  if (!ctx || t < 0 || t >= KACC_T_COUNT) return KACC_EINVAL;
  if (elem_bytes) *elem_bytes = kTables[t].elem;
  if (count) *count = ctx->counts[t];
  return KACC_OK;
}

int kacc_table_device_ptr(kacc_ctx *ctx, kacc_table t, void **dev_ptr) {
  if (!ctx || t < 0 || t >= KACC_T_COUNT || !dev_ptr) return KACC_EINVAL;
  if (kTables[t].derived) {
    *dev_ptr = nullptr;
    return fail(ctx, KACC_EINVAL, "table %d is derived on read (no device storage): see kacc_table_download", (int)t);
  }
  *dev_ptr = ctx->tables[t];
  return KACC_OK;
}

int kacc_table_row_stride(const kacc_ctx *ctx, kacc_table t, uint64_t *stride) {
  if (!ctx || t < 0 || t >= KACC_T_COUNT || !stride) return KACC_EINVAL;
  const uint64_t w = kTables[t].zoned ? ctx->cfg.zones : 1;
  *stride = pod_paired(t) ? 2 * w : w;
  return KACC_OK;
}

static int table_copy(kacc_ctx *ctx, kacc_table t, uint64_t first, uint64_t count, void *host,
                      bool down) {
  if (!ctx || t < 0 || t >= KACC_T_COUNT || (!host && count)) return KACC_EINVAL;
  if (first > ctx->counts[t] || count > ctx->counts[t] - first)
    return fail(ctx, KACC_EINVAL, "table %d range [%llu,+%llu) outside %llu", (int)t,
                (unsigned long long)first, (unsigned long long)count,
                (unsigned long long)ctx->counts[t]);
  if (kTables[t].derived && !down)
    return fail(ctx, KACC_EINVAL, "table %d is derived on read and cannot be uploaded", (int)t);
  if (!count) return KACC_OK;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  KACC_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (kTables[t].derived || pod_paired(t)) {  // derived / inside the pod records: through a dense scratch range
    void *tmp = nullptr;
    KACC_HIP(ctx, hipMalloc(&tmp, count * 8));
    hipError_t e = hipSuccess;
    int rc = KACC_OK;
    if (down) {
      rc = kacc_internal_dense_range(ctx, t, first, count, tmp, ctx->stream);
      e = rc == KACC_OK ? hipStreamSynchronize(ctx->stream) : hipSuccess;
      if (rc == KACC_OK && e == hipSuccess) e = hipMemcpy(host, tmp, count * 8, hipMemcpyDeviceToHost);
    } else {
      e = hipMemcpy(tmp, host, count * 8, hipMemcpyHostToDevice);
      if (e == hipSuccess) rc = kacc_internal_pod_scatter(ctx, t, first, count, tmp, ctx->stream);
      if (rc == KACC_OK && e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    }
    (void)hipFree(tmp);
    if (rc != KACC_OK) return rc;
    if (e != hipSuccess) return fail(ctx, KACC_EHIP, "table %d: %s", (int)t, hipGetErrorString(e));
    return KACC_OK;
  }
  char *dev = static_cast<char *>(ctx->tables[t]) + first * kTables[t].elem;
  const size_t bytes = count * kTables[t].elem;
  if (down)
    KACC_HIP(ctx, hipMemcpy(host, dev, bytes, hipMemcpyDeviceToHost));
  else
    KACC_HIP(ctx, hipMemcpy(dev, host, bytes, hipMemcpyHostToDevice));
  return KACC_OK;
}

int kacc_table_download(kacc_ctx *ctx, kacc_table t, uint64_t first, uint64_t count, void *host_dst) {
  return table_copy(ctx, t, first, count, host_dst, true);
}

int kacc_table_upload(kacc_ctx *ctx, kacc_table t, uint64_t first, uint64_t count,
                      const void *host_src) {
  return table_copy(ctx, t, first, count, const_cast<void *>(host_src), false);
}

int kacc_table_read(kacc_ctx *ctx, kacc_table t, uint64_t first, uint64_t count, void *dev_dst, void *stream) {
  if (!ctx || t < 0 || t >= KACC_T_COUNT || (!dev_dst && count)) return KACC_EINVAL;
  if (first > ctx->counts[t] || count > ctx->counts[t] - first)
    return fail(ctx, KACC_EINVAL, "table %d range [%llu,+%llu) outside %llu", (int)t, (unsigned long long)first,
                (unsigned long long)count, (unsigned long long)ctx->counts[t]);
  if (!count) return KACC_OK;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  if (kTables[t].derived || pod_paired(t)) return kacc_internal_dense_range(ctx, t, first, count, dev_dst, st);
  KACC_HIP(ctx, hipMemcpyAsync(dev_dst, static_cast<const char *>(ctx->tables[t]) + first * kTables[t].elem,
                               count * kTables[t].elem, hipMemcpyDeviceToDevice, st));
  return KACC_OK;
}

int kacc_namespace_totals(kacc_ctx *ctx, uint32_t n_ns, const uint32_t *off, const uint32_t *slots,
                          uint64_t *out_energy, double *out_power, void *stream) {
  if (!ctx) return KACC_EINVAL;
  if (!n_ns) return KACC_OK;
  if (!off || !slots || !out_energy || !out_power) return fail(ctx, KACC_EINVAL, "NULL argument");
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  (void)hipGetLastError();  // clear a stale error of an earlier call
  switch (ctx->cfg.zones) {
    case 1: launch_ns<1>(n_ns, off, slots, ctx, out_energy, out_power, st); break;
    case 2: launch_ns<2>(n_ns, off, slots, ctx, out_energy, out_power, st); break;
    case 3: launch_ns<3>(n_ns, off, slots, ctx, out_energy, out_power, st); break;
    case 4: launch_ns<4>(n_ns, off, slots, ctx, out_energy, out_power, st); break;
    case 5: launch_ns<5>(n_ns, off, slots, ctx, out_energy, out_power, st); break;
    case 6: launch_ns<6>(n_ns, off, slots, ctx, out_energy, out_power, st); break;
    case 7: launch_ns<7>(n_ns, off, slots, ctx, out_energy, out_power, st); break;
    default: launch_ns<8>(n_ns, off, slots, ctx, out_energy, out_power, st); break;
  }
  KACC_HIP(ctx, hipGetLastError());
  return KACC_OK;
}

int kacc_internal_cluster_partials(kacc_ctx *ctx, uint32_t n_ns, const uint32_t *off, const uint32_t *slots,
                                   uint64_t *out_energy, double *out_power, uint64_t *node_energy, double *node_power,
                                   void *stream) {
  return kacc_internal_export_partials(ctx, n_ns, off, slots, nullptr, 0, nullptr, 0, 0, out_energy, out_power,
                                       node_energy, node_power, stream);
}

int kacc_internal_export_partials(kacc_ctx *ctx, uint32_t n_ns, const uint32_t *off, const uint32_t *rows,
                                  const uint64_t *pod_export, uint64_t n_pods, const uint64_t *node_export,
                                  uint64_t n_nodes, int from_exports, uint64_t *out_energy, double *out_power,
                                  uint64_t *node_energy,
                                  double *node_power, void *stream) {
  if (!ctx) return KACC_EINVAL;
  const kacc::TimingScope timing(ctx);
  if (n_ns && (!off || !rows || !out_energy || !out_power)) return fail(ctx, KACC_EINVAL, "NULL argument");
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  const uint64_t Z = ctx->cfg.zones;
  // the nodes of the last interval run on the context (a node that left the
  // batch stops exporting, so PromQL's sum drops it; a fresh context sums none);
  // from an export: its n_nodes rows (an empty shard's export: none, never the
  // tables' stale nodes)
  if (from_exports && n_nodes && !node_export) return fail(ctx, KACC_EINVAL, "node export is NULL");
  const uint64_t live = from_exports ? n_nodes : std::min<uint64_t>(ctx->live_nodes, ctx->cfg.nodes);
  const uint32_t *slots = rows;
  // one block per output value (no live node: they write zero totals)
  const uint32_t node_blocks = node_energy ? static_cast<uint32_t>(5 * Z) : 0u;
  const kacc::NodeTotalsArgs na = node_totals_args(ctx, live, node_export, node_energy, node_power);
  if (!n_ns && !node_blocks) return KACC_OK;
  (void)hipGetLastError();
#define KACC_PARTIALS(Z_)                                                                                  \
  launch_cluster_partials<Z_>(n_ns, off, slots, ctx, out_energy, out_power, na, node_blocks, st, pod_export, \
                              n_pods)
  switch (ctx->cfg.zones) {
    case 1: KACC_PARTIALS(1); break;
    case 2: KACC_PARTIALS(2); break;
    case 3: KACC_PARTIALS(3); break;
    case 4: KACC_PARTIALS(4); break;
    case 5: KACC_PARTIALS(5); break;
    case 6: KACC_PARTIALS(6); break;
    case 7: KACC_PARTIALS(7); break;
    default: KACC_PARTIALS(8); break;
  }
#undef KACC_PARTIALS
  KACC_HIP(ctx, hipGetLastError());
  return KACC_OK;
}

int kacc_run_export_sums(kacc_ctx *ctx, const kacc_export_sums *x, void *stream) {
  if (!ctx) return KACC_EINVAL;
  const kacc::TimingScope timing(ctx);
  kacc::SumsArgs sa;
  int rc = sums_args(ctx, x, kacc::kBlock, sa);
  if (rc != KACC_OK) return rc;
  if (!sa.n_ns && !sa.node_blocks) return KACC_OK;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  (void)hipGetLastError();
#define KACC_XSUMS(Z_)                                                                                        \
  launch_cluster_partials<Z_>(sa.n_ns, sa.off, sa.ordered ? nullptr : sa.rows, ctx, sa.out_e, sa.out_p, sa.na, \
                              sa.node_blocks, st, sa.pe, sa.n_pods, sa.ordered != 0)
  switch (ctx->cfg.zones) {
    case 1: KACC_XSUMS(1); break;
    case 2: KACC_XSUMS(2); break;
    case 3: KACC_XSUMS(3); break;
    case 4: KACC_XSUMS(4); break;
    case 5: KACC_XSUMS(5); break;
    case 6: KACC_XSUMS(6); break;
    case 7: KACC_XSUMS(7); break;
    default: KACC_XSUMS(8); break;
  }
#undef KACC_XSUMS
  KACC_HIP(ctx, hipGetLastError());
  return KACC_OK;
}

int kacc_run_interval_sums(kacc_ctx *ctx, const kacc_interval *b, const kacc_export_sums *prev, void *stream) {
  if (!ctx) return KACC_EINVAL;
  if (!prev) return kacc_run_interval(ctx, b, stream);
  const kacc::TimingScope timing(ctx);
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  int rc = check_shape(ctx, b);
  if (rc != KACC_OK) return rc;
  kacc::SumsArgs sa;
  if ((rc = sums_args(ctx, prev, kacc::kTpb<0>, sa)) != KACC_OK) return rc;
  const uint64_t Z = ctx->cfg.zones;
  // the sums read an EARLIER interval's exports while this one writes its own, and the
  // sums' outputs are written in the same launch: no output may alias an export of
  // either interval (a silent race inside one launch otherwise)
  if (overlaps(prev->pod_export, 16 * Z * prev->n_pods, b->pod_export, 16 * Z * b->n_pods) ||
      overlaps(prev->node_export, 40 * Z * prev->n_nodes, b->node_export, 40 * Z * b->n_nodes) ||
      overlaps(prev->pod_export, 16 * Z * prev->n_pods, b->node_export, 40 * Z * b->n_nodes) ||
      overlaps(prev->node_export, 40 * Z * prev->n_nodes, b->pod_export, 16 * Z * b->n_pods))
    return fail(ctx, KACC_EINVAL, "export sums: the exports read overlap the exports this interval writes "
                                  "(double-buffer them)");
  {
    const struct { const void *p; uint64_t bytes; } outs[4] = {
        {prev->out_energy, 8 * Z * prev->n_ns}, {prev->out_power, 8 * Z * prev->n_ns},
        {prev->out_node_energy, prev->node_export ? 16 * Z : 0}, {prev->out_node_power, prev->node_export ? 24 * Z : 0}};
    const struct { const void *p; uint64_t bytes; } ins[4] = {
        {prev->pod_export, 16 * Z * prev->n_pods}, {prev->node_export, 40 * Z * prev->n_nodes},
        {b->pod_export, 16 * Z * b->n_pods}, {b->node_export, 40 * Z * b->n_nodes}};
    for (const auto &o : outs)
      for (const auto &e : ins)
        if (overlaps(o.p, o.bytes, e.p, e.bytes))
          return fail(ctx, KACC_EINVAL, "export sums: an output of the sums overlaps an export of this launch");
  }
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  const bool fuse = b->n_nodes > 0 && !(b->flags & KACC_F_SMALL_NODES) &&
                    !(sa.node_blocks && sa.na.n_nodes > kacc::kColSplitFrom) &&
                    (sa.n_ns || sa.node_blocks) &&
                    static_cast<uint64_t>(b->n_nodes) + sa.node_blocks + sa.ns_blocks <= 0x7fffffffull;
  if (!fuse) {  // the interval, then the sums as a launch of their own (the same results)
    if ((rc = run_one(ctx, b, st)) != KACC_OK) return rc;
    return kacc_run_export_sums(ctx, prev, st);  // inside this call's timing scope
  }
  if ((rc = ensure_items(ctx, b->n_nodes, b->n_procs, b->n_pods)) != KACC_OK) return rc;
  (void)hipGetLastError();  // clear a stale error of an earlier call
  launch_fused_z(ctx->cfg.zones, *b, dev_state(ctx), sa, st);
  KACC_HIP(ctx, hipGetLastError());
  ctx->live_nodes = b->n_nodes;
  return KACC_OK;
}

int kacc_internal_derived_power(kacc_ctx *ctx, int t, uint64_t first, uint64_t count, double *out, void *stream) {
  if (!ctx) return KACC_EINVAL;
  const int kind = kacc_derived_kind(t);
  if (kind < 0) return fail(ctx, KACC_EINVAL, "table %d is not derived", t);
  if (!count) return KACC_OK;
  if (!out) return fail(ctx, KACC_EINVAL, "NULL argument");
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  const uint32_t Z = ctx->cfg.zones;
  // one lane per slot, kPowWaves x 64 slots per workgroup, no grid-stride loop (a loop would
  // serialise the lanes' round trips)
  const uint64_t slots = (first + count - 1) / Z - first / Z + 1, per_block = 64ull * kacc::kPowWaves;
  const dim3 grid(static_cast<uint32_t>(std::min<uint64_t>((slots + per_block - 1) / per_block, 0x7fffffffull)));
  const kacc::ProcDerive d = kacc_derive(ctx, static_cast<kacc_kind>(kind));
  (void)hipGetLastError();
  switch (Z) {
    case 1: hipLaunchKernelGGL(kacc::proc_power_kernel<1>, grid, dim3(kacc::kBlock), 0, st, d, first, count, out); break;
    case 2: hipLaunchKernelGGL(kacc::proc_power_kernel<2>, grid, dim3(kacc::kBlock), 0, st, d, first, count, out); break;
    case 3: hipLaunchKernelGGL(kacc::proc_power_kernel<3>, grid, dim3(kacc::kBlock), 0, st, d, first, count, out); break;
    case 4: hipLaunchKernelGGL(kacc::proc_power_kernel<4>, grid, dim3(kacc::kBlock), 0, st, d, first, count, out); break;
    case 5: hipLaunchKernelGGL(kacc::proc_power_kernel<5>, grid, dim3(kacc::kBlock), 0, st, d, first, count, out); break;
    case 6: hipLaunchKernelGGL(kacc::proc_power_kernel<6>, grid, dim3(kacc::kBlock), 0, st, d, first, count, out); break;
    case 7: hipLaunchKernelGGL(kacc::proc_power_kernel<7>, grid, dim3(kacc::kBlock), 0, st, d, first, count, out); break;
    default: hipLaunchKernelGGL(kacc::proc_power_kernel<8>, grid, dim3(kacc::kBlock), 0, st, d, first, count, out); break;
  }
  KACC_HIP(ctx, hipGetLastError());
  return KACC_OK;
}

int kacc_internal_dense_range(kacc_ctx *ctx, int t, uint64_t first, uint64_t count, void *out, void *stream) {
  if (!ctx) return KACC_EINVAL;
  if (kacc_derived_kind(t) >= 0) return kacc_internal_derived_power(ctx, t, first, count, static_cast<double *>(out), stream);
  if (!count) return KACC_OK;
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  if (!pod_paired(t)) {
    KACC_HIP(ctx, hipMemcpyAsync(out, static_cast<const char *>(ctx->tables[t]) + first * 8, count * 8,
                                 hipMemcpyDeviceToDevice, st));
    return KACC_OK;
  }
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  const uint64_t blocks = (count + kacc::kBlock - 1) / kacc::kBlock;
  (void)hipGetLastError();
  hipLaunchKernelGGL(kacc::pod_pair_copy_kernel, dim3(static_cast<uint32_t>(std::min<uint64_t>(blocks, 65536))),
                     dim3(kacc::kBlock), 0, st, static_cast<uint64_t *>(ctx->tables[t]), ctx->cfg.zones, first, count,
                     static_cast<uint64_t *>(out), 0);
  KACC_HIP(ctx, hipGetLastError());
  return KACC_OK;
}

int kacc_internal_pod_scatter(kacc_ctx *ctx, int t, uint64_t first, uint64_t count, const void *in, void *stream) {
  if (!ctx || !pod_paired(t)) return KACC_EINVAL;
  if (!count) return KACC_OK;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  const uint64_t blocks = (count + kacc::kBlock - 1) / kacc::kBlock;
  (void)hipGetLastError();
  hipLaunchKernelGGL(kacc::pod_pair_copy_kernel, dim3(static_cast<uint32_t>(std::min<uint64_t>(blocks, 65536))),
                     dim3(kacc::kBlock), 0, st, static_cast<uint64_t *>(ctx->tables[t]), ctx->cfg.zones, first, count,
                     const_cast<uint64_t *>(static_cast<const uint64_t *>(in)), 1);
  KACC_HIP(ctx, hipGetLastError());
  return KACC_OK;
}

uint64_t kacc_intervals_bytes(uint32_t Z, uint64_t N, uint64_t P, uint64_t C, uint64_t V, uint64_t Q, uint32_t K,
                              int carried, uint32_t flags) {
  // K intervals of these sizes.  Carried (intervals_carry_kernel,
  // steady state): the engine state a node / row / aggregate reads back — zone
  // counters and totals, has_prev / ts, previous workload totals and CPU totals —
  // is read once, then carried on chip.
  if (!carried) return static_cast<uint64_t>(K) * kacc_interval_bytes(Z, N, P, C, V, Q, flags);
  if (K == 0) return 0;
  const uint64_t state_once = N * (12 + 24ull * Z) + P * 8ull * Z + C * (8 + 8ull * Z) + V * 8ull * Z +
                              Q * (8 + 8ull * Z);
  return static_cast<uint64_t>(K) * kacc_interval_bytes(Z, N, P, C, V, Q, flags) -
         static_cast<uint64_t>(K - 1) * state_once;
}

uint64_t kacc_interval_bytes(uint32_t Z, uint64_t N, uint64_t P, uint64_t C, uint64_t V,
                             uint64_t Q, uint32_t flags) {
  // minimal HBM bytes of one interval_kernel launch.
  const uint64_t node = 76 + 96ull * Z;
  // Δ 8 + slot 4 in, previous totals 8Z in; totals 8Z + ratio 8 + node 4 out (the node
  // only for NEW rows under KACC_F_STABLE_SLOT_NODES: not counted)
  // (small_kernel, KACC_F_SMALL_NODES, writes it anyway: KACC_SMALL_STABLE)
  const bool stable = (flags & KACC_F_STABLE_SLOT_NODES) && (KACC_SMALL_STABLE || !(flags & KACC_F_SMALL_NODES));
  const uint64_t proc = (stable ? 20 : 24) + 16ull * Z;
  // container: end 4 + slot 4 + previous CPU total 8 in, Δ 8 + total 8 out; previous
  // energies 8Z in, energies 8Z + ratio 8 + node 4 out (power derived since ABI 3)
  const uint64_t ctr = 44 + 16ull * Z;
  const uint64_t vm = 28 + 16ull * Z;  // end 4 + slot 4 in, Δ 8 out; 16Z + 12 as a container
  const uint64_t pod = 32 + 24ull * Z;
  return N * node + P * proc + C * ctr + V * vm + Q * pod;
}

// The carry kernel writes no exports (kacc_run_intervals never launches it for a
// batch that asks for them): its debug entry points refuse such batches too.
static int reject_carry_exports(kacc_ctx *ctx, const kacc_interval *b, uint32_t count) {
  for (uint32_t k = 0; k < count; ++k)
    if (b[k].pod_export || b[k].node_export)
      return fail(ctx, KACC_EINVAL, "interval %u: the carry kernel writes no pod / node exports", k);
  return KACC_OK;
}

// Internal (kacc_debug.h): timing ablations of the one-launch K-interval kernel.
int kacc_debug_carry_stamps(kacc_ctx *ctx, const kacc_interval *b, uint32_t count, void *stream, int variant,
                            uint64_t *d_out) {
  if (!ctx || !b || count == 0 || !d_out) return KACC_EINVAL;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  if (ctx->cfg.zones != 2) return fail(ctx, KACC_EINVAL, "carry variants are built for Z = 2");
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  int rc = reject_carry_exports(ctx, b, count);
  if (rc != KACC_OK) return rc;
  rc = stage_batches(ctx, b, count, st);
  if (rc != KACC_OK) return rc;
  kacc::DevState ds = dev_state(ctx);
  ds.items = reinterpret_cast<kacc::ChunkItem *>(d_out);  // [n_nodes][8 waves][8 phases] u64
  const bool medium = all_medium(b, count);
  (void)hipGetLastError();
  if (variant == 0)
    launch_carry<16>(2, medium, ctx->d_batches, count, b[0].n_nodes, ds, st);
  else if (variant == 2)
    launch_carry<18>(2, medium, ctx->d_batches, count, b[0].n_nodes, ds, st);
  else
    return fail(ctx, KACC_EINVAL, "stamp variant %d not built", variant);
  KACC_HIP(ctx, hipGetLastError());
  return KACC_OK;
}

int kacc_debug_run_intervals_variant(kacc_ctx *ctx, const kacc_interval *b, uint32_t count, void *stream,
                                     int variant) {
  if (!ctx || !b || count == 0) return KACC_EINVAL;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  if (ctx->cfg.zones != 2) return fail(ctx, KACC_EINVAL, "carry variants are built for Z = 2");
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  int rc = reject_carry_exports(ctx, b, count);
  if (rc != KACC_OK) return rc;
  rc = stage_batches(ctx, b, count, st);
  if (rc != KACC_OK) return rc;
  const kacc::DevState ds = dev_state(ctx);
  const bool medium = all_medium(b, count);
  const uint32_t nn = b[0].n_nodes;
  (void)hipGetLastError();
  switch (variant) {
    case 0: launch_carry<0>(2, medium, ctx->d_batches, count, nn, ds, st); break;
    case 1: launch_carry<1>(2, medium, ctx->d_batches, count, nn, ds, st); break;
    case 2: launch_carry<2>(2, medium, ctx->d_batches, count, nn, ds, st); break;
    case 4: launch_carry<4>(2, medium, ctx->d_batches, count, nn, ds, st); break;
    case 5: launch_carry<5>(2, medium, ctx->d_batches, count, nn, ds, st); break;
    case 8: launch_carry<8>(2, medium, ctx->d_batches, count, nn, ds, st); break;
    case 32: launch_carry<32>(2, medium, ctx->d_batches, count, nn, ds, st); break;
    default: return fail(ctx, KACC_EINVAL, "variant %d not built", variant);
  }
  KACC_HIP(ctx, hipGetLastError());
  return KACC_OK;
}

// Internal (kacc_debug.h): timing ablations of the interval kernel.  A variant
// other than 0 does NOT compute the reference semantics.
int kacc_debug_interval_stamps(kacc_ctx *ctx, const kacc_interval *b, void *stream, uint64_t *d_out) {
  if (!ctx || !d_out) return KACC_EINVAL;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  int rc = check_shape(ctx, b);
  if (rc != KACC_OK) return rc;
  if (ctx->cfg.zones != 4) return fail(ctx, KACC_EINVAL, "stamps are built for Z = 4");
  if (b->n_nodes == 0) return KACC_OK;
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  if ((rc = ensure_items(ctx, b->n_nodes, b->n_procs, b->n_pods)) != KACC_OK) return rc;
  (void)hipGetLastError();
  kacc::DevState ds = dev_state(ctx);
  ds.stamps = d_out;
  launch_zv<4, kacc::kVarStamps>(*b, ds, st);
  KACC_HIP(ctx, hipGetLastError());
  ctx->live_nodes = b->n_nodes;
  return KACC_OK;
}

int kacc_debug_run_variant(kacc_ctx *ctx, const kacc_interval *b, void *stream, int variant) {
  if (!ctx) return KACC_EINVAL;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  int rc = check_shape(ctx, b);
  if (rc != KACC_OK) return rc;
  if (b->n_nodes == 0) {  // an emptied batch: no node of it counts in the cluster totals
    ctx->live_nodes = 0;
    return KACC_OK;
  }
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  if ((rc = ensure_items(ctx, b->n_nodes, b->n_procs, b->n_pods)) != KACC_OK) return rc;
  (void)hipGetLastError();  // clear a stale error of an earlier call
  if (!launch_variant(ctx->cfg.zones, variant, *b, dev_state(ctx), st))
    return fail(ctx, KACC_EINVAL, "variant %d not built for Z=%u", variant, ctx->cfg.zones);
  KACC_HIP(ctx, hipGetLastError());
  return KACC_OK;
}

}  // extern "C"
