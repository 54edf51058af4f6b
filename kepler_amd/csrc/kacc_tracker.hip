// Terminated-workload trackers on the device, one per node.
//
// Reference: TerminatedResourceTracker (internal/monitor/
// terminated_resource_tracker.go): a min-heap of the max_size highest-energy
// terminated workloads; Add() drops a disabled tracker (:82), a tracked ID
// (:90), energy below the threshold (:102), pushes below capacity (:116) and
// evicts the minimum for a strictly higher energy at capacity (:124).  Every
// node's PowerMonitor owns its own tracker (monitor.go:123-144): it adds the
// terminated workloads of that node's previous snapshot (process.go:87-99)
// and is cleared after that node's export (process.go:80-84).  So the fleet
// engine keeps one bounded set PER NODE — the top max_size of that node
// only — never a fleet-wide top-N.
//
// One interval's batch (the slot join's per-node terminated segments, values
// read from the kind's state tables) is added as Go would add it in the map
// order "descending target-zone energy, then slot".  In that order a node's
// heap keeps the max_size best of (tracked ∪ batch), ties at the boundary
// going to tracked items first (eviction needs a strictly higher energy) and
// then to the batch order.  Each node's set is kept sorted (energy desc, then
// insertion order), so one add is, per node (one wavefront each):
//   filter  threshold, "beats the current minimum" when full, not tracked —
//           in chunks of 64 candidates in slot order (equivalent, since the
//           batch order breaks ties by slot)
//   sort    survivors by (energy desc, slot) — bitonic across the lanes
//   merge   ranks by binary search (tracked i -> i + #survivors strictly
//           above; survivor j -> j + #tracked at or above), then in place:
//           tracked items only move to later positions, so they are moved
//           in blocks of 64 from the end (a block's loads before its stores)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "kacc_derive.hpp"
#include "kacc_internal.hpp"

namespace kacc {
namespace trk {

constexpr int kThreads = 256;
constexpr uint32_t kSetLds = 512;  // tracked target-zone energies staged in LDS up to this set size
constexpr uint32_t kErrCap = 1u << 10;  // unlimited tracker past its per-node capacity

struct Args {
  const uint64_t *tab_e;
  const double *tab_p;  // NULL for processes / containers / VMs: power derived (kacc_derive.hpp) from pd
  ProcDerive pd;
  uint64_t min_e;
  int64_t max_size;
  uint32_t Z, z0, cap, n_nodes;
  uint32_t tab_stride;  // words between two slots' rows: Z (2Z for pods: energy | power records)
  const uint32_t *slot_off;
  const uint64_t *term_key;
  const uint32_t *term_slot;
  const uint32_t *term_count;
  uint64_t *set_key;  // [nodes * cap]
  uint64_t *set_e;    // [nodes * cap * Z] frozen per-zone energy
  double *set_p;      // [nodes * cap * Z] frozen per-zone power
  uint32_t *size;     // [nodes]
  uint32_t *err;
};

// One WAVE per node (four nodes per workgroup, no workgroup barriers), 64 candidates per
// chunk (one per lane).  A node's add is one dependent chain — term words -> energies ->
// tracked set -> ranks -> moves -> copies — so it pays in nodes in flight: 32 per CU
// (round 6; the workgroup-per-node kernel it replaces held 5, then 8).  Per wave in LDS:
// the tracked target-zone energies (<= kSetLds, the rank search) and the sorted survivors'
// energies.
constexpr int kWaveNodes = kThreads / 64;
template <uint32_t kZ>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(kZ <= 4 ? 8 : 4))) void node_add_wave_kernel(
    const Args a) {
  __shared__ uint64_t s_te_all[kWaveNodes][kSetLds];
  __shared__ uint64_t s_se_all[kWaveNodes][64];
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
  const uint32_t n = blockIdx.x * kWaveNodes + wv;
  if (n >= a.n_nodes) return;  // wave-uniform
  uint64_t *const s_te = s_te_all[wv];
  uint64_t *const s_se = s_se_all[wv];
  const uint32_t Z = a.Z, z0 = a.z0, cap = a.cap;
  const uint64_t base = static_cast<uint64_t>(n) * cap;
  const uint32_t b0 = a.slot_off[n];
  const uint32_t c = min(a.term_count[n], a.slot_off[n + 1] - b0);
  const uint32_t K = a.max_size > 0 ? static_cast<uint32_t>(a.max_size) : cap;
  uint32_t size = min(a.size[n], cap);
  for (uint32_t c0 = 0; c0 < c; c0 += 64) {
    const uint32_t m0 = min(64u, c - c0);
    const bool full = a.max_size > 0 && size >= K;
    const uint64_t min_full = full ? a.set_e[(base + size - 1) * Z + z0] : 0ull;
    // ---- filter (terminated_resource_tracker.go:90-124) ----------------------------
    uint64_t key = 0, e = 0;
    uint32_t slot = 0;
    bool pass = false;
    if (lane < m0) {
      slot = a.term_slot[b0 + c0 + lane];
      key = a.term_key[b0 + c0 + lane];
      e = a.tab_e[static_cast<uint64_t>(slot) * a.tab_stride + z0];
      pass = e >= a.min_e && !(full && e <= min_full);  // :102, :124
    }
    if (__ballot(pass) == 0) continue;  // the tracked set is neither read nor changed
    const bool lds_set = size <= kSetLds;  // wave-uniform
    for (uint32_t t0 = 0; t0 < size; t0 += 64) {  // :90 already tracked; the energies staged
      const uint32_t t = t0 + lane;
      const uint64_t tk = t < size ? a.set_key[base + t] : 0ull;
      if (lds_set && t < size) s_te[t] = a.set_e[(base + t) * Z + z0];
      const uint32_t tn = min(64u, size - t0);
      const uint32_t tk_lo = static_cast<uint32_t>(tk), tk_hi = static_cast<uint32_t>(tk >> 32);
      for (uint32_t j = 0; j < tn; ++j) {
        const uint64_t kj = (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(tk_hi), j))) << 32) |
                            static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(tk_lo), j));
        pass = pass && key != kj;
      }
    }
    const uint64_t pmask = __ballot(pass);
    const uint32_t m = static_cast<uint32_t>(__popcll(pmask));
    if (m == 0) continue;
    // ---- sort: survivors by (energy desc, slot) = ascending (~e, slot); the others +inf ----
    uint64_t k1 = pass ? ~e : ~0ull;
    uint32_t k2 = pass ? slot : ~0u, ix = lane;
    for (uint32_t sz = 2; sz <= 64; sz <<= 1) {
      for (uint32_t stride = sz >> 1; stride > 0; stride >>= 1) {
        const uint64_t b1 = __shfl_xor(k1, static_cast<int>(stride), 64);
        const uint32_t b2 = __shfl_xor(k2, static_cast<int>(stride), 64);
        const uint32_t b3 = __shfl_xor(ix, static_cast<int>(stride), 64);
        const bool up = (lane & sz) == 0, lower = (lane & stride) == 0;
        const bool a_gt = k1 > b1 || (k1 == b1 && k2 > b2), b_gt = b1 > k1 || (b1 == k1 && b2 > k2);
        const bool take = lower == up ? a_gt : b_gt;
        k1 = take ? b1 : k1;
        k2 = take ? b2 : k2;
        ix = take ? b3 : ix;
      }
    }
    // lane j < m: the j-th survivor (its key and slot from lane ix)
    const uint64_t skey = __shfl(key, static_cast<int>(ix), 64);
    const uint32_t sslot = static_cast<uint32_t>(__shfl(static_cast<int>(slot), static_cast<int>(ix), 64));
    const uint64_t se = ~k1;
    s_se[lane] = se;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t new_size = size + m;
    if (a.max_size > 0) {
      new_size = min(new_size, K);
    } else if (new_size > cap) {  // unlimited: per-node capacity exceeded
      if (lane == 0) atomicOr(a.err, kErrCap);
      new_size = cap;
    }
    // ---- ranks (before anything moves): survivor j -> j + #tracked with e >= its e -------
    uint32_t rank = ~0u;
    if (lane < m) {
      uint32_t lo = 0, hi = size;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((lds_set ? s_te[mid] : a.set_e[(base + mid) * Z + z0]) >= se)
          lo = mid + 1;
        else
          hi = mid;
      }
      rank = lane + lo;
    }
    // ---- tracked items move to later ranks, blocks of 64 from the end (a block's loads
    //      complete before its stores: the stores consume them) ------------------------
    if (size > 0) {
      for (int64_t blk = static_cast<int64_t>((size - 1) & ~63u); blk >= 0; blk -= 64) {
        const uint32_t i = static_cast<uint32_t>(blk) + lane;
        if (i >= size) continue;
        const uint64_t ei = lds_set ? s_te[i] : a.set_e[(base + i) * Z + z0];
        uint32_t lo = 0, hi = m;  // i + #survivors with a strictly higher energy (ties: tracked first)
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          if (s_se[mid] > ei)
            lo = mid + 1;
          else
            hi = mid;
        }
        const uint32_t r = i + lo;
        if (r == i || r >= new_size) continue;
        const uint64_t k = a.set_key[base + i];
        uint64_t E[kZ];
        double P[kZ];
        for (uint32_t z = 0; z < kZ && z < Z; ++z) {
          E[z] = a.set_e[(base + i) * Z + z];
          P[z] = a.set_p[(base + i) * Z + z];
        }
        a.set_key[base + r] = k;
        for (uint32_t z = 0; z < kZ && z < Z; ++z) {
          a.set_e[(base + r) * Z + z] = E[z];
          a.set_p[(base + r) * Z + z] = P[z];
        }
      }
    }
    // ---- survivors take their ranks (frozen copies: Add(prev.Clone())) -------------
    if (lane < m && rank < new_size) {
      a.set_key[base + rank] = skey;
      for (uint32_t z = 0; z < Z; ++z) {
        a.set_e[(base + rank) * Z + z] = a.tab_e[static_cast<uint64_t>(sslot) * a.tab_stride + z];
        a.set_p[(base + rank) * Z + z] =
            a.tab_p ? a.tab_p[static_cast<uint64_t>(sslot) * a.tab_stride + z] : proc_power(a.pd, sslot, z);
      }
    }
    size = new_size;
    // the next chunk reads the set this one wrote (minimum, keys, energies): stores complete first
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  }
  if (lane == 0) a.size[n] = size;
}

// Items(): the nodes' sets packed node by node (offsets from the host).
__global__ __launch_bounds__(kThreads) void pack_kernel(const Args a, const uint64_t *off, uint64_t *out_key,
                                                        uint32_t *out_node, uint64_t *out_e, double *out_p) {
  const uint32_t n = blockIdx.x;
  const uint64_t o = off[n], cnt = off[n + 1] - o, base = static_cast<uint64_t>(n) * a.cap;
  for (uint64_t i = threadIdx.x; i < cnt; i += kThreads) {
    out_key[o + i] = a.set_key[base + i];
    out_node[o + i] = n;
    for (uint32_t z = 0; z < a.Z; ++z) {
      out_e[(o + i) * a.Z + z] = a.set_e[(base + i) * a.Z + z];
      out_p[(o + i) * a.Z + z] = a.set_p[(base + i) * a.Z + z];
    }
  }
}

// Clear(): every node, or the nodes with mask[n] != 0 (process.go:80-84).
__global__ __launch_bounds__(kThreads) void clear_kernel(uint32_t *size, uint32_t n_nodes, const uint32_t *mask) {
  const uint32_t n = blockIdx.x * kThreads + threadIdx.x;
  if (n < n_nodes && (!mask || mask[n])) size[n] = 0;
}

}  // namespace trk
}  // namespace kacc

// =============================================================================
// C ABI
// =============================================================================
struct kacc_tracker {
  kacc_ctx *ctx = nullptr;
  int device = 0;
  kacc_kind kind = KACC_KIND_PROC;
  int64_t max_size = 0;
  uint32_t cap = 0, zone = 0, Z = 0, nodes = 0;
  uint64_t min_e = 0;
  uint64_t *d_set_key = nullptr;
  uint64_t *d_set_e = nullptr;
  double *d_set_p = nullptr;
  uint32_t *d_size = nullptr;
};

namespace {

void kind_tables(const kacc_ctx *ctx, kacc_kind k, const uint64_t **e, const double **p) {
  const int base = k == KACC_KIND_PROC ? KACC_T_PROC_ENERGY
                   : k == KACC_KIND_CTR ? KACC_T_CTR_ENERGY
                   : k == KACC_KIND_VM ? KACC_T_VM_ENERGY
                                       : KACC_T_POD_ENERGY;
  *e = static_cast<const uint64_t *>(ctx->tables[base]);
  // a process's (container's, VM's) power is derived (kacc_derive.hpp) from its
  // ratio and its node's tables of the same interval: the tracker must run before
  // that node's next one
  *p = k == KACC_KIND_POD ? static_cast<const double *>(ctx->tables[base + 1]) : nullptr;
}

kacc::trk::Args tracker_args(const kacc_tracker *t) {
  kacc::trk::Args a{};
  kind_tables(t->ctx, t->kind, &a.tab_e, &a.tab_p);
  a.pd = kacc_derive(t->ctx, t->kind);
  a.min_e = t->min_e;
  a.max_size = t->max_size;
  a.Z = t->Z;
  a.tab_stride = t->kind == KACC_KIND_POD ? 2 * t->Z : t->Z;
  a.z0 = t->zone;
  a.cap = t->cap;
  a.n_nodes = t->nodes;
  a.set_key = t->d_set_key;
  a.set_e = t->d_set_e;
  a.set_p = t->d_set_p;
  a.size = t->d_size;
  a.err = t->ctx->d_err;
  return a;
}

}  // namespace

extern "C" {

int kacc_tracker_create(kacc_ctx *ctx, kacc_kind kind, int64_t max_size, uint32_t capacity,
                        uint32_t zone, uint64_t min_energy, kacc_tracker **out) {
  if (!ctx || !out) return KACC_EINVAL;
  *out = nullptr;
  if (kind < KACC_KIND_PROC || kind > KACC_KIND_POD) return kacc_fail(ctx, KACC_EINVAL, "bad kind");
  if (zone >= ctx->cfg.zones) return kacc_fail(ctx, KACC_EINVAL, "zone %u >= Z", zone);
  if (max_size > static_cast<int64_t>(KACC_TRACKER_MAX_BOUNDED))
    return kacc_fail(ctx, KACC_EINVAL, "max_size > %u", KACC_TRACKER_MAX_BOUNDED);
  const uint32_t cap = max_size > 0 ? static_cast<uint32_t>(max_size) : max_size < 0 ? capacity : 0u;
  if (max_size < 0 && capacity == 0) return kacc_fail(ctx, KACC_EINVAL, "unlimited tracker needs a capacity");
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  auto *t = new kacc_tracker;
  t->ctx = ctx;
  t->device = ctx->device;
  t->kind = kind;
  t->max_size = max_size;
  t->cap = std::max<uint32_t>(cap, 1);
  t->zone = zone;
  t->Z = ctx->cfg.zones;
  t->nodes = static_cast<uint32_t>(std::max<uint64_t>(ctx->cfg.nodes, 1));
  t->min_e = min_energy;
  const size_t items = static_cast<size_t>(t->nodes) * t->cap, Z = t->Z;
  // nodes x per-node items x (key 8 + energy 8Z + power 8Z): refuse before the
  // allocation when it cannot fit (e.g. an unlimited tracker with a large
  // per-node capacity over a big fleet), with the cost in the message
  const size_t need = items * (8 + 16 * Z) + 4ull * t->nodes;
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && need > free_b) {
    const uint32_t nodes = t->nodes, per = t->cap;
    delete t;
    return kacc_fail(ctx, KACC_ENOMEM,
                     "tracker needs %zu B = %u nodes x %u items per node x %zu B, %zu B of device memory free",
                     need, nodes, per, static_cast<size_t>(8 + 16 * Z), free_b);
  }
  hipError_t e = hipSuccess;
  auto A = [&](void **p, size_t bytes) {
    if (e == hipSuccess) e = hipMalloc(p, std::max<size_t>(bytes, 8));
  };
  A(reinterpret_cast<void **>(&t->d_set_key), 8 * items);
  A(reinterpret_cast<void **>(&t->d_set_e), 8 * items * Z);
  A(reinterpret_cast<void **>(&t->d_set_p), 8 * items * Z);
  A(reinterpret_cast<void **>(&t->d_size), 4ull * t->nodes);
  if (e != hipSuccess) {
    kacc_tracker_destroy(t);
    return kacc_fail(ctx, KACC_ENOMEM, "tracker allocation (%u nodes x %u): %s", t->nodes, t->cap,
                     hipGetErrorString(e));
  }
  const int rc = kacc_tracker_clear(t, nullptr, nullptr);
  if (rc != KACC_OK) {
    kacc_tracker_destroy(t);
    return rc;
  }
  KACC_HIP(ctx, hipStreamSynchronize(ctx->stream));
  *out = t;
  return KACC_OK;
}

void kacc_tracker_destroy(kacc_tracker *t) {
  if (!t) return;
  (void)hipSetDevice(t->device);
  (void)hipDeviceSynchronize();
  (void)hipFree(t->d_set_key);
  (void)hipFree(t->d_set_e);
  (void)hipFree(t->d_set_p);
  (void)hipFree(t->d_size);
  delete t;
}

int kacc_tracker_clear(kacc_tracker *t, const uint32_t *node_mask, void *stream) {
  if (!t) return KACC_EINVAL;
  kacc_ctx *ctx = t->ctx;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  if (!node_mask) {
    KACC_HIP(ctx, hipMemsetAsync(t->d_size, 0, 4ull * t->nodes, st));
    return KACC_OK;
  }
  (void)hipGetLastError();
  hipLaunchKernelGGL(kacc::trk::clear_kernel, dim3((t->nodes + kacc::trk::kThreads - 1) / kacc::trk::kThreads),
                     dim3(kacc::trk::kThreads), 0, st, t->d_size, t->nodes, node_mask);
  KACC_HIP(ctx, hipGetLastError());
  return KACC_OK;
}

int kacc_tracker_add(kacc_tracker *t, const kacc_slotmap *m, const uint64_t *term_key,
                     const uint32_t *term_slot, const uint32_t *term_count, void *stream) {
  if (!t || !m) return KACC_EINVAL;
  kacc_ctx *ctx = t->ctx;
  if (m->ctx != ctx || m->kind != t->kind)
    return kacc_fail(ctx, KACC_EINVAL, "tracker and slot map differ in context or kind");
  if (t->max_size == 0 || m->n_nodes == 0) return KACC_OK;  // tracker.go:82 disabled
  if (m->n_nodes > t->nodes)
    return kacc_fail(ctx, KACC_EINVAL, "slot map has %u nodes, the tracker %u", m->n_nodes, t->nodes);
  if (!term_key || !term_slot || !term_count) return kacc_fail(ctx, KACC_EINVAL, "NULL argument");
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  kacc::trk::Args a = tracker_args(t);
  a.n_nodes = m->n_nodes;
  a.slot_off = m->d_slot_off;
  a.term_key = term_key;
  a.term_slot = term_slot;
  a.term_count = term_count;
  (void)hipGetLastError();  // clear a stale error of an earlier call
  const dim3 wgrid((m->n_nodes + kacc::trk::kWaveNodes - 1) / kacc::trk::kWaveNodes);
  if (a.Z <= 4)
    hipLaunchKernelGGL(kacc::trk::node_add_wave_kernel<4>, wgrid, dim3(kacc::trk::kThreads), 0, st, a);
  else
    hipLaunchKernelGGL(kacc::trk::node_add_wave_kernel<KACC_MAX_ZONES>, wgrid, dim3(kacc::trk::kThreads), 0, st, a);
  KACC_HIP(ctx, hipGetLastError());
  return KACC_OK;
}

int kacc_tracker_items(kacc_tracker *t, uint32_t *count, uint64_t *key, uint32_t *node,
                       uint64_t *energy, double *power) {
  if (!t || !count) return KACC_EINVAL;
  kacc_ctx *ctx = t->ctx;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  KACC_HIP(ctx, hipDeviceSynchronize());  // adds may run on any stream
  std::vector<uint32_t> sizes(t->nodes);
  KACC_HIP(ctx, hipMemcpy(sizes.data(), t->d_size, 4ull * t->nodes, hipMemcpyDeviceToHost));
  std::vector<uint64_t> off(t->nodes + 1, 0);
  for (uint32_t n = 0; n < t->nodes; ++n) off[n + 1] = off[n] + std::min(sizes[n], t->cap);
  const uint64_t total = off[t->nodes];
  if (total > 0xffffffffull) return kacc_fail(ctx, KACC_ERANGE, "tracked items exceed 2^32");
  *count = static_cast<uint32_t>(total);
  if (total == 0 || (!key && !node && !energy && !power)) return KACC_OK;
  const size_t Z = t->Z;
  void *d_off = nullptr, *d_key = nullptr, *d_node = nullptr, *d_e = nullptr, *d_p = nullptr;
  hipError_t e = hipMalloc(&d_off, 8 * off.size());
  if (e == hipSuccess) e = hipMalloc(&d_key, 8 * total);
  if (e == hipSuccess) e = hipMalloc(&d_node, 4 * total);
  if (e == hipSuccess) e = hipMalloc(&d_e, 8 * total * Z);
  if (e == hipSuccess) e = hipMalloc(&d_p, 8 * total * Z);
  if (e == hipSuccess) e = hipMemcpy(d_off, off.data(), 8 * off.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(kacc::trk::pack_kernel, dim3(t->nodes), dim3(kacc::trk::kThreads), 0, nullptr,
                       tracker_args(t), static_cast<const uint64_t *>(d_off), static_cast<uint64_t *>(d_key),
                       static_cast<uint32_t *>(d_node), static_cast<uint64_t *>(d_e), static_cast<double *>(d_p));
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess && key) e = hipMemcpy(key, d_key, 8 * total, hipMemcpyDeviceToHost);
  if (e == hipSuccess && node) e = hipMemcpy(node, d_node, 4 * total, hipMemcpyDeviceToHost);
  if (e == hipSuccess && energy) e = hipMemcpy(energy, d_e, 8 * total * Z, hipMemcpyDeviceToHost);
  if (e == hipSuccess && power) e = hipMemcpy(power, d_p, 8 * total * Z, hipMemcpyDeviceToHost);
  for (void *p : {d_off, d_key, d_node, d_e, d_p})
    if (p) (void)hipFree(p);
  if (e != hipSuccess) return kacc_fail(ctx, KACC_EHIP, "tracker items: %s", hipGetErrorString(e));
  return KACC_OK;
}

}  // extern "C"
