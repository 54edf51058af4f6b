// Terminated-workload tracker on the device.
//
// Reference: TerminatedResourceTracker (internal/monitor/
// terminated_resource_tracker.go): a min-heap of the max_size highest-energy
// terminated workloads; Add() drops a disabled tracker (:82), a tracked ID
// (:90), energy below the threshold (:102), pushes below capacity (:116) and
// evicts the minimum for a strictly higher energy at capacity (:124).  The
// monitor adds every terminated workload found in the previous snapshot
// (process.go:87-99) and clears the tracker after an export (process.go:80-84).
//
// One interval's batch (the slot join's per-node terminated segments, values
// read from the kind's state tables) is added as Go would add it in the map
// order "descending target-zone energy, then node, then slot".  In that order
// the heap simply keeps the max_size best of (tracked ∪ batch), ties at the
// boundary going to tracked items first (eviction needs a strictly higher
// energy) and then to the batch order — so the batch is a top-N selection:
//   filter    one workgroup per node: threshold, "beats the current minimum"
//             when full, not already tracked; survivors compacted in slot
//             order + a 65536-bin histogram of a monotone 16-bit energy key
//   pick      one workgroup: the boundary bin of the max_size-th item
//   collect   items above the boundary bin -> keep list, in it -> tie list
//   finalize  one workgroup: exact order of the ties (bitonic sort in LDS),
//             the new set sorted (energy desc, tracked first, node, slot),
//             frozen zone values copied, dedupe hash rebuilt
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "kacc_internal.hpp"

namespace kacc {
namespace trk {

constexpr int kThreads = 256;       // filter / collect workgroups
constexpr int kFinThreads = 1024;   // pick / finalize workgroup
constexpr uint32_t kBins = 65536;
constexpr uint32_t kSortCap = KACC_TRACKER_MAX_BOUNDED;  // ties / set sorted in LDS
constexpr uint64_t kOld = 1ull << 63;                    // sort key: 0 = tracked item
constexpr uint32_t kErrTie = 1u << 9;   // more boundary ties than kSortCap
constexpr uint32_t kErrCap = 1u << 10;  // unlimited tracker past its capacity

struct State {
  uint32_t size;      // items in the current set
  uint32_t parity;    // current set buffer
  uint64_t min_full;  // target-zone energy of the lowest item (set full)
  uint32_t keep_n, tie_n;
  uint32_t pick_bin, keep_all, need, pad;
};

struct Entry {
  uint64_t e;     // target-zone energy
  uint64_t key;   // workload ID
  uint32_t node;
  uint32_t ref;   // slot (batch item) or index in the current set (tracked)
  uint32_t old;   // 1: tracked item
  uint32_t pad;
};

struct Args {
  const uint64_t *tab_e;
  const double *tab_p;
  uint64_t min_e;
  int64_t max_size;
  uint32_t Z, z0, cap, n_nodes;
  const uint32_t *slot_off;
  const uint64_t *term_key;
  const uint32_t *term_slot;
  const uint32_t *term_count;
  uint64_t *surv_e, *surv_key;
  uint32_t *surv_slot, *surv_cnt;
  uint32_t *hist;
  Entry *keep, *ties;
  uint64_t *set_key[2];
  uint32_t *set_node[2];
  uint64_t *set_e[2];
  double *set_p[2];
  uint64_t *hkey;
  uint32_t *hnode;
  uint32_t hmask;
  State *st;
  uint32_t *err;
};

// Monotone 16-bit key: 6-bit exponent, 10-bit mantissa (e = 0 and 1 share 0).
__device__ __forceinline__ uint32_t bin_of(uint64_t e) {
  if (e == 0) return 0;
  const uint32_t msb = 63u - static_cast<uint32_t>(__clzll(static_cast<long long>(e)));
  const uint32_t mant = msb >= 10 ? static_cast<uint32_t>(e >> (msb - 10)) & 1023u
                                  : static_cast<uint32_t>(e << (10 - msb)) & 1023u;
  return msb * 1024u + mant;
}

__device__ __forceinline__ uint32_t hbucket(uint64_t key, uint32_t node, uint32_t hmask) {
  uint64_t x = key ^ (static_cast<uint64_t>(node) * 0x9E3779B97F4A7C15ull);
  x ^= x >> 31;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 29;
  return static_cast<uint32_t>(x) & hmask;
}

__device__ bool tracked(const Args &a, uint64_t key, uint32_t node) {
  uint32_t b = hbucket(key, node, a.hmask);
  for (uint32_t p = 0; p <= a.hmask; ++p, b = (b + 1) & a.hmask) {
    const uint64_t k = a.hkey[b];
    if (k == KACC_KEY_EMPTY) return false;
    if (k == key && a.hnode[b] == node) return true;
  }
  return false;
}

template <int T>
__device__ __forceinline__ uint32_t block_scan(uint32_t v, uint32_t *s_wave, uint32_t &total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) s_wave[wave] = x;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < T / 64; ++w) {
    const uint32_t t = s_wave[w];
    if (w < wave) base += t;
    tot += t;
  }
  __syncthreads();
  total = tot;
  return base + x - v;
}

// ---- filter: one workgroup per node (+ one for the tracked items) ------------------
__global__ __launch_bounds__(kThreads) void filter_kernel(const Args a) {
  __shared__ uint32_t s_wave[kThreads / 64];
  const uint32_t tid = threadIdx.x;
  const State st = *a.st;
  if (blockIdx.x == a.n_nodes) {  // tracked items stay candidates of the selection
    const uint32_t cur = st.parity & 1u;
    for (uint32_t i = tid; i < st.size; i += kThreads)
      atomicAdd(&a.hist[bin_of(a.set_e[cur][static_cast<uint64_t>(i) * a.Z + a.z0])], 1u);
    return;
  }
  const uint32_t n = blockIdx.x;
  const uint32_t base = a.slot_off[n];
  const uint32_t c = min(a.term_count[n], a.slot_off[n + 1] - base);
  const bool full = a.max_size > 0 && st.size >= static_cast<uint64_t>(a.max_size);
  uint32_t done = 0;
  for (uint32_t i0 = 0; i0 < c; i0 += kThreads) {
    const uint32_t i = i0 + tid;
    bool pass = false;
    uint64_t e = 0, key = 0;
    uint32_t slot = 0;
    if (i < c) {
      slot = a.term_slot[base + i];
      key = a.term_key[base + i];
      e = a.tab_e[static_cast<uint64_t>(slot) * a.Z + a.z0];
      pass = e >= a.min_e                       // terminated_resource_tracker.go:102
             && !(full && e <= st.min_full)     // :124 needs a strictly higher energy
             && !tracked(a, key, n);            // :90
    }
    uint32_t tot;
    const uint32_t pos = done + block_scan<kThreads>(pass ? 1u : 0u, s_wave, tot);
    if (pass) {
      a.surv_e[base + pos] = e;
      a.surv_key[base + pos] = key;
      a.surv_slot[base + pos] = slot;
      atomicAdd(&a.hist[bin_of(e)], 1u);
    }
    done += tot;
  }
  if (tid == 0) a.surv_cnt[n] = done;
}

// ---- pick: the boundary bin of the max_size-th best item --------------------------
__global__ __launch_bounds__(kFinThreads) void pick_kernel(const Args a) {
  __shared__ uint32_t s_sum[kFinThreads];
  constexpr uint32_t kPer = kBins / kFinThreads;  // 64 bins per thread
  const uint32_t tid = threadIdx.x;
  uint32_t s = 0;
  for (uint32_t j = 0; j < kPer; ++j) s += a.hist[tid * kPer + j];
  s_sum[tid] = s;
  __syncthreads();
  if (tid == 0) {
    uint32_t tot = 0;
    for (uint32_t t = 0; t < kFinThreads; ++t) tot += s_sum[t];
    State *st = a.st;
    st->keep_n = 0;
    st->tie_n = 0;
    st->need = 0;
    st->pick_bin = 0;
    if (a.max_size < 0 || tot <= static_cast<uint64_t>(a.max_size)) {
      st->keep_all = 1;
    } else {
      st->keep_all = 0;
      const uint32_t K = static_cast<uint32_t>(a.max_size);
      uint32_t above = 0, t = kFinThreads;
      while (t > 0 && above + s_sum[t - 1] < K) above += s_sum[--t];
      // thread t - 1 holds the boundary: walk its bins from the top
      const uint32_t tb = t - 1;
      uint32_t b = tb * kPer + kPer;
      while (b > tb * kPer) {
        const uint32_t h = a.hist[b - 1];
        if (above + h >= K) break;
        above += h;
        --b;
      }
      st->pick_bin = b - 1;
      st->need = K - above;
    }
  }
}

// ---- collect: above the boundary -> keep, in it -> ties ----------------------------
__device__ __forceinline__ void route(const Args &a, const State &st, const Entry &x, uint32_t lim) {
  const uint32_t b = bin_of(x.e);
  if (st.keep_all || b > st.pick_bin) {
    const uint32_t i = atomicAdd(&a.st->keep_n, 1u);
    if (i < lim) a.keep[i] = x;
    else atomicOr(a.err, kErrCap);
  } else if (b == st.pick_bin) {
    const uint32_t i = atomicAdd(&a.st->tie_n, 1u);
    if (i < kSortCap) a.ties[i] = x;
    else atomicOr(a.err, kErrTie);
  }
}

__global__ __launch_bounds__(kThreads) void collect_kernel(const Args a) {
  const State st = *a.st;
  const uint32_t tid = threadIdx.x;
  const uint32_t lim = a.cap;
  if (blockIdx.x == a.n_nodes) {
    const uint32_t cur = st.parity & 1u;
    for (uint32_t i = tid; i < st.size; i += kThreads) {
      Entry x;
      x.e = a.set_e[cur][static_cast<uint64_t>(i) * a.Z + a.z0];
      x.key = a.set_key[cur][i];
      x.node = a.set_node[cur][i];
      x.ref = i;
      x.old = 1;
      x.pad = 0;
      route(a, st, x, lim);
    }
    return;
  }
  const uint32_t n = blockIdx.x;
  const uint32_t base = a.slot_off[n];
  const uint32_t c = a.surv_cnt[n];
  for (uint32_t i = tid; i < c; i += kThreads) {
    Entry x;
    x.e = a.surv_e[base + i];
    x.key = a.surv_key[base + i];
    x.node = n;
    x.ref = a.surv_slot[base + i];
    x.old = 0;
    x.pad = 0;
    route(a, st, x, lim);
  }
}

// ---- finalize: exact order in LDS, the new set, dedupe hash -----------------------
// Sort keys: k1 = ~energy (ascending = energy desc), k2 = batch flag, node, ref.
__device__ __forceinline__ void sort_keys(const Entry &x, uint64_t &k1, uint64_t &k2) {
  k1 = ~x.e;
  k2 = (x.old ? 0ull : kOld) | (static_cast<uint64_t>(x.node) << 31) | (x.ref & 0x7fffffffu);
}

// Bitonic sort of n (<= kSortCap) (k1, k2, idx) triples in LDS, ascending.
__device__ void bitonic(uint64_t *k1, uint64_t *k2, uint16_t *ix, uint32_t n) {
  uint32_t m = 1;
  while (m < n) m <<= 1;
  for (uint32_t i = n + threadIdx.x; i < m; i += kFinThreads) {
    k1[i] = ~0ull;
    k2[i] = ~0ull;
    ix[i] = 0xffffu;
  }
  __syncthreads();
  for (uint32_t size = 2; size <= m; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t i = threadIdx.x; i < m; i += kFinThreads) {
        const uint32_t j = i ^ stride;
        if (j <= i) continue;
        const bool up = (i & size) == 0;
        const bool gt = k1[i] > k1[j] || (k1[i] == k1[j] && k2[i] > k2[j]);
        if (gt == up) {
          const uint64_t t1 = k1[i], t2 = k2[i];
          const uint16_t t3 = ix[i];
          k1[i] = k1[j];
          k2[i] = k2[j];
          ix[i] = ix[j];
          k1[j] = t1;
          k2[j] = t2;
          ix[j] = t3;
        }
      }
      __syncthreads();
    }
  }
}

__global__ __launch_bounds__(kFinThreads) void finalize_kernel(const Args a) {
  __shared__ uint64_t s_k1[kSortCap], s_k2[kSortCap];
  __shared__ uint16_t s_ix[kSortCap];
  const uint32_t tid = threadIdx.x;
  const State st = *a.st;
  const uint32_t cur = st.parity & 1u, nxt = cur ^ 1u;
  uint32_t n_keep = min(st.keep_n, a.cap);
  // 1: the first `need` ties in exact order join the keep list
  if (!st.keep_all && st.need > 0) {
    const uint32_t nt = min(st.tie_n, kSortCap);
    for (uint32_t i = tid; i < nt; i += kFinThreads) {
      sort_keys(a.ties[i], s_k1[i], s_k2[i]);
      s_ix[i] = static_cast<uint16_t>(i);
    }
    __syncthreads();
    bitonic(s_k1, s_k2, s_ix, nt);
    const uint32_t take = min(st.need, nt);
    for (uint32_t i = tid; i < take; i += kFinThreads)
      if (n_keep + i < a.cap) a.keep[n_keep + i] = a.ties[s_ix[i]];
    n_keep = min(n_keep + take, a.cap);
    __syncthreads();  // keep entries visible to the whole workgroup
  }
  // 2: the new set, sorted when it fits LDS (always for max_size > 0)
  const bool sorted = n_keep <= kSortCap;
  if (sorted) {
    for (uint32_t i = tid; i < n_keep; i += kFinThreads) {
      sort_keys(a.keep[i], s_k1[i], s_k2[i]);
      s_ix[i] = static_cast<uint16_t>(i);
    }
    __syncthreads();
    bitonic(s_k1, s_k2, s_ix, n_keep);
  }
  for (uint32_t i = tid; i < n_keep; i += kFinThreads) {
    const Entry x = a.keep[sorted ? s_ix[i] : i];
    a.set_key[nxt][i] = x.key;
    a.set_node[nxt][i] = x.node;
    for (uint32_t z = 0; z < a.Z; ++z) {  // frozen copy: Add(prev.Clone())
      const uint64_t src = static_cast<uint64_t>(x.ref) * a.Z + z;
      a.set_e[nxt][static_cast<uint64_t>(i) * a.Z + z] = x.old ? a.set_e[cur][src] : a.tab_e[src];
      a.set_p[nxt][static_cast<uint64_t>(i) * a.Z + z] = x.old ? a.set_p[cur][src] : a.tab_p[src];
    }
  }
  // 3: dedupe hash of the new set
  for (uint32_t b = tid; b <= a.hmask; b += kFinThreads) a.hkey[b] = KACC_KEY_EMPTY;
  __syncthreads();
  for (uint32_t i = tid; i < n_keep; i += kFinThreads) {
    const Entry x = a.keep[sorted ? s_ix[i] : i];
    uint32_t b = hbucket(x.key, x.node, a.hmask);
    for (uint32_t p = 0; p <= a.hmask; ++p, b = (b + 1) & a.hmask) {
      if (atomicCAS(reinterpret_cast<unsigned long long *>(a.hkey + b), KACC_KEY_EMPTY,
                    static_cast<unsigned long long>(x.key)) == KACC_KEY_EMPTY) {
        a.hnode[b] = x.node;
        break;
      }
    }
  }
  __syncthreads();
  if (tid == 0) {
    State *s = a.st;
    s->size = n_keep;
    s->parity = nxt;
    const bool full = a.max_size > 0 && n_keep >= static_cast<uint64_t>(a.max_size);
    s->min_full = full ? a.set_e[nxt][static_cast<uint64_t>(n_keep - 1) * a.Z + a.z0] : 0ull;
  }
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
  uint32_t cap = 0, zone = 0, Z = 0, hmask = 0;
  uint64_t min_e = 0;
  kacc::trk::State *d_state = nullptr;
  uint64_t *d_set_key[2] = {};
  uint32_t *d_set_node[2] = {};
  uint64_t *d_set_e[2] = {};
  double *d_set_p[2] = {};
  uint64_t *d_hkey = nullptr;
  uint32_t *d_hnode = nullptr;
  uint32_t *d_hist = nullptr;
  kacc::trk::Entry *d_keep = nullptr, *d_ties = nullptr;
  // per-node survivors, sized like the slot map that feeds the tracker
  uint32_t surv_slots = 0, surv_nodes = 0;
  uint64_t *d_surv_e = nullptr, *d_surv_key = nullptr;
  uint32_t *d_surv_slot = nullptr, *d_surv_cnt = nullptr;
};

namespace {

void kind_tables(const kacc_ctx *ctx, kacc_kind k, const uint64_t **e, const double **p) {
  const int base = k == KACC_KIND_PROC ? KACC_T_PROC_ENERGY
                   : k == KACC_KIND_CTR ? KACC_T_CTR_ENERGY
                   : k == KACC_KIND_VM ? KACC_T_VM_ENERGY
                                       : KACC_T_POD_ENERGY;
  *e = static_cast<const uint64_t *>(ctx->tables[base]);
  *p = static_cast<const double *>(ctx->tables[base + 1]);
}

void free_surv(kacc_tracker *t) {
  (void)hipFree(t->d_surv_e);
  (void)hipFree(t->d_surv_key);
  (void)hipFree(t->d_surv_slot);
  (void)hipFree(t->d_surv_cnt);
  t->d_surv_e = t->d_surv_key = nullptr;
  t->d_surv_slot = t->d_surv_cnt = nullptr;
  t->surv_slots = t->surv_nodes = 0;
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
  t->min_e = min_energy;
  uint32_t hb = 64;
  while (hb < 2 * t->cap) hb <<= 1;
  t->hmask = hb - 1;
  const size_t c = t->cap, Z = t->Z;
  hipError_t e = hipSuccess;
  auto A = [&](void **p, size_t bytes) {
    if (e == hipSuccess) e = hipMalloc(p, std::max<size_t>(bytes, 8));
  };
  A(reinterpret_cast<void **>(&t->d_state), sizeof(kacc::trk::State));
  for (int p = 0; p < 2; ++p) {
    A(reinterpret_cast<void **>(&t->d_set_key[p]), 8 * c);
    A(reinterpret_cast<void **>(&t->d_set_node[p]), 4 * c);
    A(reinterpret_cast<void **>(&t->d_set_e[p]), 8 * c * Z);
    A(reinterpret_cast<void **>(&t->d_set_p[p]), 8 * c * Z);
  }
  A(reinterpret_cast<void **>(&t->d_hkey), 8ull * hb);
  A(reinterpret_cast<void **>(&t->d_hnode), 4ull * hb);
  A(reinterpret_cast<void **>(&t->d_hist), 4ull * kacc::trk::kBins);
  A(reinterpret_cast<void **>(&t->d_keep), sizeof(kacc::trk::Entry) * (c + kacc::trk::kSortCap));
  A(reinterpret_cast<void **>(&t->d_ties), sizeof(kacc::trk::Entry) * kacc::trk::kSortCap);
  if (e != hipSuccess) {
    kacc_tracker_destroy(t);
    return kacc_fail(ctx, KACC_ENOMEM, "tracker allocation: %s", hipGetErrorString(e));
  }
  const int rc = kacc_tracker_clear(t, nullptr);
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
  (void)hipFree(t->d_state);
  for (int p = 0; p < 2; ++p) {
    (void)hipFree(t->d_set_key[p]);
    (void)hipFree(t->d_set_node[p]);
    (void)hipFree(t->d_set_e[p]);
    (void)hipFree(t->d_set_p[p]);
  }
  (void)hipFree(t->d_hkey);
  (void)hipFree(t->d_hnode);
  (void)hipFree(t->d_hist);
  (void)hipFree(t->d_keep);
  (void)hipFree(t->d_ties);
  free_surv(t);
  delete t;
}

int kacc_tracker_clear(kacc_tracker *t, void *stream) {
  if (!t) return KACC_EINVAL;
  kacc_ctx *ctx = t->ctx;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  KACC_HIP(ctx, hipMemsetAsync(t->d_state, 0, sizeof(kacc::trk::State), st));
  KACC_HIP(ctx, hipMemsetAsync(t->d_hkey, 0xff, 8ull * (t->hmask + 1), st));
  return KACC_OK;
}

int kacc_tracker_add(kacc_tracker *t, const kacc_slotmap *m, const uint64_t *term_key,
                     const uint32_t *term_slot, const uint32_t *term_count, void *stream) {
  if (!t || !m) return KACC_EINVAL;
  kacc_ctx *ctx = t->ctx;
  if (m->ctx != ctx || m->kind != t->kind)
    return kacc_fail(ctx, KACC_EINVAL, "tracker and slot map differ in context or kind");
  if (t->max_size == 0 || m->n_nodes == 0) return KACC_OK;  // tracker.go:82 disabled
  if (!term_key || !term_slot || !term_count) return kacc_fail(ctx, KACC_EINVAL, "NULL argument");
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  if (m->total_slots > t->surv_slots || m->n_nodes > t->surv_nodes) {
    KACC_HIP(ctx, hipDeviceSynchronize());
    free_surv(t);
    const size_t ns = std::max<uint32_t>(m->total_slots, 1), nn = m->n_nodes;
    hipError_t e = hipMalloc(&t->d_surv_e, 8 * ns);
    if (e == hipSuccess) e = hipMalloc(&t->d_surv_key, 8 * ns);
    if (e == hipSuccess) e = hipMalloc(&t->d_surv_slot, 4 * ns);
    if (e == hipSuccess) e = hipMalloc(&t->d_surv_cnt, 4 * nn);
    if (e != hipSuccess) {
      free_surv(t);
      return kacc_fail(ctx, KACC_ENOMEM, "tracker scratch: %s", hipGetErrorString(e));
    }
    t->surv_slots = static_cast<uint32_t>(ns);
    t->surv_nodes = m->n_nodes;
  }
  kacc::trk::Args a{};
  kind_tables(ctx, t->kind, &a.tab_e, &a.tab_p);
  a.min_e = t->min_e;
  a.max_size = t->max_size;
  a.Z = t->Z;
  a.z0 = t->zone;
  a.cap = t->cap;
  a.n_nodes = m->n_nodes;
  a.slot_off = m->d_slot_off;
  a.term_key = term_key;
  a.term_slot = term_slot;
  a.term_count = term_count;
  a.surv_e = t->d_surv_e;
  a.surv_key = t->d_surv_key;
  a.surv_slot = t->d_surv_slot;
  a.surv_cnt = t->d_surv_cnt;
  a.hist = t->d_hist;
  a.keep = t->d_keep;
  a.ties = t->d_ties;
  for (int p = 0; p < 2; ++p) {
    a.set_key[p] = t->d_set_key[p];
    a.set_node[p] = t->d_set_node[p];
    a.set_e[p] = t->d_set_e[p];
    a.set_p[p] = t->d_set_p[p];
  }
  a.hkey = t->d_hkey;
  a.hnode = t->d_hnode;
  a.hmask = t->hmask;
  a.st = t->d_state;
  a.err = ctx->d_err;
  using namespace kacc::trk;
  KACC_HIP(ctx, hipMemsetAsync(t->d_hist, 0, 4ull * kBins, st));
  (void)hipGetLastError();  // clear a stale error of an earlier call
  hipLaunchKernelGGL(filter_kernel, dim3(m->n_nodes + 1), dim3(kThreads), 0, st, a);
  hipLaunchKernelGGL(pick_kernel, dim3(1), dim3(kFinThreads), 0, st, a);
  hipLaunchKernelGGL(collect_kernel, dim3(m->n_nodes + 1), dim3(kThreads), 0, st, a);
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(kFinThreads), 0, st, a);
  KACC_HIP(ctx, hipGetLastError());
  return KACC_OK;
}

int kacc_tracker_items(kacc_tracker *t, uint32_t *count, uint64_t *key, uint32_t *node,
                       uint64_t *energy, double *power) {
  if (!t || !count) return KACC_EINVAL;
  kacc_ctx *ctx = t->ctx;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  KACC_HIP(ctx, hipDeviceSynchronize());  // adds may run on any stream
  kacc::trk::State s{};
  KACC_HIP(ctx, hipMemcpy(&s, t->d_state, sizeof(s), hipMemcpyDeviceToHost));
  *count = s.size;
  const uint32_t cur = s.parity & 1u;
  const size_t n = s.size, Z = t->Z;
  if (n == 0) return KACC_OK;
  if (key) KACC_HIP(ctx, hipMemcpy(key, t->d_set_key[cur], 8 * n, hipMemcpyDeviceToHost));
  if (node) KACC_HIP(ctx, hipMemcpy(node, t->d_set_node[cur], 4 * n, hipMemcpyDeviceToHost));
  if (energy) KACC_HIP(ctx, hipMemcpy(energy, t->d_set_e[cur], 8 * n * Z, hipMemcpyDeviceToHost));
  if (power) KACC_HIP(ctx, hipMemcpy(power, t->d_set_p[cur], 8 * n * Z, hipMemcpyDeviceToHost));
  return KACC_OK;
}

}  // extern "C"
