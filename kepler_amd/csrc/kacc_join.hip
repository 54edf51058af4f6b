// Slot join: workload IDs -> slot words, on the device.
//
// The reference decides "running total or new workload" per row with a
// string-keyed lookup of the previous snapshot (process.go:132-138,
// container.go:126, vm.go:96, pod.go:106), and the informer derives the
// terminated set as "cached before, not seen now" (informer.go:206-212,
// 236-246, 260-270, 311-322); terminated workloads found in the previous
// snapshot go to the terminated trackers (process.go:87-99).  Here a fleet
// interval does both for every node in one launch: one workgroup per node,
// the node's live-ID hash table (key u64 -> node-relative slot) rebuilt from
// the current rows every interval (no tombstones), ping-ponged between two
// device buffers.  A node whose table fits 4096 buckets (<= 2730 slots) works
// on an LDS copy; bigger nodes work on the global table directly.
//
// Per node, in order:
//   1  mark the slots held by the previous table (used bitmap, LDS)
//   2  look every row's key up: found -> its slot, bucket marked seen
//   3  unseen buckets = terminated IDs -> (key, slot) list
//   4  rows not found take the lowest free slots in row order (block scan)
//   5  the new table = exactly the current rows, written to the other buffer
// Slots of terminated IDs are marked used in step 1, so they are not handed
// out before the next interval: the tracker still reads their final values.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "kacc_internal.hpp"

namespace kacc {
namespace join {

constexpr int kThreads = 512;
constexpr uint32_t kLdsBuckets = 4096;        // small-node table in LDS
constexpr uint32_t kMaxRange = 131072;        // slots per node (bitmap words in LDS)
constexpr uint32_t kWords = kMaxRange / 32;   // big-node bitmap words
constexpr uint32_t kSmallWords = (kLdsBuckets * 2 / 3 + 31) / 32 + 1;
constexpr uint32_t kSeen = 0x80000000u;       // bucket slot field: matched this interval
constexpr uint16_t kSeen16 = 0x8000u;
constexpr uint32_t kInvalid = 0xffffffffu;    // slot word of a row in error
constexpr uint32_t kPending = 0xfffffffeu;    // row not found yet (step 2 -> 4)

constexpr uint32_t kErrOffsets = 1u << 1;
constexpr uint32_t kErrKey = 1u << 6;       // KACC_KEY_EMPTY or duplicate ID in a node
constexpr uint32_t kErrRange = 1u << 7;     // more live IDs than the node's slot range
constexpr uint32_t kErrTermCap = 1u << 8;   // terminated list overflow

struct Args {
  uint32_t n_nodes, n_rows, term_cap, pad;
  const uint32_t *row_off;
  const uint64_t *keys;
  const uint32_t *node_status;
  uint32_t *out_slot;
  uint64_t *term_key;
  uint32_t *term_slot;
  uint32_t *term_count;
  const uint32_t *slot_off;  // [N+1]
  const uint64_t *hoff;      // [N+1] bucket offsets (each node a power of two)
  uint64_t *hkeys[2];
  uint32_t *hslots[2];
  uint8_t *parity;           // [N] which buffer holds the node's live table
  uint32_t *err;
};

__device__ __forceinline__ uint64_t mix64(uint64_t x) {  // splitmix64 finalizer
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}

// Exclusive block-wide scan of v (512 threads = 8 waves); *total = sum.
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
  for (int w = 0; w < kThreads / 64; ++w) {
    const uint32_t t = s_wave[w];
    if (w < wave) base += t;
    tot += t;
  }
  __syncthreads();  // s_wave reusable
  total = tot;
  return base + x - v;
}

// Position of the j-th (0-based) set bit of w (w has more than j set bits).
__device__ __forceinline__ uint32_t select_bit(uint32_t w, uint32_t j) {
  for (uint32_t i = 0; i < j; ++i) w &= w - 1;
  return static_cast<uint32_t>(__builtin_ctz(w));
}

template <bool kSmall>
__global__ __launch_bounds__(kThreads) void join_kernel(const Args a) {
  __shared__ uint64_t s_keys[kSmall ? kLdsBuckets : 1];
  __shared__ uint16_t s_slots[kSmall ? kLdsBuckets : 1];
  __shared__ uint32_t s_used[kSmall ? kSmallWords : kWords];  // used-slot bitmap
  __shared__ uint32_t s_wpre[kSmall ? kSmallWords : kWords];  // free slots before word w
  __shared__ uint32_t s_wave[kThreads / 64];
  __shared__ uint32_t s_cnt, s_cnt2, s_base;

  const uint32_t n = blockIdx.x;
  const int tid = threadIdx.x;
  if (n >= a.n_nodes) return;
  if (a.node_status && (a.node_status[n] & KACC_NODE_READ_ERROR)) return;  // map unchanged
  const uint64_t hb = a.hoff[n];
  const uint32_t H = static_cast<uint32_t>(a.hoff[n + 1] - hb);
  if ((H <= kLdsBuckets) != kSmall) return;  // the other instance handles this node
  const uint32_t s0 = a.slot_off[n];
  const uint32_t S = a.slot_off[n + 1] - s0;
  uint32_t r0 = a.row_off[n], r1 = a.row_off[n + 1];
  if (r1 > a.n_rows || r0 > r1) {
    if (tid == 0) atomicOr(a.err, kErrOffsets);
    r1 = min(r1, a.n_rows);
    r0 = min(r0, r1);
  }
  const uint32_t par = a.parity[n] & 1u;
  uint64_t *__restrict__ Ak = a.hkeys[par] + hb;
  uint32_t *__restrict__ As = a.hslots[par] + hb;
  uint64_t *__restrict__ Bk = a.hkeys[par ^ 1u] + hb;
  uint32_t *__restrict__ Bs = a.hslots[par ^ 1u] + hb;
  const uint32_t W = (S + 31) / 32;
  const uint32_t hmask = H - 1;

  // ---- 1: previous table (LDS copy for small nodes), used bitmap -------------
  for (uint32_t w = tid; w < W; w += kThreads) s_used[w] = 0u;
  if constexpr (kSmall) {
    for (uint32_t b = tid; b < H; b += kThreads) {
      s_keys[b] = Ak[b];
      s_slots[b] = static_cast<uint16_t>(As[b]);
    }
  }
  if (tid == 0) {
    s_cnt = 0u;
    s_cnt2 = 0u;
  }
  __syncthreads();
  auto tkey = [&](uint32_t b) -> uint64_t {
    if constexpr (kSmall) return s_keys[b];
    else return Ak[b];
  };
  auto tslot = [&](uint32_t b) -> uint32_t {  // node-relative slot, seen bit stripped
    if constexpr (kSmall) return s_slots[b] & ~kSeen16;
    else return As[b] & ~kSeen;
  };
  for (uint32_t b = tid; b < H; b += kThreads) {
    if (tkey(b) == KACC_KEY_EMPTY) continue;
    const uint32_t s = tslot(b);
    if (s < S) atomicOr(&s_used[s >> 5], 1u << (s & 31));
  }
  // ---- 2: lookups (a bucket's seen bit has one writer: keys are unique) -------
  for (uint32_t r = r0 + tid; r < r1; r += kThreads) {
    const uint64_t k = a.keys[r];
    uint32_t out = kPending;
    if (k == KACC_KEY_EMPTY) {
      atomicOr(a.err, kErrKey);
      out = kInvalid;
    } else {
      uint32_t b = static_cast<uint32_t>(mix64(k)) & hmask;
      for (uint32_t probe = 0; probe < H; ++probe, b = (b + 1) & hmask) {
        const uint64_t kk = tkey(b);
        if (kk == KACC_KEY_EMPTY) break;
        if (kk == k) {
          uint32_t s;
          if constexpr (kSmall) {
            s = s_slots[b] & ~kSeen16;
            s_slots[b] = static_cast<uint16_t>(s | kSeen16);
          } else {
            s = As[b] & ~kSeen;
            As[b] = s | kSeen;
          }
          out = s < S ? s0 + s : kInvalid;
          break;
        }
      }
    }
    a.out_slot[r] = out;
  }
  __syncthreads();
  // ---- 3: terminated = previous IDs not matched ------------------------------
  auto terminated = [&](uint32_t b) -> bool {
    if (tkey(b) == KACC_KEY_EMPTY) return false;
    if constexpr (kSmall) return (s_slots[b] & kSeen16) == 0;
    else return (As[b] & kSeen) == 0u;
  };
  for (uint32_t b = tid; b < H; b += kThreads)
    if (terminated(b)) atomicAdd(&s_cnt, 1u);
  __syncthreads();
  if (tid == 0) s_base = s_cnt ? atomicAdd(a.term_count, s_cnt) : 0u;
  __syncthreads();
  if (s_cnt) {
    for (uint32_t b = tid; b < H; b += kThreads) {
      if (!terminated(b)) continue;
      const uint32_t i = s_base + atomicAdd(&s_cnt2, 1u);
      if (i < a.term_cap) {
        a.term_key[i] = tkey(b);
        a.term_slot[i] = s0 + tslot(b);
      } else {
        atomicOr(a.err, kErrTermCap);
      }
    }
  }
  // ---- 4: free-slot prefix per bitmap word, then new rows in row order --------
  uint32_t carry = 0;
  for (uint32_t w0 = 0; w0 < W; w0 += kThreads) {
    const uint32_t w = w0 + tid;
    uint32_t f = 0;
    if (w < W) {
      const uint32_t valid = (w + 1) * 32 <= S ? 0xffffffffu : ((1u << (S & 31)) - 1u);
      f = __popc(~s_used[w] & valid);
    }
    uint32_t tot;
    const uint32_t ex = block_scan(f, s_wave, tot);
    if (w < W) s_wpre[w] = carry + ex;
    carry += tot;
  }
  const uint32_t total_free = carry;
  __syncthreads();
  uint32_t taken = 0;
  for (uint32_t c0 = r0; c0 < r1; c0 += kThreads) {
    const uint32_t r = c0 + tid;
    const bool isnew = r < r1 && a.out_slot[r] == kPending;
    uint32_t tot;
    const uint32_t q = taken + block_scan(isnew ? 1u : 0u, s_wave, tot);
    if (isnew) {
      if (q < total_free) {
        uint32_t lo = 0, hi = W;  // last word with s_wpre[w] <= q
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) / 2;
          if (s_wpre[mid] <= q) lo = mid; else hi = mid;
        }
        const uint32_t valid = (lo + 1) * 32 <= S ? 0xffffffffu : ((1u << (S & 31)) - 1u);
        const uint32_t s = lo * 32 + select_bit(~s_used[lo] & valid, q - s_wpre[lo]);
        a.out_slot[r] = (s0 + s) | KACC_SLOT_NEW;
      } else {
        atomicOr(a.err, kErrRange);
        a.out_slot[r] = kInvalid;
      }
    }
    taken += tot;
  }
  // ---- 5: the new table holds exactly the current rows -----------------------
  __syncthreads();  // step 3 done reading the previous table (LDS is reused)
  for (uint32_t b = tid; b < H; b += kThreads) {
    if constexpr (kSmall) s_keys[b] = KACC_KEY_EMPTY;
    else Bk[b] = KACC_KEY_EMPTY;
  }
  __syncthreads();
  for (uint32_t r = r0 + tid; r < r1; r += kThreads) {
    const uint32_t w = a.out_slot[r];
    if (w == kInvalid) continue;
    const uint32_t rel = (w & KACC_SLOT_MASK) - s0;
    const uint64_t k = a.keys[r];
    uint32_t b = static_cast<uint32_t>(mix64(k)) & hmask;
    for (uint32_t probe = 0; probe < H; ++probe, b = (b + 1) & hmask) {
      uint64_t prev;
      if constexpr (kSmall) prev = atomicCAS(reinterpret_cast<unsigned long long *>(&s_keys[b]),
                                             KACC_KEY_EMPTY, static_cast<unsigned long long>(k));
      else prev = atomicCAS(reinterpret_cast<unsigned long long *>(&Bk[b]), KACC_KEY_EMPTY,
                            static_cast<unsigned long long>(k));
      if (prev == KACC_KEY_EMPTY) {
        if constexpr (kSmall) s_slots[b] = static_cast<uint16_t>(rel);
        else Bs[b] = rel;
        break;
      }
      if (prev == k) {  // the same ID twice in one node
        atomicOr(a.err, kErrKey);
        a.out_slot[r] = kInvalid;
        break;
      }
    }
  }
  __syncthreads();
  if constexpr (kSmall) {
    for (uint32_t b = tid; b < H; b += kThreads) {
      Bk[b] = s_keys[b];
      Bs[b] = s_slots[b];
    }
  }
  if (tid == 0) a.parity[n] = static_cast<uint8_t>(par ^ 1u);
}

}  // namespace join
}  // namespace kacc

// =============================================================================
// C ABI
// =============================================================================
struct kacc_slotmap {
  kacc_ctx *ctx = nullptr;
  kacc_kind kind = KACC_KIND_PROC;
  uint32_t n_nodes = 0;
  uint64_t buckets = 0;
  uint32_t *d_slot_off = nullptr;
  uint64_t *d_hoff = nullptr;
  uint64_t *d_keys[2] = {};
  uint32_t *d_slots[2] = {};
  uint8_t *d_parity = nullptr;
};

namespace {

uint64_t kind_capacity(const kacc_config &c, kacc_kind k) {
  switch (k) {
    case KACC_KIND_PROC: return c.proc_slots;
    case KACC_KIND_CTR: return c.ctr_slots;
    case KACC_KIND_VM: return c.vm_slots;
    default: return c.pod_slots;
  }
}

// Buckets of a node with S slots: a power of two >= 1.5 S (load <= 2/3), >= 64.
uint64_t node_buckets(uint32_t S) {
  uint64_t h = 64;
  while (h * 2 < 3ull * S) h <<= 1;
  return h;
}

}  // namespace

extern "C" {

int kacc_slotmap_create(kacc_ctx *ctx, kacc_kind kind, uint32_t n_nodes, const uint32_t *slot_off,
                        kacc_slotmap **out) {
  if (!ctx || !out || (!slot_off && n_nodes)) return KACC_EINVAL;
  *out = nullptr;
  if (kind < KACC_KIND_PROC || kind > KACC_KIND_POD) return kacc_fail(ctx, KACC_EINVAL, "bad kind %d", (int)kind);
  if (n_nodes > ctx->cfg.nodes)
    return kacc_fail(ctx, KACC_EINVAL, "n_nodes %u exceeds node capacity", n_nodes);
  const uint64_t cap = kind_capacity(ctx->cfg, kind);
  std::vector<uint64_t> hoff(n_nodes + 1, 0);
  if (n_nodes && slot_off[0] != 0) return kacc_fail(ctx, KACC_EINVAL, "slot_off[0] must be 0");
  for (uint32_t n = 0; n < n_nodes; ++n) {
    if (slot_off[n + 1] < slot_off[n]) return kacc_fail(ctx, KACC_EINVAL, "slot_off not monotonic at %u", n);
    const uint32_t S = slot_off[n + 1] - slot_off[n];
    if (S > kacc::join::kMaxRange)
      return kacc_fail(ctx, KACC_EINVAL, "node %u slot range %u > %u", n, S, kacc::join::kMaxRange);
    hoff[n + 1] = hoff[n] + node_buckets(S);
  }
  if (n_nodes && slot_off[n_nodes] > cap)
    return kacc_fail(ctx, KACC_EINVAL, "slot_off[n] = %u exceeds the kind's slot capacity %llu",
                     slot_off[n_nodes], (unsigned long long)cap);
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  auto *m = new kacc_slotmap;
  m->ctx = ctx;
  m->kind = kind;
  m->n_nodes = n_nodes;
  m->buckets = hoff[n_nodes];
  auto bail = [&](hipError_t e) {
    kacc_slotmap_destroy(m);
    return kacc_fail(ctx, e == hipErrorOutOfMemory ? KACC_ENOMEM : KACC_EHIP, "slot map allocation: %s",
                     hipGetErrorString(e));
  };
  hipError_t e;
  const size_t nb = std::max<uint64_t>(m->buckets, 1);
  if ((e = hipMalloc(&m->d_slot_off, 4ull * (n_nodes + 1))) != hipSuccess) return bail(e);
  if ((e = hipMalloc(&m->d_hoff, 8ull * (n_nodes + 1))) != hipSuccess) return bail(e);
  if ((e = hipMalloc(&m->d_parity, std::max<uint32_t>(n_nodes, 1))) != hipSuccess) return bail(e);
  for (int p = 0; p < 2; ++p) {
    if ((e = hipMalloc(&m->d_keys[p], 8 * nb)) != hipSuccess) return bail(e);
    if ((e = hipMalloc(&m->d_slots[p], 4 * nb)) != hipSuccess) return bail(e);
  }
  if (n_nodes) {
    if ((e = hipMemcpy(m->d_slot_off, slot_off, 4ull * (n_nodes + 1), hipMemcpyHostToDevice)) != hipSuccess)
      return bail(e);
    if ((e = hipMemcpy(m->d_hoff, hoff.data(), 8ull * (n_nodes + 1), hipMemcpyHostToDevice)) != hipSuccess)
      return bail(e);
  }
  int rc = kacc_slotmap_reset(m);
  if (rc != KACC_OK) {
    kacc_slotmap_destroy(m);
    return rc;
  }
  *out = m;
  return KACC_OK;
}

void kacc_slotmap_destroy(kacc_slotmap *m) {
  if (!m) return;
  (void)hipSetDevice(m->ctx->device);
  (void)hipStreamSynchronize(m->ctx->stream);
  (void)hipFree(m->d_slot_off);
  (void)hipFree(m->d_hoff);
  (void)hipFree(m->d_parity);
  for (int p = 0; p < 2; ++p) {
    (void)hipFree(m->d_keys[p]);
    (void)hipFree(m->d_slots[p]);
  }
  delete m;
}

int kacc_slotmap_reset(kacc_slotmap *m) {
  if (!m) return KACC_EINVAL;
  kacc_ctx *ctx = m->ctx;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  const size_t nb = std::max<uint64_t>(m->buckets, 1);
  for (int p = 0; p < 2; ++p) KACC_HIP(ctx, hipMemsetAsync(m->d_keys[p], 0xff, 8 * nb, ctx->stream));
  KACC_HIP(ctx, hipMemsetAsync(m->d_parity, 0, std::max<uint32_t>(m->n_nodes, 1), ctx->stream));
  KACC_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return KACC_OK;
}

int kacc_slot_join(kacc_slotmap *m, uint32_t n_rows, const uint32_t *row_off, const uint64_t *keys,
                   const uint32_t *node_status, uint32_t *out_slot, uint64_t *term_key,
                   uint32_t *term_slot, uint32_t *term_count, uint32_t term_cap, void *stream) {
  if (!m) return KACC_EINVAL;
  kacc_ctx *ctx = m->ctx;
  if (!m->n_nodes) return KACC_OK;
  if (!row_off || !out_slot || !term_count || (term_cap && (!term_key || !term_slot)))
    return kacc_fail(ctx, KACC_EINVAL, "slot join: NULL argument");
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  if (n_rows && !keys) return kacc_fail(ctx, KACC_EINVAL, "slot join: keys is NULL");
  KACC_HIP(ctx, hipMemsetAsync(term_count, 0, 4, st));
  kacc::join::Args a{};
  a.n_nodes = m->n_nodes;
  a.n_rows = n_rows;
  a.term_cap = term_cap;
  a.row_off = row_off;
  a.keys = keys;
  a.node_status = node_status;
  a.out_slot = out_slot;
  a.term_key = term_key;
  a.term_slot = term_slot;
  a.term_count = term_count;
  a.slot_off = m->d_slot_off;
  a.hoff = m->d_hoff;
  for (int p = 0; p < 2; ++p) {
    a.hkeys[p] = m->d_keys[p];
    a.hslots[p] = m->d_slots[p];
  }
  a.parity = m->d_parity;
  a.err = ctx->d_err;
  hipLaunchKernelGGL((kacc::join::join_kernel<true>), dim3(m->n_nodes), dim3(kacc::join::kThreads), 0, st, a);
  hipLaunchKernelGGL((kacc::join::join_kernel<false>), dim3(m->n_nodes), dim3(kacc::join::kThreads), 0, st, a);
  KACC_HIP(ctx, hipGetLastError());
  return KACC_OK;
}

}  // extern "C"
