// Slot join: workload IDs -> slot words, on the device.
//
// The reference decides "running total or new workload" per row with a
// string-keyed lookup of the previous snapshot (process.go:132-138,
// container.go:126, vm.go:96, pod.go:106), and the informer derives the
// terminated set as "cached before, not seen now" (informer.go:206-212,
// 236-246, 260-270, 311-322); terminated workloads found in the previous
// snapshot go to the terminated trackers (process.go:87-99).  Here a fleet
// interval does both for every node in one launch: one workgroup per node,
// over the node's private open-addressing table of live IDs (key -> node-
// relative slot, linear probing, load <= 2/3), updated in place: terminated
// IDs become tombstones, new IDs claim empty or tombstone buckets, and only
// the buckets that changed are written back.  When live + tombstones pass
// 3/4 of the table it is rebuilt from the current rows.  PIDs are u32 keys
// packed with their slot in one 8-B bucket; 64-bit IDs use a key array and a
// slot array.  A node whose table has <= 4096 buckets (<= 2730 slots) works on
// an LDS copy with its rows' keys in registers; bigger nodes work on the
// global table.
//
// Per node, in order:
//   1  load the table (LDS) and the rows' keys
//   2  used-slot bitmap of the live IDs; look every row up (seen-slot bitmap)
//   3  live IDs whose slot was not seen = terminated: the node's segment of
//      the (key, slot) list in slot order (bitmap prefix, no global atomic),
//      bucket -> tombstone
//   4  rows not found take the lowest slots free at step 2, in row order
//   5  new IDs claim buckets; a re-probe flags an ID given twice in a node
//   6  write back the changed buckets (or rebuild the table)
// Terminated slots are in the step-2 bitmap, so they are not handed out
// before the next interval: the tracker still reads their final values.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <type_traits>
#include <vector>

#include "kacc_debug.h"
#include "kacc_internal.hpp"

namespace kacc {
namespace join {

constexpr int kThreads = 512;
constexpr uint32_t kLdsBuckets = 4096;           // small-node table in LDS
constexpr int kRpl = 6;                          // small-node rows per lane (contiguous)
constexpr uint32_t kSmallRows = kRpl * kThreads;
constexpr uint32_t kMaxRange = 131072;           // slots per node
constexpr uint32_t kWords = kMaxRange / 32;      // big-node slot bitmap words
constexpr uint32_t kSmallWords = (kLdsBuckets * 2 / 3 + 31) / 32 + 1;
constexpr uint32_t kInvalid = 0xffffffffu;       // slot word of a row in error
constexpr uint32_t kPending = 0xfffffffeu;       // row not found (step 2 -> 4)

constexpr uint32_t kErrOffsets = 1u << 1;
constexpr uint32_t kErrKey = 1u << 6;      // reserved key or an ID given twice in a node
constexpr uint32_t kErrRange = 1u << 7;    // more live IDs than the node's slot range

struct Args {
  uint32_t n_nodes, n_rows;
  uint32_t stop_after;  // timing ablation (kacc_debug_join_variant): 0 = full join
  uint32_t reuse;       // KACC_JOIN_REUSE_TERMINATED
  uint32_t fmt6;        // PID tables of small nodes are 6-B buckets (join_small's kJ6B)
  uint32_t uniform;     // every node's table has kLdsBuckets buckets (hoff[n] = n kLdsBuckets)
  const uint32_t *row_off;
  const void *keys;
  const uint32_t *node_status;
  uint32_t *out_slot;
  uint64_t *term_key;
  uint32_t *term_slot;
  uint32_t *term_count;
  uint32_t *out_span;        // optional [2N]: {min, max} slot of the node's rows
  const uint32_t *slot_off;  // [N+1]
  const uint64_t *hoff;      // [N+1] bucket offsets (each node a power of two)
  uint64_t *ent;             // u32 keys: packed (key << 32 | slot); u64 keys: the keys
  uint32_t *slots;           // u64 keys: the slots
  uint32_t *err;
};

// Fibonacci hashing: the top log2(H) bits of fold(k) * 2^32/phi (PIDs are
// near-sequential; 64-bit IDs are already hashed by the packer).
template <typename K>
__device__ __forceinline__ uint32_t bucket(K k, uint32_t shift) {
  uint32_t x = static_cast<uint32_t>(k);
  if constexpr (sizeof(K) == 8) x ^= static_cast<uint32_t>(static_cast<uint64_t>(k) >> 32);
  return (x * 0x9E3779B1u) >> shift;
}

// Bucket views over generic (LDS or global) pointers.  raw(b) is the word a
// claim compares: the packed entry (u32 keys) or the key (u64 keys).
template <typename K>
struct Tab;
template <>
struct Tab<uint32_t> {
  static constexpr uint32_t kEmpty = 0xffffffffu, kTomb = 0xfffffffeu;
  uint64_t *e;
  __device__ uint64_t raw(uint32_t b) const { return e[b]; }
  __device__ static uint32_t key_of(uint64_t r) { return static_cast<uint32_t>(r >> 32); }
  __device__ uint32_t key(uint32_t b) const { return key_of(e[b]); }
  __device__ uint32_t slot(uint32_t b) const { return static_cast<uint32_t>(e[b]); }
  __device__ void tomb(uint32_t b) const { e[b] = static_cast<uint64_t>(kTomb) << 32; }
  __device__ bool claim(uint32_t b, uint64_t seen, uint32_t k, uint32_t s) const {
    const unsigned long long v = (static_cast<unsigned long long>(k) << 32) | s;
    return atomicCAS(reinterpret_cast<unsigned long long *>(e + b), seen, v) == seen;
  }
  __device__ void clear(uint32_t b) const { e[b] = ~0ull; }
};
template <>
struct Tab<uint64_t> {
  static constexpr uint64_t kEmpty = ~0ull, kTomb = ~0ull - 1;
  uint64_t *k;
  uint32_t *s;
  __device__ uint64_t raw(uint32_t b) const { return k[b]; }
  __device__ static uint64_t key_of(uint64_t r) { return r; }
  __device__ uint64_t key(uint32_t b) const { return k[b]; }
  __device__ uint32_t slot(uint32_t b) const { return s[b]; }
  __device__ void tomb(uint32_t b) const { k[b] = kTomb; }
  __device__ bool claim(uint32_t b, uint64_t seen, uint64_t kk, uint32_t ss) const {
    if (atomicCAS(reinterpret_cast<unsigned long long *>(k + b), seen, kk) != seen) return false;
    s[b] = ss;
    return true;
  }
  __device__ void clear(uint32_t b) const { k[b] = kEmpty; }
};

// The PID table of a small node (H <= kLdsBuckets) in 6-B buckets: H u32 keys,
// then H u16 node-relative slots (S <= 2730), in the node's 8H-byte region;
// a claim is a CAS on the key, then the slot store (as Tab<uint64_t>).
struct TabP {
  static constexpr uint32_t kEmpty = 0xffffffffu, kTomb = 0xfffffffeu;
  uint32_t *k;
  uint16_t *s;
  __device__ uint32_t raw(uint32_t b) const { return k[b]; }
  __device__ static uint32_t key_of(uint32_t r) { return r; }
  __device__ uint32_t key(uint32_t b) const { return k[b]; }
  __device__ uint32_t slot(uint32_t b) const { return s[b]; }
  __device__ void tomb(uint32_t b) const { k[b] = kTomb; }
  __device__ bool claim(uint32_t b, uint32_t seen, uint32_t kk, uint32_t ss) const {
    if (atomicCAS(k + b, seen, kk) != seen) return false;
    s[b] = static_cast<uint16_t>(ss);
    return true;
  }
  __device__ void clear(uint32_t b) const { k[b] = kEmpty; }
};

template <typename T, typename R>
__device__ __forceinline__ bool is_live(R raw) {
  const auto k = T::key_of(raw);
  return k != T::kEmpty && k != T::kTomb;
}

// Linear-probing operations shared by both kernels (hmask = H - 1).
template <typename K, typename T = Tab<K>>
struct Probe {
  T t;
  uint32_t shift, hmask, H;
  // bucket holding k, or ~0u (stops at the first empty bucket, skips tombstones)
  __device__ uint32_t find(K k) const {
    uint32_t b = bucket(k, shift);
    for (uint32_t p = 0; p < H; ++p, b = (b + 1) & hmask) {
      const K kk = static_cast<K>(t.key(b));
      if (kk == k) return b;
      if (kk == T::kEmpty) break;
    }
    return ~0u;
  }
  // claim the first empty or tombstone bucket on k's path; returns it (or ~0u);
  // *fresh: the bucket was empty (the table's occupancy grew)
  __device__ uint32_t insert(K k, uint32_t rel, uint32_t *fresh = nullptr) const {
    uint32_t b = bucket(k, shift);
    for (uint32_t p = 0; p < H;) {
      const auto raw = t.raw(b);
      const K kk = static_cast<K>(T::key_of(raw));
      if (kk == T::kEmpty || kk == T::kTomb) {
        if (t.claim(b, raw, k, rel)) {
          if (fresh) *fresh += kk == T::kEmpty ? 1u : 0u;
          return b;
        }
        continue;  // lost the race for this bucket: look at it again
      }
      ++p;
      b = (b + 1) & hmask;
    }
    return ~0u;
  }
};

// Exclusive block-wide scan of v (512 threads = 8 waves); total = sum.
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

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}

// Position of the j-th (0-based) set bit of w (w has more than j set bits).
__device__ __forceinline__ uint32_t select_bit(uint32_t w, uint32_t j) {
  for (uint32_t i = 0; i < j; ++i) w &= w - 1;
  return static_cast<uint32_t>(__builtin_ctz(w));
}

// Node geometry shared by both kernels; false when this kernel skips the node.
struct NodeView {
  uint64_t hb;
  uint32_t H, S, s0, r0, r1, shift;
};
template <bool kSmall>
__device__ __forceinline__ bool node_view(const Args &a, uint32_t n, NodeView &v) {
  // every node word is loaded up front (independent loads, one round trip)
  const uint32_t status = a.node_status ? a.node_status[n] : 0u;
  v.hb = a.hoff[n];
  const uint64_t he = a.hoff[n + 1];
  v.r0 = a.row_off[n];
  v.r1 = a.row_off[n + 1];
  v.s0 = a.slot_off[n];
  const uint32_t s1 = a.slot_off[n + 1];
  if (status & KACC_NODE_READ_ERROR) {  // map unchanged
    if (kSmall && threadIdx.x == 0) a.term_count[n] = 0u;
    return false;
  }
  v.H = static_cast<uint32_t>(he - v.hb);
  if (v.r1 > a.n_rows || v.r0 > v.r1) {
    if (kSmall && threadIdx.x == 0) atomicOr(a.err, kErrOffsets);
    v.r1 = min(v.r1, a.n_rows);
    v.r0 = min(v.r0, v.r1);
  }
  // every small-table node is join_small's, whatever its kind and row count: more
  // rows than kSmallRows cannot fit its <= 2730 slots, an ERANGE there (join_big
  // only runs for maps with a big table, so routing such a node to it would leave
  // its slot words and terminated count unwritten for the other maps)
  if ((v.H <= kLdsBuckets) != kSmall) return false;
  v.S = s1 - v.s0;
  v.shift = 32u - static_cast<uint32_t>(__builtin_ctz(v.H));
  return true;
}

// {min, max} over the block (lane values; no row = {1, 0}) -> out_span[2n..]
__device__ __forceinline__ void span_out(const Args &a, uint32_t n, uint32_t lo, uint32_t hi,
                                         uint32_t *s_lo, uint32_t *s_hi) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    lo = min(lo, static_cast<uint32_t>(__shfl_xor(static_cast<int>(lo), d, 64)));
    hi = max(hi, static_cast<uint32_t>(__shfl_xor(static_cast<int>(hi), d, 64)));
  }
  if ((threadIdx.x & 63) == 0) {
    s_lo[threadIdx.x >> 6] = lo;
    s_hi[threadIdx.x >> 6] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 1; w < kThreads / 64; ++w) {
      lo = min(lo, s_lo[w]);
      hi = max(hi, s_hi[w]);
    }
    const bool none = lo > hi;
    a.out_span[2 * n] = none ? 1u : lo;
    a.out_span[2 * n + 1] = none ? 0u : hi;
  }
}

// ============================ small nodes (LDS) ====================================
// Table in LDS, rows' keys / slot words in registers (lane owns kRpl
// consecutive rows), per-slot mark bitmaps in LDS (LDS atomics): s_used
// (slot held at the start), s_seen (a row found the slot; the second finder
// of the same ID sees the bit already set: duplicate).  Bitmaps keep the
// workgroup at <= 40 KiB of LDS, i.e. 4 workgroups (8 waves/SIMD) per CU.
constexpr uint32_t kNewCap = 512;  // new rows handled as a compact list

// Variant bits of join_small (timing ablations; production = kJoinDefault):
constexpr int kJLock = 1;      // lookups of a lane's rows in lock-step (one LDS round trip per depth)
constexpr int kJErrReg = 2;    // error bits gathered in a register, one atomic per lane at the end
constexpr int kJLdsBar = 4;    // LDS-only barriers (never wait for the node's global stores)
constexpr int kJInsDup = 8;    // duplicates found by the insert itself (no re-probe pass)
constexpr int kJScan2 = 16;    // the two block scans of step 3 share their barrier
constexpr int kJ6B = 32;       // PID tables in 6-B buckets (u32 keys, u16 slots), vector table loads
constexpr int kJSeenNR = 64;   // seen marks without return; duplicates found by counting (step 3)
constexpr int kJVec = 128;     // a lane's keys loaded / slot words stored as vectors
constexpr int kJGroup = 256;   // kJ6B lookups read four buckets per LDS read
constexpr int kJDpp = 1024;    // block scans by DPP moves instead of LDS permutes
constexpr uint32_t kPendWords = (kSmallRows + 31) / 32;  // rows-not-found bitmap (kJLean)
// The block-wide tail without its table pass (round 6): step 3's word prefixes come from
// wave 0 (two DPP scans over the slot bitmaps, two over the rows-not-found bitmap), a new
// row's rank is its row's position in that bitmap, and step 4 lists the terminated IDs
// from the terminated bits through the held slots' buckets (s_bkt) instead of every lane
// walking the node's whole table; the other steps are join_small's.
constexpr int kJLean = 8192;
// Two-choice cuckoo placement of the 6-B PID table (round 6): a key lives in one of the
// 4-bucket groups ck_g1(k) / ck_g2(k), so a lookup reads exactly those two 16-B groups —
// no probe loop, whose lock-step depth is the deepest of a wave's 384 rows — and a
// terminated key's bucket is simply emptied (no tombstones, no rebuild).  New keys claim
// an empty bucket of their two groups (CAS); the rare key whose groups are both full is
// placed by lane 0 alone, moving keys to their other group (cuckoo kicks).  At most
// 2730 live keys in 4096 buckets (load <= 2/3), far below 4-way 2-choice cuckoo's limit.
constexpr int kJCuckoo = 16384;
constexpr int kCkMaxKicks = 512;
// the key's two groups among G (>= 2): the high word of hash x G (a power-of-two G takes the
// hash's top bits), the second moved off the first
__device__ __forceinline__ uint32_t ck_g1(uint32_t k, uint32_t G) { return __umulhi(k * 0x9E3779B1u, G); }
__device__ __forceinline__ uint32_t ck_g2(uint32_t k, uint32_t G) {
  uint32_t x = k ^ (k >> 15);
  x *= 0x2C1B3C6Du;
  x ^= x >> 12;
  x *= 0x297A2D39u;
  x ^= x >> 15;
  const uint32_t g = __umulhi(x, G), g1 = ck_g1(k, G);
  return g != g1 ? g : g1 + 1 == G ? 0u : g1 + 1;
}
// kJCkSmall: the cuckoo table fills only 4 ceil(3S / 8) of the node's H buckets (1.5 S: load
// <= 2/3 as before, but of a table sized by the slots, not the next power of two)
constexpr int kJCkSmall = 32768;
// kJCkFast: the join is VALU-issue-bound (eight waves per SIMD, 821 VALU instructions per
// wave: 85 % of its quad-cycles), so (a) the two groups from ONE quarter-rate multiply each
// (the top bits of k x C for the power-of-two group count of format 3, the second group
// flipped off the first on a clash) instead of five multiplies per key, (b) a wave without
// rows skips the lookups (R = 2000 leaves waves 6-7 idle there), (c) no occupancy count
// (a six-step cross-lane sum per wave; only linear probing's rebuild rule reads it)
constexpr int kJCkFast = 65536;
// kJUni: on a map whose every node has a kLdsBuckets table (hoff[n] = n kLdsBuckets) the
// node's table address needs no node word, so its loads issue at the kernel's first
// instruction, beside the node words' round trip instead of after it
constexpr int kJUni = 131072;

// bit e: key word e of a group equals k
__device__ __forceinline__ uint32_t ck_match(const uint4 &g, uint32_t k) {
  return (g.x == k ? 1u : 0u) | (g.y == k ? 2u : 0u) | (g.z == k ? 4u : 0u) | (g.w == k ? 8u : 0u);
}

__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <int V>
__device__ __forceinline__ void jbar() {
  if constexpr ((V & kJLdsBar) != 0)
    lds_barrier();
  else
    __syncthreads();
}

// Inclusive scan over the 64 lanes of a wave in DPP moves (no LDS round trips): within
// rows of 16 by row_shr 1, 2, 4, 8, then row_bcast:15 into rows 1 and 3 and
// row_bcast:31 into rows 2 and 3.  A lane without a source (or outside the row mask)
// adds the `old` operand, 0.
template <typename Op>
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t x, uint32_t identity, Op op) {
  int v = static_cast<int>(x);
  const int id = static_cast<int>(identity);
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x111, 0xf, 0xf, false));  // row_shr:1
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x112, 0xf, 0xf, false));  // row_shr:2
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x114, 0xf, 0xf, false));  // row_shr:4
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x118, 0xf, 0xf, false));  // row_shr:8
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x142, 0xa, 0xf, false));  // row_bcast:15
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return static_cast<uint32_t>(v);
}
struct DppAdd {
  __device__ int operator()(int a, int b) const { return static_cast<int>(static_cast<uint32_t>(a) + static_cast<uint32_t>(b)); }
};
struct DppMin {
  __device__ int operator()(int a, int b) const { return static_cast<int>(min(static_cast<uint32_t>(a), static_cast<uint32_t>(b))); }
};
struct DppMax {
  __device__ int operator()(int a, int b) const { return static_cast<int>(max(static_cast<uint32_t>(a), static_cast<uint32_t>(b))); }
};
// the wave's reduction (lane 63 of the inclusive scan), uniform
template <typename Op>
__device__ __forceinline__ uint32_t wave_reduce_dpp(uint32_t x, uint32_t identity, Op op) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(wave_scan_dpp(x, identity, op)), 63));
}

// Two exclusive block-wide scans at once (one barrier; s_wave [2 * waves]).
// The caller puts a barrier between this and the next write of s_wave.
template <int V>
__device__ __forceinline__ void block_scan2(uint32_t v0, uint32_t v1, uint32_t *s_wave, uint32_t &ex0,
                                            uint32_t &ex1, uint32_t &tot0, uint32_t &tot1) {
  constexpr int kW = kThreads / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t x0 = v0, x1 = v1;
  if constexpr ((V & kJDpp) != 0) {
    x0 = wave_scan_dpp(x0, 0u, DppAdd{});
    x1 = wave_scan_dpp(x1, 0u, DppAdd{});
  } else {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y0 = __shfl_up(x0, d, 64), y1 = __shfl_up(x1, d, 64);
      if (lane >= d) {
        x0 += y0;
        x1 += y1;
      }
    }
  }
  if (lane == 63) {
    s_wave[wave] = x0;
    s_wave[kW + wave] = x1;
  }
  jbar<V>();
  uint32_t b0 = 0, b1 = 0, t0 = 0, t1 = 0;
#pragma unroll
  for (int w = 0; w < kW; ++w) {
    const uint32_t a0 = s_wave[w], a1 = s_wave[kW + w];
    if (w < wave) {
      b0 += a0;
      b1 += a1;
    }
    t0 += a0;
    t1 += a1;
  }
  ex0 = b0 + x0 - v0;
  ex1 = b1 + x1 - v1;
  tot0 = t0;
  tot1 = t1;
}

template <typename K, int V>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(sizeof(K) == 8 ? 4 : 8))) void join_small(const Args a) {
  constexpr bool kWide = sizeof(K) == 8;
  constexpr bool k6 = !kWide && (V & kJ6B) != 0;
  constexpr bool kSplit = kWide || k6;  // a key array and a slot array (else packed entries)
  constexpr bool kLock = (V & kJLock) != 0, kErrReg = (V & kJErrReg) != 0, kInsDup = (V & kJInsDup) != 0;
  constexpr bool kScan2 = (V & kJScan2) != 0, kSeenNR = (V & kJSeenNR) != 0, kVec = (V & kJVec) != 0;
  constexpr bool kGroup = k6 && (V & kJGroup) != 0;
  constexpr bool kLean = (V & kJLean) != 0;
  static_assert(!kLean || (kSeenNR && kLock && kErrReg && kInsDup && kScan2),
                "kJLean builds on the lock-step lookups with counted duplicates");
  constexpr bool kBkt = kLean;  // held slots' buckets and the rows-not-found bitmap
  constexpr bool kCuckoo = k6 && kGroup && (V & kJCuckoo) != 0;  // PID tables only
  constexpr bool kCkSmall = kCuckoo && (V & kJCkSmall) != 0;
  constexpr bool kCkFast = kCuckoo && !kCkSmall && (V & kJCkFast) != 0;
  static_assert(!kCuckoo || kLean, "kJCuckoo empties terminated buckets through kJLean's step 4");
  using T = std::conditional_t<kWide, Tab<uint64_t>, std::conditional_t<k6, TabP, Tab<uint32_t>>>;
  using EntT = std::conditional_t<k6, uint32_t, uint64_t>;   // a bucket's entry / key word
  using SlotT = std::conditional_t<k6, uint16_t, uint32_t>;
  __shared__ __align__(16) EntT s_ent[kLdsBuckets];               // entries (packed PIDs) / keys
  __shared__ __align__(16) SlotT s_slot[kSplit ? kLdsBuckets : 1];  // slots (split tables)
  __shared__ uint32_t s_used[kSmallWords];  // bit s: slot s held by a live ID
  __shared__ uint32_t s_seen[kSmallWords];  // bit s: a row found slot s
  __shared__ uint32_t s_dup[kSeenNR ? kSmallWords : 1];  // kSeenNR's error path: marks with return
  __shared__ uint32_t s_fmask[kSmallWords], s_tmask[kSmallWords];  // free / terminated bits
  __shared__ uint32_t s_wpre[kSmallWords];                          // (free << 16 | term) before w
  __shared__ uint16_t s_free[kNewCap];                              // the first free slots
  __shared__ K s_newkey[kNewCap];
  __shared__ uint8_t s_newbad[kNewCap];
  __shared__ uint32_t s_dirty[kLdsBuckets / 32];
  __shared__ uint32_t s_wave[2 * kThreads / 64], s_lo[kThreads / 64], s_hi[kThreads / 64];
  __shared__ uint32_t s_occ;
  // kJLean: slot -> bucket of its live ID (valid where s_used is set), rows not found;
  // block totals (found rows), the rows' span (kJCuckoo)
  __shared__ uint16_t s_bkt[kBkt ? kSmallWords * 32 : 1];
  __shared__ uint32_t s_pend[kBkt ? kPendWords : 1];
  __shared__ uint32_t s_ppre[kLean ? kPendWords : 1];  // kJLean: rows not found before word w
  __shared__ uint32_t s_ckkey[kCuckoo ? kNewCap : 1];    // kJCuckoo: keys left to kick in
  __shared__ uint16_t s_ckrel[kCuckoo ? kNewCap : 1];
  __shared__ uint32_t s_ckn, s_ckfail;
  __shared__ uint32_t s_tot[1], s_flo, s_fhi;

  const uint32_t tid = threadIdx.x;
  constexpr int kPer = kLdsBuckets / kThreads;
  // node n's words, keys and table, loaded into registers (the loads issued, not waited for)
  struct Pf {
    bool ok;
    NodeView v;
    K key[kRpl];
    EntT ev[kPer];
    SlotT sv[kSplit ? kPer : 1];
  };
  const auto prefetch = [&](uint32_t n, Pf &p) {
    bool early = false;
    if constexpr (k6 && (V & kJUni) != 0) {
      if (a.uniform && n < a.n_nodes) {  // the table before the node words (map-uniform)
        const uint32_t *gk = reinterpret_cast<const uint32_t *>(a.ent + static_cast<uint64_t>(n) * kLdsBuckets);
        const uint16_t *gs = reinterpret_cast<const uint16_t *>(gk + kLdsBuckets);
        __builtin_memcpy(p.ev, __builtin_assume_aligned(gk + tid * kPer, 16), sizeof(p.ev));
        __builtin_memcpy(p.sv, __builtin_assume_aligned(gs + tid * kPer, 16), sizeof(p.sv));
        early = true;
      }
    }
    p.ok = n < a.n_nodes && node_view<true>(a, n, p.v);
    if (!p.ok) return;
    const NodeView &v = p.v;
    const uint32_t R = v.r1 - v.r0, H = v.H, S = v.S;
    const uint32_t Hu = kCkSmall ? min(H, max(8u, 4 * ((3 * S + 7) / 8))) : H;
    const K *__restrict__ keys = static_cast<const K *>(a.keys) + v.r0;
    if (kVec && tid * kRpl + kRpl <= R) {  // the lane's rows as one vector (4-B aligned)
      __builtin_memcpy(p.key, keys + tid * kRpl, sizeof(p.key));
    } else {
#pragma unroll
      for (int j = 0; j < kRpl; ++j) {
        const uint32_t r = tid * kRpl + j;
        p.key[j] = r < R ? keys[r] : T::kEmpty;
      }
    }
    if constexpr (k6) {
      const uint32_t *gk = reinterpret_cast<const uint32_t *>(a.ent + v.hb);
      const uint16_t *gs = reinterpret_cast<const uint16_t *>(gk + H);
      if (!early && tid * kPer < Hu) {
        __builtin_memcpy(p.ev, __builtin_assume_aligned(gk + tid * kPer, 16), sizeof(p.ev));
        __builtin_memcpy(p.sv, __builtin_assume_aligned(gs + tid * kPer, 16), sizeof(p.sv));
      }
    } else if (H) {  // node-uniform; clamped addresses keep the loads unconditional
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const uint32_t b = tid + j * kThreads, bb = b < H ? b : 0u;
        if constexpr (kWide) {
          p.ev[j] = a.ent[v.hb + bb];
          p.sv[j] = a.slots[v.hb + bb];
        } else {
          p.ev[j] = static_cast<EntT>(a.ent[v.hb + bb]);
        }
      }
    }
  };
  // the join of node n from the registers prefetch() loaded (round 6: the loads behind one
  // function and the join behind another — the same work, 3-4 % faster than the inline form,
  // 50 VGPRs instead of 53: profiles/r06/join/r06v_*.json)
  const auto join_one = [&](uint32_t n, const Pf &cur) {
  if (!cur.ok) return;
  const NodeView v = cur.v;
  const uint32_t R = v.r1 - v.r0, S = v.S, s0 = v.s0, H = v.H, hmask = H - 1;
  const uint32_t W = (S + 31) / 32;
  // kJCuckoo: the buckets in use (Hu <= H) and their 4-bucket groups
  const uint32_t Hu = kCkSmall ? min(H, max(8u, 4 * ((3 * S + 7) / 8))) : H, CG = Hu / 4;
  // the key's two groups (kJCkFast: CG = H / 4 is a power of two >= 16, csh = 32 - log2 CG)
  const uint32_t csh = kCkFast ? static_cast<uint32_t>(__builtin_clz(CG)) + 1u : 0u;
  const auto h1 = [&](uint32_t k) -> uint32_t {
    if constexpr (kCkFast) return (k * 0x9E3779B1u) >> csh;
    else return ck_g1(k, CG);
  };
  const auto h2 = [&](uint32_t k) -> uint32_t {
    if constexpr (kCkFast) {
      const uint32_t g1 = (k * 0x9E3779B1u) >> csh, g = ((k ^ (k >> 16)) * 0x85EBCA6Bu) >> csh;
      return g != g1 ? g : g1 ^ 1u;
    } else {
      return ck_g2(k, CG);
    }
  };
  if (R > kSmallRows) {  // more rows than the table's <= 2730 slots: ERANGE, map unchanged
    for (uint32_t r = tid; r < R; r += kThreads) a.out_slot[v.r0 + r] = kInvalid;
    if (tid == 0) {
      atomicOr(a.err, kErrRange);
      a.term_count[n] = 0u;
      if (a.out_span) {
        a.out_span[2 * n] = 1u;
        a.out_span[2 * n + 1] = 0u;
      }
    }
    return;
  }
  T G, L;
  if constexpr (kWide) {
    G.k = a.ent + v.hb;
    G.s = a.slots + v.hb;
    L.k = s_ent;
    L.s = s_slot;
  } else if constexpr (k6) {
    G.k = reinterpret_cast<uint32_t *>(a.ent + v.hb);
    G.s = reinterpret_cast<uint16_t *>(G.k + H);
    L.k = s_ent;
    L.s = s_slot;
  } else {
    G.e = a.ent + v.hb;
    L.e = s_ent;
  }
  auto lslot = [&](uint32_t b) -> uint32_t { return L.slot(b); };
  const Probe<K, T> pr{L, v.shift, hmask, H};
  uint32_t errs = 0;  // kErrReg: this lane's error bits
  auto raise = [&](uint32_t bits) {
    if constexpr (kErrReg)
      errs |= bits;
    else
      atomicOr(a.err, bits);
  };

  // ---- 1: table -> LDS, keys -> registers, marks cleared ---------------------------
  // All loads of the phase were issued before the first LDS store (register staging, in
  // prefetch): the node pays one memory round trip, not one per bucket.
  // kJ6B: lane tid owns buckets [kPer tid, kPer tid + kPer) — 32 B of keys and
  // 16 B of slots, 16-B aligned (H >= 64 and every node's hb a multiple of 64)
  auto bucket_of = [&](int j) -> uint32_t { return k6 ? tid * kPer + j : tid + j * kThreads; };
  K key[kRpl];
  uint32_t res[kRpl];
#pragma unroll
  for (int j = 0; j < kRpl; ++j) key[j] = cur.key[j];
  const EntT (&ev)[kPer] = cur.ev;
  const SlotT (&sv)[kSplit ? kPer : 1] = cur.sv;
  {
    for (uint32_t i = tid; i < W; i += kThreads) {
      s_used[i] = 0u;
      s_seen[i] = 0u;
      if constexpr (kSeenNR) s_dup[i] = 0u;
    }
    for (uint32_t w = tid; w < kLdsBuckets / 32; w += kThreads) s_dirty[w] = 0u;
    if (tid == 0) {
      s_occ = 0u;
      s_ckn = 0u;
      s_ckfail = 0u;
    }
    if constexpr (kBkt) {
      if (tid < kPendWords) s_pend[tid] = 0u;
      if (tid == 0) {
        s_tot[0] = 0u;
        s_flo = 0xffffffffu;
        s_fhi = 0u;
      }
    }
    if constexpr (k6) {
      if (tid * kPer < Hu) {
        __builtin_memcpy(s_ent + tid * kPer, ev, sizeof(ev));
        __builtin_memcpy(s_slot + tid * kPer, sv, sizeof(sv));
      }
    } else if (H) {
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const uint32_t b = tid + j * kThreads;
        if (b >= H) break;
        s_ent[b] = ev[j];
        if constexpr (kWide) s_slot[b] = sv[j];
      }
    }
  }
  jbar<V>();
  if (a.stop_after == 1u) return;  // timing ablation

  // ---- 2: held slots and the occupancy, from this lane's buckets still in registers;
  //         lookups ---------------------------------------------------------------------
  {
    uint32_t occ = 0;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      if (bucket_of(j) >= Hu) break;
      const auto k = T::key_of(ev[j]);
      occ += k != T::kEmpty ? 1u : 0u;
      if (k == T::kEmpty || k == T::kTomb) continue;
      uint32_t sl;
      if constexpr (kSplit)
        sl = sv[j];
      else
        sl = static_cast<uint32_t>(ev[j]);
      if (sl < S) {
        atomicOr(&s_used[sl >> 5], 1u << (sl & 31));
        if constexpr (kBkt) s_bkt[sl] = static_cast<uint16_t>(bucket_of(j));
      }
    }
    if constexpr (!kCkFast) {  // (the cuckoo table never rebuilds: kJCkFast drops the count)
      occ = (V & kJDpp) ? wave_reduce_dpp(occ, 0u, DppAdd{}) : wave_sum(occ);
      if ((tid & 63) == 0 && occ) atomicAdd(&s_occ, occ);  // buckets not empty at load
    }
  }
  uint32_t mine = 0;   // new rows of this lane
  uint32_t found = 0;  // kSeenNR: rows of this lane that found their ID
  uint32_t pm = 0;     // kJLean: bit j = row j of this lane not found
  if constexpr (kLock) {
    // every row of the lane probes in lock-step: unconditional LDS reads per depth
    uint32_t pb[kRpl];
    uint32_t state = 0;  // 2 bits per row: 0 idle, 1 probing, 2 found, 3 absent
#pragma unroll
    for (int j = 0; j < kRpl; ++j) {
      const uint32_t r = tid * kRpl + j;
      res[j] = kInvalid;
      pb[j] = kCuckoo ? 0u : bucket(key[j], v.shift);
      if (r >= R) continue;
      if (key[j] == T::kEmpty || key[j] == T::kTomb) {
        raise(kErrKey);
        continue;
      }
      state |= 1u << (2 * j);
    }
    if constexpr (kCuckoo) {
      // the key's two groups; found in either or absent (three rows at a time)
      const uint32_t wrow0 = __builtin_amdgcn_readfirstlane((tid & ~63u) * kRpl);
#pragma unroll
      for (int hh = 0; hh < kRpl; hh += kRpl / 2) {
        if (kCkFast && wrow0 >= R) break;  // wave-uniform: no row of this wave
        uint4 ga[kRpl / 2], gb[kRpl / 2];
        uint32_t g1[kRpl / 2], g2[kRpl / 2];
#pragma unroll
        for (int j = 0; j < kRpl / 2; ++j) {
          const uint32_t k = static_cast<uint32_t>(key[hh + j]);
          g1[j] = h1(k);
          g2[j] = h2(k);
          ga[j] = *reinterpret_cast<const uint4 *>(s_ent + g1[j] * 4);
          gb[j] = *reinterpret_cast<const uint4 *>(s_ent + g2[j] * 4);
        }
#pragma unroll
        for (int j = 0; j < kRpl / 2; ++j) {
          const uint32_t k = static_cast<uint32_t>(key[hh + j]);
          const uint32_t m1 = ck_match(ga[j], k), m2 = ck_match(gb[j], k);
          const uint32_t b = m1 ? g1[j] * 4 + __builtin_ctz(m1) : g2[j] * 4 + __builtin_ctz(m2 | 16u);
          const uint32_t nv = (m1 | m2) ? 2u : 3u;
          const bool act = ((state >> (2 * (hh + j))) & 3u) == 1u;
          state = act ? (state & ~(3u << (2 * (hh + j)))) | (nv << (2 * (hh + j))) : state;
          pb[hh + j] = b;
        }
      }
    } else if constexpr (kGroup) {
      // four consecutive buckets per LDS read (16 B, aligned): the probe ends at the
      // first bucket at or after pb holding the key or empty (where linear probing
      // stops; tombstones are skipped); <= H / 4 + 1 groups cover the whole table
      for (uint32_t depth = 0; depth <= H; depth += 4) {
        uint4 g[kRpl];
#pragma unroll
        for (int j = 0; j < kRpl; ++j) g[j] = *reinterpret_cast<const uint4 *>(s_ent + (pb[j] & ~3u));
        uint32_t probing = 0;
#pragma unroll
        for (int j = 0; j < kRpl; ++j) {
          const uint32_t k = static_cast<uint32_t>(key[j]), e = T::kEmpty;
          const uint32_t hm = (g[j].x == k ? 1u : 0u) | (g[j].y == k ? 2u : 0u) | (g[j].z == k ? 4u : 0u) |
                              (g[j].w == k ? 8u : 0u);
          const uint32_t em = (g[j].x == e ? 1u : 0u) | (g[j].y == e ? 2u : 0u) | (g[j].z == e ? 4u : 0u) |
                              (g[j].w == e ? 8u : 0u);
          const uint32_t o = pb[j] & 3u;
          const uint32_t f = static_cast<uint32_t>(__builtin_ctz((((hm | em) >> o) << o) | 16u));
          const bool act = ((state >> (2 * j)) & 3u) == 1u, end = f < 4u, hit = end && ((hm >> f) & 1u);
          const uint32_t nv = hit ? 2u : end ? 3u : 1u;  // found / absent / next group
          state = act ? (state & ~(3u << (2 * j))) | (nv << (2 * j)) : state;
          pb[j] = !act ? pb[j] : end ? (pb[j] & ~3u) + f : ((pb[j] | 3u) + 1u) & hmask;
          probing |= act && !end ? 1u : 0u;
        }
        if (__ballot(probing) == 0) break;
      }
    } else
    for (uint32_t depth = 0; depth < H; ++depth) {
      K kk[kRpl];
#pragma unroll
      for (int j = 0; j < kRpl; ++j) kk[j] = static_cast<K>(L.key(pb[j]));
      uint32_t probing = 0;
#pragma unroll
      for (int j = 0; j < kRpl; ++j) {
        const uint32_t sj = (state >> (2 * j)) & 3u;
        const bool hit = kk[j] == key[j], empty = kk[j] == T::kEmpty;
        const bool act = sj == 1u;
        const uint32_t nv = hit ? 2u : empty ? 3u : 1u;  // found / absent / next bucket
        state = act ? (state & ~(3u << (2 * j))) | (nv << (2 * j)) : state;
        const bool step = act && !hit && !empty;
        pb[j] = step ? ((pb[j] + 1) & hmask) : pb[j];
        probing |= step ? 1u : 0u;
      }
      if (__ballot(probing) == 0) break;
    }
#pragma unroll
    for (int j = 0; j < kRpl; ++j) {
      const uint32_t sj = (state >> (2 * j)) & 3u;
      if (sj == 3u) {
        res[j] = kPending;
        ++mine;
        pm |= 1u << j;
      } else if (sj == 2u) {
        const uint32_t sl = lslot(pb[j]);
        if (sl >= S) continue;
        const uint32_t bit = 1u << (sl & 31);
        if constexpr (kSeenNR) {
          atomicOr(&s_seen[sl >> 5], bit);
          ++found;
        } else if (atomicOr(&s_seen[sl >> 5], bit) & bit) {  // a second row with this ID
          raise(kErrKey);
          continue;
        }
        res[j] = s0 + sl;
      }
    }
    if constexpr (kBkt) {  // the rows not found (row bitmap) and the found rows' count
      if (pm) {  // this lane's rows not found: <= 2 words of the row bitmap
        uint32_t base = tid * kRpl;
        asm volatile("" : "+v"(base));  // computed here, not hoisted above the probe loop
        const uint32_t w0 = base >> 5, o = base & 31u;
        atomicOr(&s_pend[w0], pm << o);
        if (o + kRpl > 32u) atomicOr(&s_pend[w0 + 1], pm >> (32u - o));
      }
      // the found rows (duplicates included) for step 3's counting check
      const uint32_t f = wave_reduce_dpp(found, 0u, DppAdd{});
      if ((tid & 63) == 0 && f) atomicAdd(&s_tot[0], f);
    }
  } else {
#pragma unroll
    for (int j = 0; j < kRpl; ++j) {
      const uint32_t r = tid * kRpl + j;
      res[j] = kInvalid;
      if (r >= R) continue;
      const K k = key[j];
      if (k == T::kEmpty || k == T::kTomb) {
        raise(kErrKey);
        continue;
      }
      const uint32_t b = pr.find(k);
      if (b == ~0u) {
        res[j] = kPending;
        ++mine;
        continue;
      }
      const uint32_t sl = lslot(b);
      if (sl >= S) continue;
      const uint32_t bit = 1u << (sl & 31);
      if constexpr (kSeenNR) {
        atomicOr(&s_seen[sl >> 5], bit);
        ++found;
      } else if (atomicOr(&s_seen[sl >> 5], bit) & bit) {  // a second row with this ID
        raise(kErrKey);
        continue;
      }
      res[j] = s0 + sl;
    }
  }
  jbar<V>();
  if (a.stop_after == 2u) return;  // timing ablation
  // ---- 3: per-word free / terminated bits and their prefixes -------------------------
  uint32_t packed = 0;
  if (!kLean && tid < W) {
    const uint32_t used = s_used[tid], seen = s_seen[tid];
    const uint32_t valid = (tid + 1) * 32 <= S ? 0xffffffffu : ((1u << (S & 31)) - 1u);
    const uint32_t fm = ~used & valid, tm = used & ~seen & valid;
    s_fmask[tid] = fm;
    s_tmask[tid] = tm;
    packed = (static_cast<uint32_t>(__popc(fm)) << 16) | static_cast<uint32_t>(__popc(tm));
  }
  uint32_t ptot, ntot, pex = 0, rank0;  // rank0: this lane's first new-row rank
  // kSeenNR: the found rows ride in the new-row channel's high half (<= 3072 each)
  const uint32_t chan = kSeenNR ? mine | (found << 16) : mine;
  if constexpr (kLean) {
    // wave 0: the slot-bitmap words (lane, lane + 64) and their prefixes, the prefixes of
    // the rows-not-found bitmap; everyone reads them after the barrier
    if (tid < 64) {
      uint32_t base = 0, pbase = 0;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const uint32_t w = tid + 64u * i;
        uint32_t fm = 0, tm = 0;
        if (w < W) {
          const uint32_t used = s_used[w], seen = s_seen[w];
          const uint32_t valid = (w + 1) * 32 <= S ? 0xffffffffu : ((1u << (S & 31)) - 1u);
          fm = ~used & valid;
          tm = used & ~seen & valid;
          s_fmask[w] = fm;
          s_tmask[w] = tm;
        }
        const uint32_t pk = (static_cast<uint32_t>(__popc(fm)) << 16) | static_cast<uint32_t>(__popc(tm));
        const uint32_t inc = wave_scan_dpp(pk, 0u, DppAdd{});
        if (w < W) s_wpre[w] = base + inc - pk;
        base += static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(inc), 63));
        const uint32_t c = w < kPendWords ? static_cast<uint32_t>(__popc(s_pend[w])) : 0u;
        const uint32_t pinc = wave_scan_dpp(c, 0u, DppAdd{});
        if (w < kPendWords) s_ppre[w] = pbase + pinc - c;
        pbase += static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(pinc), 63));
      }
      if (tid == 0) {
        s_wave[0] = base;
        s_wave[1] = pbase;
      }
    }
    jbar<V>();
    ptot = s_wave[0];
    ntot = s_wave[1] | (s_tot[0] << 16);
    rank0 = 0;
    if (pm) {  // rows not found before this lane's first row
      uint32_t r = tid * kRpl;
      asm volatile("" : "+v"(r));
      const uint32_t w = r >> 5, below = (1u << (r & 31)) - 1u;
      rank0 = s_ppre[w] + static_cast<uint32_t>(__popc(s_pend[w] & below));
    }
  } else if constexpr (kScan2) {
    block_scan2<V>(packed, chan, s_wave, pex, rank0, ptot, ntot);
  } else {
    pex = block_scan(packed, s_wave, ptot);
    rank0 = block_scan(chan, s_wave, ntot);
  }
  if (!kLean && tid < W) s_wpre[tid] = pex;
  const uint32_t total_free = ptot >> 16, n_term = ptot & 0xffffu, n_new = ntot & 0xffffu;
  if constexpr (kSeenNR) {
    rank0 &= 0xffffu;
    // every found row set its slot's seen bit and the seen slots are exactly the
    // held ones not terminated: fewer of those than found rows = an ID given twice
    if ((ntot >> 16) != S - total_free - n_term) {  // block-uniform; the error path only
#pragma unroll
      for (int j = 0; j < kRpl; ++j) {
        if (res[j] >= kPending) continue;
        const uint32_t sl = res[j] - s0, bit = 1u << (sl & 31);
        if (atomicOr(&s_dup[sl >> 5], bit) & bit) {  // a second row with this ID
          raise(kErrKey);
          res[j] = kInvalid;
        }
      }
    }
  }
  // KACC_JOIN_REUSE_TERMINATED: new rows take this call's terminated slots first
  // (slot order), then the free ones; otherwise terminated slots are held
  const uint32_t t_first = a.reuse ? n_term : 0u, n_avail = total_free + t_first;
  if (tid == 0) a.term_count[n] = n_term;
  if constexpr (!kLean) jbar<V>();  // (kJLean: step 4's inputs were written before its barrier)
  if (a.stop_after == 3u) return;  // timing ablation

  // ---- 4: terminated list (slot order) + tombstones; the first free slots ------------
  if (kLean && n_term && tid < W) {  // the word's terminated slots, their buckets from s_bkt
    uint32_t rank = s_wpre[tid] & 0xffffu;
    for (uint32_t tm = s_tmask[tid]; tm; tm &= tm - 1, ++rank) {
      const uint32_t sl = tid * 32 + static_cast<uint32_t>(__builtin_ctz(tm));
      const uint32_t b = s_bkt[sl], pos = s0 + rank;
      a.term_key[pos] = static_cast<uint64_t>(L.key(b));
      a.term_slot[pos] = s0 + sl;
      if (a.reuse && rank < kNewCap) s_free[rank] = static_cast<uint16_t>(sl);
      if constexpr (kCuckoo)
        L.clear(b);  // no probe chain passes through a bucket: empty it
      else
        L.tomb(b);
      atomicOr(&s_dirty[b >> 5], 1u << (b & 31));
    }
  } else if (!kLean && n_term) {
    for (uint32_t b = tid; b < H; b += kThreads) {
      if (!is_live<T>(L.raw(b))) continue;
      const uint32_t sl = lslot(b);
      if (sl >= S) continue;
      const uint32_t w = sl >> 5, bit = 1u << (sl & 31);
      const uint32_t tm = s_tmask[w];
      if (!(tm & bit)) continue;
      const uint32_t rank = (s_wpre[w] & 0xffffu) + __popc(tm & (bit - 1u)), pos = s0 + rank;
      a.term_key[pos] = static_cast<uint64_t>(L.key(b));
      a.term_slot[pos] = s0 + sl;
      if (a.reuse && rank < kNewCap) s_free[rank] = static_cast<uint16_t>(sl);
      L.tomb(b);
      atomicOr(&s_dirty[b >> 5], 1u << (b & 31));
    }
  }
  const uint32_t want = min(min(n_new, n_avail), kNewCap);
  if (tid < W) {
    uint32_t p = t_first + (s_wpre[tid] >> 16);
    for (uint32_t fm = s_fmask[tid]; fm && p < want; fm &= fm - 1, ++p)
      s_free[p] = static_cast<uint16_t>(tid * 32 + __builtin_ctz(fm));
  }
  jbar<V>();
  if (a.stop_after == 4u) return;  // timing ablation

  // ---- 5: new rows take slots in row order ------------------------------------------
  auto take_slow = [&](uint32_t q) -> uint32_t {  // q-th available slot, q >= kNewCap
    const bool term = q < t_first;
    const uint32_t sh = term ? 0u : 16u, msk = term ? 0xffffu : 0xffffffffu;
    if (!term) q -= t_first;
    uint32_t lo = 0, hi = W;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) / 2;
      if (((s_wpre[mid] >> sh) & msk) <= q) lo = mid; else hi = mid;
    }
    return lo * 32 + select_bit(term ? s_tmask[lo] : s_fmask[lo], q - ((s_wpre[lo] >> sh) & msk));
  };
  const bool compact = n_new <= kNewCap;
  uint32_t q = rank0;
  uint32_t rk[kRpl];
#pragma unroll
  for (int j = 0; j < kRpl; ++j) {
    rk[j] = ~0u;
    if (res[j] != kPending) continue;
    if (q >= n_avail) {
      raise(kErrRange);
      res[j] = kInvalid;
      ++q;
      continue;
    }
    const uint32_t sl = q < kNewCap ? s_free[q] : take_slow(q);
    res[j] = (s0 + sl) | KACC_SLOT_NEW;
    rk[j] = q;
    if (compact) {
      s_newkey[q] = key[j];
      s_newbad[q] = 0;
    }
    ++q;
  }
  if constexpr (kCuckoo) {
    // the span of the rows' slots, here with the slots just handed out (an ID given twice
    // fails the call, whose outputs are then unspecified: a dropped row may widen it)
    if (a.out_span) {
      uint32_t lo = 0xffffffffu, hi = 0u;
#pragma unroll
      for (int j = 0; j < kRpl; ++j) {
        if (res[j] != kInvalid) {
          lo = min(lo, res[j] & KACC_SLOT_MASK);
          hi = max(hi, res[j] & KACC_SLOT_MASK);
        }
      }
      lo = wave_reduce_dpp(lo, 0xffffffffu, DppMin{});
      hi = wave_reduce_dpp(hi, 0u, DppMax{});
      if ((tid & 63) == 0 && lo <= hi) {
        atomicMin(&s_flo, lo);
        atomicMax(&s_fhi, hi);
      }
    }
  }
  jbar<V>();
  if (a.stop_after == 5u) return;  // timing ablation

  // ---- 6: inserts (one lane per new row); an ID given twice in the node is flagged ---
  // kJInsDup: by the insert that meets its own key on the probe path (buckets only
  // fill during this step, so of two rows with one ID the later claimant always
  // passes the earlier's bucket); otherwise by a re-probe after every insert.
  const uint32_t n_ins = min(n_new, n_avail);
  uint32_t fresh = 0;  // inserts into empty buckets (occupancy)
  auto insert_dup = [&](K k, uint32_t rel) -> uint32_t {  // bucket, ~0u full, ~1u duplicate
    uint32_t b = bucket(k, v.shift);
    for (uint32_t p = 0; p < H;) {
      const uint64_t raw = L.raw(b);
      const K kk = static_cast<K>(T::key_of(raw));
      if (kk == k) return ~1u;
      if (kk == T::kEmpty || kk == T::kTomb) {
        if (L.claim(b, raw, k, rel)) {
          fresh += kk == T::kEmpty ? 1u : 0u;
          return b;
        }
        continue;  // lost the race for this bucket: look at it again
      }
      ++p;
      b = (b + 1) & hmask;
    }
    return ~0u;
  };
  if constexpr (kCuckoo) {
    auto dirty = [&](uint32_t b) { atomicOr(&s_dirty[b >> 5], 1u << (b & 31)); };
    const uint4 *const s_grp = reinterpret_cast<const uint4 *>(s_ent);
    // an empty bucket of the emptier of k's two groups (both read at once), claimed by CAS;
    // ~0u: both groups full (the serial kicks below), ~1u: k is already there — an ID given
    // twice.  Filling the emptier group keeps the groups balanced, so a new key rarely finds
    // both full.  Two rows of one ID inserting in ONE wave read the same groups in the same
    // instruction, choose the same bucket and collide on it: the loser's retry finds the key
    const auto ck_direct = [&](uint32_t k, uint32_t rel) -> uint32_t {
      const uint32_t ga = h1(k), gb = h2(k);
      for (int tries = 0; tries < 16; ++tries) {
        const uint4 va = s_grp[ga], vb = s_grp[gb];
        if (ck_match(va, k) | ck_match(vb, k)) return ~1u;
        const uint32_t ea = ck_match(va, T::kEmpty), eb = ck_match(vb, T::kEmpty);
        if (!(ea | eb)) return ~0u;
        const bool use_a = __popc(ea) >= __popc(eb);
        const uint32_t b = (use_a ? ga : gb) * 4 + __builtin_ctz(use_a ? ea : eb);
        if (L.claim(b, T::kEmpty, k, rel)) return b;
      }
      return ~0u;  // lost the race 16 times: the kicks place it
    };
    const auto defer = [&](uint32_t k, uint32_t rel) {
      const uint32_t d = atomicAdd(&s_ckn, 1u);
      if (d < kNewCap) {
        s_ckkey[d] = k;
        s_ckrel[d] = static_cast<uint16_t>(rel);
      } else {
        atomicOr(&s_ckfail, 1u);
      }
    };
    // the new rows in windows of kNewCap ranks (one window unless mass churn): the window's
    // keys and slots listed by rank (step 5 listed the first window when it is the only one),
    // one lane per new row inserting
    for (uint32_t w0 = 0; w0 < n_ins; w0 += kNewCap) {  // block-uniform
      const uint32_t wn = min(kNewCap, n_ins - w0);
      if (!compact) {
#pragma unroll
        for (int j = 0; j < kRpl; ++j) {
          if (rk[j] == ~0u || rk[j] - w0 >= wn) continue;
          s_newkey[rk[j] - w0] = key[j];
          s_free[rk[j] - w0] = static_cast<uint16_t>((res[j] & KACC_SLOT_MASK) - s0);
          s_newbad[rk[j] - w0] = 0;
        }
        jbar<V>();
      }
      for (uint32_t i = tid; i < wn; i += kThreads) {
        const uint32_t k = static_cast<uint32_t>(s_newkey[i]), rel = s_free[i], b = ck_direct(k, rel);
        if (b == ~1u) s_newbad[i] = 1;
        else if (b == ~0u) defer(k, rel);
        else dirty(b);
      }
      jbar<V>();
      if (a.stop_after == 6u) return;  // timing ablation: direct inserts done
      if (s_ckn) {  // block-uniform: lane 0 alone places each key whose groups were full, by kicks
        if (tid == 0) {
          const uint32_t nd = min(s_ckn, kNewCap);
          for (uint32_t d = 0; d < nd; ++d) {
            uint32_t k = s_ckkey[d], rel = s_ckrel[d];
            if (ck_match(s_grp[h1(k)], k) | ck_match(s_grp[h2(k)], k)) {
              s_ckfail |= 2u;  // an ID given twice among the deferred: the check below finds it
              continue;
            }
            bool placed = false;
            for (int kick = 0; kick < kCkMaxKicks && !placed; ++kick) {
              const uint32_t ga = h1(k), gb = h2(k);
              const uint32_t ea = ck_match(s_grp[ga], T::kEmpty), eb = ck_match(s_grp[gb], T::kEmpty);
              if (ea | eb) {
                const uint32_t b = ea ? ga * 4 + __builtin_ctz(ea) : gb * 4 + __builtin_ctz(eb);
                L.k[b] = k;
                L.s[b] = static_cast<uint16_t>(rel);
                dirty(b);
                placed = true;
                break;
              }
              // evict a key of one of the groups (alternating, rotating) to its other group
              const uint32_t b = ((kick & 1) ? gb : ga) * 4 + ((kick >> 1) & 3);
              const uint32_t vk = L.k[b], vr = L.s[b];
              L.k[b] = k;
              L.s[b] = static_cast<uint16_t>(rel);
              dirty(b);
              k = vk;
              rel = vr;
            }
            if (!placed) s_ckfail |= 1u;  // a homeless key: the call fails (not reached at load <= 2/3)
          }
          s_ckn = 0u;
        }
        jbar<V>();
      }
      // inserts from more than one wave, or a deferred duplicate: an ID given twice within the
      // window may have escaped the inline check (an earlier window's entry never does: it was
      // in place before this window's inserts) — both entries sit in the ID's two groups, the
      // larger slot gives way (block-uniform; rare)
      if (wn > 64 || (s_ckfail & 2u)) {
        for (uint32_t i = tid; i < wn; i += kThreads) {
          if (s_newbad[i]) continue;
          const uint32_t k = static_cast<uint32_t>(s_newkey[i]), rel = s_free[i];
          bool drop = false;
          uint32_t mine_b = ~0u;
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const uint32_t g = t ? h2(k) : h1(k);
            for (uint32_t m = ck_match(s_grp[g], k); m; m &= m - 1) {
              const uint32_t b = g * 4 + __builtin_ctz(m), sl = L.slot(b);
              if (sl == rel) mine_b = b;
              else if (sl < rel) drop = true;
            }
          }
          if (drop && mine_b != ~0u) L.clear(mine_b);
          if (drop || mine_b == ~0u) s_newbad[i] = 1;
        }
        jbar<V>();  // the dropped duplicates' buckets are empty before step 7 writes them back
      }
#pragma unroll
      for (int j = 0; j < kRpl; ++j)
        if (rk[j] != ~0u && rk[j] - w0 < wn && s_newbad[rk[j] - w0]) {
          raise(kErrKey);
          res[j] = kInvalid;
        }
      if (w0 + kNewCap < n_ins) jbar<V>();  // the list is refilled for the next window
    }
    if (tid == 0 && (s_ckfail & 1u)) raise(kErrRange);
    if (a.stop_after == 7u) return;  // timing ablation: kicks and duplicate check done
  } else if (compact) {
    for (uint32_t i = tid; i < n_ins; i += kThreads) {
      if constexpr (kInsDup) {
        const uint32_t b = insert_dup(s_newkey[i], s_free[i]);
        if (b >= ~1u) s_newbad[i] = 1;
        else atomicOr(&s_dirty[b >> 5], 1u << (b & 31));
      } else {
        const uint32_t b = pr.insert(s_newkey[i], s_free[i], &fresh);
        if (b != ~0u) atomicOr(&s_dirty[b >> 5], 1u << (b & 31));
      }
    }
    if (fresh) atomicAdd(&s_occ, fresh);
    jbar<V>();
    if constexpr (!kInsDup) {
      for (uint32_t i = tid; i < n_ins; i += kThreads) {
        const uint32_t b = pr.find(s_newkey[i]);
        if (b == ~0u || lslot(b) != s_free[i]) s_newbad[i] = 1;
      }
      jbar<V>();
    }
#pragma unroll
    for (int j = 0; j < kRpl; ++j)
      if (rk[j] != ~0u && s_newbad[rk[j]]) {
        raise(kErrKey);
        res[j] = kInvalid;
      }
  } else {  // first interval / mass churn: each lane inserts its own rows
#pragma unroll
    for (int j = 0; j < kRpl; ++j) {
      if (rk[j] == ~0u) continue;
      if constexpr (kInsDup) {
        const uint32_t b = insert_dup(key[j], (res[j] & KACC_SLOT_MASK) - s0);
        if (b >= ~1u) {
          raise(kErrKey);
          res[j] = kInvalid;
          rk[j] = ~0u;
        } else {
          atomicOr(&s_dirty[b >> 5], 1u << (b & 31));
        }
      } else {
        const uint32_t b = pr.insert(key[j], (res[j] & KACC_SLOT_MASK) - s0, &fresh);
        if (b != ~0u) atomicOr(&s_dirty[b >> 5], 1u << (b & 31));
      }
    }
    if (fresh) atomicAdd(&s_occ, fresh);
    jbar<V>();
    if constexpr (!kInsDup) {
#pragma unroll
      for (int j = 0; j < kRpl; ++j) {
        if (rk[j] == ~0u) continue;
        const uint32_t b = pr.find(key[j]);
        if (b == ~0u || lslot(b) != (res[j] & KACC_SLOT_MASK) - s0) {
          raise(kErrKey);
          res[j] = kInvalid;
        }
      }
    }
  }

  // ---- 7: write back the changed buckets (or rebuild); slot words -------------------
  // s_occ: the buckets not empty at load (step 2) + inserts into empty buckets (step 6;
  // tombstones of step 4 keep their buckets occupied) — every write of s_occ is
  // behind step 6's barriers
  const bool rebuild = !kCuckoo && s_occ * 4 > H * 3;  // tombstones crowd the table (kJCuckoo has none)
  if (rebuild) {
    for (uint32_t b = tid; b < H; b += kThreads) L.clear(b);
    jbar<V>();
#pragma unroll
    for (int j = 0; j < kRpl; ++j) {
      if (res[j] != kInvalid) pr.insert(key[j], (res[j] & KACC_SLOT_MASK) - s0);
    }
    jbar<V>();
    for (uint32_t b = tid; b < H; b += kThreads) {
      if constexpr (kSplit) {
        G.k[b] = s_ent[b];
        G.s[b] = s_slot[b];
      } else {
        G.e[b] = s_ent[b];
      }
    }
  } else if constexpr (kCuckoo) {  // lane tid: its 8 buckets as two vector stores when any changed
    if (tid * kPer < Hu && ((s_dirty[tid >> 2] >> ((tid & 3) * 8)) & 0xffu)) {
      using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;
      const u32x4 *ks = reinterpret_cast<const u32x4 *>(s_ent + tid * kPer);
      u32x4 *kd = reinterpret_cast<u32x4 *>(G.k + tid * kPer);
      kd[0] = ks[0];
      kd[1] = ks[1];
      *reinterpret_cast<u32x4 *>(G.s + tid * kPer) = *reinterpret_cast<const u32x4 *>(s_slot + tid * kPer);
    }
  } else {
    for (uint32_t w = tid; w < H / 32; w += kThreads) {
      for (uint32_t d = s_dirty[w]; d; d &= d - 1) {
        const uint32_t b = w * 32 + __builtin_ctz(d);
        if constexpr (kSplit) {
          G.k[b] = s_ent[b];
          G.s[b] = s_slot[b];
        } else {
          G.e[b] = s_ent[b];
        }
      }
    }
  }
  if (a.stop_after == 8u) return;  // timing ablation: the changed buckets written back
  uint32_t *__restrict__ out = a.out_slot + v.r0;
  if (kVec && tid * kRpl + kRpl <= R) {
    __builtin_memcpy(out + tid * kRpl, res, sizeof(res));
  } else {
#pragma unroll
    for (int j = 0; j < kRpl; ++j)
      if (tid * kRpl + j < R) out[tid * kRpl + j] = res[j];
  }
  uint32_t lo = 0xffffffffu, hi = 0u;
#pragma unroll
  for (int j = 0; j < kRpl; ++j) {
    if (res[j] != kInvalid) {
      lo = min(lo, res[j] & KACC_SLOT_MASK);
      hi = max(hi, res[j] & KACC_SLOT_MASK);
    }
  }
  if constexpr (kErrReg) {
    if (errs) atomicOr(a.err, errs);
  }
  if (kCuckoo && a.out_span) {  // reduced before step 6's last barrier
    if (tid == 0) {
      const uint32_t flo = s_flo, fhi = s_fhi;
      a.out_span[2 * n] = flo > fhi ? 1u : flo;
      a.out_span[2 * n + 1] = flo > fhi ? 0u : fhi;
    }
  } else if (a.out_span) {
    if constexpr ((V & kJDpp) != 0) {
      lo = wave_reduce_dpp(lo, 0xffffffffu, DppMin{});
      hi = wave_reduce_dpp(hi, 0u, DppMax{});
    } else {
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) {
        lo = min(lo, static_cast<uint32_t>(__shfl_xor(static_cast<int>(lo), d, 64)));
        hi = max(hi, static_cast<uint32_t>(__shfl_xor(static_cast<int>(hi), d, 64)));
      }
    }
    if ((tid & 63) == 0) {
      s_lo[tid >> 6] = lo;
      s_hi[tid >> 6] = hi;
    }
    jbar<V>();
    if (tid == 0) {
#pragma unroll
      for (int w = 1; w < kThreads / 64; ++w) {
        lo = min(lo, s_lo[w]);
        hi = max(hi, s_hi[w]);
      }
      const bool none = lo > hi;
      a.out_span[2 * n] = none ? 1u : lo;
      a.out_span[2 * n + 1] = none ? 0u : hi;
    }
  }
  };
  {
    if (blockIdx.x >= a.n_nodes) return;
    Pf cur;
    prefetch(blockIdx.x, cur);
    join_one(blockIdx.x, cur);
  }
}

// ============================ big nodes (global table) =============================
// Same steps on the node's table in global memory; per-slot bitmaps in LDS
// (slot ranges up to kMaxRange); rows processed in chunks of kThreads.
template <typename K>
__global__ __launch_bounds__(kThreads) void join_big(const Args a) {
  using T = Tab<K>;
  __shared__ uint32_t s_used[kWords];  // slots held by live IDs
  __shared__ uint32_t s_seen[kWords];  // slots of rows found
  __shared__ uint32_t s_wpre[kWords];  // free slots before word w
  __shared__ uint32_t s_tpre[kWords];  // terminated before word w
  __shared__ uint32_t s_wave[kThreads / 64], s_lo[kThreads / 64], s_hi[kThreads / 64];
  __shared__ uint32_t s_occ;

  const uint32_t n = blockIdx.x, tid = threadIdx.x;
  if (n >= a.n_nodes) return;
  NodeView v;
  if (!node_view<false>(a, n, v)) return;
  const uint32_t r0 = v.r0, r1 = v.r1, S = v.S, s0 = v.s0, H = v.H;
  const uint32_t W = (S + 31) / 32;
  const K *__restrict__ keys = static_cast<const K *>(a.keys);
  T L;
  if constexpr (sizeof(K) == 8) {
    L.k = a.ent + v.hb;
    L.s = a.slots + v.hb;
  } else {
    L.e = a.ent + v.hb;
  }
  const Probe<K, T> pr{L, v.shift, H - 1, H};
  auto bit_set = [](uint32_t *bm, uint32_t i) {
    return (atomicOr(&bm[i >> 5], 1u << (i & 31)) >> (i & 31)) & 1u;
  };

  // ---- 1-2: bitmaps, held slots, lookups ----------------------------------------------
  for (uint32_t w = tid; w < W; w += kThreads) {
    s_used[w] = 0u;
    s_seen[w] = 0u;
  }
  if (tid == 0) s_occ = 0u;
  __syncthreads();
  if (a.stop_after == 1) return;
  for (uint32_t b = tid; b < H; b += kThreads) {
    if (!is_live<T>(L.raw(b))) continue;
    const uint32_t s = L.slot(b);
    if (s < S) atomicOr(&s_used[s >> 5], 1u << (s & 31));
  }
  for (uint32_t r = r0 + tid; r < r1; r += kThreads) {
    const K k = keys[r];
    uint32_t out = kPending;
    if (k == T::kEmpty || k == T::kTomb) {
      atomicOr(a.err, kErrKey);
      out = kInvalid;
    } else {
      const uint32_t b = pr.find(k);
      if (b != ~0u) {
        const uint32_t s = L.slot(b);
        if (s >= S) {
          out = kInvalid;
        } else if (bit_set(s_seen, s)) {  // the same ID on two rows of the node
          atomicOr(a.err, kErrKey);
          out = kInvalid;
        } else {
          out = s0 + s;
        }
      }
    }
    a.out_slot[r] = out;
  }
  __syncthreads();
  if (a.stop_after == 2) return;

  // ---- 3: terminated = held slots not seen, listed in slot order; tombstones --------
  uint32_t carry = 0;
  for (uint32_t w0 = 0; w0 < W; w0 += kThreads) {
    const uint32_t w = w0 + tid;
    const uint32_t t = w < W ? __popc(s_used[w] & ~s_seen[w]) : 0u;
    uint32_t tot;
    const uint32_t ex = block_scan(t, s_wave, tot);
    if (w < W) s_tpre[w] = carry + ex;
    carry += tot;
  }
  if (tid == 0) a.term_count[n] = carry;
  const uint32_t t_first = a.reuse ? carry : 0u;  // KACC_JOIN_REUSE_TERMINATED: terminated slots first
  __syncthreads();
  if (carry) {
    for (uint32_t b = tid; b < H; b += kThreads) {
      if (!is_live<T>(L.raw(b))) continue;
      const uint32_t s = L.slot(b);
      if (s >= S) continue;
      const uint32_t w = s >> 5, bit = 1u << (s & 31);
      const uint32_t term = s_used[w] & ~s_seen[w];
      if (!(term & bit)) continue;
      const uint32_t pos = s0 + s_tpre[w] + __popc(term & (bit - 1u));
      a.term_key[pos] = static_cast<uint64_t>(L.key(b));
      a.term_slot[pos] = s0 + s;
      L.tomb(b);
    }
  }
  if (a.stop_after == 3) return;

  // ---- 4: free slots (held at step 2), new rows in row order -------------------------
  carry = 0;
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
  auto take = [&](uint32_t q) -> uint32_t {  // q-th available slot, as a slot word
    if (q >= total_free + t_first) {
      atomicOr(a.err, kErrRange);
      return kInvalid;
    }
    if (q < t_first) {  // the q-th terminated slot (last word with s_tpre[w] <= q)
      uint32_t lo = 0, hi = W;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (s_tpre[mid] <= q) lo = mid; else hi = mid;
      }
      return (s0 + lo * 32 + select_bit(s_used[lo] & ~s_seen[lo], q - s_tpre[lo])) | KACC_SLOT_NEW;
    }
    q -= t_first;
    uint32_t lo = 0, hi = W;  // last word with s_wpre[w] <= q
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) / 2;
      if (s_wpre[mid] <= q) lo = mid; else hi = mid;
    }
    const uint32_t valid = (lo + 1) * 32 <= S ? 0xffffffffu : ((1u << (S & 31)) - 1u);
    return (s0 + lo * 32 + select_bit(~s_used[lo] & valid, q - s_wpre[lo])) | KACC_SLOT_NEW;
  };
  uint32_t taken = 0;
  for (uint32_t c0 = r0; c0 < r1; c0 += kThreads) {
    const uint32_t r = c0 + tid;
    const bool isnew = r < r1 && a.out_slot[r] == kPending;
    uint32_t tot;
    const uint32_t q = taken + block_scan(isnew ? 1u : 0u, s_wave, tot);
    if (isnew) a.out_slot[r] = take(q);
    taken += tot;
  }
  __syncthreads();  // step 3's tombstones are in place
  if (a.stop_after == 4) return;

  // ---- 5: new IDs claim buckets; a re-probe flags an ID given twice ------------------
  for (uint32_t r = r0 + tid; r < r1; r += kThreads) {
    const uint32_t w = a.out_slot[r];
    if (w != kInvalid && (w & KACC_SLOT_NEW)) pr.insert(keys[r], (w & KACC_SLOT_MASK) - s0);
  }
  __syncthreads();
  for (uint32_t r = r0 + tid; r < r1; r += kThreads) {
    const uint32_t w = a.out_slot[r];
    if (w == kInvalid || !(w & KACC_SLOT_NEW)) continue;
    const uint32_t b = pr.find(keys[r]);
    if (b == ~0u || L.slot(b) != (w & KACC_SLOT_MASK) - s0) {
      atomicOr(a.err, kErrKey);
      a.out_slot[r] = kInvalid;
    }
  }
  if (a.stop_after == 5) return;

  // ---- 6: occupancy; rebuild when tombstones crowd the table -------------------------
  {
    uint32_t occ = 0;
    for (uint32_t b = tid; b < H; b += kThreads) occ += L.key(b) != T::kEmpty ? 1u : 0u;
    occ = wave_sum(occ);
    if ((tid & 63) == 0) atomicAdd(&s_occ, occ);
  }
  __syncthreads();
  if (s_occ * 4 > H * 3) {
    for (uint32_t b = tid; b < H; b += kThreads) L.clear(b);
    __syncthreads();
    for (uint32_t r = r0 + tid; r < r1; r += kThreads) {
      const uint32_t w = a.out_slot[r];
      if (w != kInvalid) pr.insert(keys[r], (w & KACC_SLOT_MASK) - s0);
    }
  }
  if (a.out_span) {
    uint32_t lo = 0xffffffffu, hi = 0u;
    for (uint32_t r = r0 + tid; r < r1; r += kThreads) {
      const uint32_t w = a.out_slot[r];
      if (w == kInvalid) continue;
      lo = min(lo, w & KACC_SLOT_MASK);
      hi = max(hi, w & KACC_SLOT_MASK);
    }
    span_out(a, n, lo, hi, s_lo, s_hi);
  }
}

}  // namespace join
}  // namespace kacc

// =============================================================================
// C ABI
// =============================================================================

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

namespace {
// round 2's kernel (8-B packed PID buckets) and the production one
constexpr int kJoinR2 = kacc::join::kJLock | kacc::join::kJErrReg | kacc::join::kJLdsBar |
                        kacc::join::kJInsDup | kacc::join::kJScan2;
constexpr int kJoinGroup = kJoinR2 | kacc::join::kJ6B | kacc::join::kJSeenNR | kacc::join::kJVec | kacc::join::kJGroup;
constexpr int kJoinLean = kJoinGroup | kacc::join::kJLean;
constexpr int kJoinCuckoo = kJoinLean | kacc::join::kJCuckoo;
constexpr int kJoinCuckooS = kJoinCuckoo | kacc::join::kJCkSmall;
constexpr int kJoinCuckooF = kJoinCuckoo | kacc::join::kJCkFast;
constexpr int kJoinUni = kJoinCuckooF | kacc::join::kJUni;


constexpr int kJoinDefault = kJoinUni;  // production: PID tables (the u64-keyed kinds: kJoinLean)
// the PID small-table format a variant works on (kacc_slotmap.fmt)
int variant_fmt(int v) {
  return (v & kacc::join::kJCuckoo) ? ((v & kacc::join::kJCkSmall) ? 4 : (v & kacc::join::kJCkFast) ? 5 : 3)
                                    : (v & kacc::join::kJ6B) ? 1 : 0;
}
const char *fmt_name(int f) {
  return f == 5 ? "6-B cuckoo, shift hashes" : f == 4 ? "6-B cuckoo, 1.5 S buckets" : f == 3 ? "6-B cuckoo" : f == 1 ? "6-B" : "8-B";
}
int g_join_variant = -1;  // kacc_debug_set_join_variant: -1 = production (kJoinDefault)
// the variant join_small is launched with (the instantiated ones; else production)
int launched_variant(int v) {
  switch (v) {
    case 0: case 1: case 3: case 6: case 7: case 15: case kJoinR2:
    case kJoinR2 | kacc::join::kJ6B:
    case kJoinR2 | kacc::join::kJ6B | kacc::join::kJSeenNR:
    case kJoinR2 | kacc::join::kJSeenNR | kacc::join::kJVec:
    case kJoinR2 | kacc::join::kJ6B | kacc::join::kJSeenNR | kacc::join::kJVec:
    case kJoinGroup:
    case kJoinGroup | kacc::join::kJDpp:
    case kJoinLean:
    case kJoinCuckoo:
    case kJoinCuckooS:
    case kJoinCuckooF:
    case kJoinUni:
      return v;
    default: return kJoinDefault;
  }
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
  bool has_big = false;
  bool uniform = n_nodes > 0;
  for (uint32_t n = 0; n < n_nodes; ++n) {
    has_big |= hoff[n + 1] - hoff[n] > kacc::join::kLdsBuckets;
    uniform &= hoff[n] == static_cast<uint64_t>(n) * kacc::join::kLdsBuckets &&
               hoff[n + 1] - hoff[n] == kacc::join::kLdsBuckets;
  }
  if (n_nodes && slot_off[n_nodes] > cap)
    return kacc_fail(ctx, KACC_EINVAL, "slot_off[n] = %u exceeds the kind's slot capacity %llu",
                     slot_off[n_nodes], (unsigned long long)cap);
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  auto *m = new kacc_slotmap;
  m->ctx = ctx;
  m->device = ctx->device;
  m->kind = kind;
  m->n_nodes = n_nodes;
  m->total_slots = n_nodes ? slot_off[n_nodes] : 0;
  m->buckets = hoff[n_nodes];
  m->has_big = has_big;
  m->uniform = uniform;
  auto bail = [&](hipError_t e) {
    kacc_slotmap_destroy(m);
    return kacc_fail(ctx, e == hipErrorOutOfMemory ? KACC_ENOMEM : KACC_EHIP, "slot map allocation: %s",
                     hipGetErrorString(e));
  };
  hipError_t e;
  const size_t nb = std::max<uint64_t>(m->buckets, 1);
  if ((e = hipMalloc(&m->d_slot_off, 4ull * (n_nodes + 1))) != hipSuccess) return bail(e);
  if ((e = hipMalloc(&m->d_hoff, 8ull * (n_nodes + 1))) != hipSuccess) return bail(e);
  if ((e = hipMalloc(&m->d_ent, 8 * nb)) != hipSuccess) return bail(e);
  if (kind != KACC_KIND_PROC && (e = hipMalloc(&m->d_slots, 4 * nb)) != hipSuccess) return bail(e);
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
  (void)hipSetDevice(m->device);
  (void)hipDeviceSynchronize();  // no launch of this map may still be running
  (void)hipFree(m->d_slot_off);
  (void)hipFree(m->d_hoff);
  (void)hipFree(m->d_ent);
  (void)hipFree(m->d_slots);
  delete m;
}

int kacc_slotmap_reset(kacc_slotmap *m) {
  if (!m) return KACC_EINVAL;
  kacc_ctx *ctx = m->ctx;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  const size_t nb = std::max<uint64_t>(m->buckets, 1);
  // the bucket format of the PID small tables follows the join variant in force now;
  // slot_join refuses a later launch in the other format (it would misread the table)
  m->fmt = m->kind == KACC_KIND_PROC ? variant_fmt(launched_variant(g_join_variant)) : 0;
  KACC_HIP(ctx, hipMemsetAsync(m->d_ent, 0xff, 8 * nb, ctx->stream));  // every bucket empty
  KACC_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return KACC_OK;
}

static int slot_join(kacc_slotmap *m, uint32_t n_rows, const uint32_t *row_off, const void *keys,
                     const uint32_t *node_status, uint32_t *out_slot, uint64_t *term_key,
                     uint32_t *term_slot, uint32_t *term_count, uint32_t *out_span, void *stream,
                     uint32_t stop_after);


int kacc_slot_join(kacc_slotmap *m, uint32_t n_rows, const uint32_t *row_off, const void *keys,
                   const uint32_t *node_status, uint32_t *out_slot, uint64_t *term_key,
                   uint32_t *term_slot, uint32_t *term_count, uint32_t *out_span, void *stream) {
  return slot_join(m, n_rows, row_off, keys, node_status, out_slot, term_key, term_slot, term_count,
                   out_span, stream, 0u);
}

int kacc_debug_join_variant(kacc_slotmap *m, uint32_t n_rows, const uint32_t *row_off, const void *keys,
                            uint32_t *out_slot, uint64_t *term_key, uint32_t *term_slot,
                            uint32_t *term_count, void *stream, uint32_t stop_after) {
  return slot_join(m, n_rows, row_off, keys, nullptr, out_slot, term_key, term_slot, term_count,
                   nullptr, stream, stop_after);
}

int kacc_slotmap_set_policy(kacc_slotmap *m, uint32_t policy) {
  if (!m) return KACC_EINVAL;
  if (policy & ~KACC_JOIN_REUSE_TERMINATED)
    return kacc_fail(m->ctx, KACC_EINVAL, "slot map policy: unknown bits 0x%x", policy & ~KACC_JOIN_REUSE_TERMINATED);
  m->policy = policy;
  return KACC_OK;
}

int kacc_debug_set_join_variant(int variant) {
  const int prev = g_join_variant;
  g_join_variant = variant;
  return prev;
}

}  // extern "C"

static int slot_join(kacc_slotmap *m, uint32_t n_rows, const uint32_t *row_off, const void *keys,
                     const uint32_t *node_status, uint32_t *out_slot, uint64_t *term_key,
                     uint32_t *term_slot, uint32_t *term_count, uint32_t *out_span, void *stream,
                     uint32_t stop_after) {
  if (!m) return KACC_EINVAL;
  kacc_ctx *ctx = m->ctx;
  if (!m->n_nodes) return KACC_OK;
  if (!row_off || !out_slot || !term_count || !term_key || !term_slot)
    return kacc_fail(ctx, KACC_EINVAL, "slot join: NULL argument");
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  if (n_rows && !keys) return kacc_fail(ctx, KACC_EINVAL, "slot join: keys is NULL");
  kacc::join::Args a{};
  a.n_nodes = m->n_nodes;
  a.n_rows = n_rows;
  a.stop_after = stop_after;
  a.reuse = (m->policy & KACC_JOIN_REUSE_TERMINATED) ? 1u : 0u;
  a.row_off = row_off;
  a.keys = keys;
  a.node_status = node_status;
  a.out_slot = out_slot;
  a.term_key = term_key;
  a.term_slot = term_slot;
  a.term_count = term_count;
  a.out_span = out_span;
  a.slot_off = m->d_slot_off;
  a.hoff = m->d_hoff;
  a.ent = m->d_ent;
  a.slots = m->d_slots;
  a.err = ctx->d_err;
  (void)hipGetLastError();  // a stale error of an earlier call must not be blamed on this launch
  using namespace kacc::join;
  const dim3 grid(m->n_nodes), block(kThreads);
  // the table format follows the variant: a map keeps the format of its reset
  const int var = launched_variant(g_join_variant);
  const int fmt = m->kind == KACC_KIND_PROC ? variant_fmt(var) : 0;
  a.fmt6 = fmt == 1 ? 1u : 0u;
  a.uniform = m->uniform ? 1u : 0u;
  if (fmt != m->fmt)
    return kacc_fail(ctx, KACC_EINVAL,
                     "slot join: the join variant's table format (%s) differs from the map's "
                     "(%s, fixed at its last reset): reset the map first",
                     fmt_name(fmt), fmt_name(m->fmt));
  auto small = [&](auto key) {
    using K = decltype(key);
    switch (var) {
      case 0: hipLaunchKernelGGL((join_small<K, 0>), grid, block, 0, st, a); break;
      case 1: hipLaunchKernelGGL((join_small<K, 1>), grid, block, 0, st, a); break;
      case 3: hipLaunchKernelGGL((join_small<K, 3>), grid, block, 0, st, a); break;
      case 7: hipLaunchKernelGGL((join_small<K, 7>), grid, block, 0, st, a); break;
      case 15: hipLaunchKernelGGL((join_small<K, 15>), grid, block, 0, st, a); break;
      case 6: hipLaunchKernelGGL((join_small<K, 6>), grid, block, 0, st, a); break;
      case kJoinR2: hipLaunchKernelGGL((join_small<K, kJoinR2>), grid, block, 0, st, a); break;
      case kJoinR2 | kJ6B: hipLaunchKernelGGL((join_small<K, kJoinR2 | kJ6B>), grid, block, 0, st, a); break;
      case kJoinR2 | kJ6B | kJSeenNR:
        hipLaunchKernelGGL((join_small<K, kJoinR2 | kJ6B | kJSeenNR>), grid, block, 0, st, a);
        break;
      case kJoinR2 | kJSeenNR | kJVec:
        hipLaunchKernelGGL((join_small<K, kJoinR2 | kJSeenNR | kJVec>), grid, block, 0, st, a);
        break;
      case kJoinR2 | kJ6B | kJSeenNR | kJVec:
        hipLaunchKernelGGL((join_small<K, kJoinR2 | kJ6B | kJSeenNR | kJVec>), grid, block, 0, st, a);
        break;
      case kJoinGroup | kJDpp: hipLaunchKernelGGL((join_small<K, kJoinGroup | kJDpp>), grid, block, 0, st, a); break;
      case kJoinGroup: hipLaunchKernelGGL((join_small<K, kJoinGroup>), grid, block, 0, st, a); break;
      case kJoinLean: hipLaunchKernelGGL((join_small<K, kJoinLean>), grid, block, 0, st, a); break;
      case kJoinCuckoo: hipLaunchKernelGGL((join_small<K, kJoinCuckoo>), grid, block, 0, st, a); break;
      case kJoinCuckooS: hipLaunchKernelGGL((join_small<K, kJoinCuckooS>), grid, block, 0, st, a); break;
      case kJoinCuckooF: hipLaunchKernelGGL((join_small<K, kJoinCuckooF>), grid, block, 0, st, a); break;
      case kJoinUni: hipLaunchKernelGGL((join_small<K, kJoinUni>), grid, block, 0, st, a); break;
      default:
        if constexpr (sizeof(K) == 4)
          hipLaunchKernelGGL((join_small<K, kJoinDefault>), grid, block, 0, st, a);
        else  // kJCuckoo places 6-B PID tables only
          hipLaunchKernelGGL((join_small<K, kJoinLean>), grid, block, 0, st, a);
        break;
    }
  };
  if (m->kind == KACC_KIND_PROC) {
    small(uint32_t{});
    if (m->has_big) hipLaunchKernelGGL((join_big<uint32_t>), grid, block, 0, st, a);
  } else {
    small(uint64_t{});
    if (m->has_big) hipLaunchKernelGGL((join_big<uint64_t>), grid, block, 0, st, a);
  }
  KACC_HIP(ctx, hipGetLastError());
  return KACC_OK;
}


