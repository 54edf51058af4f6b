// Exposition values: the numbers of Kepler's Prometheus
// exposition, formatted on the device exactly as Go writes them.
//
// power_collector.go:306-436 emits, per workload and zone,
// usage.EnergyTotal.Joules() (device/energy.go:30-32: float64(e) / 1e6) and
// usage.Power.Watts() (:57-59: p / 1e6), which the text exposition writes with
// expfmt writeFloat (prometheus/common v0.62.0): 1 / 0 / -1 / NaN / ±Inf
// spelled out, everything else strconv.AppendFloat(f, 'g', -1, 64) — the
// shortest round-trip digits, in %e form ("d.ddde±XX") when the decimal
// exponent is < -4 or >= 6, else %f form.  The labels are strings owned by
// the Go side; this kernel produces the value field of every sample line.
//
// Shortest digits: Adams' Ryū method (PLDI 2018) — the interval of decimals
// that round to the input, scaled by a 125-bit power of five
// (kacc_pow5_tables.h), shortened digit by digit; ties round to even.
// Attribution: shortest() below follows the structure of the published
// algorithm and of its reference implementation's d2s routine (Ulf Adams,
// "Ryū: fast float-to-string conversion", PLDI 2018; reference code under
// Apache-2.0 / Boost-1.0), restated for the device from the paper — the
// power-of-five tables are generated here (tools/gen_pow5_tables.py), not copied.
// Go's strconv uses the same shortest-digit definition (ryuFtoaShortest), which
// is what the exposition needs byte for byte.
// One thread per value; each writes a fixed kFmtWidth-byte field (three
// 8-byte stores) and its length.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "kacc_derive.hpp"
#include "kacc_internal.hpp"
#include "kacc_pow5_tables.h"

namespace kacc {
namespace fmt {

constexpr int kThreads = 256;
static_assert(KACC_FMT_WIDTH == 24, "three 8-byte stores per field");

__device__ __forceinline__ uint32_t pow5bits(int32_t e) {  // bit length of 5^e (e >= 1)
  return static_cast<uint32_t>((static_cast<uint32_t>(e) * 1217359u) >> 19) + 1u;
}
__device__ __forceinline__ uint32_t log10_pow2(int32_t e) {  // floor(e log10 2)
  return (static_cast<uint32_t>(e) * 78913u) >> 18;
}
__device__ __forceinline__ uint32_t log10_pow5(int32_t e) {  // floor(e log10 5)
  return (static_cast<uint32_t>(e) * 732923u) >> 20;
}
// Exact u64 division by 5 / 10 / 100 via multiply-high (no software divide).
__device__ __forceinline__ uint64_t div5(uint64_t x) { return __umul64hi(x, 0xCCCCCCCCCCCCCCCDull) >> 2; }
__device__ __forceinline__ uint64_t div10(uint64_t x) { return __umul64hi(x, 0xCCCCCCCCCCCCCCCDull) >> 3; }
__device__ __forceinline__ uint64_t div100(uint64_t x) { return __umul64hi(x >> 2, 0x28F5C28F5C28F5C3ull) >> 2; }

__device__ __forceinline__ uint32_t pow5_factor(uint64_t v) {
  uint32_t c = 0;
  for (;;) {
    const uint64_t q = div5(v);
    if (v - 5 * q != 0) break;
    v = q;
    ++c;
  }
  return c;
}
__device__ __forceinline__ bool multiple_of_pow5(uint64_t v, uint32_t p) { return pow5_factor(v) >= p; }
__device__ __forceinline__ bool multiple_of_pow2(uint64_t v, uint32_t p) {
  return (v & ((1ull << p) - 1)) == 0;
}

// (m * mul) >> j for a 125-bit multiplier, j >= 64
__device__ __forceinline__ uint64_t mul_shift(uint64_t m, const uint64_t *mul, int32_t j) {
  const unsigned __int128 b0 = static_cast<unsigned __int128>(m) * mul[0];
  const unsigned __int128 b2 = static_cast<unsigned __int128>(m) * mul[1];
  return static_cast<uint64_t>(((b0 >> 64) + b2) >> (j - 64));
}

struct Dec {
  uint64_t m;  // digits
  int32_t e;   // value = m * 10^e
};

// Shortest decimal of a positive finite double given its IEEE fields.
__device__ Dec shortest(uint64_t frac, uint32_t bexp) {
  int32_t e2;
  uint64_t m2;
  if (bexp == 0) {
    e2 = 1 - 1023 - 52 - 2;
    m2 = frac;
  } else {
    e2 = static_cast<int32_t>(bexp) - 1023 - 52 - 2;
    m2 = (1ull << 52) | frac;
  }
  const bool even = (m2 & 1) == 0;
  const uint64_t mv = 4 * m2;
  const uint32_t mm_shift = (frac != 0 || bexp <= 1) ? 1u : 0u;  // lower gap halves at a power of 2
  uint64_t vr, vp, vm;
  int32_t e10;
  bool vm_tz = false, vr_tz = false;
  if (e2 >= 0) {
    const uint32_t q = log10_pow2(e2) - (e2 > 3 ? 1u : 0u);
    e10 = static_cast<int32_t>(q);
    const int32_t k = kPow5InvBits + static_cast<int32_t>(pow5bits(static_cast<int32_t>(q))) - 1;
    const int32_t i = -e2 + static_cast<int32_t>(q) + k;
    vr = mul_shift(mv, kPow5Inv[q], i);
    vp = mul_shift(mv + 2, kPow5Inv[q], i);
    vm = mul_shift(mv - 1 - mm_shift, kPow5Inv[q], i);
    if (q <= 21) {
      if (mv - 5 * div5(mv) == 0)
        vr_tz = multiple_of_pow5(mv, q);
      else if (even)
        vm_tz = multiple_of_pow5(mv - 1 - mm_shift, q);
      else
        vp -= multiple_of_pow5(mv + 2, q) ? 1 : 0;
    }
  } else {
    const uint32_t q = log10_pow5(-e2) - (-e2 > 1 ? 1u : 0u);
    e10 = static_cast<int32_t>(q) + e2;
    const int32_t i = -e2 - static_cast<int32_t>(q);
    const int32_t k = static_cast<int32_t>(pow5bits(i)) - kPow5Bits;
    const int32_t j = static_cast<int32_t>(q) - k;
    vr = mul_shift(mv, kPow5[i], j);
    vp = mul_shift(mv + 2, kPow5[i], j);
    vm = mul_shift(mv - 1 - mm_shift, kPow5[i], j);
    if (q <= 1) {
      vr_tz = true;
      if (even)
        vm_tz = mm_shift == 1;
      else
        --vp;
    } else if (q < 63) {
      vr_tz = multiple_of_pow2(mv, q);
    }
  }
  int32_t removed = 0;
  uint32_t last = 0;
  uint64_t out;
  if (vm_tz || vr_tz) {  // rare: exact trailing zeros matter
    for (;;) {
      const uint64_t vp10 = div10(vp), vm10 = div10(vm);
      if (vp10 <= vm10) break;
      const uint32_t vm_mod = static_cast<uint32_t>(vm - 10 * vm10);
      const uint64_t vr10 = div10(vr);
      const uint32_t vr_mod = static_cast<uint32_t>(vr - 10 * vr10);
      vm_tz &= vm_mod == 0;
      vr_tz &= last == 0;
      last = vr_mod;
      vr = vr10;
      vp = vp10;
      vm = vm10;
      ++removed;
    }
    if (vm_tz) {
      for (;;) {
        const uint64_t vm10 = div10(vm);
        if (vm - 10 * vm10 != 0) break;
        const uint64_t vp10 = div10(vp), vr10 = div10(vr);
        const uint32_t vr_mod = static_cast<uint32_t>(vr - 10 * vr10);
        vr_tz &= last == 0;
        last = vr_mod;
        vr = vr10;
        vp = vp10;
        vm = vm10;
        ++removed;
      }
    }
    if (vr_tz && last == 5 && vr % 2 == 0) last = 4;  // exactly ...50..0: round half to even
    out = vr + (((vr == vm && (!even || !vm_tz)) || last >= 5) ? 1 : 0);
  } else {
    bool up = false;
    const uint64_t vp100 = div100(vp), vm100 = div100(vm);
    if (vp100 > vm100) {
      const uint64_t vr100 = div100(vr);
      up = vr - 100 * vr100 >= 50;
      vr = vr100;
      vp = vp100;
      vm = vm100;
      removed += 2;
    }
    for (;;) {
      const uint64_t vp10 = div10(vp), vm10 = div10(vm);
      if (vp10 <= vm10) break;
      const uint64_t vr10 = div10(vr);
      up = vr - 10 * vr10 >= 5;
      vr = vr10;
      vp = vp10;
      vm = vm10;
      ++removed;
    }
    out = vr + ((vr == vm || up) ? 1 : 0);
  }
  return Dec{out, e10 + removed};
}

// The value field in registers: a 24-byte little-endian byte string (byte k
// of the text = bits 8(k & 7) of word k >> 3), assembled with whole-word
// shifts and masks — no per-byte indexing (a dynamically indexed register
// array compiles to select chains: ~4k instructions per value before).
struct Text {
  uint64_t w[3];
  uint32_t n;  // bytes
};

__device__ __forceinline__ void shl_bytes(uint64_t (&w)[3], uint32_t k) {  // bytes move up by k (< 24)
  const uint32_t s = 8 * k;
  if (s >= 128) {
    w[2] = w[0] << (s - 128);
    w[1] = 0;
    w[0] = 0;
  } else if (s >= 64) {
    const uint32_t t = s - 64;
    w[2] = (w[1] << t) | (t ? w[0] >> (64 - t) : 0);
    w[1] = w[0] << t;
    w[0] = 0;
  } else if (s) {
    w[2] = (w[2] << s) | (w[1] >> (64 - s));
    w[1] = (w[1] << s) | (w[0] >> (64 - s));
    w[0] <<= s;
  }
}
__device__ __forceinline__ void shr_bytes(uint64_t (&w)[3], uint32_t k) {  // bytes move down by k (< 24)
  const uint32_t s = 8 * k;
  if (s >= 128) {
    w[0] = w[2] >> (s - 128);
    w[1] = 0;
    w[2] = 0;
  } else if (s >= 64) {
    const uint32_t t = s - 64;
    w[0] = (w[1] >> t) | (t ? w[2] << (64 - t) : 0);
    w[1] = w[2] >> t;
    w[2] = 0;
  } else if (s) {
    w[0] = (w[0] >> s) | (w[1] << (64 - s));
    w[1] = (w[1] >> s) | (w[2] << (64 - s));
    w[2] >>= s;
  }
}
// bytes [0, k) of w stay, the rest are cleared (k <= 24)
__device__ __forceinline__ void keep_bytes(uint64_t (&w)[3], uint32_t k) {
  const uint32_t s = 8 * k;
  w[0] &= s >= 64 ? ~0ull : (1ull << s) - 1;
  w[1] &= s >= 128 ? ~0ull : s <= 64 ? 0ull : (1ull << (s - 64)) - 1;
  w[2] &= s >= 192 ? ~0ull : s <= 128 ? 0ull : (1ull << (s - 128)) - 1;
}
// the byte string c (up to 8 bytes, at most 24 - k of them) ORed in at byte k
__device__ __forceinline__ void or_at(uint64_t (&w)[3], uint32_t k, uint64_t c) {
  uint64_t v[3] = {c, 0, 0};
  shl_bytes(v, k);
  w[0] |= v[0];
  w[1] |= v[1];
  w[2] |= v[2];
}
// byte c inserted at position p: bytes [p, 23) move up by one
__device__ __forceinline__ void insert_byte(uint64_t (&w)[3], uint32_t p, uint8_t c) {
  uint64_t hi[3] = {w[0], w[1], w[2]};
  shl_bytes(hi, 1);
  uint64_t m[3] = {~0ull, ~0ull, ~0ull};
  keep_bytes(m, p + 1);  // bytes [0, p] of the shifted copy are dropped
  keep_bytes(w, p);
  w[0] |= hi[0] & ~m[0];
  w[1] |= hi[1] & ~m[1];
  w[2] |= hi[2] & ~m[2];
  or_at(w, p, c);
}

// Four / eight ASCII digits of v (leading zeros kept), most significant at byte 0.
__device__ __forceinline__ uint32_t ascii4(uint32_t v) {  // v < 10^4
  const uint32_t a = (v * 5243u) >> 19;                    // v / 100 (exact for v < 43699)
  const uint32_t b = v - a * 100u;
  const uint32_t a1 = (a * 103u) >> 10, b1 = (b * 103u) >> 10;  // / 10 (exact below 179)
  return 0x30303030u | a1 | ((a - a1 * 10u) << 8) | (b1 << 16) | ((b - b1 * 10u) << 24);
}
__device__ __forceinline__ uint64_t ascii8(uint32_t v) {  // v < 10^8
  const uint32_t hi = __umulhi(v, 0xD1B71759u) >> 13;      // v / 10^4
  return static_cast<uint64_t>(ascii4(hi)) | (static_cast<uint64_t>(ascii4(v - hi * 10000u)) << 32);
}

// Digit count of m (1 <= m < 10^17).
__device__ __forceinline__ uint32_t digits10(uint64_t m) {
  uint32_t nd = 1;
  uint64_t p = 10;
#pragma unroll
  for (int k = 1; k < 17; ++k, p *= 10) nd += m >= p ? 1u : 0u;
  return nd;
}

// strconv 'g' -1 layout (the %e / %f choice of Go's %g with shortest digits) of
// the decimal m x 10^e10 (m < 10^17 with no trailing zero), after the sign.
__device__ void write_dec(bool neg, Dec d, Text &t) {
  const uint64_t m = d.m;
  const uint64_t q = __umul64hi(m, 0xABCC77118461CEFDull) >> 26;  // m / 10^8 (m < 2^64)
  const uint32_t r = static_cast<uint32_t>(m - q * 100000000ull);
  const uint32_t q32 = static_cast<uint32_t>(q);                  // < 10^9
  const uint32_t q1 = __umulhi(q32, 0xABCC7712u) >> 26;          // q / 10^8 (< 10)
  const uint32_t q0 = q32 - q1 * 100000000u;
  const uint64_t a0 = ascii8(q0), a1 = ascii8(r);
  // the 17 digits, most significant first, then drop the leading zeros
  uint64_t w[3] = {(0x30ull + q1) | (a0 << 8), (a0 >> 56) | (a1 << 8), a1 >> 56};
  const uint32_t nd = digits10(m);
  shr_bytes(w, 17 - nd);
  keep_bytes(w, nd);
  const int32_t dp = static_cast<int32_t>(nd) + d.e;  // value = 0.DIGITS x 10^dp
  const int32_t x = dp - 1;
  uint32_t n;
  if (x < -4 || x >= 6) {  // %e with nd - 1 fraction digits
    n = nd;
    if (nd > 1) {
      insert_byte(w, 1, '.');
      ++n;
    }
    const uint32_t ax = static_cast<uint32_t>(x < 0 ? -x : x);
    const uint32_t h = ax / 100, tt = (ax / 10) % 10, u = ax % 10;
    uint64_t suf = 'e' | (static_cast<uint64_t>(x < 0 ? '-' : '+') << 8);
    uint32_t sl = 2;
    if (h) suf |= static_cast<uint64_t>('0' + h) << (8 * sl++);
    suf |= static_cast<uint64_t>('0' + tt) << (8 * sl++);
    suf |= static_cast<uint64_t>('0' + u) << (8 * sl++);
    or_at(w, n, suf);
    n += sl;
  } else if (dp >= static_cast<int32_t>(nd)) {  // integer: dp - nd zeros (at most 5)
    or_at(w, nd, 0x303030303030ull & ((1ull << (8 * (dp - nd))) - 1));
    n = static_cast<uint32_t>(dp);
  } else if (dp > 0) {  // d.ddd
    insert_byte(w, static_cast<uint32_t>(dp), '.');
    n = nd + 1;
  } else {  // 0.000ddd: 2 - dp bytes before the digits (dp >= -3)
    const uint32_t pre = static_cast<uint32_t>(2 - dp);
    shl_bytes(w, pre);
    w[0] |= 0x303030302E30ull & ((1ull << (8 * pre)) - 1);  // "0." then zeros
    n = nd + pre;
  }
  if (neg) {
    shl_bytes(w, 1);
    w[0] |= '-';
    ++n;
  }
  t.w[0] = w[0];
  t.w[1] = w[1];
  t.w[2] = w[2];
  t.n = n;
}

// expfmt writeFloat / strconv.AppendFloat(f, 'g', -1, 64)
__device__ void write_float(double f, Text &t) {
  t.w[1] = t.w[2] = 0;
  if (f == 1.0) { t.w[0] = '1'; t.n = 1; return; }
  if (f == 0.0) { t.w[0] = '0'; t.n = 1; return; }
  if (f == -1.0) { t.w[0] = 0x312Dull; t.n = 2; return; }        // "-1"
  if (f != f) { t.w[0] = 0x4E614Eull; t.n = 3; return; }          // "NaN"
  const uint64_t bits = static_cast<uint64_t>(__double_as_longlong(f));
  const bool neg = (bits >> 63) != 0;
  const uint32_t bexp = static_cast<uint32_t>((bits >> 52) & 0x7ff);
  const uint64_t frac = bits & ((1ull << 52) - 1);
  if (bexp == 0x7ff) { t.w[0] = neg ? 0x666E492Dull : 0x666E492Bull; t.n = 4; return; }  // "-Inf" / "+Inf"
  write_dec(neg, shortest(frac, bexp), t);
}

// Joules() of a u64 µJ energy, float64(e) / 1e6 (energy.go:30-32), written as
// write_float writes it.  Below 10^15 µJ the decimal e·10^-6 has at most 15
// significant digits, and it rounds to the quotient (a correctly rounded
// division); distinct decimals of <= 15 significant digits are distinct
// doubles (DBL_DIG = 15), so no other decimal of that length or shorter lies
// in the quotient's rounding interval: the shortest round-trip digits are e's
// own digits with the trailing zeros dropped — no Ryū step needed.
__device__ void write_joules(uint64_t e, Text &t) {
  if (e == 0 || e == 1000000u || e >= 1000000000000000ull) return write_float(static_cast<double>(e) / 1e6, t);
  uint64_t m = e;
  int32_t x = -6;
  for (;;) {
    const uint64_t q = div10(m);
    if (m - 10 * q != 0) break;
    m = q;
    ++x;
  }
  write_dec(false, Dec{m, x}, t);
}

struct Args {
  const void *src;
  uint64_t count;
  uint32_t is_energy;  // u64 µJ -> Joules(); else f64 / div
  double div;          // 1e6: µW -> Watts(); 1: a plain float64 (Node.UsageRatio)
  char *out;
  uint8_t *len;
};

__global__ __launch_bounds__(kThreads) void format_kernel(const Args a) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (i >= a.count) return;
  Text o;
  if (a.is_energy)
    write_joules(static_cast<const uint64_t *>(a.src)[i], o);  // energy.go:30-32
  else
    write_float(static_cast<const double *>(a.src)[i] / a.div, o);  // energy.go:57-59 (x / 1 == x)
  uint64_t *dst = reinterpret_cast<uint64_t *>(a.out + i * KACC_FMT_WIDTH);
  dst[0] = o.w[0];
  dst[1] = o.w[1];
  dst[2] = o.w[2];
  a.len[i] = static_cast<uint8_t>(o.n);
}

// ---- sample lines: NAME{LABELS,zone="ZONE"} VALUE\n ------------------------------
// Constants of one call, staged in LDS: the metric name, then the zone names.
constexpr uint32_t kConstCap = 1024;
constexpr int kLineWaves = 2;  // line_write_kernel: waves per workgroup (16 KiB of LDS each)

struct LineArgs {
  uint64_t src_first;  // element index of src[0] (a derived table materialised from its row `first`)
  const void *src;       // table base
  uint32_t Z;            // table zones
  uint32_t is_energy;
  uint64_t first, count;  // rows (slots) [first, first + count)
  uint32_t n_zones;
  const uint32_t *row_order;  // device [count] or NULL
  const char *labels;         // device
  const uint64_t *label_off;  // device [count + 1]
  const char *consts;         // device: name, then zone names
  uint32_t name_len;
  uint32_t zone_table[KACC_MAX_ZONES];  // table zone of line zone j
  uint32_t zone_pos[KACC_MAX_ZONES + 1];  // zone name j = consts[zone_pos[j], + zone_len[j]) (4-aligned)
  uint32_t zone_len[KACC_MAX_ZONES];
  uint32_t const_len;
  uint64_t *len;     // temp [lines + 1]
  uint64_t *line_off;  // [lines + 1]
  char *out;
  uint64_t out_cap;
  uint32_t *err;       // context error word (a line past out_cap is not written)
};

__device__ __forceinline__ uint64_t line_row(const LineArgs &a, uint64_t r) {
  // a row_order entry past the range is clamped: wrong text, never a fault
  return a.row_order ? min(static_cast<uint64_t>(a.row_order[r]), a.count - 1) : r;
}

// The value field of table entry e (the write pass formats it again instead
// of reading a stored copy: the formatting is cheaper than 2 x 24 B of traffic).
__device__ __forceinline__ void line_value(const LineArgs &a, uint64_t e, Text &o) {
  if (a.is_energy)
    write_joules(static_cast<const uint64_t *>(a.src)[e - a.src_first], o);  // energy.go:30-32
  else
    write_float(static_cast<const double *>(a.src)[e - a.src_first] / 1e6, o);  // energy.go:57-59
}

// Pass 1: the length of every line.
__global__ __launch_bounds__(kThreads) void line_len_kernel(const LineArgs a) {
  const uint64_t lines = a.count * a.n_zones;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x; i < lines;
       i += static_cast<uint64_t>(gridDim.x) * kThreads) {
    const uint64_t ri = i / a.n_zones;
    const uint32_t j = static_cast<uint32_t>(i - ri * a.n_zones);
    const uint64_t r = line_row(a, ri);
    const uint64_t e = (a.first + r) * a.Z + a.zone_table[j];
    Text o;
    line_value(a, e, o);
    const uint64_t ll = a.label_off[r + 1] - a.label_off[r];
    const uint32_t zl = a.zone_len[j];
    // NAME { LABELS ,zone=" ZONE "}<sp> VALUE \n
    a.len[i] = a.name_len + 1 + ll + 7 + zl + 3 + o.n + 1;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) a.len[lines] = 0;
}

// Pass 2: a wave takes 64 consecutive lines: lane l loads line (base + l)'s
// offsets in one round trip, then the wave writes the 64 lines one after the
// other, lane l writing bytes l, l + 64, ... of the line (64 contiguous bytes
// per store instruction); each line's words are broadcast with readlane.
__device__ __forceinline__ uint64_t bcast64(uint64_t x, int k) {
  const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(x), k);
  const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(x >> 32), k);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// Pass 2: a wave takes 64 consecutive lines (one contiguous byte range of the
// text).  Lane l assembles line base + l in a wave-private LDS buffer laid
// out so that buffer offset ≡ text offset (mod 16): its pieces (name, labels,
// zone, value, punctuation) are appended a dword at a time through a byte
// packer (v_alignbyte for unaligned label bytes, ds_write_b32 per full dword,
// byte stores only for the dwords it shares with its neighbour lines); then
// the wave stores the range with 16-byte stores (1 KiB per instruction).
// Lines are taken in the longest prefix that fits the buffer; a single line
// longer than the buffer is written with per-line 64-byte-wide byte stores.
#ifndef KACC_LINE_BUF
#define KACC_LINE_BUF 12288
#endif
constexpr uint32_t kLineBuf = KACC_LINE_BUF;  // bytes per wave

__device__ __forceinline__ void write_lines_bytewise(const LineArgs &a, const char *s_c, uint64_t base, uint32_t k_beg,
                                                     uint32_t k_end, uint64_t l0, uint64_t l1, uint64_t o0,
                                                     uint64_t o1, uint32_t vl, uint32_t zpair, uint64_t v0,
                                                     uint64_t v1, uint64_t v2) {
  const uint32_t lane = threadIdx.x & 63u;
  for (uint32_t k = k_beg; k < k_end; ++k) {
    const uint64_t L0 = bcast64(l0, k), LL = bcast64(l1, k) - L0;
    const uint64_t O0 = bcast64(o0, k), N = bcast64(o1, k) - O0;
    const uint32_t VL = __builtin_amdgcn_readlane(vl, k), ZP = __builtin_amdgcn_readlane(zpair, k);
    const uint32_t z0 = ZP >> 16, zl = ZP & 0xffffu;
    if (O0 > a.out_cap || N > a.out_cap - O0) {  // cannot happen with a consistent scan
      if (lane == 0) atomicOr(a.err, 1u << 8);
      continue;
    }
    const uint64_t V0 = bcast64(v0, k), V1 = bcast64(v1, k), V2 = bcast64(v2, k);
    const uint64_t cL = a.name_len + 1, cD = cL + LL, cE = cD + 7, cF = cE + zl, cG = cF + 3, cH = cG + VL;
    for (uint64_t p = lane; p < N; p += 64) {
      char c;
      if (p < a.name_len) c = s_c[p];
      else if (p < cL) c = '{';
      else if (p < cD) c = a.labels[L0 + (p - cL)];
      else if (p < cE) c = ",zone=\""[p - cD];
      else if (p < cF) c = s_c[z0 + (p - cE)];
      else if (p < cG) c = "\"} "[p - cF];
      else if (p < cH) {
        const uint32_t q = static_cast<uint32_t>(p - cG);
        c = static_cast<char>((q < 8 ? V0 : q < 16 ? V1 : V2) >> (8 * (q & 7)));
      }
      else c = '\n';
      a.out[O0 + p] = c;
    }
  }
}

// One lane's line in LDS: bytes appended to `acc` (nb of them valid), full
// dwords stored; the first `skip` bytes of the first dword belong to the line
// before, so that dword (and the last, partial one) is stored byte by byte.
struct Packer {
  uint32_t *buf;
  uint32_t d, nb, skip;
  uint64_t acc;
};

__device__ __forceinline__ void pk_put(Packer &p, uint32_t src, uint32_t k) {  // the low k (1..4) bytes of src
  const uint64_t m = k >= 4 ? 0xffffffffull : ((1ull << (8 * k)) - 1ull);
  p.acc |= (static_cast<uint64_t>(src) & m) << (8 * p.nb);
  p.nb += k;
  if (p.nb >= 4) {
    const uint32_t w = static_cast<uint32_t>(p.acc);
    if (p.skip) {
      char *c = reinterpret_cast<char *>(p.buf + p.d);
      for (uint32_t b = p.skip; b < 4; ++b) c[b] = static_cast<char>(w >> (8 * b));
      p.skip = 0;
    } else {
      p.buf[p.d] = w;
    }
    ++p.d;
    p.acc >>= 32;
    p.nb -= 4;
  }
}

__device__ __forceinline__ void pk_finish(Packer &p) {
  char *c = reinterpret_cast<char *>(p.buf + p.d);
  const uint32_t w = static_cast<uint32_t>(p.acc);
  for (uint32_t b = p.skip; b < p.nb; ++b) c[b] = static_cast<char>(w >> (8 * b));
}

__device__ __forceinline__ void pk_lds(Packer &p, const char *s_c, uint32_t pos, uint32_t len) {  // pos 4-aligned
  const uint32_t *w = reinterpret_cast<const uint32_t *>(s_c + pos);
  for (uint32_t i = 0; i < len; i += 4) pk_put(p, w[i >> 2], min(4u, len - i));
}

__global__ __launch_bounds__(64 * kLineWaves) void line_write_kernel(const LineArgs a) {
  __shared__ __attribute__((aligned(16))) char s_c[kConstCap];
  __shared__ __attribute__((aligned(16))) char s_buf[kLineWaves][kLineBuf];
  for (uint32_t k = threadIdx.x; k < a.const_len; k += 64 * kLineWaves) s_c[k] = a.consts[k];
  __syncthreads();
  const uint64_t lines = a.count * a.n_zones;
  const uint32_t lane = threadIdx.x & 63u;
  char *buf = s_buf[threadIdx.x >> 6];
  // label bytes as aligned dwords when the label buffer is dword-aligned: the
  // last readable dword is the one holding the final label byte
  const uint64_t label_bytes = a.label_off[a.count];
  const bool dw_labels = (reinterpret_cast<uintptr_t>(a.labels) & 3u) == 0 && label_bytes > 0;
  const uint64_t last_dw = label_bytes ? (label_bytes - 1) >> 2 : 0;
  const uint32_t *lw = reinterpret_cast<const uint32_t *>(a.labels);
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * kLineWaves * 64;
  // this lane's line of the batch at `bs`: its offsets and the raw table value,
  // all loads in flight together (indices clamped: the loads stay unconditional)
  struct Pre {
    uint64_t l0, l1, o0, o1, raw;
    uint32_t j;
  };
  auto fetch = [&](uint64_t bs) {
    Pre p;
    const uint64_t i = min(bs + lane, lines - 1);
    const uint64_t ri = i / a.n_zones;
    p.j = static_cast<uint32_t>(i - ri * a.n_zones);
    const uint64_t r = line_row(a, ri);
    p.l0 = a.label_off[r];
    p.l1 = a.label_off[r + 1];
    p.o0 = a.line_off[i];
    p.o1 = a.line_off[i + 1];
    p.raw = static_cast<const uint64_t *>(a.src)[(a.first + r) * a.Z + a.zone_table[p.j] - a.src_first];
    return p;
  };
  const uint64_t base0 = (static_cast<uint64_t>(blockIdx.x) * kLineWaves + (threadIdx.x >> 6)) * 64;
  Pre nxt = fetch(min(base0, lines - 1));
  for (uint64_t base = base0; base < lines; base += step) {
    // ---- this lane's line (loaded one batch ahead); the next batch's loads go out now
    const Pre cur = nxt;
    nxt = fetch(min(base + step, lines - 1));
    const uint64_t l0 = cur.l0, l1 = cur.l1, o0 = cur.o0, o1 = cur.o1;
    const uint32_t j = cur.j;
    const uint32_t zpair = (a.zone_pos[j] << 16) | a.zone_len[j];  // z0 | zl
    Text val;
    if (a.is_energy)
      write_joules(cur.raw, val);  // energy.go:30-32
    else
      write_float(__longlong_as_double(static_cast<long long>(cur.raw)) / 1e6, val);  // energy.go:57-59
    const uint32_t vl = val.n;
    const uint64_t v0 = val.w[0], v1 = val.w[1], v2 = val.w[2];
    const uint32_t nl = static_cast<uint32_t>(min<uint64_t>(lines - base, 64));
    for (uint32_t k0 = 0; k0 < nl;) {
      const uint64_t t0 = bcast64(o0, k0);
      const uint32_t shift = static_cast<uint32_t>(t0 & 15u);
      // lanes [k0, k1): the longest run of lines that fits the buffer (and out_cap)
      const bool fit = lane >= k0 && lane < nl && o1 >= t0 && o1 - t0 + shift <= kLineBuf && o1 <= a.out_cap &&
                       o0 <= o1;
      const uint64_t miss = ~__ballot(fit) >> k0;
      const uint32_t k1 = k0 + (miss ? static_cast<uint32_t>(__builtin_ctzll(miss)) : 64u - k0);
      if (k1 == k0) {  // one line longer than the buffer (or an inconsistent offset)
        write_lines_bytewise(a, s_c, base, k0, k0 + 1, l0, l1, o0, o1, vl, zpair, v0, v1, v2);
        ++k0;
        continue;
      }
      const uint64_t t1 = bcast64(o1, k1 - 1);
      if (lane >= k0 && lane < k1) {  // assemble line base + lane
        const uint32_t st = static_cast<uint32_t>(o0 - t0) + shift;
        Packer p{reinterpret_cast<uint32_t *>(buf), st >> 2, st & 3u, st & 3u, 0ull};
        pk_lds(p, s_c, 0, a.name_len);
        pk_put(p, '{', 1);
        const uint64_t n = l1 - l0;
        if (dw_labels) {  // 4 label bytes per dword pair (v_alignbyte), 8 dwords in flight
          const uint64_t q0 = l0 >> 2;
          const uint32_t sh = static_cast<uint32_t>(l0 & 3u);
          uint32_t w[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) w[q] = lw[min(q0 + q, last_dw)];
          for (uint64_t p0 = 0; p0 < n; p0 += 28) {
            uint32_t wn[8];  // the next 28 bytes' dwords go out before these are packed
#pragma unroll
            for (int q = 0; q < 8; ++q) wn[q] = lw[min(q0 + ((p0 + 28) >> 2) + q, last_dw)];
#pragma unroll
            for (int q = 0; q < 7; ++q) {
              const uint64_t at = p0 + 4u * q;
              if (at < n) pk_put(p, __builtin_amdgcn_alignbyte(w[q + 1], w[q], sh), static_cast<uint32_t>(min<uint64_t>(4, n - at)));
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) w[q] = wn[q];
          }
        } else {
          const char *lb = a.labels + l0;
          for (uint64_t p0 = 0; p0 < n; ++p0) pk_put(p, static_cast<uint8_t>(lb[p0]), 1);
        }
        pk_put(p, 0x6e6f7a2cu, 4);  // ",zon"
        pk_put(p, 0x00223d65u, 3);  // "e=\""
        pk_lds(p, s_c, zpair >> 16, zpair & 0xffffu);
        pk_put(p, 0x00207d22u, 3);  // "\"} "
        const uint32_t vd[6] = {static_cast<uint32_t>(v0), static_cast<uint32_t>(v0 >> 32), static_cast<uint32_t>(v1),
                                static_cast<uint32_t>(v1 >> 32), static_cast<uint32_t>(v2), static_cast<uint32_t>(v2 >> 32)};
#pragma unroll
        for (int q = 0; q < 6; ++q)
          if (4u * q < vl) pk_put(p, vd[q], min(4u, vl - 4u * q));
        pk_put(p, '\n', 1);
        pk_finish(p);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // ---- the range [t0, t1) out of LDS (word w = text bytes [t0 - shift + 16w, +16))
      const uint64_t g0 = t0 - shift;
      const uint32_t words = static_cast<uint32_t>((t1 - g0 + 15) / 16);
      using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;
      for (uint32_t w = lane; w < words; w += 64) {
        const uint64_t g = g0 + 16ull * w;
        if (g >= t0 && g + 16 <= t1) {
          __builtin_nontemporal_store(*reinterpret_cast<const u32x4 *>(buf + 16 * w),
                                      reinterpret_cast<u32x4 *>(a.out + g));
        } else {
          for (uint32_t b = 0; b < 16; ++b)
            if (g + b >= t0 && g + b < t1) a.out[g + b] = buf[16 * w + b];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();  // the buffer is rewritten next
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      k0 = k1;
    }
  }
}

// Exclusive scan of the u64 line lengths (reduce-then-scan, three launches,
// no inter-workgroup communication inside a launch): tiles of kTile lengths.
constexpr int kScanThreads = 256;
constexpr int kScanPer = 16;
constexpr uint64_t kTile = static_cast<uint64_t>(kScanThreads) * kScanPer;

__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t *s_w, uint64_t &total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) s_w[wave] = x;
  __syncthreads();
  uint64_t base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kScanThreads / 64; ++w) {
    if (w < wave) base += s_w[w];
    tot += s_w[w];
  }
  __syncthreads();
  total = tot;
  return base + x - v;
}

__global__ __launch_bounds__(kScanThreads) void scan_tile_sums(const uint64_t *in, uint64_t n, uint64_t *tile_sum) {
  __shared__ uint64_t s_w[kScanThreads / 64];
  const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * kTile + static_cast<uint64_t>(threadIdx.x) * kScanPer;
  uint64_t x = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) x += t0 + k < n ? in[t0 + k] : 0;
  uint64_t total;
  (void)block_excl_scan(x, s_w, total);
  if (threadIdx.x == 0) tile_sum[blockIdx.x] = total;
}

// one workgroup: tile_sum -> exclusive prefixes, in place
__global__ __launch_bounds__(kScanThreads) void scan_tile_prefix(uint64_t *tile_sum, uint64_t tiles) {
  __shared__ uint64_t s_w[kScanThreads / 64];
  uint64_t carry = 0;
  for (uint64_t b = 0; b < tiles; b += kScanThreads) {
    const uint64_t i = b + threadIdx.x;
    const uint64_t v = i < tiles ? tile_sum[i] : 0;
    uint64_t total;
    const uint64_t ex = block_excl_scan(v, s_w, total);
    if (i < tiles) tile_sum[i] = carry + ex;
    carry += total;
  }
}

__global__ __launch_bounds__(kScanThreads) void scan_tiles(const uint64_t *in, uint64_t n, const uint64_t *tile_prefix,
                                                            uint64_t *out) {
  __shared__ uint64_t s_w[kScanThreads / 64];
  const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * kTile + static_cast<uint64_t>(threadIdx.x) * kScanPer;
  uint64_t v[kScanPer], x = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    v[k] = t0 + k < n ? in[t0 + k] : 0;
    x += v[k];
  }
  uint64_t total;
  uint64_t run = tile_prefix[blockIdx.x] + block_excl_scan(x, s_w, total);
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    if (t0 + k < n) out[t0 + k] = run;
    run += v[k];
  }
}

}  // namespace fmt
}  // namespace kacc

extern "C" {

int kacc_format_values(kacc_ctx *ctx, kacc_table t, uint64_t first, uint64_t count, char *out,
                       uint8_t *len, void *stream) {
  if (!ctx || t < 0 || t >= KACC_T_COUNT) return KACC_EINVAL;
  const bool energy = t == KACC_T_NODE_ENERGY_TOTAL || t == KACC_T_NODE_ACTIVE_ENERGY ||
                      t == KACC_T_NODE_ACTIVE_TOTAL || t == KACC_T_NODE_IDLE_TOTAL ||
                      t == KACC_T_PROC_ENERGY || t == KACC_T_CTR_ENERGY || t == KACC_T_VM_ENERGY ||
                      t == KACC_T_POD_ENERGY;
  const bool power = t == KACC_T_NODE_POWER || t == KACC_T_NODE_ACTIVE_POWER || t == KACC_T_NODE_IDLE_POWER ||
                     t == KACC_T_PROC_POWER || t == KACC_T_CTR_POWER || t == KACC_T_VM_POWER ||
                     t == KACC_T_POD_POWER;
  // kepler_node_cpu_usage_ratio (power_collector.go:280-285): Node.UsageRatio as is
  const bool plain = t == KACC_T_NODE_USAGE_RATIO;
  if (!energy && !power && !plain)
    return kacc_fail(ctx, KACC_EINVAL, "table %d is not an energy, power or usage-ratio table", (int)t);
  if (first > ctx->counts[t] || count > ctx->counts[t] - first)
    return kacc_fail(ctx, KACC_EINVAL, "format range outside table %d", (int)t);
  if (!count) return KACC_OK;
  if (!out || !len) return kacc_fail(ctx, KACC_EINVAL, "format: NULL output");
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  kacc::fmt::Args a{};
  a.src = static_cast<const char *>(ctx->tables[t]) + first * 8;
  // a derived power table (kacc_derive.hpp) or a pod table (inside the pod records):
  // the range made dense first
  double *derived = nullptr;
  if (kacc_derived_kind(t) >= 0 || t == KACC_T_POD_ENERGY || t == KACC_T_POD_POWER) {
    KACC_HIP(ctx, hipMallocAsync(reinterpret_cast<void **>(&derived), count * 8, st));
    const int rc = kacc_internal_dense_range(ctx, t, first, count, derived, st);
    if (rc != KACC_OK) {
      (void)hipFreeAsync(derived, st);
      return rc;
    }
    a.src = derived;
  }
  a.count = count;
  a.is_energy = energy ? 1u : 0u;
  a.div = plain ? 1.0 : 1e6;
  a.out = out;
  a.len = len;
  (void)hipGetLastError();  // clear a stale error of an earlier call
  const uint64_t grid = (count + kacc::fmt::kThreads - 1) / kacc::fmt::kThreads;
  if (grid > 0x7fffffffull) {
    if (derived) (void)hipFreeAsync(derived, st);
    return kacc_fail(ctx, KACC_EINVAL, "format: count too large for one launch");
  }
  hipLaunchKernelGGL(kacc::fmt::format_kernel, dim3(static_cast<uint32_t>(grid)), dim3(kacc::fmt::kThreads), 0,
                     st, a);
  if (derived) (void)hipFreeAsync(derived, st);
  KACC_HIP(ctx, hipGetLastError());
  return KACC_OK;
}

int kacc_format_lines(kacc_ctx *ctx, kacc_table t, uint64_t first, uint64_t count, const char *name,
                      const char *const *zone_names, const uint32_t *zone_order, uint32_t n_zones,
                      const char *labels, const uint64_t *label_off, const uint32_t *row_order,
                      uint64_t *line_off, char *out, uint64_t out_cap, uint64_t *total, void *stream) {
  if (!ctx || t < 0 || t >= KACC_T_COUNT || !total) return KACC_EINVAL;
  *total = 0;
  const uint32_t Z = ctx->cfg.zones;
  // workload tables (rows = slots) and the node x zone tables (rows = nodes: the node
  // families of power_collector.go:246-278, one call per zone for their path label)
  const bool energy = t == KACC_T_PROC_ENERGY || t == KACC_T_CTR_ENERGY || t == KACC_T_VM_ENERGY ||
                      t == KACC_T_POD_ENERGY || t == KACC_T_NODE_ENERGY_TOTAL || t == KACC_T_NODE_ACTIVE_TOTAL ||
                      t == KACC_T_NODE_IDLE_TOTAL;
  const bool power = t == KACC_T_PROC_POWER || t == KACC_T_CTR_POWER || t == KACC_T_VM_POWER ||
                     t == KACC_T_POD_POWER || t == KACC_T_NODE_POWER || t == KACC_T_NODE_ACTIVE_POWER ||
                     t == KACC_T_NODE_IDLE_POWER;
  if (!energy && !power)
    return kacc_fail(ctx, KACC_EINVAL, "table %d is not a workload or node energy / power table", (int)t);
  const uint64_t slots = ctx->counts[t] / Z;
  if (first > slots || count > slots - first)
    return kacc_fail(ctx, KACC_EINVAL, "format_lines: rows outside table %d", (int)t);
  if (!name || !zone_names || n_zones == 0 || n_zones > Z)
    return kacc_fail(ctx, KACC_EINVAL, "format_lines: name / zone names missing or n_zones > %u", Z);
  if (count && (!labels || !label_off || !line_off))
    return kacc_fail(ctx, KACC_EINVAL, "format_lines: NULL device array");
  kacc::fmt::LineArgs a{};
  std::string consts(name);
  a.name_len = static_cast<uint32_t>(consts.size());
  auto pad4 = [&consts]() { consts.resize((consts.size() + 3) & ~size_t{3}, '\0'); };  // dword-aligned pieces
  pad4();
  for (uint32_t j = 0; j < n_zones; ++j) {
    const uint32_t z = zone_order ? zone_order[j] : j;
    if (z >= Z || !zone_names[j]) return kacc_fail(ctx, KACC_EINVAL, "format_lines: bad zone %u", j);
    a.zone_table[j] = z;
    a.zone_pos[j] = static_cast<uint32_t>(consts.size());
    a.zone_len[j] = static_cast<uint32_t>(strlen(zone_names[j]));
    consts += zone_names[j];
    pad4();
  }
  a.zone_pos[n_zones] = static_cast<uint32_t>(consts.size());
  if (consts.size() > kacc::fmt::kConstCap)
    return kacc_fail(ctx, KACC_EINVAL, "format_lines: name + zone names exceed %u bytes", kacc::fmt::kConstCap);
  if (!count) return KACC_OK;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  const uint64_t lines = count * n_zones;
  a.src = ctx->tables[t];
  a.Z = Z;
  a.is_energy = energy ? 1u : 0u;
  a.first = first;
  a.count = count;
  a.n_zones = n_zones;
  a.row_order = row_order;
  a.labels = labels;
  a.label_off = label_off;
  a.const_len = static_cast<uint32_t>(consts.size());
  a.line_off = line_off;
  a.out = out;
  a.out_cap = out_cap;
  a.err = ctx->d_err;
  // temporaries, stream ordered: consts, lengths, tile sums (+ the derived rows of
  // a derived power table, rows [first, first + count), kacc_derive.hpp)
  const uint64_t tiles = (lines + 1 + kacc::fmt::kTile - 1) / kacc::fmt::kTile;
  if (tiles > 0x7fffffffull) return kacc_fail(ctx, KACC_EINVAL, "format_lines: too many lines");
  const size_t scan_bytes = 8 * tiles;
  char *tmp = nullptr;
  // every sub-buffer 256-B aligned (the scan's look-back state needs aligned storage)
  auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
  const uint64_t off_len = 1024, off_scan = al(off_len + 8 * (lines + 1));
  const bool derived = kacc_derived_kind(t) >= 0 || t == KACC_T_POD_ENERGY || t == KACC_T_POD_POWER;
  const uint64_t off_derived = al(off_scan + scan_bytes);
  KACC_HIP(ctx, hipMallocAsync(reinterpret_cast<void **>(&tmp), derived ? off_derived + 8 * count * Z : off_scan + scan_bytes,
                               st));
  a.consts = tmp;
  a.len = reinterpret_cast<uint64_t *>(tmp + off_len);
  int rc = KACC_OK;
  auto done = [&](int code) {
    (void)hipFreeAsync(tmp, st);
    return code;
  };
  if (derived) {
    a.src = tmp + off_derived;
    a.src_first = first * Z;
    if ((rc = kacc_internal_dense_range(ctx, t, first * Z, count * Z, tmp + off_derived, st)) != KACC_OK)
      return done(rc);
  }
  if (hipMemcpyAsync(tmp, consts.data(), consts.size(), hipMemcpyHostToDevice, st) != hipSuccess)
    return done(kacc_fail(ctx, KACC_EHIP, "format_lines: constants upload"));
  (void)hipGetLastError();
  const uint64_t g1 = std::min<uint64_t>((lines + kacc::fmt::kThreads - 1) / kacc::fmt::kThreads, 1u << 20);
  hipLaunchKernelGGL(kacc::fmt::line_len_kernel, dim3(static_cast<uint32_t>(g1)), dim3(kacc::fmt::kThreads), 0, st, a);
  uint64_t *tile_sum = reinterpret_cast<uint64_t *>(tmp + off_scan);
  const dim3 gt(static_cast<uint32_t>(tiles)), bt(kacc::fmt::kScanThreads);
  hipLaunchKernelGGL(kacc::fmt::scan_tile_sums, gt, bt, 0, st, a.len, lines + 1, tile_sum);
  hipLaunchKernelGGL(kacc::fmt::scan_tile_prefix, dim3(1), bt, 0, st, tile_sum, tiles);
  hipLaunchKernelGGL(kacc::fmt::scan_tiles, gt, bt, 0, st, a.len, lines + 1, tile_sum, line_off);
  if (hipGetLastError() != hipSuccess) return done(kacc_fail(ctx, KACC_EHIP, "format_lines: scan launch"));
  if (hipMemcpyAsync(total, line_off + lines, sizeof(uint64_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return done(kacc_fail(ctx, KACC_EHIP, "format_lines: %s", hipGetErrorString(hipGetLastError())));
  if (!out) return done(KACC_OK);  // sizing call
  if (out_cap < *total)
    return done(kacc_fail(ctx, KACC_ERANGE, "format_lines: %llu bytes of text, out_cap %llu",
                          (unsigned long long)*total, (unsigned long long)out_cap));
  const uint64_t g2 = std::min<uint64_t>((lines + 64 * kacc::fmt::kLineWaves - 1) / (64 * kacc::fmt::kLineWaves),
                                         1u << 14);
  hipLaunchKernelGGL(kacc::fmt::line_write_kernel, dim3(static_cast<uint32_t>(g2)), dim3(64 * kacc::fmt::kLineWaves),
                     0, st, a);
  if (hipGetLastError() != hipSuccess) rc = kacc_fail(ctx, KACC_EHIP, "format_lines: launch");
  return done(rc);
}

}  // extern "C"
