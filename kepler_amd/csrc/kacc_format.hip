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
// One thread per value; each writes a fixed kFmtWidth-byte field (three
// 8-byte stores) and its length.
#include <hip/hip_runtime.h>

#include <algorithm>

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

// Field writer: up to kFmtWidth bytes in registers.
struct Field {
  char c[KACC_FMT_WIDTH];
  uint32_t n = 0;
  __device__ void put(char ch) { c[n++] = ch; }
  __device__ void puts(const char *s) {
    while (*s) put(*s++);
  }
};

// expfmt writeFloat / strconv.AppendFloat(f, 'g', -1, 64)
__device__ void write_float(double f, Field &o) {
  if (f == 1.0) return o.put('1');
  if (f == 0.0) return o.put('0');
  if (f == -1.0) return o.puts("-1");
  if (f != f) return o.puts("NaN");
  const uint64_t bits = static_cast<uint64_t>(__double_as_longlong(f));
  const bool neg = (bits >> 63) != 0;
  const uint32_t bexp = static_cast<uint32_t>((bits >> 52) & 0x7ff);
  const uint64_t frac = bits & ((1ull << 52) - 1);
  if (bexp == 0x7ff) return o.puts(neg ? "-Inf" : "+Inf");
  const Dec d = shortest(frac, bexp);
  // digits of d.m, most significant first
  char dig[20];
  int nd = 0;
  for (uint64_t m = d.m; m;) {
    const uint64_t q = div10(m);
    dig[nd++] = static_cast<char>('0' + (m - 10 * q));
    m = q;
  }
  for (int i = 0; i < nd / 2; ++i) {
    const char t = dig[i];
    dig[i] = dig[nd - 1 - i];
    dig[nd - 1 - i] = t;
  }
  const int dp = nd + d.e;  // value = 0.dig x 10^dp
  const int x = dp - 1;
  if (neg) o.put('-');
  if (x < -4 || x >= 6) {  // %e with nd-1 fraction digits
    o.put(dig[0]);
    if (nd > 1) {
      o.put('.');
      for (int i = 1; i < nd; ++i) o.put(dig[i]);
    }
    o.put('e');
    o.put(x < 0 ? '-' : '+');
    const int a = x < 0 ? -x : x;
    if (a >= 100) o.put(static_cast<char>('0' + a / 100));
    o.put(static_cast<char>('0' + (a / 10) % 10));
    o.put(static_cast<char>('0' + a % 10));
    return;
  }
  if (dp > 0) {  // %f with max(nd - dp, 0) fraction digits
    for (int i = 0; i < dp; ++i) o.put(i < nd ? dig[i] : '0');
  } else {
    o.put('0');
  }
  if (nd > dp) {
    o.put('.');
    for (int i = dp; i < nd; ++i) o.put(i >= 0 ? dig[i] : '0');
  }
}

struct Args {
  const void *src;
  uint64_t count;
  uint32_t is_energy;  // u64 µJ -> Joules(); else f64 µW -> Watts()
  char *out;
  uint8_t *len;
};

__global__ __launch_bounds__(kThreads) void format_kernel(const Args a) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (i >= a.count) return;
  double f;
  if (a.is_energy)
    f = static_cast<double>(static_cast<const uint64_t *>(a.src)[i]) / 1e6;  // energy.go:30-32
  else
    f = static_cast<const double *>(a.src)[i] / 1e6;  // energy.go:57-59
  Field o;
  write_float(f, o);
  uint64_t w[3] = {0, 0, 0};
  for (uint32_t k = 0; k < o.n; ++k) w[k >> 3] |= static_cast<uint64_t>(static_cast<uint8_t>(o.c[k])) << (8 * (k & 7));
  uint64_t *dst = reinterpret_cast<uint64_t *>(a.out + i * KACC_FMT_WIDTH);
  dst[0] = w[0];
  dst[1] = w[1];
  dst[2] = w[2];
  a.len[i] = static_cast<uint8_t>(o.n);
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
  if (!energy && !power) return kacc_fail(ctx, KACC_EINVAL, "table %d is not an energy or power table", (int)t);
  if (first > ctx->counts[t] || count > ctx->counts[t] - first)
    return kacc_fail(ctx, KACC_EINVAL, "format range outside table %d", (int)t);
  if (!count) return KACC_OK;
  if (!out || !len) return kacc_fail(ctx, KACC_EINVAL, "format: NULL output");
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  kacc::fmt::Args a{};
  a.src = static_cast<const char *>(ctx->tables[t]) + first * 8;
  a.count = count;
  a.is_energy = energy ? 1u : 0u;
  a.out = out;
  a.len = len;
  (void)hipGetLastError();  // clear a stale error of an earlier call
  const uint64_t grid = (count + kacc::fmt::kThreads - 1) / kacc::fmt::kThreads;
  if (grid > 0x7fffffffull) return kacc_fail(ctx, KACC_EINVAL, "format: count too large for one launch");
  hipLaunchKernelGGL(kacc::fmt::format_kernel, dim3(static_cast<uint32_t>(grid)), dim3(kacc::fmt::kThreads), 0,
                     st, a);
  KACC_HIP(ctx, hipGetLastError());
  return KACC_OK;
}

}  // extern "C"
