// Device-side Go arithmetic for the attribution engine (gfx950).
//
// Go on amd64 (GOAMD64=v1) evaluates float64 with SSE2 and never contracts
// a*b+c into an FMA; the engine is compiled with -ffp-contract=off so every
// product and sum below rounds exactly once, as in Go.  f64 division and the
// u64->f64 conversion are correctly rounded on AMDGPU (div_scale/div_fmas/
// div_fixup; cvt_f64_u32 hi*2^32 + lo with one rounding), matching Go.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kacc {

constexpr double kTwo63 = 9223372036854775808.0;

// CVTTSD2SQ semantics: truncate toward zero, NaN / out of range -> INT64_MIN.
__device__ __forceinline__ int64_t cvttsd2sq(double x) {
  if (!(x >= -kTwo63 && x < kTwo63)) return INT64_MIN;
  return static_cast<int64_t>(x);
}

// Go float64 -> uint64 conversion on amd64 (cmd/compile ssagen
// float64ToUint64): x < 2^63 ? int64(x) : int64(x - 2^63) | 1<<63.
// Energies of one interval fit 32 bits (4.29e9 µJ) almost always: for x in
// (-1, 2^32) truncation is one v_cvt_u32_f64 (the same value as CVTTSD2SQ), and
// the general expansion runs only when some lane of the wave needs it.
__device__ __forceinline__ uint64_t go_f64_to_u64(double x) {
  if (__builtin_expect(x > -1.0 && x < 4294967296.0, 1)) return static_cast<uint32_t>(x);
  if (x < kTwo63) return static_cast<uint64_t>(cvttsd2sq(x));
  return static_cast<uint64_t>(cvttsd2sq(x - kTwo63)) | 0x8000000000000000ull;
}

__device__ __forceinline__ double u2f(uint64_t v) { return static_cast<double>(v); }

// time.Time.Sub on monotonic readings: saturating int64 difference.
__device__ __forceinline__ int64_t go_sub_mono(int64_t t, int64_t u) {
  int64_t d;
  if (__builtin_sub_overflow(t, u, &d)) return t > u ? INT64_MAX : INT64_MIN;
  return d;
}

// time.Duration.Seconds(): float64(d/1e9) + float64(d%1e9)/1e9
__device__ __forceinline__ double go_duration_seconds(int64_t d) {
  const int64_t sec = d / 1000000000LL;
  const int64_t nsec = d % 1000000000LL;
  return static_cast<double>(sec) + static_cast<double>(nsec) / 1e9;
}

// internal/monitor/node.go:87-98 calculateEnergyDelta
__device__ __forceinline__ uint64_t energy_delta(uint64_t cur, uint64_t prev, uint64_t max_j) {
  if (cur >= prev) return cur - prev;
  if (max_j > 0) return (max_j - prev) + cur;
  return 0;
}

}  // namespace kacc
