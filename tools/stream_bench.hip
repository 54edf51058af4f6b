// Achievable-bandwidth probes for the attribution kernel's access mix (gfx950).
//
// Per "row" the process pass reads 8 B (Δ) + 4 B (slot) + 32 B (prev energy,
// Z = 4) and writes 32 B (energy) + 32 B (power).  These probes move the same
// bytes with different instruction shapes so the interval kernel can be
// priced against what the chip actually sustains for this mix:
//   copy16   : float4 copy (the classic HBM probe)
//   mix_rows : one lane per row, 2x16-B loads / 4x16-B stores at a 32-B row
//              stride (the interval kernel's shape), + 8-B and 4-B loads
//   mix_lin  : same bytes, every wave instruction touching 1 KiB contiguous
//   mix_zmaj : zone-major tables, 8-B per lane per zone (fully coalesced)
// Build: hipcc -O3 --offload-arch=gfx950 -o stream_bench stream_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));      \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

using u64x2 = __attribute__((ext_vector_type(2))) unsigned long long;
using f64x2 = __attribute__((ext_vector_type(2))) double;

__global__ void copy16(const float4 *__restrict__ a, float4 *__restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    b[i] = a[i];
}

// row-per-lane, Z = 4
__global__ void mix_rows(const double *__restrict__ d, const unsigned *__restrict__ slot,
                         u64x2 *__restrict__ energy, f64x2 *__restrict__ power, size_t rows) {
  for (size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r < rows; r += (size_t)gridDim.x * blockDim.x) {
    const double x = d[r];
    const size_t s = slot[r];
    u64x2 e0 = energy[2 * s], e1 = energy[2 * s + 1];
    e0.x += (unsigned long long)x;
    e0.y += 1;
    e1.x += 2;
    e1.y += 3;
    energy[2 * s] = e0;
    energy[2 * s + 1] = e1;
    f64x2 p0, p1;
    p0.x = x;
    p0.y = x * 2;
    p1.x = x * 3;
    p1.y = x * 4;
    power[2 * s] = p0;
    power[2 * s + 1] = p1;
  }
}

// same bytes, each wave instruction 1 KiB contiguous: lane l of a wave handles
// the 16-B piece l of a 64-row group's energy block (2 KiB), etc.
__global__ void mix_lin(const double *__restrict__ d, const unsigned *__restrict__ slot,
                        u64x2 *__restrict__ energy, f64x2 *__restrict__ power, size_t rows) {
  const size_t lane = threadIdx.x & 63;
  const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t g = wave; g * 64 < rows; g += waves) {
    const size_t r = g * 64 + lane;
    const double x = r < rows ? d[r] : 0.0;
    const unsigned s = r < rows ? slot[r] : 0;
    // 64 rows x 32 B = 2 KiB of energy = 2 wave instructions of 1 KiB
    u64x2 e0 = energy[g * 128 + lane], e1 = energy[g * 128 + 64 + lane];
    e0.x += (unsigned long long)x + s;
    e1.y += 1;
    energy[g * 128 + lane] = e0;
    energy[g * 128 + 64 + lane] = e1;
    f64x2 p0, p1;
    p0.x = x;
    p0.y = x * 2;
    p1.x = x * 3;
    p1.y = x * 4;
    power[g * 128 + lane] = p0;
    power[g * 128 + 64 + lane] = p1;
  }
}

// zone-major: energy[z][slot], power[z][slot]
__global__ void mix_zmaj(const double *__restrict__ d, const unsigned *__restrict__ slot,
                         unsigned long long *__restrict__ energy, double *__restrict__ power,
                         size_t rows) {
  for (size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r < rows; r += (size_t)gridDim.x * blockDim.x) {
    const double x = d[r];
    const size_t s = slot[r];
#pragma unroll
    for (int z = 0; z < 4; ++z) {
      energy[z * rows + s] += (unsigned long long)x + z;
      power[z * rows + s] = x * (z + 1);
    }
  }
}

// 4 float4 per thread in flight
__global__ void copy16x4(const float4 *__restrict__ a, float4 *__restrict__ b, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += 4 * stride) {
    float4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = i + k * stride < n ? a[i + k * stride] : float4{};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i + k * stride < n) b[i + k * stride] = v[k];
  }
}

// zone-major with 4 rows per lane in flight
__global__ void mix_zmaj4(const double *__restrict__ d, const unsigned *__restrict__ slot,
                          unsigned long long *__restrict__ energy, double *__restrict__ power,
                          size_t rows) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t r0 = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r0 < rows; r0 += 4 * stride) {
    double x[4];
    size_t s[4];
    unsigned long long e[4][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const size_t r = r0 + k * stride;
      x[k] = r < rows ? d[r] : 0.0;
      s[k] = r < rows ? slot[r] : 0;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int z = 0; z < 4; ++z) e[k][z] = r0 + k * stride < rows ? energy[z * rows + s[k]] : 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (r0 + k * stride >= rows) continue;
#pragma unroll
      for (int z = 0; z < 4; ++z) {
        energy[z * rows + s[k]] = e[k][z] + (unsigned long long)x[k] + z;
        power[z * rows + s[k]] = x[k] * (z + 1);
      }
    }
  }
}

// row-major (the interval kernel's shape) with 4 rows per lane in flight
__global__ void mix_rows4(const double *__restrict__ d, const unsigned *__restrict__ slot,
                          u64x2 *__restrict__ energy, f64x2 *__restrict__ power, size_t rows) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t r0 = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r0 < rows; r0 += 4 * stride) {
    double x[4];
    size_t s[4];
    u64x2 e[4][2];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const size_t r = r0 + k * stride;
      x[k] = r < rows ? d[r] : 0.0;
      s[k] = r < rows ? slot[r] : 0;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      e[k][0] = energy[2 * s[k]];
      e[k][1] = energy[2 * s[k] + 1];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (r0 + k * stride >= rows) continue;
      e[k][0].x += (unsigned long long)x[k];
      e[k][1].y += 1;
      energy[2 * s[k]] = e[k][0];
      energy[2 * s[k] + 1] = e[k][1];
      f64x2 p0, p1;
      p0.x = x[k];
      p0.y = x[k] * 2;
      p1.x = x[k] * 3;
      p1.y = x[k] * 4;
      power[2 * s[k]] = p0;
      power[2 * s[k] + 1] = p1;
    }
  }
}

// 1 KiB-contiguous shape with 4 groups per wave in flight; NT: nontemporal
// stores (and loads of the streamed inputs) for the tables that are not re-read
template <bool NT>
__global__ void mix_lin4(const double *__restrict__ d, const unsigned *__restrict__ slot,
                         u64x2 *__restrict__ energy, f64x2 *__restrict__ power, size_t rows) {
  const size_t lane = threadIdx.x & 63;
  const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
  const size_t groups = (rows + 63) / 64;
  for (size_t g0 = wave; g0 < groups; g0 += 4 * waves) {
    double x[4];
    unsigned s[4];
    u64x2 e[4][2];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const size_t g = g0 + k * waves;
      const size_t r = g * 64 + lane;
      const bool ok = g < groups && r < rows;
      x[k] = ok ? (NT ? __builtin_nontemporal_load(d + r) : d[r]) : 0.0;
      s[k] = ok ? (NT ? __builtin_nontemporal_load(slot + r) : slot[r]) : 0u;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const size_t g = min(g0 + k * waves, groups - 1);
      e[k][0] = energy[g * 128 + lane];
      e[k][1] = energy[g * 128 + 64 + lane];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const size_t g = g0 + k * waves;
      if (g >= groups) continue;
      e[k][0].x += (unsigned long long)x[k] + s[k];
      e[k][1].y += 1;
      f64x2 p0, p1;
      p0.x = x[k];
      p0.y = x[k] * 2;
      p1.x = x[k] * 3;
      p1.y = x[k] * 4;
      if (NT) {
        __builtin_nontemporal_store(e[k][0], energy + g * 128 + lane);
        __builtin_nontemporal_store(e[k][1], energy + g * 128 + 64 + lane);
        __builtin_nontemporal_store(p0, power + g * 128 + lane);
        __builtin_nontemporal_store(p1, power + g * 128 + 64 + lane);
      } else {
        energy[g * 128 + lane] = e[k][0];
        energy[g * 128 + 64 + lane] = e[k][1];
        power[g * 128 + lane] = p0;
        power[g * 128 + 64 + lane] = p1;
      }
    }
  }
}

__global__ void copy16x4_nt(const u64x2 *__restrict__ a, u64x2 *__restrict__ b, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += 4 * stride) {
    u64x2 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = i + k * stride < n ? __builtin_nontemporal_load(a + i + k * stride) : u64x2{};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i + k * stride < n) __builtin_nontemporal_store(v[k], b + i + k * stride);
  }
}

__global__ void fill16x4(float4 *__restrict__ b, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride) b[i] = float4{1.f, 2.f, 3.f, (float)i};
}

__global__ void read16x4(const float4 *__restrict__ a, float *__restrict__ out, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  float acc = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += 4 * stride) {
    float4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = i + k * stride < n ? a[i + k * stride] : float4{};
#pragma unroll
    for (int k = 0; k < 4; ++k) acc += v[k].x + v[k].w;
  }
  if (acc == 12345.f) out[0] = acc;
}

int main(int argc, char **argv) {
  const size_t rows = argc > 1 ? strtoull(argv[1], nullptr, 10) : 20000000ull;
  const int reps = 20;
  double *d;
  unsigned *slot;
  void *energy, *power;
  CHECK(hipMalloc(&d, rows * 8));
  CHECK(hipMalloc(&slot, rows * 4));
  CHECK(hipMalloc(&energy, rows * 32));
  CHECK(hipMalloc(&power, rows * 32));
  std::vector<unsigned> hs(rows);
  for (size_t i = 0; i < rows; ++i) hs[i] = (unsigned)i;
  CHECK(hipMemcpy(slot, hs.data(), rows * 4, hipMemcpyHostToDevice));
  CHECK(hipMemset(d, 0, rows * 8));
  CHECK(hipMemset(energy, 0, rows * 32));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double mix_bytes = rows * (8.0 + 4 + 32 + 64);
  const int grids[] = {1024, 2048, 4096, 16384};
  for (int g : grids) {
    for (int k = 0; k < 12; ++k) {
      float best = 1e30f;
      for (int rep = 0; rep < reps; ++rep) {
        CHECK(hipEventRecord(e0, 0));
        if (k == 0)
          hipLaunchKernelGGL(copy16, dim3(g), dim3(256), 0, 0, (const float4 *)energy, (float4 *)power, rows * 2);
        if (k == 1) hipLaunchKernelGGL(mix_rows, dim3(g), dim3(256), 0, 0, d, slot, (u64x2 *)energy, (f64x2 *)power, rows);
        if (k == 2) hipLaunchKernelGGL(mix_lin, dim3(g), dim3(256), 0, 0, d, slot, (u64x2 *)energy, (f64x2 *)power, rows);
        if (k == 3)
          hipLaunchKernelGGL(mix_zmaj, dim3(g), dim3(256), 0, 0, d, slot, (unsigned long long *)energy,
                             (double *)power, rows);
        if (k == 4)
          hipLaunchKernelGGL(copy16x4, dim3(g), dim3(256), 0, 0, (const float4 *)energy, (float4 *)power, rows * 2);
        if (k == 5)
          hipLaunchKernelGGL(mix_zmaj4, dim3(g), dim3(256), 0, 0, d, slot, (unsigned long long *)energy,
                             (double *)power, rows);
        if (k == 6) hipLaunchKernelGGL(mix_rows4, dim3(g), dim3(256), 0, 0, d, slot, (u64x2 *)energy, (f64x2 *)power, rows);
        if (k == 7) hipLaunchKernelGGL(mix_lin4<false>, dim3(g), dim3(256), 0, 0, d, slot, (u64x2 *)energy, (f64x2 *)power, rows);
        if (k == 8) hipLaunchKernelGGL(mix_lin4<true>, dim3(g), dim3(256), 0, 0, d, slot, (u64x2 *)energy, (f64x2 *)power, rows);
        if (k == 9)
          hipLaunchKernelGGL(copy16x4_nt, dim3(g), dim3(256), 0, 0, (const u64x2 *)energy, (u64x2 *)power, rows * 2);
        if (k == 10) hipLaunchKernelGGL(fill16x4, dim3(g), dim3(256), 0, 0, (float4 *)power, rows * 2);
        if (k == 11) hipLaunchKernelGGL(read16x4, dim3(g), dim3(256), 0, 0, (const float4 *)energy, (float *)d, rows * 2);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (rep > 2 && ms < best) best = ms;
      }
      const char *name[] = {"copy16",    "mix_rows",  "mix_lin",     "mix_zmaj",  "copy16x4", "mix_zmaj4",
                            "mix_rows4", "mix_lin4", "mix_lin4_nt", "copy16x4_nt", "fill16",  "read16x4"};
      const double bytes = (k == 0 || k == 4 || k == 9) ? rows * 64.0 : (k == 10 || k == 11) ? rows * 32.0 : mix_bytes;
      printf("{\"kernel\":\"%s\",\"grid\":%d,\"ms\":%.4f,\"GBps\":%.1f}\n", name[k], g, best, bytes / (best * 1e-3) / 1e9);
    }
  }
  return 0;
}
