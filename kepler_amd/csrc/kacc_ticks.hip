// CPU-tick input format (kepler_accel.h, "CPU-tick input format"): Go's
// CPUTimeDelta computed on the device from per-slot cumulative ticks.
//
// The reference, per process and interval (internal/resource/informer.go:512-524,
// procfs_reader.go:75-82):
//   cpuTotalTime := float64(st.STime+st.UTime) / userHZ   // userHZ = 100
//   p.CPUTimeDelta = cpuTotalTime - p.CPUTotalTime         // 0 for a new process
//   p.CPUTotalTime = cpuTotalTime
// The tick map keeps the ticks behind p.CPUTotalTime per process slot, so the
// caller ships a 2-byte increment per row (plus rare 8-byte escapes) instead of
// the 8-byte float64 Δ, and the device reproduces both float64 values exactly:
// float64(uint64) correctly rounded (one rounding of hi*2^32 + lo), one IEEE
// division by 100 (never a reciprocal: -ffp-contract=off, no fast-math), one
// subtraction.
//
// One workgroup per node: a READ_ERROR node is skipped whole (the reference
// skips Refresh for it, monitor.go:399-410), its escapes are node-local
// (esc_off), and no two rows of a batch share a slot (kacc_slot_join), so rows
// never race.  HBM-bound integer/byte work: 2 B increment + 4 B slot word + 8 B
// previous ticks in, 8 B ticks + 8 B Δ out per row (30 B).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "../../include/kepler_accel.h"
#include "kacc_device.hpp"
#include "kacc_internal.hpp"

struct kacc_tickmap {
  kacc_ctx *ctx = nullptr;
  int device = 0;
  uint64_t slots = 0;
  uint64_t *d_ticks = nullptr;  // [slots] ticks of each slot's last reading
};

namespace kacc {
namespace ticks {

constexpr int kThreads = 256;
constexpr int kUnroll = 4;  // rows in flight per lane
constexpr uint32_t kErrOffsets = 1u << 1, kErrSlot = 1u << 2;

struct Args {
  kacc_ticks t;
  uint64_t *map;
  uint64_t slots;
  uint32_t *err;
};

// Go's CPUTimeDelta of one row: float64(now)/100 - float64(prev)/100.
__device__ __forceinline__ double go_cpu_delta(uint64_t prev, uint64_t now) {
  const double hz = static_cast<double>(KACC_USER_HZ);
  return u2f(now) / hz - u2f(prev) / hz;
}

__global__ __launch_bounds__(kThreads) void ticks_kernel(const Args a) {
  const uint32_t n = blockIdx.x, tid = threadIdx.x;
  const kacc_ticks &t = a.t;
  if (t.node_status && (t.node_status[n] & KACC_NODE_READ_ERROR)) return;  // Refresh skipped
  uint32_t p0 = t.proc_off[n], p1 = t.proc_off[n + 1];
  if (p1 > t.n_procs || p0 > p1) {
    if (tid == 0) atomicOr(a.err, kErrOffsets);
    p1 = min(p1, t.n_procs);
    p0 = min(p0, p1);
  }
  __shared__ uint32_t s_escaped;  // escaped rows of the node (each needs exactly one escape)
  if (tid == 0) s_escaped = 0;
  __syncthreads();
  uint32_t errs = 0, escaped = 0;
  // regular rows: every load of kUnroll rows issued before their use (clamped, unconditional)
  for (uint32_t r0 = p0 + tid; r0 < p1; r0 += kThreads * kUnroll) {
    uint32_t w[kUnroll];
    uint16_t d[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const uint32_t r = min(r0 + u * kThreads, p1 - 1);
      w[u] = t.proc_slot[r];
      d[u] = t.dticks[r];
    }
    uint64_t prev[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const uint64_t s = w[u] & KACC_SLOT_MASK;
      prev[u] = a.map[s < a.slots ? s : 0];
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const uint32_t r = r0 + u * kThreads;
      if (r >= p1) continue;
      if (d[u] == KACC_TICKS_ESCAPED) {  // its escape writes it below (0 if it has none: an error)
        ++escaped;
        t.proc_cpu_delta[r] = 0.0;
        continue;
      }
      const uint64_t s = w[u] & KACC_SLOT_MASK;
      if (s >= a.slots) {
        errs |= kErrSlot;
        t.proc_cpu_delta[r] = 0.0;
        continue;
      }
      const uint64_t p = (w[u] & KACC_SLOT_NEW) ? 0ull : prev[u];  // a new process: p.CPUTotalTime = 0
      const uint64_t now = p + d[u];
      t.proc_cpu_delta[r] = go_cpu_delta(p, now);
      a.map[s] = now;
    }
  }
  if (escaped) atomicAdd(&s_escaped, escaped);
  __syncthreads();  // the zeroed escaped rows and s_escaped before the escapes
  // escapes of this node: [esc_off[n], esc_off[n+1]), rows strictly ascending, each an
  // escaped row of the node; with as many entries as escaped rows that covers each once
  uint32_t e0 = 0, e1 = 0;
  if (t.n_escapes && t.esc_off) {
    e0 = t.esc_off[n];
    e1 = t.esc_off[n + 1];
    if (e1 > t.n_escapes || e0 > e1) {
      errs |= kErrOffsets;
      e1 = min(e1, t.n_escapes);
      e0 = min(e0, e1);
    }
  }
  if (tid == 0 && e1 - e0 != s_escaped) errs |= kErrOffsets;
  {
    for (uint32_t e = e0 + tid; e < e1; e += kThreads) {
      const uint32_t r = t.esc_row[e];
      if (r < p0 || r >= p1 || t.dticks[r] != KACC_TICKS_ESCAPED || (e > e0 && t.esc_row[e - 1] >= r)) {
        errs |= kErrOffsets;
        continue;
      }
      const uint32_t w = t.proc_slot[r];
      const uint64_t s = w & KACC_SLOT_MASK;
      if (s >= a.slots) {
        errs |= kErrSlot;
        t.proc_cpu_delta[r] = 0.0;
        continue;
      }
      const uint64_t p = (w & KACC_SLOT_NEW) ? 0ull : a.map[s];
      const uint64_t now = p + static_cast<uint64_t>(t.esc_ticks[e]);  // mod 2^64, as Go's uint
      t.proc_cpu_delta[r] = go_cpu_delta(p, now);
      a.map[s] = now;
    }
  }
  if (errs) atomicOr(a.err, errs);
}

}  // namespace ticks
}  // namespace kacc

extern "C" {

int kacc_tickmap_create(kacc_ctx *ctx, kacc_tickmap **out) {
  if (!ctx || !out) return KACC_EINVAL;
  *out = nullptr;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  auto *m = new kacc_tickmap;
  m->ctx = ctx;
  m->device = ctx->device;
  m->slots = ctx->cfg.proc_slots;
  const hipError_t e = hipMalloc(&m->d_ticks, 8 * std::max<uint64_t>(m->slots, 1));
  if (e != hipSuccess) {
    delete m;
    return kacc_fail(ctx, e == hipErrorOutOfMemory ? KACC_ENOMEM : KACC_EHIP, "tick map allocation: %s",
                     hipGetErrorString(e));
  }
  const int rc = kacc_tickmap_reset(m);
  if (rc != KACC_OK) {
    kacc_tickmap_destroy(m);
    return rc;
  }
  *out = m;
  return KACC_OK;
}

void kacc_tickmap_destroy(kacc_tickmap *m) {
  if (!m) return;
  (void)hipSetDevice(m->device);
  (void)hipDeviceSynchronize();  // no launch on this map may still be running
  (void)hipFree(m->d_ticks);
  delete m;
}

int kacc_tickmap_reset(kacc_tickmap *m) {
  if (!m) return KACC_EINVAL;
  kacc_ctx *ctx = m->ctx;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  KACC_HIP(ctx, hipMemsetAsync(m->d_ticks, 0, 8 * std::max<uint64_t>(m->slots, 1), ctx->stream));
  KACC_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return KACC_OK;
}

int kacc_ticks_delta(kacc_tickmap *m, const kacc_ticks *t, void *stream) {
  if (!m) return KACC_EINVAL;
  kacc_ctx *ctx = m->ctx;
  if (!t) return kacc_fail(ctx, KACC_EINVAL, "ticks: NULL descriptor");
  if (!t->n_nodes) return KACC_OK;
  if (t->n_nodes > ctx->cfg.nodes) return kacc_fail(ctx, KACC_EINVAL, "ticks: n_nodes %u exceeds capacity", t->n_nodes);
  if (!t->proc_off || (t->n_procs && (!t->proc_slot || !t->dticks || !t->proc_cpu_delta)))
    return kacc_fail(ctx, KACC_EINVAL, "ticks: NULL array");
  if (t->n_escapes && (!t->esc_off || !t->esc_row || !t->esc_ticks))
    return kacc_fail(ctx, KACC_EINVAL, "ticks: escapes without esc_off / esc_row / esc_ticks");
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  kacc::ticks::Args a{*t, m->d_ticks, m->slots, ctx->d_err};
  (void)hipGetLastError();
  hipLaunchKernelGGL(kacc::ticks::ticks_kernel, dim3(t->n_nodes), dim3(kacc::ticks::kThreads), 0, st, a);
  KACC_HIP(ctx, hipGetLastError());
  return KACC_OK;
}

int kacc_tickmap_download(kacc_tickmap *m, uint64_t first, uint64_t count, uint64_t *host_dst) {
  if (!m) return KACC_EINVAL;
  kacc_ctx *ctx = m->ctx;
  if (first > m->slots || count > m->slots - first || (count && !host_dst))
    return kacc_fail(ctx, KACC_EINVAL, "tick map download: range past %llu slots", (unsigned long long)m->slots);
  if (!count) return KACC_OK;
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  KACC_HIP(ctx, hipStreamSynchronize(ctx->stream));
  KACC_HIP(ctx, hipMemcpy(host_dst, m->d_ticks + first, 8 * count, hipMemcpyDeviceToHost));
  return KACC_OK;
}

}  // extern "C"
