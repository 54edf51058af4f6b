// Multi-socket aggregated RAPL zones on the device.
//
// Reference: device.AggregatedZone (internal/device/energy_zone.go:47-148):
// the zones of one type on a multi-socket node (package-0, package-1, ...)
// read as one counter.  Per Energy() call, sub-zone by sub-zone in order: a
// read error returns at once, leaving the earlier sub-zones' last readings
// updated and the aggregate untouched (:104-108); a first reading adds the
// raw value (:130-131); otherwise the wrap-safe delta (:115-125), with a
// MaxEnergy of 0 keeping the uint64 underflow (:127-128); the aggregate
// accumulates modulo the summed MaxEnergy (:136-145), that sum saturating at
// MaxUint64 (:55-67).  The monitor reads every zone of a node even after one
// fails and then fails the node's interval (monitor/node.go:37-44).
//
// One thread per node, its zones in order; S sub-zones each, stored
// [node][zone][socket].  The outputs are the interval batch's zone_energy /
// zone_max and the KACC_NODE_READ_ERROR bit of the batch's node_status, set
// when one of the node's zones failed and cleared otherwise (other bits kept).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "kacc_internal.hpp"

namespace kacc {
namespace zagg {

constexpr int kThreads = 256;

struct Args {
  uint32_t n;  // nodes * zones
  uint32_t Z, S;
  const uint64_t *readings;
  const uint32_t *sub_status;
  const uint64_t *sub_max;
  const uint64_t *agg_max;
  uint64_t *last;
  uint32_t *seen;
  uint64_t *current;
  uint64_t *out_energy, *out_max;
  uint32_t *node_status;
};

// One thread per node: its Z aggregated zones in order; the node's read-error
// bit is written (set or cleared) every call, so a node fails only the
// intervals whose reads failed (monitor/node.go:37-44: every zone is read,
// then the interval fails).
__global__ __launch_bounds__(kThreads) void zone_agg_kernel(const Args a) {
  const uint32_t node = blockIdx.x * kThreads + threadIdx.x;
  if (node >= a.n / a.Z) return;
  bool failed = false;
  for (uint32_t z = 0; z < a.Z; ++z) {
    const uint32_t i = node * a.Z + z;
    const uint64_t base = static_cast<uint64_t>(i) * a.S;
    const uint64_t amax = a.agg_max[i];
    a.out_max[i] = amax;
    uint64_t total = 0;
    bool ok = true;
    for (uint32_t s = 0; s < a.S && ok; ++s) {
      const uint64_t k = base + s;
      if (a.sub_status && a.sub_status[k]) {  // energy_zone.go:104-108: return at once
        ok = false;
        break;
      }
      const uint64_t r = a.readings[k];
      if (a.seen[k]) {
        const uint64_t prev = a.last[k], mx = a.sub_max[k];
        total += r >= prev ? r - prev : mx > 0 ? (mx - prev) + r : r - prev;  // :115-128
      } else {
        total += r;  // :130-131 first reading
      }
      a.last[k] = r;
      a.seen[k] = 1u;
    }
    if (!ok) {
      a.out_energy[i] = 0;
      failed = true;
      continue;
    }
    uint64_t cur = a.current[i] + total;  // :136
    if (amax > 0) cur %= amax;            // :139-145
    a.current[i] = cur;
    a.out_energy[i] = cur;
  }
  const uint32_t st = a.node_status[node];
  a.node_status[node] = failed ? (st | KACC_NODE_READ_ERROR) : (st & ~KACC_NODE_READ_ERROR);
}

}  // namespace zagg
}  // namespace kacc

struct kacc_zone_agg {
  kacc_ctx *ctx = nullptr;
  int device = 0;
  uint32_t n_nodes = 0, S = 0;
  uint64_t *d_sub_max = nullptr, *d_agg_max = nullptr, *d_last = nullptr, *d_current = nullptr;
  uint32_t *d_seen = nullptr;
};

extern "C" {

int kacc_zone_agg_create(kacc_ctx *ctx, uint32_t n_nodes, uint32_t sockets, const uint64_t *sub_max,
                         kacc_zone_agg **out) {
  if (!ctx || !out || (!sub_max && n_nodes && sockets)) return KACC_EINVAL;
  *out = nullptr;
  if (sockets == 0) return kacc_fail(ctx, KACC_EINVAL, "an aggregated zone needs >= 1 sub-zone");
  const uint64_t Z = ctx->cfg.zones, nz = static_cast<uint64_t>(n_nodes) * Z, nsub = nz * sockets;
  if (nz > 0xffffffffull) return kacc_fail(ctx, KACC_EINVAL, "too many zones");
  // NewAggregatedZone (energy_zone.go:55-67): summed MaxEnergy, saturating
  std::vector<uint64_t> agg(nz);
  for (uint64_t i = 0; i < nz; ++i) {
    uint64_t total = 0;
    for (uint32_t s = 0; s < sockets; ++s) {
      const uint64_t m = sub_max[i * sockets + s];
      if (total > 0 && m > UINT64_MAX - total) {
        total = UINT64_MAX;
        break;
      }
      total += m;
    }
    agg[i] = total;
  }
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  auto *z = new kacc_zone_agg;
  z->ctx = ctx;
  z->device = ctx->device;
  z->n_nodes = n_nodes;
  z->S = sockets;
  hipError_t e = hipSuccess;
  auto A = [&](void **p, size_t bytes) {
    if (e == hipSuccess) e = hipMalloc(p, std::max<size_t>(bytes, 8));
  };
  A(reinterpret_cast<void **>(&z->d_sub_max), 8 * nsub);
  A(reinterpret_cast<void **>(&z->d_last), 8 * nsub);
  A(reinterpret_cast<void **>(&z->d_seen), 4 * nsub);
  A(reinterpret_cast<void **>(&z->d_agg_max), 8 * nz);
  A(reinterpret_cast<void **>(&z->d_current), 8 * nz);
  if (e == hipSuccess && nsub) e = hipMemcpy(z->d_sub_max, sub_max, 8 * nsub, hipMemcpyHostToDevice);
  if (e == hipSuccess && nz) e = hipMemcpy(z->d_agg_max, agg.data(), 8 * nz, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemset(z->d_seen, 0, std::max<size_t>(4 * nsub, 8));
  if (e == hipSuccess) e = hipMemset(z->d_current, 0, std::max<size_t>(8 * nz, 8));
  if (e != hipSuccess) {
    kacc_zone_agg_destroy(z);
    return kacc_fail(ctx, KACC_ENOMEM, "zone aggregation allocation: %s", hipGetErrorString(e));
  }
  *out = z;
  return KACC_OK;
}

void kacc_zone_agg_destroy(kacc_zone_agg *z) {
  if (!z) return;
  (void)hipSetDevice(z->device);
  (void)hipDeviceSynchronize();
  (void)hipFree(z->d_sub_max);
  (void)hipFree(z->d_last);
  (void)hipFree(z->d_seen);
  (void)hipFree(z->d_agg_max);
  (void)hipFree(z->d_current);
  delete z;
}

int kacc_zone_agg_read(kacc_zone_agg *z, const uint64_t *readings, const uint32_t *sub_status,
                       uint64_t *out_energy, uint64_t *out_max, uint32_t *node_status, void *stream) {
  if (!z) return KACC_EINVAL;
  kacc_ctx *ctx = z->ctx;
  if (!z->n_nodes) return KACC_OK;
  if (!readings || !out_energy || !out_max || !node_status)
    return kacc_fail(ctx, KACC_EINVAL, "zone aggregation: NULL argument");
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  kacc::zagg::Args a{};
  a.Z = ctx->cfg.zones;
  a.n = z->n_nodes * a.Z;
  a.S = z->S;
  a.readings = readings;
  a.sub_status = sub_status;
  a.sub_max = z->d_sub_max;
  a.agg_max = z->d_agg_max;
  a.last = z->d_last;
  a.seen = z->d_seen;
  a.current = z->d_current;
  a.out_energy = out_energy;
  a.out_max = out_max;
  a.node_status = node_status;
  (void)hipGetLastError();  // clear a stale error of an earlier call
  const uint32_t grid = (z->n_nodes + kacc::zagg::kThreads - 1) / kacc::zagg::kThreads;
  hipLaunchKernelGGL(kacc::zagg::zone_agg_kernel, dim3(grid), dim3(kacc::zagg::kThreads), 0, st, a);
  KACC_HIP(ctx, hipGetLastError());
  return KACC_OK;
}

}  // extern "C"
