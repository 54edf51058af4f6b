// Derived process / container / VM power (device + host helpers; not part of the public ABI).
//
// The engine's process state is the energy totals plus, per slot, the row's
// cpuTimeRatio and its node (kacc_engine.hip attribute_proc / store_proc):
// Kepler's process power is
//     Power = cpuTimeRatio · NodeUsage.ActivePower          process.go:142
// for a zone that passed the guard
//     ActivePower != 0 && activeEnergy != 0 && nodeCPUTimeDelta != 0   process.go:124
// and the zero Usage otherwise (process.go:58-63).  Every operand besides the
// ratio is a node table of the same interval (KACC_T_NODE_ACTIVE_POWER,
// KACC_T_NODE_ACTIVE_ENERGY, KACC_T_NODE_CPU_DELTA), so the power is one f64
// multiply wherever it is read — bit-identical to storing it, 8Z - 12 bytes
// per process row less HBM traffic in the interval kernels.  The derivation is
// valid for a slot its node attributed in the node's LAST processed interval
// (the running processes of the snapshot); a terminated slot's final power is
// read before its node's next interval (kacc_tracker_add's contract).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kacc_internal.hpp"

namespace kacc {

struct ProcDerive {
  const double *ratio;           // [Sp]
  const uint32_t *node;          // [Sp]
  const uint64_t *active_energy;  // [N*Z] NodeUsage.activeEnergy
  const double *active_power;    // [N*Z] NodeUsage.ActivePower
  const double *cpu_delta;       // [N]   ProcessTotalCPUTimeDelta
  uint64_t nodes;
  uint32_t zones;
};

// Usage.Power of process slot s in zone z (process.go:124-142).
__device__ __forceinline__ double proc_power(const ProcDerive &d, uint64_t s, uint32_t z) {
  const uint32_t n = d.node[s];
  if (n >= d.nodes) return 0.0;
  const uint64_t i = static_cast<uint64_t>(n) * d.zones + z;
  const double aP = d.active_power[i];
  if (d.active_energy[i] == 0 || !(d.cpu_delta[n] != 0) || !(aP != 0)) return 0.0;  // the guard
  return d.ratio[s] * aP;
}

}  // namespace kacc

// The context's derivation inputs for a workload kind (host): processes,
// containers or VMs (their power has the same form and guard:
// container.go:114, 134; vm.go:84, 103).
inline kacc::ProcDerive kacc_derive(const kacc_ctx *ctx, kacc_kind kind) {
  kacc::ProcDerive d;
  const int tr = kind == KACC_KIND_CTR ? KACC_T_CTR_RATIO : kind == KACC_KIND_VM ? KACC_T_VM_RATIO : KACC_T_PROC_RATIO;
  d.ratio = static_cast<const double *>(ctx->tables[tr]);
  d.node = static_cast<const uint32_t *>(ctx->tables[tr + 1]);
  d.active_energy = static_cast<const uint64_t *>(ctx->tables[KACC_T_NODE_ACTIVE_ENERGY]);
  d.active_power = static_cast<const double *>(ctx->tables[KACC_T_NODE_ACTIVE_POWER]);
  d.cpu_delta = static_cast<const double *>(ctx->tables[KACC_T_NODE_CPU_DELTA]);
  d.nodes = ctx->cfg.nodes;
  d.zones = ctx->cfg.zones;
  return d;
}
inline kacc::ProcDerive kacc_proc_derive(const kacc_ctx *ctx) { return kacc_derive(ctx, KACC_KIND_PROC); }

// The kind whose power table t is derived (KACC_T_PROC_POWER / CTR / VM), or -1.
inline int kacc_derived_kind(int t) {
  return t == KACC_T_PROC_POWER ? KACC_KIND_PROC : t == KACC_T_CTR_POWER ? KACC_KIND_CTR
                                                 : t == KACC_T_VM_POWER ? KACC_KIND_VM : -1;
}

// Elements [first, first + count) of the derived power table t ([slot*Z + z])
// into out (device), async on `stream` (kacc_engine.hip).
extern "C" int kacc_internal_derived_power(kacc_ctx *ctx, int t, uint64_t first, uint64_t count, double *out,
                                           void *stream);
