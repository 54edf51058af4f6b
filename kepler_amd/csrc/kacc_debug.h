// Internal debug entry points of libkepler_accel.so (not part of the public ABI).
#pragma once
#include "../../include/kepler_accel.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Launch a timing-ablation variant of the interval kernel (Z = 4 only):
 * 0 = production, 1 = skip containers/VMs/pods, 2 = skip processes,
 * 3 = node phases only, 4 = never stage Δ in LDS, 8 = non-temporal stores,
 * 9 = 1|8.  Variants != 0 do not compute the reference semantics.          */
int kacc_debug_run_variant(kacc_ctx *ctx, const kacc_interval *dev_batch, void *stream, int variant);

#ifdef __cplusplus
}
#endif
