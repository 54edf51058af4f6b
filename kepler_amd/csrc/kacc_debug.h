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

/* interval_kernel (Z = 4) with per-workgroup real-time stamps into d_out
 * [grid][8] u64: start, rows staged, attribution start, end, XCC_ID, HW_ID, block,
 * 0 (s_memrealtime ticks, 100 MHz; diagnostic, results are the reference's).  */
int kacc_debug_interval_stamps(kacc_ctx *ctx, const kacc_interval *dev_batch, void *stream, uint64_t *d_out);

/* Per-wave s_memtime phase totals of the carry kernel (Z = 2; variant 0 or 2) into
 * d_out[n_nodes][8][8] (diagnostic; results are the reference's).             */
int kacc_debug_carry_stamps(kacc_ctx *ctx, const kacc_interval *batches, uint32_t count, void *stream,
                            int variant, uint64_t *d_out);
/* One-launch K-interval kernel ablation (Z = 2; the FAST or MEDIUM shape from the
 * flags): 0 = production, 1 = no process-row stores, 2 = rows prefetched an interval
 * ahead into registers, 4 = no aggregates, 5 = 1|4, 8 = never take the moved path.
 * Variants 1, 4, 5, 8 do not compute the reference results.                   */
int kacc_debug_run_intervals_variant(kacc_ctx *ctx, const kacc_interval *batches, uint32_t count, void *stream,
                                     int variant);

/* Slot join timing ablation: stop_after = k returns after phase k (1 load,
 * 2 lookups, 3 terminated, 4 allocation, 5 inserts); 0 = the full join.    */
int kacc_debug_join_variant(kacc_slotmap *m, uint32_t n_rows, const uint32_t *row_off, const void *keys,
                            uint32_t *out_slot, uint64_t *term_key, uint32_t *term_slot,
                            uint32_t *term_count, void *stream, uint32_t stop_after);
/* Small-node join variant (bits: 1 lock-step lookups, 2 error bits in a register,
 * 4 LDS-only barriers, 8 duplicates found by the insert, 16 shared scan barrier);
 * -1 = production.  Every variant computes the same results.  Returns the old value. */
int kacc_debug_set_join_variant(int variant);

#ifdef __cplusplus
}
#endif
