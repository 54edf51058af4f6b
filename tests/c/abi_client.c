/* A plain C99 client of the C ABI, the way the cgo shim uses
 * it: context, pinned host batch, submit / wait, table download.  Two
 * intervals of one node, two zones and two processes:
 *   interval 1: first read (node.go:101-131), nothing attributed;
 *   interval 2: +100 J / +50 J over exactly 5 s at usage ratio 0.6 (the
 *   reference's node_test.go:349-521 split: 100 J x 0.6 -> 60 J active,
 *   40 J idle; 20 W -> 12 W active), process CPU deltas 30 s and 10 s of a
 *   40 s node total -> ratios 0.75 / 0.25 (process_power_test.go:87-166
 *   style): energies 45 / 15 J (zone 0) and 22.5 / 7.5 J (zone 1), powers
 *   9 / 3 W and 4.5 / 1.5 W.
 * Exit status 0 and "abi_client ok" when every value matches exactly. */
#include <stdio.h>
#include <string.h>

#include "kepler_accel.h"

#define CHECK(call)                                                                  \
  do {                                                                               \
    int rc_ = (call);                                                                \
    if (rc_ != KACC_OK) {                                                            \
      fprintf(stderr, "%s -> %d: %s\n", #call, rc_, kacc_last_error(ctx));          \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

static int fill(kacc_interval *v, int64_t ts, double ratio, uint64_t e0, uint64_t e1, uint32_t slot_flags) {
  ((int64_t *)v->node_ts_ns)[0] = ts;
  ((double *)v->node_usage_ratio)[0] = ratio;
  ((uint32_t *)v->node_status)[0] = 0;
  ((uint64_t *)v->zone_energy)[0] = e0;
  ((uint64_t *)v->zone_energy)[1] = e1;
  ((uint64_t *)v->zone_max)[0] = 262143328850ull; /* max_energy_range_uj of device/testdata */
  ((uint64_t *)v->zone_max)[1] = 262143328850ull;
  uint32_t *po = (uint32_t *)v->proc_off, *co = (uint32_t *)v->ctr_off, *vo = (uint32_t *)v->vm_off,
           *qo = (uint32_t *)v->pod_off;
  po[0] = 0, po[1] = 2;
  co[0] = co[1] = vo[0] = vo[1] = qo[0] = qo[1] = 0;
  ((double *)v->proc_cpu_delta)[0] = 30.0;
  ((double *)v->proc_cpu_delta)[1] = 10.0;
  ((uint32_t *)v->proc_slot)[0] = 0u | slot_flags;
  ((uint32_t *)v->proc_slot)[1] = 1u | slot_flags;
  v->node_cpu_delta = NULL;
  v->node_order = NULL;
  v->node_proc_span = NULL;
  v->flags = 0;
  return 0;
}

int main(void) {
  kacc_ctx *ctx = NULL;
  if (kacc_abi_version() != KACC_ABI_VERSION) {
    fprintf(stderr, "ABI version mismatch\n");
    return 1;
  }
  kacc_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.zones = 2;
  cfg.nodes = 1;
  cfg.proc_slots = 4;
  cfg.ctr_slots = cfg.vm_slots = cfg.pod_slots = 1;
  if (kacc_create(0, &cfg, &ctx) != KACC_OK) {
    char msg[256];
    kacc_last_error_copy(NULL, msg, sizeof msg); /* the cgo form: no thread affinity */
    fprintf(stderr, "kacc_create: %s\n", msg);
    return 1;
  }
  kacc_batch *b = NULL;
  kacc_interval *v = NULL;
  kacc_shape shape;
  memset(&shape, 0, sizeof shape);
  shape.n_nodes = 1;
  shape.n_procs = 2;
  shape.intervals = 1;
  CHECK(kacc_batch_alloc(ctx, &shape, &b, &v));
  const int64_t t0 = 1000000000000ll;
  fill(v, t0, 0.0, 1000000000ull, 500000000ull, KACC_SLOT_NEW);
  CHECK(kacc_batch_submit(ctx, b));
  CHECK(kacc_batch_wait(ctx, b));
  fill(v, t0 + 5000000000ll, 0.6, 1100000000ull, 550000000ull, 0u);
  CHECK(kacc_batch_submit(ctx, b));
  CHECK(kacc_batch_wait(ctx, b));

  uint64_t pe[4], act[2], idle[2];
  double pp[4], np[2], nap[2];
  CHECK(kacc_table_download(ctx, KACC_T_PROC_ENERGY, 0, 4, pe));
  CHECK(kacc_table_download(ctx, KACC_T_PROC_POWER, 0, 4, pp));
  CHECK(kacc_table_download(ctx, KACC_T_NODE_ACTIVE_TOTAL, 0, 2, act));
  CHECK(kacc_table_download(ctx, KACC_T_NODE_IDLE_TOTAL, 0, 2, idle));
  CHECK(kacc_table_download(ctx, KACC_T_NODE_POWER, 0, 2, np));
  CHECK(kacc_table_download(ctx, KACC_T_NODE_ACTIVE_POWER, 0, 2, nap));
  const uint64_t want_pe[4] = {45000000ull, 22500000ull, 15000000ull, 7500000ull};
  const double want_pp[4] = {9e6, 4.5e6, 3e6, 1.5e6};
  int bad = 0;
  for (int i = 0; i < 4; ++i) {
    if (pe[i] != want_pe[i]) fprintf(stderr, "proc_energy[%d] = %llu, want %llu\n", i, (unsigned long long)pe[i], (unsigned long long)want_pe[i]), bad = 1;
    if (pp[i] != want_pp[i]) fprintf(stderr, "proc_power[%d] = %.17g, want %.17g\n", i, pp[i], want_pp[i]), bad = 1;
  }
  /* first read: ActiveEnergyTotal = trunc(abs x 0) = 0, Idle = abs; then +60/40 J and +30/20 J */
  if (act[0] != 60000000ull || act[1] != 30000000ull) fprintf(stderr, "active totals %llu %llu\n", (unsigned long long)act[0], (unsigned long long)act[1]), bad = 1;
  if (idle[0] != 1040000000ull || idle[1] != 520000000ull) fprintf(stderr, "idle totals %llu %llu\n", (unsigned long long)idle[0], (unsigned long long)idle[1]), bad = 1;
  if (np[0] != 2e7 || np[1] != 1e7 || nap[0] != 1.2e7 || nap[1] != 6e6) fprintf(stderr, "node powers %.17g %.17g %.17g %.17g\n", np[0], np[1], nap[0], nap[1]), bad = 1;
  kacc_batch_free(ctx, b);
  kacc_destroy(ctx);
  if (bad) return 1;
  printf("abi_client ok\n");
  return 0;
}
