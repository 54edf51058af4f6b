/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of Kepler's power-attribution path (reference:
 * sthaha/kepler @ 2025-08-24, internal/monitor + internal/device +
 * internal/resource).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the CPU
 * baseline.  The product path (kepler_amd/, libkepler_accel.so) never links or
 * calls it.
 *
 * Parity pinning: the restatement is checked against every known-answer test
 * the reference's own Go tests hold for this path (tests/golden/kat_*.json,
 * transcribed with file:line by tests/golden/make_golden.py).  The Go
 * reference itself cannot be built here (no Go toolchain).
 */
#ifndef KEPLER_ORACLE_H
#define KEPLER_ORACLE_H

#include <stdint.h>

#include "../include/kepler_accel.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Order used for the node total ProcessTotalCPUTimeDelta (informer.go:330-333).
 * Go sums over a map, so its order is random; the engine's canonical order is
 * KOR_SUM_TREE256 (256 strided lane sums, then a halving tree) and the oracle
 * reproduces it bit for bit.  KOR_SUM_LISTING sums in row (listing) order,
 * which is one of the orders Go may take; tests compare it at 1e-12 rel.   */
#define KOR_SUM_TREE256 0
#define KOR_SUM_LISTING 1

/* Host mirror of the device state tables (same layout, see kacc_table). */
typedef struct kor_state {
  uint32_t zones;
  uint32_t reserved0;
  uint64_t nodes, proc_slots, ctr_slots, vm_slots, pod_slots;
  uint64_t *node_energy_total, *node_active_energy, *node_active_total, *node_idle_total;
  double *node_power, *node_active_power, *node_idle_power;
  int64_t *node_ts;
  uint32_t *node_has_prev;
  double *node_usage_ratio, *node_cpu_delta;
  uint32_t *node_status;
  uint64_t *proc_energy;
  double *proc_power;
  uint64_t *ctr_energy;
  double *ctr_power, *ctr_cpu_delta, *ctr_cpu_total;
  uint64_t *vm_energy;
  double *vm_power, *vm_cpu_delta;
  uint64_t *pod_energy;
  double *pod_power, *pod_cpu_delta, *pod_cpu_total;
  /* the engine's process storage behind the derived power (kacc_derive.hpp):
   * the row's cpuTimeRatio (process.go:128) and its node, per slot */
  double *proc_ratio;
  uint32_t *proc_node;
  double *ctr_ratio; /* the same for containers and VMs (container.go:118, vm.go:89) */
  uint32_t *ctr_node;
  double *vm_ratio;
  uint32_t *vm_node;
} kor_state;

/* Scalar Go-semantics helpers (exported so the KATs can pin them directly). */
uint64_t kor_go_f64_to_u64(double x);
double kor_go_duration_seconds(int64_t ns);
uint64_t kor_calculate_energy_delta(uint64_t current, uint64_t previous, uint64_t max_joules);

/* One interval for every node of a host batch; returns 0 or KACC_E*. */
int kor_interval(kor_state *st, const kacc_interval *b, int sum_mode);
/* the same over `threads` host threads (node ranges): the CPU baseline */
int kor_interval_mt(kor_state *st, const kacc_interval *b, int sum_mode, int threads);

int kor_namespace_totals(const kor_state *st, uint32_t n_ns, const uint32_t *ns_pod_off,
                         const uint32_t *ns_pod_slot, uint64_t *out_energy, double *out_power);

/* Multi-socket aggregated zone (device/energy_zone.go:97-148), one call =
 * one AggregatedZone.Energy() over `n` sub-zones.  last[] / seen[] / current
 * are the zone's persistent state.                                          */
uint64_t kor_aggregated_max(uint32_t n, const uint64_t *sub_max);
uint64_t kor_aggregated_energy(uint32_t n, const uint64_t *reading, const uint64_t *sub_max,
                               uint64_t *last, uint8_t *seen, uint64_t *current,
                               uint64_t agg_max);
/* With per-sub-zone read errors (status nonzero): returns KACC_ERANGE at the
 * first failing sub-zone, as Energy() returns its error; else 0 and *out.   */
int kor_aggregated_energy_st(uint32_t n, const uint64_t *reading, const uint32_t *status,
                             const uint64_t *sub_max, uint64_t *last, uint8_t *seen, uint64_t *current,
                             uint64_t agg_max, uint64_t *out);

/* Go-faithful CPU baseline: the same interval computed with the reference's
 * data structures (string-keyed maps of heap objects with per-object zone
 * maps, rebuilt every interval, prev snapshot looked up by string ID, as in
 * process.go:118-148 / container.go:106-140 / vm.go:78-109 / pod.go:87-118).
 * Single threaded like the Go goroutine.  Results are written to the same
 * state tables so tests can check it against kor_interval.                  */
typedef struct kor_gofaithful kor_gofaithful;
kor_gofaithful *kor_gf_create(uint32_t zones);
void kor_gf_destroy(kor_gofaithful *g);
int kor_gf_interval(kor_gofaithful *g, kor_state *st, const kacc_interval *b);

/* Slot join restatement (kor_join.cpp): same contract as kacc_slot_join on
 * host arrays (term_* sized slot_off[n], term_count [n_nodes]); returns 0, or
 * KACC_ERANGE after an error row.                                          */
typedef struct kor_slotmap kor_slotmap;
kor_slotmap *kor_slotmap_create(uint32_t n_nodes, const uint32_t *slot_off);
void kor_slotmap_destroy(kor_slotmap *m);
void kor_slotmap_set_policy(kor_slotmap *m, uint32_t policy);
int kor_slot_join(kor_slotmap *m, uint32_t n_rows, const uint32_t *row_off, const uint64_t *keys,
                  const uint32_t *node_status, uint32_t *out_slot, uint64_t *term_key,
                  uint32_t *term_slot, uint32_t *term_count);

/* TerminatedResourceTracker restatement (kor_tracker.cpp), Go's heap exactly.
 * add_one = one Add(); add_batch = a batch in kacc_tracker_add's order.     */
typedef struct kor_tracker kor_tracker;
kor_tracker *kor_tracker_create(int64_t max_size, uint64_t min_energy, uint32_t zones, uint32_t zone);
void kor_tracker_destroy(kor_tracker *t);
void kor_tracker_clear(kor_tracker *t);
void kor_tracker_clear_node(kor_tracker *t, uint32_t node);
void kor_tracker_add_one(kor_tracker *t, uint32_t node, uint64_t key, const uint64_t *energy,
                         const double *power);
void kor_tracker_add_batch(kor_tracker *t, uint32_t n, const uint32_t *node, const uint64_t *key,
                           const uint32_t *slot, const uint64_t *tab_e, const double *tab_p);
uint32_t kor_tracker_items(const kor_tracker *t, uint64_t *key, uint32_t *node, uint64_t *energy,
                           double *power);

#ifdef __cplusplus
}
#endif
#endif
