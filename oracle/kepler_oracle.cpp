// ORACLE — TEST INFRASTRUCTURE ONLY (see kepler_oracle.h).
//
// A line-by-line CPU restatement of the reference's attribution semantics.
// Every function cites the Go source it follows (sthaha/kepler @ 2025-08-24).
// Built with g++ -O2 -ffp-contract=off (SSE2 doubles, no FMA), so float64
// arithmetic matches Go on amd64 (GOAMD64=v1 never contracts a*b+c).
#include "kepler_oracle.h"

#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

constexpr double kTwo63 = 9223372036854775808.0;

// CVTTSD2SQ: truncating float64 -> int64; NaN and out-of-range give INT64_MIN.
int64_t cvttsd2sq(double x) {
  if (std::isnan(x) || x >= kTwo63 || x < -kTwo63) return INT64_MIN;
  return static_cast<int64_t>(x);
}

// Go's uint64 -> float64 (ssagen uint64Tofloat64) is correctly rounded, as is
// the C conversion on x86-64.
inline double u2f(uint64_t v) { return static_cast<double>(v); }

// time.Time.Sub with monotonic readings (time/time.go subMono): saturating.
int64_t go_sub_mono(int64_t t, int64_t u) {
  int64_t d;
  if (__builtin_sub_overflow(t, u, &d)) return t > u ? INT64_MAX : INT64_MIN;
  return d;
}

struct NodeZ {  // the fields of monitor.NodeUsage the workload passes read
  uint64_t active_energy[KACC_MAX_ZONES];
  double power[KACC_MAX_ZONES];
  double active_power[KACC_MAX_ZONES];
};

struct Ranges {
  uint32_t p0, p1, c0, c1, v0, v1, q0, q1;
};

Ranges node_ranges(const kacc_interval *b, uint32_t n) {
  Ranges r;
  r.p0 = b->proc_off[n];
  r.p1 = b->proc_off[n + 1];
  r.c0 = b->ctr_off[n];
  r.c1 = b->ctr_off[n + 1];
  r.v0 = b->vm_off[n];
  r.v1 = b->vm_off[n + 1];
  r.q0 = b->pod_off[n];
  r.q1 = b->pod_off[n + 1];
  return r;
}
inline uint32_t ctr_begin(const kacc_interval *b, const Ranges &r, uint32_t c) {
  return c == r.c0 ? r.p0 : b->ctr_proc_end[c - 1];
}
inline uint32_t vm_begin(const kacc_interval *b, const Ranges &r, uint32_t v) {
  if (v != r.v0) return b->vm_proc_end[v - 1];
  return r.c1 > r.c0 ? b->ctr_proc_end[r.c1 - 1] : r.p0;
}
inline uint32_t pod_begin(const kacc_interval *b, const Ranges &r, uint32_t q) {
  return q == r.q0 ? r.c0 : b->pod_ctr_end[q - 1];
}

// resource/informer.go:328-345 refreshNode: procCPUDeltaTotal over Running.
double node_cpu_delta_sum(const double *d, uint32_t p0, uint32_t p1, int mode) {
  if (mode == KOR_SUM_LISTING) {
    double s = 0;
    for (uint32_t i = p0; i < p1; ++i) s += d[i];
    return s;
  }
  // canonical engine order: lane l sums rows p0+l, p0+l+256, ... in order,
  // then the 256 lane sums are halved pairwise (l += l+s for s=128..1).
  double lane[256];
  for (int l = 0; l < 256; ++l) lane[l] = 0.0;
  for (uint32_t i = p0; i < p1; ++i) lane[(i - p0) & 255u] += d[i];
  for (int s = 128; s >= 1; s >>= 1)
    for (int l = 0; l < s; ++l) lane[l] += lane[l + s];
  return lane[0];
}

// The per-zone workload formula shared by process.go:118-148,
// container.go:106-140, vm.go:78-109 and pod.go:87-118 (and their first*Read
// variants process.go:21-36, container.go:22-34, vm.go:22-34, pod.go:22-34).
void attribute(uint32_t Z, double cpu_delta, double node_delta, const NodeZ &nz, bool is_pod,
               bool first_read, bool is_new, uint64_t *energy, double *power) {
  for (uint32_t z = 0; z < Z; ++z) {
    // pod.go:96 guards on nodeZoneUsage.Power; every other pass (and
    // firstPodRead, pod.go:23) guards on ActivePower.
    const double guard_power = (is_pod && !first_read) ? nz.power[z] : nz.active_power[z];
    if (guard_power == 0 || nz.active_energy[z] == 0 || node_delta == 0) {
      // zone keeps newProcess/newContainer/newVM/newPod's zero Usage
      // (process.go:58-63): the cumulative total resets to 0.
      energy[z] = 0;
      power[z] = 0;
      continue;
    }
    const double ratio = cpu_delta / node_delta;  // process.go:127
    // process.go:129 Energy(cpuTimeRatio * float64(activeEnergy));
    // pod.go:102 writes float64(activeEnergy) * cpuTimeRatio (same product).
    const uint64_t e = is_pod ? kor_go_f64_to_u64(u2f(nz.active_energy[z]) * ratio)
                              : kor_go_f64_to_u64(ratio * u2f(nz.active_energy[z]));
    if (first_read) {  // first*Read: EnergyTotal = interval energy, Power(0)
      energy[z] = e;
      power[z] = 0;
      continue;
    }
    // process.go:132-138: absolute = interval + prev.Zones[zone].EnergyTotal
    // when the previous snapshot has this ID (and zone).
    const uint64_t prev = is_new ? 0 : energy[z];
    energy[z] = e + prev;
    // process.go:142: Power(cpuTimeRatio * ActivePower.MicroWatts())
    power[z] = ratio * nz.active_power[z];
  }
}

}  // namespace

// One node of kor_interval (nodes are independent: disjoint state rows).
static void node_interval(kor_state *st, const kacc_interval *b, uint32_t n, int sum_mode) {
  const uint32_t Z = st->zones;
  const uint32_t status = b->node_status ? b->node_status[n] : 0u;
  if (status & KACC_NODE_READ_ERROR) {
    // node.go:39-44 joins the read error; calculatePower returns it
    // (monitor.go:401-403) and refreshSnapshot keeps the old snapshot
    // (monitor.go:332-334) without calling Refresh.
    st->node_status[n] = KACC_NODE_SKIPPED;
    return;
  }
  const bool first_read = st->node_has_prev[n] == 0;  // monitor.go:326-330
  const double ratio = b->node_usage_ratio[n];
  const int64_t now = b->node_ts_ns[n];
  NodeZ nz;

  // ---- node zones: node.go:10-84 (calculateNodePower) / node.go:101-131 (firstNodeRead)
  double time_diff = 0;
  if (!first_read) time_diff = kor_go_duration_seconds(go_sub_mono(now, st->node_ts[n]));
  for (uint32_t z = 0; z < Z; ++z) {
    const uint64_t i = static_cast<uint64_t>(n) * Z + z;
    const uint64_t abs_energy = b->zone_energy[i];
    if (first_read) {
      const uint64_t active = kor_go_f64_to_u64(u2f(abs_energy) * ratio);  // node.go:118
      st->node_energy_total[i] = abs_energy;
      st->node_active_total[i] = active;
      st->node_idle_total[i] = abs_energy - active;  // node.go:119
      st->node_active_energy[i] = active;
      st->node_power[i] = 0;  // node.go:126: no power on the first read
      st->node_active_power[i] = 0;
      st->node_idle_power[i] = 0;
    } else {
      const uint64_t delta =
          kor_calculate_energy_delta(abs_energy, st->node_energy_total[i], b->zone_max[i]);
      const uint64_t active = kor_go_f64_to_u64(u2f(delta) * ratio);  // node.go:58
      const uint64_t idle = delta - active;                           // node.go:59
      st->node_active_total[i] += active;                             // node.go:61
      st->node_idle_total[i] += idle;                                 // node.go:62
      const double p = u2f(delta) / time_diff;                        // node.go:64
      st->node_power[i] = p;
      st->node_active_power[i] = p * ratio;  // node.go:66
      st->node_idle_power[i] = st->node_power[i] - st->node_active_power[i];
      st->node_energy_total[i] = abs_energy;
      st->node_active_energy[i] = active;
    }
    nz.active_energy[z] = st->node_active_energy[i];
    nz.power[z] = st->node_power[i];
    nz.active_power[z] = st->node_active_power[i];
  }
  st->node_ts[n] = now;                             // node.go:16 / node.go:102
  st->node_usage_ratio[n] = first_read ? 0 : ratio;  // node.go:26 (firstNodeRead leaves 0)
  st->node_has_prev[n] = 1;
  st->node_status[n] = first_read ? KACC_NODE_FIRST_READ : KACC_NODE_OK;

  // ---- resources.Refresh(): informer.go:349-410
  const Ranges r = node_ranges(b, n);
  const double *d = b->proc_cpu_delta;
  // refreshContainers + updateContainerCache (informer.go:223-249, 469-489)
  for (uint32_t c = r.c0; c < r.c1; ++c) {
    const uint32_t w = b->ctr_slot[c];
    const uint32_t s = w & KACC_SLOT_MASK;
    double delta = 0;  // resetCPUTime on the container's first process
    double total = (w & KACC_SLOT_NEW) ? 0.0 : st->ctr_cpu_total[s];  // Clone() drops totals
    for (uint32_t i = ctr_begin(b, r, c); i < b->ctr_proc_end[c]; ++i) {
      delta += d[i];
      total += d[i];
    }
    st->ctr_cpu_delta[s] = delta;
    st->ctr_cpu_total[s] = total;
  }
  // refreshVMs + updateVMCache (informer.go:251-273, 433-449): last writer wins
  for (uint32_t v = r.v0; v < r.v1; ++v) {
    const uint32_t s = b->vm_slot[v] & KACC_SLOT_MASK;
    double delta = 0;
    for (uint32_t i = vm_begin(b, r, v); i < b->vm_proc_end[v]; ++i) delta = d[i];
    st->vm_cpu_delta[s] = delta;
  }
  // refreshPods + updatePodCache (informer.go:275-326, 491-510)
  for (uint32_t q = r.q0; q < r.q1; ++q) {
    const uint32_t w = b->pod_slot[q];
    const uint32_t s = w & KACC_SLOT_MASK;
    double delta = 0;
    double total = (w & KACC_SLOT_NEW) ? 0.0 : st->pod_cpu_total[s];
    for (uint32_t c = pod_begin(b, r, q); c < b->pod_ctr_end[q]; ++c) {
      const uint32_t cs = b->ctr_slot[c] & KACC_SLOT_MASK;
      delta += st->ctr_cpu_delta[cs];
      total += st->ctr_cpu_total[cs];  // quirk: adds the container's running total
    }
    st->pod_cpu_delta[s] = delta;
    st->pod_cpu_total[s] = total;
  }
  // refreshNode (informer.go:328-345)
  const double node_delta = (b->flags & KACC_F_NODE_CPU_DELTA_GIVEN)
                                ? b->node_cpu_delta[n]
                                : node_cpu_delta_sum(d, r.p0, r.p1, sum_mode);
  st->node_cpu_delta[n] = node_delta;

  // ---- workloads: process.go:79-161, container.go:71-153, vm.go:46-121, pod.go:46-131
  for (uint32_t i = r.p0; i < r.p1; ++i) {
    const uint32_t w = b->proc_slot[i];
    const uint64_t s = w & KACC_SLOT_MASK;
    attribute(Z, d[i], node_delta, nz, false, first_read, (w & KACC_SLOT_NEW) != 0,
              st->proc_energy + s * Z, st->proc_power + s * Z);
    if (st->proc_ratio) st->proc_ratio[s] = d[i] / node_delta;  // process.go:128
    if (st->proc_node) st->proc_node[s] = n;
  }
  for (uint32_t c = r.c0; c < r.c1; ++c) {
    const uint32_t w = b->ctr_slot[c];
    const uint64_t s = w & KACC_SLOT_MASK;
    attribute(Z, st->ctr_cpu_delta[s], node_delta, nz, false, first_read,
              (w & KACC_SLOT_NEW) != 0, st->ctr_energy + s * Z, st->ctr_power + s * Z);
    if (st->ctr_ratio) st->ctr_ratio[s] = st->ctr_cpu_delta[s] / node_delta;  // container.go:118
    if (st->ctr_node) st->ctr_node[s] = n;
  }
  for (uint32_t v = r.v0; v < r.v1; ++v) {
    const uint32_t w = b->vm_slot[v];
    const uint64_t s = w & KACC_SLOT_MASK;
    attribute(Z, st->vm_cpu_delta[s], node_delta, nz, false, first_read,
              (w & KACC_SLOT_NEW) != 0, st->vm_energy + s * Z, st->vm_power + s * Z);
    if (st->vm_ratio) st->vm_ratio[s] = st->vm_cpu_delta[s] / node_delta;  // vm.go:89
    if (st->vm_node) st->vm_node[s] = n;
  }
  // pod.go:70-73 returns early when no pod is running: nothing to write.
  for (uint32_t q = r.q0; q < r.q1; ++q) {
    const uint32_t w = b->pod_slot[q];
    const uint64_t s = w & KACC_SLOT_MASK;
    attribute(Z, st->pod_cpu_delta[s], node_delta, nz, true, first_read,
              (w & KACC_SLOT_NEW) != 0, st->pod_energy + s * Z, st->pod_power + s * Z);
  }
}

extern "C" {

// cmd/compile ssagen float64ToUint64 (amd64): x < 2^63 ? CVTTSD2SQ(x)
//                                     : CVTTSD2SQ(x - 2^63) | 1<<63.
uint64_t kor_go_f64_to_u64(double x) {
  if (x < kTwo63) return static_cast<uint64_t>(cvttsd2sq(x));
  return static_cast<uint64_t>(cvttsd2sq(x - kTwo63)) | 0x8000000000000000ull;
}

// time.Duration.Seconds(): float64(d/Second) + float64(d%Second)/1e9
double kor_go_duration_seconds(int64_t d) {
  const int64_t sec = d / 1000000000LL;
  const int64_t nsec = d % 1000000000LL;
  return static_cast<double>(sec) + static_cast<double>(nsec) / 1e9;
}

// internal/monitor/node.go:87-98 calculateEnergyDelta
uint64_t kor_calculate_energy_delta(uint64_t current, uint64_t previous, uint64_t max_joules) {
  if (current >= previous) return current - previous;
  if (max_joules > 0) return (max_joules - previous) + current;  // counter wraparound
  return 0;                                                        // unable to calculate
}

int kor_interval(kor_state *st, const kacc_interval *b, int sum_mode) {
  if (!st || !b) return KACC_EINVAL;
  const uint32_t Z = st->zones;
  if (Z == 0 || Z > KACC_MAX_ZONES || b->n_nodes > st->nodes) return KACC_EINVAL;
  for (uint32_t n = 0; n < b->n_nodes; ++n) node_interval(st, b, n, sum_mode);
  return KACC_OK;
}

// The same on `threads` host threads over contiguous node ranges (CPU
// baseline only; results identical to kor_interval).
int kor_interval_mt(kor_state *st, const kacc_interval *b, int sum_mode, int threads) {
  if (!st || !b) return KACC_EINVAL;
  const uint32_t Z = st->zones;
  if (Z == 0 || Z > KACC_MAX_ZONES || b->n_nodes > st->nodes) return KACC_EINVAL;
  const uint32_t N = b->n_nodes, T = threads < 1 ? 1u : static_cast<uint32_t>(threads);
  std::vector<std::thread> pool;
  for (uint32_t t = 0; t < T; ++t) {
    const uint32_t n0 = static_cast<uint32_t>(uint64_t(N) * t / T), n1 = static_cast<uint32_t>(uint64_t(N) * (t + 1) / T);
    pool.emplace_back([=] {
      for (uint32_t n = n0; n < n1; ++n) node_interval(st, b, n, sum_mode);
    });
  }
  for (auto &th : pool) th.join();
  return KACC_OK;
}

// North-star namespace totals: sum of per-pod values grouped by
// resource.Pod.Namespace (resource/types.go:106-110).  Kepler itself leaves
// this to PromQL, so there is no Go order to follow; the engine's canonical
// order is: lane l of 16 sums pods l, l+16, ... of the namespace in list
// order, then the 16 lane sums are halved pairwise (l += l+s, s = 8..1).
// The u64 energy sums are order independent.
int kor_namespace_totals(const kor_state *st, uint32_t n_ns, const uint32_t *ns_pod_off,
                         const uint32_t *ns_pod_slot, uint64_t *out_energy, double *out_power) {
  const uint32_t Z = st->zones;
  for (uint32_t k = 0; k < n_ns; ++k) {
    for (uint32_t z = 0; z < Z; ++z) {
      uint64_t e = 0;
      double lane[16];
      for (int l = 0; l < 16; ++l) lane[l] = 0.0;
      for (uint32_t j = ns_pod_off[k]; j < ns_pod_off[k + 1]; ++j) {
        const uint64_t s = ns_pod_slot[j] & KACC_SLOT_MASK;
        e += st->pod_energy[s * Z + z];
        const uint32_t l = (j - ns_pod_off[k]) & 15u;
        lane[l] = lane[l] + st->pod_power[s * Z + z];
      }
      for (int sft = 8; sft >= 1; sft >>= 1)
        for (int l = 0; l < sft; ++l) lane[l] = lane[l] + lane[l + sft];
      out_energy[static_cast<uint64_t>(k) * Z + z] = e;
      out_power[static_cast<uint64_t>(k) * Z + z] = lane[0];
    }
  }
  return KACC_OK;
}

// device/energy_zone.go:57-67: cached ΣMaxEnergy, saturating at MaxUint64.
uint64_t kor_aggregated_max(uint32_t n, const uint64_t *sub_max) {
  uint64_t total = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (total > 0 && sub_max[i] > UINT64_MAX - total) return UINT64_MAX;
    total += sub_max[i];
  }
  return total;
}

// device/energy_zone.go:97-148 AggregatedZone.Energy
uint64_t kor_aggregated_energy(uint32_t n, const uint64_t *reading, const uint64_t *sub_max,
                               uint64_t *last, uint8_t *seen, uint64_t *current,
                               uint64_t agg_max) {
  uint64_t total_delta = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (seen[i]) {
      uint64_t delta;
      if (reading[i] >= last[i]) {
        delta = reading[i] - last[i];
      } else if (sub_max[i] > 0) {
        delta = (sub_max[i] - last[i]) + reading[i];  // :124-125 wrap
      } else {
        delta = reading[i] - last[i];  // :127-128 max==0: u64 underflow kept
      }
      total_delta += delta;
    } else {
      total_delta += reading[i];  // :130-131 first reading
    }
    last[i] = reading[i];
    seen[i] = 1;
  }
  *current += total_delta;  // :136
  if (agg_max > 0) *current %= agg_max;  // :139-145
  return *current;
}

// The same with per-sub-zone read errors: Energy() returns the error at the
// first failing sub-zone (energy_zone.go:104-108) after updating the last
// readings of the sub-zones before it; the aggregate is not updated.
int kor_aggregated_energy_st(uint32_t n, const uint64_t *reading, const uint32_t *status,
                             const uint64_t *sub_max, uint64_t *last, uint8_t *seen, uint64_t *current,
                             uint64_t agg_max, uint64_t *out) {
  uint64_t total_delta = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (status && status[i]) return KACC_ERANGE;
    if (seen[i]) {
      uint64_t delta;
      if (reading[i] >= last[i])
        delta = reading[i] - last[i];
      else if (sub_max[i] > 0)
        delta = (sub_max[i] - last[i]) + reading[i];
      else
        delta = reading[i] - last[i];
      total_delta += delta;
    } else {
      total_delta += reading[i];
    }
    last[i] = reading[i];
    seen[i] = 1;
  }
  *current += total_delta;
  if (agg_max > 0) *current %= agg_max;
  *out = *current;
  return KACC_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Go-faithful baseline: the reference's data structures, one goroutine.
// ---------------------------------------------------------------------------
namespace {

using ZoneUsageMap = std::unordered_map<int, std::pair<uint64_t, double>>;  // zone -> {E, P}

struct GfWorkload {  // monitor.Process / Container / VirtualMachine / Pod
  std::string id;
  uint64_t slot;
  double cpu_delta = 0, cpu_total = 0;
  ZoneUsageMap zones;
};
using GfMap = std::unordered_map<std::string, std::unique_ptr<GfWorkload>>;

struct GfNode {  // one node's PowerMonitor: previous snapshot + informer caches
  bool has_prev = false;
  GfMap procs, ctrs, vms, pods;
  std::unordered_map<std::string, double> ctr_cache_total, pod_cache_total;
};

}  // namespace

struct kor_gofaithful {
  uint32_t zones;
  std::vector<GfNode> nodes;
};

namespace {

std::string itoa_id(const char *prefix, uint64_t v) { return std::string(prefix) + std::to_string(v); }

void gf_attribute(uint32_t Z, const GfMap &prev_map, GfMap &out, const std::string &id,
                  uint64_t slot, double cpu_delta, double node_delta, const NodeZ &nz,
                  bool is_pod, bool first_read, bool is_new) {
  auto wl = std::make_unique<GfWorkload>();  // newProcess/newContainer/...
  wl->id = id;
  wl->slot = slot;
  wl->cpu_delta = cpu_delta;
  for (uint32_t z = 0; z < Z; ++z) wl->zones[z] = {0, 0.0};
  const GfWorkload *prev = nullptr;
  if (!is_new) {
    auto it = prev_map.find(id);
    if (it != prev_map.end()) prev = it->second.get();
  }
  for (uint32_t z = 0; z < Z; ++z) {
    const double guard_power = (is_pod && !first_read) ? nz.power[z] : nz.active_power[z];
    if (guard_power == 0 || nz.active_energy[z] == 0 || node_delta == 0) continue;
    const double ratio = cpu_delta / node_delta;
    const uint64_t e = is_pod ? kor_go_f64_to_u64(u2f(nz.active_energy[z]) * ratio)
                              : kor_go_f64_to_u64(ratio * u2f(nz.active_energy[z]));
    if (first_read) {
      wl->zones[z] = {e, 0.0};
      continue;
    }
    uint64_t abs_e = e;
    if (prev) {
      auto pz = prev->zones.find(static_cast<int>(z));
      if (pz != prev->zones.end()) abs_e += pz->second.first;
    }
    wl->zones[z] = {abs_e, ratio * nz.active_power[z]};
  }
  out[id] = std::move(wl);
}

}  // namespace

extern "C" {

kor_gofaithful *kor_gf_create(uint32_t zones) {
  auto *g = new kor_gofaithful;
  g->zones = zones;
  return g;
}

void kor_gf_destroy(kor_gofaithful *g) { delete g; }

int kor_gf_interval(kor_gofaithful *g, kor_state *st, const kacc_interval *b) {
  const uint32_t Z = g->zones;
  if (g->nodes.size() < b->n_nodes) g->nodes.resize(b->n_nodes);
  std::vector<std::string> proc_ctr_id, proc_vm_id;
  for (uint32_t n = 0; n < b->n_nodes; ++n) {
    GfNode &gn = g->nodes[n];
    const uint32_t status = b->node_status ? b->node_status[n] : 0u;
    if (status & KACC_NODE_READ_ERROR) {
      st->node_status[n] = KACC_NODE_SKIPPED;
      continue;
    }
    const bool first_read = !gn.has_prev;
    const double ratio = b->node_usage_ratio[n];
    const int64_t now = b->node_ts_ns[n];
    NodeZ nz;
    // node zones: a per-zone map as in NodeZoneUsageMap (types.go:56)
    std::map<int, uint64_t> zone_abs;
    for (uint32_t z = 0; z < Z; ++z) zone_abs[z] = b->zone_energy[static_cast<uint64_t>(n) * Z + z];
    const double time_diff =
        first_read ? 0.0 : kor_go_duration_seconds(go_sub_mono(now, st->node_ts[n]));
    for (auto &kv : zone_abs) {
      const uint64_t i = static_cast<uint64_t>(n) * Z + kv.first;
      const uint64_t abs_energy = kv.second;
      if (first_read) {
        const uint64_t active = kor_go_f64_to_u64(u2f(abs_energy) * ratio);
        st->node_active_total[i] = active;
        st->node_idle_total[i] = abs_energy - active;
        st->node_active_energy[i] = active;
        st->node_power[i] = st->node_active_power[i] = st->node_idle_power[i] = 0;
      } else {
        const uint64_t delta =
            kor_calculate_energy_delta(abs_energy, st->node_energy_total[i], b->zone_max[i]);
        const uint64_t active = kor_go_f64_to_u64(u2f(delta) * ratio);
        st->node_active_total[i] += active;
        st->node_idle_total[i] += delta - active;
        const double p = u2f(delta) / time_diff;
        st->node_power[i] = p;
        st->node_active_power[i] = p * ratio;
        st->node_idle_power[i] = p - st->node_active_power[i];
        st->node_active_energy[i] = active;
      }
      st->node_energy_total[i] = abs_energy;
      nz.active_energy[kv.first] = st->node_active_energy[i];
      nz.power[kv.first] = st->node_power[i];
      nz.active_power[kv.first] = st->node_active_power[i];
    }
    st->node_ts[n] = now;
    st->node_usage_ratio[n] = first_read ? 0 : ratio;
    st->node_has_prev[n] = 1;
    st->node_status[n] = first_read ? KACC_NODE_FIRST_READ : KACC_NODE_OK;

    // informer: per-process container/VM membership by string ID, then the
    // containersRunning / podsRunning maps (informer.go:223-326)
    const Ranges r = node_ranges(b, n);
    const double *d = b->proc_cpu_delta;
    proc_ctr_id.assign(r.p1 - r.p0, std::string());
    proc_vm_id.assign(r.p1 - r.p0, std::string());
    std::unordered_map<std::string, uint64_t> ctr_slot_of, vm_slot_of, pod_slot_of;
    std::unordered_map<std::string, bool> ctr_new, pod_new;
    std::unordered_map<std::string, std::string> ctr_pod;
    for (uint32_t c = r.c0; c < r.c1; ++c) {
      const std::string cid = itoa_id("ctr-", b->ctr_slot[c] & KACC_SLOT_MASK);
      ctr_slot_of[cid] = b->ctr_slot[c] & KACC_SLOT_MASK;
      ctr_new[cid] = (b->ctr_slot[c] & KACC_SLOT_NEW) != 0;
      for (uint32_t i = ctr_begin(b, r, c); i < b->ctr_proc_end[c]; ++i) proc_ctr_id[i - r.p0] = cid;
    }
    for (uint32_t v = r.v0; v < r.v1; ++v) {
      const std::string vid = itoa_id("vm-", b->vm_slot[v] & KACC_SLOT_MASK);
      vm_slot_of[vid] = b->vm_slot[v] & KACC_SLOT_MASK;
      for (uint32_t i = vm_begin(b, r, v); i < b->vm_proc_end[v]; ++i) proc_vm_id[i - r.p0] = vid;
    }
    for (uint32_t q = r.q0; q < r.q1; ++q) {
      const std::string pid = itoa_id("pod-", b->pod_slot[q] & KACC_SLOT_MASK);
      pod_slot_of[pid] = b->pod_slot[q] & KACC_SLOT_MASK;
      pod_new[pid] = (b->pod_slot[q] & KACC_SLOT_NEW) != 0;
      for (uint32_t c = pod_begin(b, r, q); c < b->pod_ctr_end[q]; ++c)
        ctr_pod[itoa_id("ctr-", b->ctr_slot[c] & KACC_SLOT_MASK)] = pid;
    }
    // refreshContainers: container cache updated per process in listing order
    std::unordered_map<std::string, std::pair<double, double>> ctr_running;  // id -> {delta,total}
    std::vector<std::string> ctr_order;
    for (uint32_t i = r.p0; i < r.p1; ++i) {
      const std::string &cid = proc_ctr_id[i - r.p0];
      if (cid.empty()) continue;
      auto it = ctr_running.find(cid);
      if (it == ctr_running.end()) {
        if (ctr_new[cid]) gn.ctr_cache_total.erase(cid);
        double total = gn.ctr_cache_total.count(cid) ? gn.ctr_cache_total[cid] : 0.0;
        it = ctr_running.emplace(cid, std::make_pair(0.0, total)).first;
        ctr_order.push_back(cid);
      }
      it->second.first += d[i];
      it->second.second += d[i];
    }
    for (auto &kv : ctr_running) gn.ctr_cache_total[kv.first] = kv.second.second;
    // refreshVMs: last writer wins
    std::unordered_map<std::string, double> vm_running;
    for (uint32_t i = r.p0; i < r.p1; ++i) {
      const std::string &vid = proc_vm_id[i - r.p0];
      if (!vid.empty()) vm_running[vid] = d[i];
    }
    // refreshPods: pods accumulate their containers (container order)
    std::unordered_map<std::string, std::pair<double, double>> pod_running;
    for (const std::string &cid : ctr_order) {
      auto pit = ctr_pod.find(cid);
      if (pit == ctr_pod.end()) continue;  // ContainersNoPod
      const std::string &pid = pit->second;
      auto it = pod_running.find(pid);
      if (it == pod_running.end()) {
        if (pod_new[pid]) gn.pod_cache_total.erase(pid);
        double total = gn.pod_cache_total.count(pid) ? gn.pod_cache_total[pid] : 0.0;
        it = pod_running.emplace(pid, std::make_pair(0.0, total)).first;
      }
      it->second.first += ctr_running[cid].first;
      it->second.second += ctr_running[cid].second;
    }
    for (auto &kv : pod_running) gn.pod_cache_total[kv.first] = kv.second.second;
    // refreshNode: map-ordered sum over running processes (here: listing)
    double node_delta = 0;
    if (b->flags & KACC_F_NODE_CPU_DELTA_GIVEN) {
      node_delta = b->node_cpu_delta[n];
    } else {
      std::unordered_map<std::string, double> running;
      for (uint32_t i = r.p0; i < r.p1; ++i)
        running[std::to_string(b->proc_slot[i] & KACC_SLOT_MASK)] = d[i];
      for (uint32_t i = r.p0; i < r.p1; ++i)
        node_delta += running[std::to_string(b->proc_slot[i] & KACC_SLOT_MASK)];
    }
    st->node_cpu_delta[n] = node_delta;

    // calculateProcessPower & co: new maps keyed by string ID, prev lookups
    GfMap new_procs, new_ctrs, new_vms, new_pods;
    for (uint32_t i = r.p0; i < r.p1; ++i) {
      const uint32_t w = b->proc_slot[i];
      gf_attribute(Z, gn.procs, new_procs, std::to_string(w & KACC_SLOT_MASK), w & KACC_SLOT_MASK,
                   d[i], node_delta, nz, false, first_read, (w & KACC_SLOT_NEW) != 0);
    }
    for (auto &kv : ctr_running)
      gf_attribute(Z, gn.ctrs, new_ctrs, kv.first, ctr_slot_of[kv.first], kv.second.first,
                   node_delta, nz, false, first_read, ctr_new[kv.first]);
    for (auto &kv : vm_running) {
      bool is_new = false;
      for (uint32_t v = r.v0; v < r.v1; ++v)
        if ((b->vm_slot[v] & KACC_SLOT_MASK) == vm_slot_of[kv.first])
          is_new = (b->vm_slot[v] & KACC_SLOT_NEW) != 0;
      gf_attribute(Z, gn.vms, new_vms, kv.first, vm_slot_of[kv.first], kv.second, node_delta,
                   nz, false, first_read, is_new);
    }
    for (auto &kv : pod_running)
      gf_attribute(Z, gn.pods, new_pods, kv.first, pod_slot_of[kv.first], kv.second.first,
                   node_delta, nz, true, first_read, pod_new[kv.first]);

    // store the snapshot (monitor.go:341-342) and mirror it into the tables
    auto dump = [Z](const GfMap &m, uint64_t *E, double *P) {
      for (const auto &kv : m)
        for (const auto &zu : kv.second->zones) {
          E[kv.second->slot * Z + zu.first] = zu.second.first;
          P[kv.second->slot * Z + zu.first] = zu.second.second;
        }
    };
    dump(new_procs, st->proc_energy, st->proc_power);
    dump(new_ctrs, st->ctr_energy, st->ctr_power);
    dump(new_vms, st->vm_energy, st->vm_power);
    dump(new_pods, st->pod_energy, st->pod_power);
    for (auto &kv : ctr_running) {
      st->ctr_cpu_delta[ctr_slot_of[kv.first]] = kv.second.first;
      st->ctr_cpu_total[ctr_slot_of[kv.first]] = kv.second.second;
    }
    for (auto &kv : vm_running) st->vm_cpu_delta[vm_slot_of[kv.first]] = kv.second;
    for (auto &kv : pod_running) {
      st->pod_cpu_delta[pod_slot_of[kv.first]] = kv.second.first;
      st->pod_cpu_total[pod_slot_of[kv.first]] = kv.second.second;
    }
    gn.procs = std::move(new_procs);
    gn.ctrs = std::move(new_ctrs);
    gn.vms = std::move(new_vms);
    gn.pods = std::move(new_pods);
    gn.has_prev = true;
  }
  return KACC_OK;
}

}  // extern "C"
