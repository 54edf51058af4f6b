// ORACLE — TEST INFRASTRUCTURE ONLY (see kepler_oracle.h).
//
// CPU restatement of the slot join (include/kepler_accel.h kacc_slot_join)
// in terms of the reference's own data structures: per node, the set of IDs
// of the previous snapshot is a map (Go: prev.Processes keyed by PID string,
// process.go:132-138; prev.Containers / VirtualMachines / Pods by ID,
// container.go:126, vm.go:96, pod.go:106), and the terminated set is
// "cached before, not running now" (informer.go:206-212 for processes,
// :236-246 containers, :260-270 VMs, :311-322 pods).  The slot numbering rule
// is the engine's own (the reference has no slots): a new ID takes the lowest
// slot of its node's range not held by any ID of the previous set, new rows
// taking slots in row order; with KACC_JOIN_REUSE_TERMINATED the slots of the
// IDs terminated in the same call come first (ascending by slot).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "kepler_oracle.h"

struct kor_slotmap {
  std::vector<uint32_t> slot_off;
  std::vector<std::unordered_map<uint64_t, uint32_t>> live;  // per node: ID -> slot
  uint32_t policy = 0;  // KACC_JOIN_REUSE_TERMINATED
};

extern "C" {

kor_slotmap *kor_slotmap_create(uint32_t n_nodes, const uint32_t *slot_off) {
  auto *m = new kor_slotmap;
  m->slot_off.assign(slot_off, slot_off + n_nodes + 1);
  m->live.resize(n_nodes);
  return m;
}

void kor_slotmap_destroy(kor_slotmap *m) { delete m; }

void kor_slotmap_set_policy(kor_slotmap *m, uint32_t policy) { m->policy = policy; }

int kor_slot_join(kor_slotmap *m, uint32_t n_rows, const uint32_t *row_off, const uint64_t *keys,
                  const uint32_t *node_status, uint32_t *out_slot, uint64_t *term_key,
                  uint32_t *term_slot, uint32_t *term_count) {
  const uint32_t N = static_cast<uint32_t>(m->live.size());
  int rc = KACC_OK;
  for (uint32_t n = 0; n < N; ++n) {
    term_count[n] = 0;
    if (node_status && (node_status[n] & KACC_NODE_READ_ERROR)) continue;  // Refresh skipped
    const uint32_t r0 = row_off[n], r1 = row_off[n + 1];
    if (r1 > n_rows || r0 > r1) return KACC_EINVAL;
    const uint32_t s0 = m->slot_off[n], S = m->slot_off[n + 1] - s0;
    auto &prev = m->live[n];
    std::vector<uint8_t> used(S, 0);
    for (const auto &kv : prev) used[kv.second] = 1;  // held until the next interval
    std::unordered_map<uint64_t, uint32_t> cur;
    cur.reserve(r1 - r0);
    uint32_t next_free = 0;
    // KACC_JOIN_REUSE_TERMINATED: the previous IDs absent from this batch, their
    // slots ascending, go to the new rows first (in row order)
    std::vector<uint32_t> reuse;
    size_t next_reuse = 0;
    if (m->policy & KACC_JOIN_REUSE_TERMINATED) {
      std::unordered_map<uint64_t, uint8_t> now;
      now.reserve(r1 - r0);
      for (uint32_t r = r0; r < r1; ++r) now.emplace(keys[r], 1);
      for (const auto &kv : prev)
        if (!now.count(kv.first)) reuse.push_back(kv.second);
      std::sort(reuse.begin(), reuse.end());
    }
    for (uint32_t r = r0; r < r1; ++r) {
      const uint64_t k = keys[r];
      if (k == KACC_KEY_EMPTY || k == KACC_KEY_TOMB || cur.count(k)) {
        out_slot[r] = 0xffffffffu;
        rc = KACC_ERANGE;
        continue;
      }
      auto it = prev.find(k);
      if (it != prev.end()) {  // running total continues (process.go:134-137)
        out_slot[r] = s0 + it->second;
        cur.emplace(k, it->second);
        continue;
      }
      if (next_reuse < reuse.size()) {  // a slot terminated in this call
        const uint32_t sl = reuse[next_reuse++];
        out_slot[r] = (s0 + sl) | KACC_SLOT_NEW;
        cur.emplace(k, sl);
        continue;
      }
      while (next_free < S && used[next_free]) ++next_free;
      if (next_free >= S) {
        out_slot[r] = 0xffffffffu;
        rc = KACC_ERANGE;
        continue;
      }
      used[next_free] = 1;
      out_slot[r] = (s0 + next_free) | KACC_SLOT_NEW;
      cur.emplace(k, next_free);
    }
    // terminated (informer.go:206-212): the node's segment, ascending by slot
    std::vector<std::pair<uint32_t, uint64_t>> term;
    for (const auto &kv : prev)
      if (!cur.count(kv.first)) term.emplace_back(kv.second, kv.first);
    std::sort(term.begin(), term.end());
    for (size_t i = 0; i < term.size(); ++i) {
      term_key[s0 + i] = term[i].second;
      term_slot[s0 + i] = s0 + term[i].first;
    }
    term_count[n] = static_cast<uint32_t>(term.size());
    prev.swap(cur);
  }
  return rc;
}

}  // extern "C"
