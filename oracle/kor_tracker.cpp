// ORACLE — TEST INFRASTRUCTURE ONLY (see kepler_oracle.h).
//
// CPU restatement of TerminatedResourceTracker
// (internal/monitor/terminated_resource_tracker.go) with Go's container/heap
// algorithms (Push = append + up, Pop = swap(0, n-1) + down + remove last;
// Less = EnergyTotal <, :188-191), item by item as Add() does it — one tracker
// per node, as every node's PowerMonitor owns its own (monitor.go:123-144).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <utility>
#include <vector>

#include "kepler_oracle.h"

namespace {

struct Item {
  uint64_t e;  // EnergyTotal of the target zone
  uint32_t node;
  uint64_t key;
  std::vector<uint64_t> energy;
  std::vector<double> power;
};

}  // namespace

// One node's TerminatedResourceTracker.
struct NodeTracker {
  int64_t max_size;
  uint64_t min_energy;
  std::vector<Item> heap;                                       // Heap[T]
  std::map<std::pair<uint32_t, uint64_t>, size_t> resources;   // ID -> present (index unused)

  bool less(size_t i, size_t j) const { return heap[i].e < heap[j].e; }
  void up(size_t j) {  // container/heap up
    while (j > 0) {
      const size_t i = (j - 1) / 2;
      if (!less(j, i)) break;
      std::swap(heap[i], heap[j]);
      j = i;
    }
  }
  void down(size_t i0, size_t n) {  // container/heap down
    size_t i = i0;
    for (;;) {
      const size_t j1 = 2 * i + 1;
      if (j1 >= n) break;
      size_t j = j1;
      if (j1 + 1 < n && less(j1 + 1, j1)) j = j1 + 1;
      if (!less(j, i)) break;
      std::swap(heap[i], heap[j]);
      i = j;
    }
  }
  void push(Item it) {
    heap.push_back(std::move(it));
    up(heap.size() - 1);
  }
  Item pop() {
    const size_t n = heap.size() - 1;
    std::swap(heap[0], heap[n]);
    down(0, n);
    Item it = std::move(heap.back());
    heap.pop_back();
    return it;
  }
  // terminated_resource_tracker.go:80-137
  void add(Item it) {
    if (max_size == 0) return;                                   // :82
    const auto id = std::make_pair(it.node, it.key);
    if (resources.count(id)) return;                             // :90
    if (it.e < min_energy) return;                               // :102
    if (static_cast<int64_t>(heap.size()) < max_size || max_size < 0) {  // :116
      resources[id] = 1;
      push(std::move(it));
      return;
    }
    if (!heap.empty() && it.e > heap[0].e) {                     // :124
      Item gone = pop();
      resources.erase(std::make_pair(gone.node, gone.key));
      resources[id] = 1;
      push(std::move(it));
    }
  }
};

struct kor_tracker {
  int64_t max_size;
  uint64_t min_energy;
  uint32_t zones, zone;
  std::map<uint32_t, NodeTracker> nodes;  // node -> its own tracker
  void add(Item it) {
    auto f = nodes.find(it.node);
    if (f == nodes.end()) f = nodes.emplace(it.node, NodeTracker{max_size, min_energy, {}, {}}).first;
    f->second.add(std::move(it));
  }
};

extern "C" {

kor_tracker *kor_tracker_create(int64_t max_size, uint64_t min_energy, uint32_t zones, uint32_t zone) {
  auto *t = new kor_tracker;
  t->max_size = max_size;
  t->min_energy = min_energy;
  t->zones = zones;
  t->zone = zone;
  return t;
}

void kor_tracker_destroy(kor_tracker *t) { delete t; }

void kor_tracker_clear(kor_tracker *t) {  // :156-160, every node
  t->nodes.clear();
}

void kor_tracker_clear_node(kor_tracker *t, uint32_t node) { t->nodes.erase(node); }

void kor_tracker_add_one(kor_tracker *t, uint32_t node, uint64_t key, const uint64_t *energy,
                         const double *power) {
  Item it;
  it.node = node;
  it.key = key;
  it.energy.assign(energy, energy + t->zones);
  it.power.assign(power, power + t->zones);
  it.e = it.energy[t->zone];
  t->add(std::move(it));
}

void kor_tracker_add_batch(kor_tracker *t, uint32_t n, const uint32_t *node, const uint64_t *key,
                           const uint32_t *slot, const uint64_t *tab_e, const double *tab_p) {
  // one of Go's map orders for procs.Terminated (process.go:89): energy desc, node, slot
  std::vector<uint32_t> ord(n);
  for (uint32_t i = 0; i < n; ++i) ord[i] = i;
  const uint32_t Z = t->zones, z0 = t->zone;
  std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) {
    const uint64_t ea = tab_e[static_cast<uint64_t>(slot[a]) * Z + z0];
    const uint64_t eb = tab_e[static_cast<uint64_t>(slot[b]) * Z + z0];
    if (ea != eb) return ea > eb;
    if (node[a] != node[b]) return node[a] < node[b];
    return slot[a] < slot[b];
  });
  for (uint32_t i : ord)
    kor_tracker_add_one(t, node[i], key[i], tab_e + static_cast<uint64_t>(slot[i]) * Z,
                        tab_p + static_cast<uint64_t>(slot[i]) * Z);
}

uint32_t kor_tracker_items(const kor_tracker *t, uint64_t *key, uint32_t *node, uint64_t *energy,
                           double *power) {
  // Items() is a map: returned here sorted by (node, key)
  std::vector<const Item *> v;
  for (const auto &nt : t->nodes)
    for (const auto &it : nt.second.heap) v.push_back(&it);
  std::sort(v.begin(), v.end(), [](const Item *a, const Item *b) {
    return a->node != b->node ? a->node < b->node : a->key < b->key;
  });
  const uint32_t Z = t->zones;
  for (size_t i = 0; i < v.size(); ++i) {
    if (key) key[i] = v[i]->key;
    if (node) node[i] = v[i]->node;
    for (uint32_t z = 0; z < Z; ++z) {
      if (energy) energy[i * Z + z] = v[i]->energy[z];
      if (power) power[i * Z + z] = v[i]->power[z];
    }
  }
  return static_cast<uint32_t>(v.size());
}

}  // extern "C"
