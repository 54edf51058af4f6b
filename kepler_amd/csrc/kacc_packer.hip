// Host SoA packer (the step before the path) and the
// device unpack of per-workload results.
//
// kacc_pack turns informer-shaped records — per node, the running processes
// in /proc listing order with their resource.Process fields — into the
// kacc_interval CSR layout, reproducing the informer's segment membership
// and summation orders (internal/resource/informer.go):
//   * refreshProcesses (:167-220) walks AllProcs() in listing order and
//     collects container / VM processes in that order;
//   * refreshContainers (:223-249): a container's CPUTimeDelta is the sum of
//     its processes' deltas in listing order, reset at its first process —
//     so a container's rows keep their listing order;
//   * refreshVMs (:251-273): last writer wins — a VM's rows keep their
//     listing order (its last row is the writer);
//   * refreshPods (:275-326) walks the running containers (a Go map: random
//     order) and looks up each container's pod; containers without a pod go
//     to ContainersNoPod.  The packer fixes that order: pods in the order of
//     their containers' first appearance, each pod's containers in first-
//     appearance order, ContainersNoPod after the pods (pod sums over a map
//     agree with any fixed order to <= 1e-12).
// Rows inside a node: container processes grouped by container (containers
// grouped by pod), then VM processes grouped by VM, then the others — the
// layout kepler_accel.h requires.  The per-row / per-aggregate keys it emits
// are the inputs of kacc_slot_join (PIDs, container / VM / pod IDs), and
// row_record maps every row back to its input record for kacc_unpack.
//
// Two passes over node ranges on host threads (count, then write at the
// prefix-summed offsets); per node a reusable open-addressing map per kind.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "kacc_derive.hpp"
#include "kacc_internal.hpp"

namespace {

constexpr uint32_t kNone = 0xffffffffu;

// Open-addressing map u64 key -> u32 (first-appearance index), reused per node.
struct KeyMap {
  std::vector<uint64_t> keys;
  std::vector<uint32_t> vals;
  uint64_t mask = 0;
  void reset(size_t n) {
    size_t cap = 16;
    while (cap < 2 * n) cap <<= 1;
    if (keys.size() < cap) {
      keys.assign(cap, KACC_KEY_EMPTY);
      vals.assign(cap, 0);
    } else {
      std::fill(keys.begin(), keys.begin() + cap, KACC_KEY_EMPTY);
    }
    mask = cap - 1;
  }
  // index of `k`, inserting `next` when absent (then *added = true)
  uint32_t get(uint64_t k, uint32_t next, bool *added) {
    uint64_t x = k * 0x9E3779B97F4A7C15ull;
    uint64_t b = (x ^ (x >> 29)) & mask;
    for (;;) {
      if (keys[b] == k) {
        *added = false;
        return vals[b];
      }
      if (keys[b] == KACC_KEY_EMPTY) {
        keys[b] = k;
        vals[b] = next;
        *added = true;
        return next;
      }
      b = (b + 1) & mask;
    }
  }
};

struct Agg {
  uint64_t key;
  uint64_t pod;  // containers: pod key of the first process (KACC_KEY_EMPTY: no pod)
  uint32_t ns;
  uint32_t rows;
  uint32_t group;  // containers: pod index (kNone: ContainersNoPod)
  uint32_t pos;    // position in the node's output order
  uint32_t cursor; // next row while writing
};

struct Scratch {
  KeyMap cmap, vmap, pmap;
  std::vector<Agg> ctrs, vms, pods;
  std::vector<uint32_t> grp;  // per record: container / VM index
  std::vector<uint32_t> order;
};

struct Counts {
  uint32_t c = 0, v = 0, q = 0;
};

struct Bases {
  uint32_t p, c, v, q;
};

// One node: membership (pass 1) and, when `o` is given, the output at `b`.
int pack_node(const kacc_records &in, uint32_t n, Scratch &s, Counts *cnt, kacc_packed *o, const Bases *b) {
  const uint32_t r0 = in.rec_off[n], r1 = in.rec_off[n + 1], R = r1 - r0;
  s.cmap.reset(R);
  s.vmap.reset(R);
  s.ctrs.clear();
  s.vms.clear();
  s.pods.clear();
  s.grp.resize(R);
  uint32_t regular = 0;
  for (uint32_t r = r0; r < r1; ++r) {  // informer.go:182-205, listing order
    const uint8_t t = in.type[r];
    bool added = false;
    if (t == KACC_PROC_CONTAINER) {
      const uint64_t k = in.ctr_key[r];
      if (k >= KACC_KEY_TOMB) return -1;
      // KACC_KEY_EMPTY = the pod lookup found none (ContainersNoPod); the other reserved key is an error
      if (in.pod_key && in.pod_key[r] == KACC_KEY_TOMB) return -1;
      const uint32_t i = s.cmap.get(k, static_cast<uint32_t>(s.ctrs.size()), &added);
      if (added)
        s.ctrs.push_back(Agg{k, in.pod_key ? in.pod_key[r] : KACC_KEY_EMPTY, in.pod_ns ? in.pod_ns[r] : 0u, 0,
                             kNone, 0, 0});
      ++s.ctrs[i].rows;
      s.grp[r - r0] = i;
    } else if (t == KACC_PROC_VM) {
      const uint64_t k = in.vm_key[r];
      if (k >= KACC_KEY_TOMB) return -1;
      const uint32_t i = s.vmap.get(k, static_cast<uint32_t>(s.vms.size()), &added);
      if (added) s.vms.push_back(Agg{k, 0, 0, 0, 0, 0, 0});
      ++s.vms[i].rows;
      s.grp[r - r0] = i;
    } else if (t == KACC_PROC_REGULAR) {
      ++regular;
    } else {
      return -2;
    }
  }
  // pods in the order of their containers' first appearance (informer.go:284-310)
  s.pmap.reset(s.ctrs.size());
  for (Agg &c : s.ctrs) {
    if (c.pod == KACC_KEY_EMPTY) continue;  // ContainersNoPod
    bool added = false;
    const uint32_t q = s.pmap.get(c.pod, static_cast<uint32_t>(s.pods.size()), &added);
    if (added) s.pods.push_back(Agg{c.pod, 0, c.ns, 0, 0, 0, 0});
    c.group = q;
    ++s.pods[q].rows;  // containers of the pod
  }
  cnt->c = static_cast<uint32_t>(s.ctrs.size());
  cnt->v = static_cast<uint32_t>(s.vms.size());
  cnt->q = static_cast<uint32_t>(s.pods.size());
  if (!o) return 0;
  // container order: grouped by pod (pod order), ContainersNoPod last; stable
  const uint32_t C = cnt->c, Q = cnt->q;
  std::vector<uint32_t> &ord = s.order;
  ord.assign(Q + 2, 0);
  for (const Agg &c : s.ctrs) ++ord[(c.group == kNone ? Q : c.group) + 1];
  for (uint32_t q = 0; q <= Q; ++q) ord[q + 1] += ord[q];
  for (Agg &c : s.ctrs) c.pos = ord[c.group == kNone ? Q : c.group]++;
  // row ranges: containers in output order, then VMs, then the rest
  std::vector<uint32_t> by_pos(C);
  for (uint32_t i = 0; i < C; ++i) by_pos[s.ctrs[i].pos] = i;
  uint32_t row = b->p;
  for (uint32_t j = 0; j < C; ++j) {
    Agg &c = s.ctrs[by_pos[j]];
    c.cursor = row;
    row += c.rows;
    o->ctr_proc_end[b->c + j] = row;
    o->ctr_key[b->c + j] = c.key;
  }
  for (uint32_t j = 0; j < cnt->v; ++j) {
    Agg &v = s.vms[j];
    v.cursor = row;
    row += v.rows;
    o->vm_proc_end[b->v + j] = row;
    o->vm_key[b->v + j] = v.key;
  }
  uint32_t rest = row;
  uint32_t cend = b->c;
  for (uint32_t q = 0; q < Q; ++q) {
    cend += s.pods[q].rows;
    o->pod_ctr_end[b->q + q] = cend;
    o->pod_key[b->q + q] = s.pods[q].key;
    o->pod_ns[b->q + q] = s.pods[q].ns;
  }
  for (uint32_t r = r0; r < r1; ++r) {  // listing order inside every segment
    const uint8_t t = in.type[r];
    uint32_t dst;
    if (t == KACC_PROC_CONTAINER)
      dst = s.ctrs[s.grp[r - r0]].cursor++;
    else if (t == KACC_PROC_VM)
      dst = s.vms[s.grp[r - r0]].cursor++;
    else
      dst = rest++;
    o->proc_cpu_delta[dst] = in.cpu_delta[r];
    o->proc_key[dst] = in.pid[r];
    if (o->row_record) o->row_record[dst] = r;
  }
  (void)regular;
  return 0;
}

template <typename F>
void for_node_ranges(const kacc_records &in, uint32_t threads, F fn) {
  const uint32_t N = in.n_nodes;
  const uint32_t T = std::max<uint32_t>(1, std::min<uint32_t>(threads, std::max<uint32_t>(N, 1)));
  if (T == 1) {
    fn(0u, N, 0u);
    return;
  }
  // cuts balanced by records
  std::vector<uint32_t> cut(T + 1, N);
  cut[0] = 0;
  const uint64_t total = in.rec_off[N];
  uint32_t n = 0;
  for (uint32_t t = 1; t < T; ++t) {
    const uint64_t target = total * t / T;
    while (n < N && in.rec_off[n] < target) ++n;
    cut[t] = n;
  }
  std::vector<std::thread> pool;
  for (uint32_t t = 0; t < T; ++t) pool.emplace_back(fn, cut[t], std::max(cut[t], cut[t + 1]), t);
  for (auto &th : pool) th.join();
}

}  // namespace

namespace kacc {
namespace unpack {

constexpr int kThreads = 256;

// out[dest ? dest[i] : i] = the tables' row of slot word w[i] (energy, power per zone).
// Processes / containers / VMs (tp NULL): power derived from the slot's ratio and
// its node's tables (kacc_derive.hpp).  Pods (tp given): te / tp point into the
// pod records, a slot's row `stride` = 2Z words after the previous one's.
template <int Z>
__global__ __launch_bounds__(kThreads) void unpack_kernel(uint32_t n, const uint32_t *w, const uint32_t *dest,
                                                          uint64_t cap, const uint64_t *te, const double *tp,
                                                          uint32_t stride, const ProcDerive pd, uint64_t *oe,
                                                          double *op, uint32_t *err) {
  const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const uint64_t s = w[i] & KACC_SLOT_MASK;
  const uint64_t o = static_cast<uint64_t>(dest ? dest[i] : i) * Z;
  if (s >= cap) {
    atomicOr(err, 1u << 2);  // the slot bit of kacc_sync
    return;
  }
#pragma unroll
  for (int z = 0; z < Z; ++z) {
    oe[o + z] = te[s * stride + z];
    op[o + z] = tp ? tp[s * stride + z] : proc_power(pd, s, z);
  }
}

}  // namespace unpack
}  // namespace kacc

extern "C" {

int kacc_pack(const kacc_records *in, kacc_packed *out, uint32_t threads) {
  if (!in || !out) return kacc_fail(nullptr, KACC_EINVAL, "kacc_pack: NULL argument");
  const uint32_t N = in->n_nodes;
  if (!in->rec_off) return kacc_fail(nullptr, KACC_EINVAL, "kacc_pack: rec_off is NULL");
  const uint32_t R = in->rec_off[N];
  if (in->rec_off[0] != 0) return kacc_fail(nullptr, KACC_EINVAL, "kacc_pack: rec_off[0] != 0");
  for (uint32_t n = 0; n < N; ++n)
    if (in->rec_off[n + 1] < in->rec_off[n]) return kacc_fail(nullptr, KACC_EINVAL, "kacc_pack: rec_off not monotonic");
  if (R && (!in->pid || !in->cpu_delta || !in->type || !in->ctr_key || !in->vm_key))
    return kacc_fail(nullptr, KACC_EINVAL, "kacc_pack: NULL record array");
  if (!out->proc_off || !out->ctr_off || !out->vm_off || !out->pod_off)
    return kacc_fail(nullptr, KACC_EINVAL, "kacc_pack: NULL offset array");
  // pass 1: counts per node
  std::vector<Counts> cnt(N);
  std::atomic<int> bad{0};
  std::atomic<uint32_t> bad_node{0};
  for_node_ranges(*in, threads ? threads : 1, [&](uint32_t nb, uint32_t ne, uint32_t) {
    Scratch s;
    for (uint32_t n = nb; n < ne; ++n) {
      const int rc = pack_node(*in, n, s, &cnt[n], nullptr, nullptr);
      if (rc) {
        bad = rc;
        bad_node = n;
        return;
      }
    }
  });
  if (bad == -1)
    return kacc_fail(nullptr, KACC_EINVAL, "kacc_pack: node %u: a container / VM key, or a pod key other than KACC_KEY_EMPTY, is a reserved value",
                     bad_node.load());
  if (bad == -2) return kacc_fail(nullptr, KACC_EINVAL, "kacc_pack: node %u: unknown process type", bad_node.load());
  // offsets
  uint64_t C = 0, V = 0, Q = 0;
  out->proc_off[0] = out->ctr_off[0] = out->vm_off[0] = out->pod_off[0] = 0;
  for (uint32_t n = 0; n < N; ++n) {
    C += cnt[n].c;
    V += cnt[n].v;
    Q += cnt[n].q;
    if (C > 0xffffffffull || V > 0xffffffffull || Q > 0xffffffffull)
      return kacc_fail(nullptr, KACC_EINVAL, "kacc_pack: more than 2^32 aggregates");
    out->proc_off[n + 1] = in->rec_off[n + 1];
    out->ctr_off[n + 1] = static_cast<uint32_t>(C);
    out->vm_off[n + 1] = static_cast<uint32_t>(V);
    out->pod_off[n + 1] = static_cast<uint32_t>(Q);
  }
  const bool fits = R <= out->n_procs && C <= out->n_ctrs && V <= out->n_vms && Q <= out->n_pods;
  const uint32_t cap_p = out->n_procs, cap_c = out->n_ctrs, cap_v = out->n_vms, cap_q = out->n_pods;
  out->n_procs = R;
  out->n_ctrs = static_cast<uint32_t>(C);
  out->n_vms = static_cast<uint32_t>(V);
  out->n_pods = static_cast<uint32_t>(Q);
  if (!fits)
    return kacc_fail(nullptr, KACC_ERANGE,
                     "kacc_pack: needs %u rows / %llu containers / %llu VMs / %llu pods, capacity %u / %u / %u / %u", R,
                     (unsigned long long)C, (unsigned long long)V, (unsigned long long)Q, cap_p, cap_c, cap_v, cap_q);
  if ((R && (!out->proc_cpu_delta || !out->proc_key)) || (C && (!out->ctr_proc_end || !out->ctr_key)) ||
      (V && (!out->vm_proc_end || !out->vm_key)) || (Q && (!out->pod_ctr_end || !out->pod_key || !out->pod_ns)))
    return kacc_fail(nullptr, KACC_EINVAL, "kacc_pack: NULL output array");
  // pass 2: write at the offsets
  for_node_ranges(*in, threads ? threads : 1, [&](uint32_t nb, uint32_t ne, uint32_t) {
    Scratch s;
    for (uint32_t n = nb; n < ne; ++n) {
      const Bases b{out->proc_off[n], out->ctr_off[n], out->vm_off[n], out->pod_off[n]};
      Counts c;
      pack_node(*in, n, s, &c, out, &b);
    }
  });
  return KACC_OK;
}

int kacc_unpack(kacc_ctx *ctx, kacc_kind kind, uint32_t n, const uint32_t *slot_words, const uint32_t *dest,
                uint64_t *out_energy, double *out_power, void *stream) {
  if (!ctx) return KACC_EINVAL;
  if (!n) return KACC_OK;
  if (!slot_words || !out_energy || !out_power) return kacc_fail(ctx, KACC_EINVAL, "kacc_unpack: NULL argument");
  if (kind < KACC_KIND_PROC || kind > KACC_KIND_POD) return kacc_fail(ctx, KACC_EINVAL, "bad kind");
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  const int te = kind == KACC_KIND_PROC ? KACC_T_PROC_ENERGY
                 : kind == KACC_KIND_CTR ? KACC_T_CTR_ENERGY
                 : kind == KACC_KIND_VM ? KACC_T_VM_ENERGY
                                        : KACC_T_POD_ENERGY;
  const uint64_t cap = kind == KACC_KIND_PROC ? ctx->cfg.proc_slots
                       : kind == KACC_KIND_CTR ? ctx->cfg.ctr_slots
                       : kind == KACC_KIND_VM ? ctx->cfg.vm_slots
                                              : ctx->cfg.pod_slots;
  const uint64_t *e = static_cast<const uint64_t *>(ctx->tables[te]);
  // processes, containers, VMs: power derived (kacc_derive.hpp); pods: the table
  const double *p = kind == KACC_KIND_POD ? static_cast<const double *>(ctx->tables[te + 1]) : nullptr;
  const kacc::ProcDerive pd = kacc_derive(ctx, kind);
  const uint32_t grid = (n + kacc::unpack::kThreads - 1) / kacc::unpack::kThreads;
  (void)hipGetLastError();
#define KACC_UNPACK(Z)                                                                                          \
  hipLaunchKernelGGL((kacc::unpack::unpack_kernel<Z>), dim3(grid), dim3(kacc::unpack::kThreads), 0, st, n,   \
                     slot_words, dest, cap, e, p, kind == KACC_KIND_POD ? 2 * Z : Z, pd, out_energy, out_power,   \
                     ctx->d_err)
  switch (ctx->cfg.zones) {
    case 1: KACC_UNPACK(1); break;
    case 2: KACC_UNPACK(2); break;
    case 3: KACC_UNPACK(3); break;
    case 4: KACC_UNPACK(4); break;
    case 5: KACC_UNPACK(5); break;
    case 6: KACC_UNPACK(6); break;
    case 7: KACC_UNPACK(7); break;
    default: KACC_UNPACK(8); break;
  }
#undef KACC_UNPACK
  KACC_HIP(ctx, hipGetLastError());
  return KACC_OK;
}

}  // extern "C"
