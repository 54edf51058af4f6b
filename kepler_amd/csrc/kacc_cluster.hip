// Cluster totals across GPUs over RCCL (SURVEY §8(b) kacc_create_multi /
// kacc_allreduce_namespaces, §8(e)).
//
// Kepler has no collectives: every node exports its own metrics and cluster
// sums are left to PromQL (`sum by (namespace)`).  The north star moves the
// fleet onto GPUs as contiguous node shards (kepler_amd/shard.py), so the
// attribution itself never crosses a GPU; the only cross-GPU quantities are
//   * per-namespace totals over pods (grouped by Pod.Namespace,
//     internal/resource/types.go:106-110): u64 energy per zone (modular, exact
//     in any order) and f64 power per zone;
//   * cluster node totals per zone: Σ NodeUsage.ActiveEnergyTotal /
//     IdleEnergyTotal (u64) and Σ Power / ActivePower / IdlePower (f64)
//     (monitor/types.go:27-40);
//   * the pods themselves (a pod lives on exactly one node, so "cluster pod
//     totals" are a gather, not a reduction).
//
// A cluster is a set of shards (engine contexts).  RCCL ranks are GPUs: a
// process may hold several shards on one GPU (their partial vectors are first
// added on that GPU, in shard order) and several GPUs (ncclCommInitAll), or
// one shard per process (ncclCommInitRank, the one-process-per-GPU launch).
// Every collective is enqueued on the shard's stream: nothing here blocks the
// host except kacc_gather_pods' count exchange.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "kacc_internal.hpp"

// RCCL is loaded on first use (dlopen), not linked: single-GPU users of the
// library (and the C99 ABI client) need no librccl at load time.  The library
// binds the RCCL that the process already holds under the soname librccl.so.1
// (e.g. torch's), else the first on the search path (the build's RUNPATH,
// /opt/rocm/lib); KACC_RCCL_PATH names another file.  The version is read with
// ncclGetVersion and a major version other than the headers' (NCCL_MAJOR) is
// refused; kacc_cluster_rccl() reports the version and the file in use.
namespace {
struct Rccl {
  bool ok = false;
  std::string err;
  int version = 0;
  std::string path;
  decltype(&ncclGetVersion) GetVersion = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommInitAll) CommInitAll = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclAllReduce) AllReduce = nullptr;
  decltype(&ncclAllGather) AllGather = nullptr;
  decltype(&ncclBroadcast) Broadcast = nullptr;
};

const Rccl &rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char *env = std::getenv("KACC_RCCL_PATH");
    const char *names[] = {env && *env ? env : "librccl.so.1", "librccl.so"};
    void *h = nullptr;
    for (const char *n : names)
      if ((h = dlopen(n, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
    if (!h) {
      const char *e = dlerror();
      r.err = std::string("dlopen(librccl.so.1): ") + (e ? e : "not found");
      return;
    }
    bool all = true;
    auto sym = [&](auto &fn, const char *name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      if (!fn) {
        all = false;
        r.err += std::string(r.err.empty() ? "" : ", ") + "missing " + name;
      }
    };
    sym(r.GetVersion, "ncclGetVersion");
    sym(r.GetErrorString, "ncclGetErrorString");
    sym(r.GetUniqueId, "ncclGetUniqueId");
    sym(r.CommInitRank, "ncclCommInitRank");
    sym(r.CommInitAll, "ncclCommInitAll");
    sym(r.CommDestroy, "ncclCommDestroy");
    sym(r.GroupStart, "ncclGroupStart");
    sym(r.GroupEnd, "ncclGroupEnd");
    sym(r.AllReduce, "ncclAllReduce");
    sym(r.AllGather, "ncclAllGather");
    sym(r.Broadcast, "ncclBroadcast");
    if (!all) return;
    Dl_info info{};
    if (dladdr(reinterpret_cast<void *>(r.GetVersion), &info) && info.dli_fname) r.path = info.dli_fname;
    if (r.GetVersion(&r.version) != ncclSuccess) {
      r.err = "ncclGetVersion failed";
      return;
    }
    // NCCL_VERSION(X,Y,Z) = X*10000 + Y*100 + Z since 2.9 (X*1000 + Y*100 + Z before)
    const int major = r.version >= 10000 ? r.version / 10000 : r.version / 1000;
    if (major != NCCL_MAJOR) {
      r.err = "RCCL " + std::to_string(r.version) + " at " + r.path + ": major version " + std::to_string(major) +
              " != " + std::to_string(NCCL_MAJOR) + " of the headers this library was built with";
      return;
    }
    r.ok = true;
  });
  return r;
}
}  // namespace

namespace kacc {
namespace cluster {

constexpr int kThreads = 256;

// acc += add, element-wise (u64 modular, f64 one rounding per element).
__global__ __launch_bounds__(kThreads) void accumulate_kernel(uint64_t n_e, uint64_t *acc_e, const uint64_t *add_e,
                                                              uint64_t n_p, double *acc_p, const double *add_p) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (i < n_e) acc_e[i] += add_e[i];
  if (i < n_p) acc_p[i] = acc_p[i] + add_p[i];
}

// Pod rows of one shard into the gathered vector: row base + i = the pod in
// slot pod_slot[i] (energy and power per zone, bit copies).
template <int Z>
__global__ __launch_bounds__(kThreads) void pod_pack_kernel(uint32_t q, const uint32_t *pod_slot, uint64_t cap,
                                                            const uint64_t *pe, const double *pp, uint64_t base,
                                                            uint64_t *out_e, double *out_p, uint32_t *err) {
  const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= q) return;
  const uint64_t s = pod_slot[i] & KACC_SLOT_MASK;
  const uint64_t o = (base + i) * Z;
  if (s >= cap) {
    atomicOr(err, 1u << 3);  // the namespace / pod-list range bit of kacc_sync
#pragma unroll
    for (int z = 0; z < Z; ++z) {
      out_e[o + z] = 0;
      out_p[o + z] = 0.0;
    }
    return;
  }
#pragma unroll
  for (int z = 0; z < Z; ++z) {  // a pod slot's row: one [energy Z | power Z] record (kacc_table_row_stride)
    out_e[o + z] = pe[s * 2 * Z + z];
    out_p[o + z] = pp[s * 2 * Z + z];
  }
}

}  // namespace cluster
}  // namespace kacc

struct kacc_cluster {
  int nranks = 0;          // RCCL ranks (GPUs) in the whole cluster
  int rank0 = 0;           // rank of this process's first local GPU
  bool owns_shards = false;
  uint32_t zones = 0;
  std::vector<kacc_ctx *> shards;    // local shards, in order
  std::vector<int> dev_first;        // per local GPU: its first shard (shards of a GPU are contiguous)
  std::vector<int> dev_count;        //                and how many
  std::vector<ncclComm_t> comms;     // per local GPU
  std::vector<hipEvent_t> events;    // per shard
  std::vector<uint64_t *> d_count;   // per local GPU: [1 + nranks] u64 (pod-gather count exchange)
  std::vector<double *> d_gather;    // per local GPU: the f64 rows of every rank (ordered sums)
  uint64_t gather_n = 0;             // doubles each d_gather holds
};

namespace {

int nccl_fail(kacc_ctx *ctx, ncclResult_t r, const char *what) {
  return kacc_fail(ctx, KACC_EHIP, "%s: %s", what, rccl().GetErrorString(r));
}

#define KACC_NCCL(ctx, call)                                  \
  do {                                                        \
    ncclResult_t r_ = (call);                                 \
    if (r_ != ncclSuccess) return nccl_fail((ctx), r_, #call); \
  } while (0)

// Events and the count-exchange scratch of a new cluster.
int cluster_scratch(kacc_cluster *c) {
  kacc_ctx *c0 = c->shards[0];
  c->events.assign(c->shards.size(), nullptr);
  for (size_t s = 0; s < c->shards.size(); ++s) {
    KACC_HIP(c0, hipSetDevice(c->shards[s]->device));
    KACC_HIP(c0, hipEventCreateWithFlags(&c->events[s], hipEventDisableTiming));
  }
  c->d_count.assign(c->dev_first.size(), nullptr);
  for (size_t d = 0; d < c->dev_first.size(); ++d) {
    KACC_HIP(c0, hipSetDevice(c->shards[c->dev_first[d]]->device));
    KACC_HIP(c0, hipMalloc(&c->d_count[d], 8 * (1 + static_cast<size_t>(c->nranks))));
  }
  return KACC_OK;
}

hipStream_t shard_stream(const kacc_cluster *c, void *const *streams, size_t s) {
  return (streams && streams[s]) ? static_cast<hipStream_t>(streams[s]) : c->shards[s]->stream;
}

template <int Z>
void launch_pod_pack(kacc_ctx *x, uint32_t q, const uint32_t *slot, uint64_t base, uint64_t *oe, double *op,
                     hipStream_t st) {
  const uint32_t grid = (q + kacc::cluster::kThreads - 1) / kacc::cluster::kThreads;
  hipLaunchKernelGGL((kacc::cluster::pod_pack_kernel<Z>), dim3(grid), dim3(kacc::cluster::kThreads), 0, st, q,
                     slot, x->cfg.pod_slots, (const uint64_t *)x->tables[KACC_T_POD_ENERGY],
                     (const double *)x->tables[KACC_T_POD_POWER], base, oe, op, x->d_err);
}

void pod_pack(kacc_ctx *x, uint32_t q, const uint32_t *slot, uint64_t base, uint64_t *oe, double *op,
              hipStream_t st) {
  switch (x->cfg.zones) {
    case 1: launch_pod_pack<1>(x, q, slot, base, oe, op, st); break;
    case 2: launch_pod_pack<2>(x, q, slot, base, oe, op, st); break;
    case 3: launch_pod_pack<3>(x, q, slot, base, oe, op, st); break;
    case 4: launch_pod_pack<4>(x, q, slot, base, oe, op, st); break;
    case 5: launch_pod_pack<5>(x, q, slot, base, oe, op, st); break;
    case 6: launch_pod_pack<6>(x, q, slot, base, oe, op, st); break;
    case 7: launch_pod_pack<7>(x, q, slot, base, oe, op, st); break;
    default: launch_pod_pack<8>(x, q, slot, base, oe, op, st); break;
  }
}

void accumulate(uint64_t n_e, uint64_t *acc_e, const uint64_t *add_e, uint64_t n_p, double *acc_p,
                const double *add_p, hipStream_t st) {
  const uint64_t n = std::max(n_e, n_p);
  if (!n) return;
  const uint32_t grid = static_cast<uint32_t>((n + kacc::cluster::kThreads - 1) / kacc::cluster::kThreads);
  hipLaunchKernelGGL(kacc::cluster::accumulate_kernel, dim3(grid), dim3(kacc::cluster::kThreads), 0, st, n_e,
                     acc_e, add_e, n_p, acc_p, add_p);
}

// Shards of one GPU: the later shards' vectors are added into the first one's
// (in shard order), on the first shard's stream after the others' work.
int local_combine(kacc_cluster *c, void *const *streams, uint64_t *const *e, uint64_t n_e, double *const *p,
                  uint64_t n_p) {
  kacc_ctx *c0 = c->shards[0];
  for (size_t d = 0; d < c->dev_first.size(); ++d) {
    const int f = c->dev_first[d], cnt = c->dev_count[d];
    if (cnt < 2) continue;
    KACC_HIP(c0, hipSetDevice(c->shards[f]->device));
    hipStream_t sf = shard_stream(c, streams, f);
    for (int s = f + 1; s < f + cnt; ++s) {
      hipStream_t ss = shard_stream(c, streams, s);
      if (ss != sf) {
        KACC_HIP(c0, hipEventRecord(c->events[s], ss));
        KACC_HIP(c0, hipStreamWaitEvent(sf, c->events[s], 0));
      }
      accumulate(n_e, e[f], e[s], n_p, p[f], p[s], sf);
    }
  }
  return KACC_OK;
}

// The first shard's result of each GPU copied to the GPU's other shards.
int local_broadcast(kacc_cluster *c, void *const *streams, uint64_t *const *e, uint64_t n_e, double *const *p,
                    uint64_t n_p) {
  kacc_ctx *c0 = c->shards[0];
  for (size_t d = 0; d < c->dev_first.size(); ++d) {
    const int f = c->dev_first[d], cnt = c->dev_count[d];
    if (cnt < 2) continue;
    KACC_HIP(c0, hipSetDevice(c->shards[f]->device));
    hipStream_t sf = shard_stream(c, streams, f);
    KACC_HIP(c0, hipEventRecord(c->events[f], sf));
    for (int s = f + 1; s < f + cnt; ++s) {
      hipStream_t ss = shard_stream(c, streams, s);
      KACC_HIP(c0, hipStreamWaitEvent(ss, c->events[f], 0));
      if (n_e) KACC_HIP(c0, hipMemcpyAsync(e[s], e[f], 8 * n_e, hipMemcpyDeviceToDevice, ss));
      if (n_p) KACC_HIP(c0, hipMemcpyAsync(p[s], p[f], 8 * n_p, hipMemcpyDeviceToDevice, ss));
    }
  }
  return KACC_OK;
}

// f64 sums in RANK order, ((x_0 + x_1) + x_2) + ...: every rank's row gathered, then
// added here, so the result does not depend on RCCL's ring / tree order (round 6: the
// loopback tests' order is the one every run has)
__global__ void ordered_sum_kernel(const double *__restrict__ rows, uint64_t n, int nranks, double *out) {
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    double s = rows[i];
    for (int r = 1; r < nranks; ++r) s = s + rows[static_cast<uint64_t>(r) * n + i];
    out[i] = s;
  }
}

// In-place all-reduces (sum) of the vectors of `reqs` (u64 e [n_e], f64 p
// [n_p] of each local GPU's first shard) as ONE RCCL group: one launch of
// RCCL's kernels per step however many vectors cross the GPUs.  The u64 sums
// are exact in any order (all-reduce); the f64 rows are all-gathered and summed
// in rank order (ordered_sum_kernel) so every run gives the same bits.
struct ReduceReq {
  uint64_t *const *e;
  uint64_t n_e;
  double *const *p;
  uint64_t n_p;
};
int allreduce(kacc_cluster *c, void *const *streams, const ReduceReq *reqs, int n_reqs) {
  kacc_ctx *c0 = c->shards[0];
  uint64_t need = 0;  // every request's f64 rows of every rank
  for (int q = 0; q < n_reqs; ++q) need += reqs[q].n_p * static_cast<uint64_t>(c->nranks);
  if (need > c->gather_n) {
    c->d_gather.resize(c->dev_first.size(), nullptr);
    for (size_t d = 0; d < c->dev_first.size(); ++d) {
      KACC_HIP(c0, hipSetDevice(c->shards[c->dev_first[d]]->device));
      KACC_HIP(c0, hipDeviceSynchronize());
      (void)hipFree(c->d_gather[d]);
      c->d_gather[d] = nullptr;
      KACC_HIP(c0, hipMalloc(&c->d_gather[d], 8 * need));
    }
    c->gather_n = need;
  }
  KACC_NCCL(c0, rccl().GroupStart());
  uint64_t off = 0;
  for (int q = 0; q < n_reqs; ++q) {
    const ReduceReq &rq = reqs[q];
    for (size_t d = 0; d < c->dev_first.size(); ++d) {
      const int f = c->dev_first[d];
      hipStream_t sf = shard_stream(c, streams, f);
      if (rq.n_e) {
        const ncclResult_t r = rccl().AllReduce(rq.e[f], rq.e[f], rq.n_e, ncclUint64, ncclSum, c->comms[d], sf);
        if (r != ncclSuccess) {
          (void)rccl().GroupEnd();
          return nccl_fail(c0, r, "ncclAllReduce(u64)");
        }
      }
      if (rq.n_p) {
        const ncclResult_t r = rccl().AllGather(rq.p[f], c->d_gather[d] + off, rq.n_p, ncclFloat64, c->comms[d], sf);
        if (r != ncclSuccess) {
          (void)rccl().GroupEnd();
          return nccl_fail(c0, r, "ncclAllGather(f64)");
        }
      }
    }
    off += rq.n_p * static_cast<uint64_t>(c->nranks);
  }
  KACC_NCCL(c0, rccl().GroupEnd());
  off = 0;
  for (int q = 0; q < n_reqs; ++q) {
    const ReduceReq &rq = reqs[q];
    if (rq.n_p) {
      for (size_t d = 0; d < c->dev_first.size(); ++d) {
        const int f = c->dev_first[d];
        KACC_HIP(c0, hipSetDevice(c->shards[f]->device));
        const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>((rq.n_p + 255) / 256, 1024));
        hipLaunchKernelGGL(ordered_sum_kernel, dim3(grid), dim3(256), 0, shard_stream(c, streams, f),
                           c->d_gather[d] + off, rq.n_p, c->nranks, rq.p[f]);
        KACC_HIP(c0, hipGetLastError());
      }
    }
    off += rq.n_p * static_cast<uint64_t>(c->nranks);
  }
  return KACC_OK;
}

// RCCL loaded and usable, else the loader's message on ctx (or the create error).
int need_rccl(kacc_ctx *ctx) {
  const Rccl &r = rccl();
  return r.ok ? KACC_OK : kacc_fail(ctx, KACC_EHIP, "RCCL unavailable: %s", r.err.c_str());
}

}  // namespace

extern "C" {

int kacc_create_multi(const int *devices, int n, const kacc_config *cfgs, kacc_cluster **out, kacc_ctx **ctxs) {
  if (!devices || n <= 0 || !cfgs || !out || !ctxs) return kacc_fail(nullptr, KACC_EINVAL, "NULL argument");
  *out = nullptr;
  for (int i = 0; i < n; ++i) {
    ctxs[i] = nullptr;
    if (cfgs[i].zones != cfgs[0].zones) return kacc_fail(nullptr, KACC_EINVAL, "shards must share Z");
    for (int j = 0; j < i; ++j)  // shards of one GPU contiguous: the gather order is the shard order
      if (devices[j] == devices[i] && devices[i - 1] != devices[i])
        return kacc_fail(nullptr, KACC_EINVAL, "shards of device %d are not contiguous", devices[i]);
  }
  if (need_rccl(nullptr) != KACC_OK) return KACC_EHIP;
  auto *c = new kacc_cluster;
  c->owns_shards = true;
  c->zones = cfgs[0].zones;
  std::vector<int> devlist;
  for (int i = 0; i < n; ++i) {
    kacc_ctx *x = nullptr;
    const int rc = kacc_create(devices[i], &cfgs[i], &x);
    if (rc != KACC_OK) {
      const std::string why = kacc_last_error(nullptr);
      kacc_cluster_destroy(c);
      return kacc_fail(nullptr, rc, "shard %d: %s", i, why.c_str());
    }
    c->shards.push_back(x);
    if (i == 0 || devices[i] != devices[i - 1]) {
      c->dev_first.push_back(i);
      c->dev_count.push_back(0);
      devlist.push_back(devices[i]);
    }
    ++c->dev_count.back();
  }
  c->nranks = static_cast<int>(devlist.size());
  c->rank0 = 0;
  c->comms.assign(devlist.size(), nullptr);
  const ncclResult_t r = rccl().CommInitAll(c->comms.data(), c->nranks, devlist.data());
  if (r != ncclSuccess) {
    c->comms.clear();
    kacc_cluster_destroy(c);
    return kacc_fail(nullptr, KACC_EHIP, "ncclCommInitAll over %d GPUs: %s", static_cast<int>(devlist.size()),
                     rccl().GetErrorString(r));
  }
  if (cluster_scratch(c) != KACC_OK) {
    const std::string why = c->shards[0]->err;
    kacc_cluster_destroy(c);
    return kacc_fail(nullptr, KACC_EHIP, "cluster scratch: %s", why.c_str());
  }
  for (int i = 0; i < n; ++i) ctxs[i] = c->shards[i];
  *out = c;
  return KACC_OK;
}

int kacc_cluster_unique_id(uint8_t id[KACC_UNIQUE_ID_BYTES]) {
  if (!id) return kacc_fail(nullptr, KACC_EINVAL, "NULL argument");
  static_assert(sizeof(ncclUniqueId) == KACC_UNIQUE_ID_BYTES, "unique id size");
  if (need_rccl(nullptr) != KACC_OK) return KACC_EHIP;
  ncclUniqueId u;
  const ncclResult_t r = rccl().GetUniqueId(&u);
  if (r != ncclSuccess) return kacc_fail(nullptr, KACC_EHIP, "ncclGetUniqueId: %s", rccl().GetErrorString(r));
  std::memcpy(id, &u, sizeof(u));
  return KACC_OK;
}

int kacc_cluster_join(kacc_ctx *ctx, const uint8_t id[KACC_UNIQUE_ID_BYTES], int nranks, int rank,
                      kacc_cluster **out) {
  if (!ctx || !id || !out) return KACC_EINVAL;
  *out = nullptr;
  if (nranks <= 0 || rank < 0 || rank >= nranks)
    return kacc_fail(ctx, KACC_EINVAL, "rank %d of %d", rank, nranks);
  KACC_HIP(ctx, hipSetDevice(ctx->device));
  if (need_rccl(ctx) != KACC_OK) return KACC_EHIP;
  auto *c = new kacc_cluster;
  c->owns_shards = false;
  c->zones = ctx->cfg.zones;
  c->shards.push_back(ctx);
  c->dev_first.push_back(0);
  c->dev_count.push_back(1);
  c->nranks = nranks;
  c->rank0 = rank;
  c->comms.assign(1, nullptr);
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  const ncclResult_t r = rccl().CommInitRank(&c->comms[0], nranks, u, rank);
  if (r != ncclSuccess) {
    c->comms.clear();
    kacc_cluster_destroy(c);
    return kacc_fail(ctx, KACC_EHIP, "ncclCommInitRank(%d of %d): %s", rank, nranks, rccl().GetErrorString(r));
  }
  const int rc = cluster_scratch(c);
  if (rc != KACC_OK) {
    kacc_cluster_destroy(c);
    return rc;
  }
  *out = c;
  return KACC_OK;
}

void kacc_cluster_destroy(kacc_cluster *c) {
  if (!c) return;
  for (size_t d = 0; d < c->comms.size(); ++d) {
    if (!c->comms[d]) continue;
    (void)hipSetDevice(c->shards[c->dev_first[d]]->device);
    (void)hipDeviceSynchronize();
    if (rccl().CommDestroy) (void)rccl().CommDestroy(c->comms[d]);
  }
  for (size_t d = 0; d < c->d_count.size(); ++d)
    if (c->d_count[d]) {
      (void)hipSetDevice(c->shards[c->dev_first[d]]->device);
      (void)hipFree(c->d_count[d]);
    }
  for (size_t d = 0; d < c->d_gather.size(); ++d)
    if (c->d_gather[d]) {
      (void)hipSetDevice(c->shards[c->dev_first[d]]->device);
      (void)hipFree(c->d_gather[d]);
    }
  for (size_t s = 0; s < c->events.size(); ++s)
    if (c->events[s]) {
      (void)hipSetDevice(c->shards[s]->device);
      (void)hipEventDestroy(c->events[s]);
    }
  if (c->owns_shards)
    for (kacc_ctx *x : c->shards) kacc_destroy(x);
  delete c;
}

int kacc_cluster_rccl(int *version, char *path, size_t len) {
  const Rccl &r = rccl();
  if (version) *version = r.version;
  if (path && len) {
    const size_t n = std::min(len - 1, r.path.size());
    std::memcpy(path, r.path.data(), n);
    path[n] = '\0';
  }
  return r.ok ? KACC_OK : kacc_fail(nullptr, KACC_EHIP, "RCCL unavailable: %s", r.err.c_str());
}

int kacc_cluster_info(const kacc_cluster *c, int *nranks, int *rank, int *n_shards) {
  if (!c) return KACC_EINVAL;
  if (nranks) *nranks = c->nranks;
  if (rank) *rank = c->rank0;
  if (n_shards) *n_shards = static_cast<int>(c->shards.size());
  return KACC_OK;
}

}  // extern "C"

namespace {
// Step 1 of kacc_allreduce_namespaces / kacc_cluster_partials: the checked
// arguments, then every shard's partial vectors (namespace sums and node totals
// in one launch per shard) on its stream.
int shard_partials(kacc_cluster *c, uint32_t n_ns, const uint32_t *const *ns_pod_off,
                   const uint32_t *const *ns_pod_slot, uint64_t *const *out_energy, double *const *out_power,
                   uint64_t *const *out_node_energy, double *const *out_node_power, void *const *streams) {
  kacc_ctx *c0 = c->shards[0];
  const size_t ns = c->shards.size();
  const bool nodes = out_node_energy && out_node_power;
  if ((out_node_energy != nullptr) != (out_node_power != nullptr))
    return kacc_fail(c0, KACC_EINVAL, "node totals need both output arrays");
  if (n_ns && (!ns_pod_off || !ns_pod_slot || !out_energy || !out_power))
    return kacc_fail(c0, KACC_EINVAL, "NULL argument");
  for (size_t s = 0; s < ns; ++s) {
    if (n_ns && (!ns_pod_off[s] || !ns_pod_slot[s] || !out_energy[s] || !out_power[s]))
      return kacc_fail(c0, KACC_EINVAL, "shard %zu: NULL namespace array", s);
    if (nodes && (!out_node_energy[s] || !out_node_power[s]))
      return kacc_fail(c0, KACC_EINVAL, "shard %zu: NULL node-total array", s);
  }
  for (size_t s = 0; s < ns; ++s) {
    kacc_ctx *x = c->shards[s];
    hipStream_t st = shard_stream(c, streams, s);
    const int rc = kacc_internal_cluster_partials(
        x, n_ns, n_ns ? ns_pod_off[s] : nullptr, n_ns ? ns_pod_slot[s] : nullptr, n_ns ? out_energy[s] : nullptr,
        n_ns ? out_power[s] : nullptr, nodes ? out_node_energy[s] : nullptr, nodes ? out_node_power[s] : nullptr, st);
    if (rc != KACC_OK) return kacc_fail(c0, rc, "shard %zu: %s", s, std::string(x->err).c_str());
  }
  return KACC_OK;
}

// The comm streams wait for the work queued on the compute streams so far (one
// event packet on each compute stream).
int handoff(kacc_cluster *c, void *const *streams, void *const *comm_streams) {
  kacc_ctx *c0 = c->shards[0];
  if (!comm_streams) return KACC_OK;
  for (size_t s = 0; s < c->shards.size(); ++s) {
    hipStream_t a = shard_stream(c, streams, s), b = shard_stream(c, comm_streams, s);
    if (a == b) continue;
    KACC_HIP(c0, hipSetDevice(c->shards[s]->device));
    KACC_HIP(c0, hipEventRecord(c->events[s], a));
    KACC_HIP(c0, hipStreamWaitEvent(b, c->events[s], 0));
  }
  return KACC_OK;
}
}  // namespace

extern "C" {

int kacc_cluster_partials(kacc_cluster *c, uint32_t n_ns, const uint32_t *const *ns_pod_off,
                          const uint32_t *const *ns_pod_slot, uint64_t *const *out_energy, double *const *out_power,
                          uint64_t *const *out_node_energy, double *const *out_node_power, void *const *streams) {
  if (!c) return KACC_EINVAL;
  return shard_partials(c, n_ns, ns_pod_off, ns_pod_slot, out_energy, out_power, out_node_energy, out_node_power,
                        streams);
}

int kacc_allreduce_sums(kacc_cluster *c, uint64_t *const *energy, uint64_t n_e, double *const *power, uint64_t n_p,
                        void *const *streams, void *const *comm_streams) {
  if (!c) return KACC_EINVAL;
  kacc_ctx *c0 = c->shards[0];
  const size_t ns = c->shards.size();
  if ((n_e && !energy) || (n_p && !power)) return kacc_fail(c0, KACC_EINVAL, "NULL argument");
  for (size_t s = 0; s < ns; ++s)
    if ((n_e && !energy[s]) || (n_p && !power[s])) return kacc_fail(c0, KACC_EINVAL, "shard %zu: NULL vector", s);
  if ((c->nranks == 1 && ns == 1) || (!n_e && !n_p)) return KACC_OK;
  int rc = local_combine(c, streams, energy, n_e, power, n_p);
  if (rc != KACC_OK) return rc;
  if ((rc = handoff(c, streams, comm_streams)) != KACC_OK) return rc;
  void *const *cs = comm_streams ? comm_streams : streams;
  const ReduceReq req{energy, n_e, power, n_p};
  if ((rc = allreduce(c, cs, &req, 1)) != KACC_OK) return rc;
  return local_broadcast(c, cs, energy, n_e, power, n_p);
}

int kacc_allreduce_namespaces(kacc_cluster *c, uint32_t n_ns, const uint32_t *const *ns_pod_off,
                              const uint32_t *const *ns_pod_slot, uint64_t *const *out_energy,
                              double *const *out_power, uint64_t *const *out_node_energy,
                              double *const *out_node_power, void *const *streams,
                              void *const *comm_streams) {
  if (!c) return KACC_EINVAL;
  const size_t ns = c->shards.size();
  const uint64_t Z = c->zones;
  const bool nodes = out_node_energy && out_node_power;
  // 1. partial vectors of every shard, on its stream: namespace sums and node
  //    totals in one launch per shard
  int rc = shard_partials(c, n_ns, ns_pod_off, ns_pod_slot, out_energy, out_power, out_node_energy, out_node_power,
                          streams);
  if (rc != KACC_OK) return rc;
  // one rank, one shard: the partial sums are the cluster totals (no combine, no
  // collective, and no cross-stream packets between the caller's intervals)
  if (c->nranks == 1 && ns == 1) return KACC_OK;
  // 2. shards of one GPU (on the compute streams)
  if (n_ns && (rc = local_combine(c, streams, out_energy, n_ns * Z, out_power, n_ns * Z)) != KACC_OK) return rc;
  if (nodes && (rc = local_combine(c, streams, out_node_energy, 2 * Z, out_node_power, 3 * Z)) != KACC_OK) return rc;
  // the collective may run on other streams: they wait for the partial sums,
  // and the caller's next interval on the compute stream overlaps it
  void *const *cs = comm_streams ? comm_streams : streams;
  if ((rc = handoff(c, streams, comm_streams)) != KACC_OK) return rc;
  // 3. across GPUs (RCCL: every vector in one group), 4. back to every shard
  ReduceReq reqs[2];
  int n_reqs = 0;
  if (n_ns) reqs[n_reqs++] = ReduceReq{out_energy, n_ns * Z, out_power, n_ns * Z};
  if (nodes) reqs[n_reqs++] = ReduceReq{out_node_energy, 2 * Z, out_node_power, 3 * Z};
  if (n_reqs && (rc = allreduce(c, cs, reqs, n_reqs)) != KACC_OK) return rc;
  if (n_ns && (rc = local_broadcast(c, cs, out_energy, n_ns * Z, out_power, n_ns * Z)) != KACC_OK) return rc;
  if (nodes && (rc = local_broadcast(c, cs, out_node_energy, 2 * Z, out_node_power, 3 * Z)) != KACC_OK)
    return rc;
  return KACC_OK;
}

int kacc_allreduce_exports(kacc_cluster *c, uint32_t n_ns, const uint32_t *const *ns_pod_off,
                           const uint32_t *const *ns_pod_row, const uint32_t *n_pods,
                           const uint64_t *const *pod_export, const uint32_t *n_nodes,
                           const uint64_t *const *node_export, uint64_t *const *out_energy,
                           double *const *out_power, uint64_t *const *out_node_energy,
                           double *const *out_node_power, void *const *streams, void *const *comm_streams) {
  if (!c) return KACC_EINVAL;
  kacc_ctx *c0 = c->shards[0];
  const size_t ns = c->shards.size();
  const uint64_t Z = c->zones;
  const bool nodes = out_node_energy && out_node_power;
  if ((out_node_energy != nullptr) != (out_node_power != nullptr))
    return kacc_fail(c0, KACC_EINVAL, "node totals need both output arrays");
  if (n_ns && (!ns_pod_off || !ns_pod_row || !n_pods || !pod_export || !out_energy || !out_power))
    return kacc_fail(c0, KACC_EINVAL, "NULL argument");
  if (nodes && (!n_nodes || !node_export)) return kacc_fail(c0, KACC_EINVAL, "node totals need node exports");
  for (size_t s = 0; s < ns; ++s) {
    if (n_ns && (!ns_pod_off[s] || !ns_pod_row[s] || !out_energy[s] || !out_power[s] || (n_pods[s] && !pod_export[s])))
      return kacc_fail(c0, KACC_EINVAL, "shard %zu: NULL namespace / pod export array", s);
    if (nodes && (!out_node_energy[s] || !out_node_power[s] || (n_nodes[s] && !node_export[s])))
      return kacc_fail(c0, KACC_EINVAL, "shard %zu: NULL node-total / node export array", s);
  }
  // everything on the comm streams, after the work queued on the compute streams
  void *const *cs = comm_streams ? comm_streams : streams;
  for (size_t s = 0; s < ns; ++s) {
    kacc_ctx *x = c->shards[s];
    hipStream_t a = shard_stream(c, streams, s), b = shard_stream(c, cs, s);
    KACC_HIP(c0, hipSetDevice(x->device));
    if (a != b) {
      KACC_HIP(c0, hipEventRecord(c->events[s], a));
      KACC_HIP(c0, hipStreamWaitEvent(b, c->events[s], 0));
    }
    // 1. partial vectors of every shard from its exports
    const int rc = kacc_internal_export_partials(
        x, n_ns, n_ns ? ns_pod_off[s] : nullptr, n_ns ? ns_pod_row[s] : nullptr, n_ns ? pod_export[s] : nullptr,
        n_ns ? n_pods[s] : 0, nodes ? node_export[s] : nullptr, nodes ? n_nodes[s] : 0, nodes ? 1 : 0,
        n_ns ? out_energy[s] : nullptr,
        n_ns ? out_power[s] : nullptr, nodes ? out_node_energy[s] : nullptr, nodes ? out_node_power[s] : nullptr, b);
    if (rc != KACC_OK) return kacc_fail(c0, rc, "shard %zu: %s", s, std::string(x->err).c_str());
  }
  if (c->nranks == 1 && ns == 1) return KACC_OK;
  // 2. shards of one GPU, 3. across GPUs, 4. back to every shard — all on the comm streams
  int rc = KACC_OK;
  if (n_ns && (rc = local_combine(c, cs, out_energy, n_ns * Z, out_power, n_ns * Z)) != KACC_OK) return rc;
  if (nodes && (rc = local_combine(c, cs, out_node_energy, 2 * Z, out_node_power, 3 * Z)) != KACC_OK) return rc;
  ReduceReq reqs[2];
  int n_reqs = 0;
  if (n_ns) reqs[n_reqs++] = ReduceReq{out_energy, n_ns * Z, out_power, n_ns * Z};
  if (nodes) reqs[n_reqs++] = ReduceReq{out_node_energy, 2 * Z, out_node_power, 3 * Z};
  if (n_reqs && (rc = allreduce(c, cs, reqs, n_reqs)) != KACC_OK) return rc;
  if (n_ns && (rc = local_broadcast(c, cs, out_energy, n_ns * Z, out_power, n_ns * Z)) != KACC_OK) return rc;
  if (nodes && (rc = local_broadcast(c, cs, out_node_energy, 2 * Z, out_node_power, 3 * Z)) != KACC_OK) return rc;
  return KACC_OK;
}

int kacc_gather_pods(kacc_cluster *c, const uint32_t *n_pods, const uint32_t *const *pod_slot, uint64_t out_cap,
                     uint64_t *const *out_energy, double *const *out_power, uint64_t *total, uint64_t *first,
                     void *const *streams) {
  if (!c) return KACC_EINVAL;
  kacc_ctx *c0 = c->shards[0];
  if (!n_pods || !pod_slot || !out_energy || !out_power || !total) return kacc_fail(c0, KACC_EINVAL, "NULL argument");
  const size_t nd = c->dev_first.size();
  const uint64_t Z = c->zones;
  // 1. pods per local GPU, exchanged: every rank learns every rank's count
  std::vector<uint64_t> local(nd, 0);
  for (size_t d = 0; d < nd; ++d)
    for (int s = c->dev_first[d]; s < c->dev_first[d] + c->dev_count[d]; ++s) local[d] += n_pods[s];
  for (size_t d = 0; d < nd; ++d) {
    KACC_HIP(c0, hipSetDevice(c->shards[c->dev_first[d]]->device));
    KACC_HIP(c0, hipMemcpyAsync(c->d_count[d], &local[d], 8, hipMemcpyHostToDevice,
                                shard_stream(c, streams, c->dev_first[d])));
  }
  KACC_NCCL(c0, rccl().GroupStart());
  for (size_t d = 0; d < nd; ++d) {
    const ncclResult_t r = rccl().AllGather(c->d_count[d], c->d_count[d] + 1, 1, ncclUint64, c->comms[d],
                                         shard_stream(c, streams, c->dev_first[d]));
    if (r != ncclSuccess) {
      (void)rccl().GroupEnd();
      return nccl_fail(c0, r, "ncclAllGather(counts)");
    }
  }
  KACC_NCCL(c0, rccl().GroupEnd());
  std::vector<uint64_t> counts(c->nranks, 0);
  {
    const int f = c->dev_first[0];
    KACC_HIP(c0, hipSetDevice(c->shards[f]->device));
    hipStream_t sf = shard_stream(c, streams, f);
    KACC_HIP(c0, hipStreamSynchronize(sf));
    KACC_HIP(c0, hipMemcpy(counts.data(), c->d_count[0] + 1, 8 * counts.size(), hipMemcpyDeviceToHost));
  }
  std::vector<uint64_t> off(c->nranks + 1, 0);
  for (int r = 0; r < c->nranks; ++r) off[r + 1] = off[r] + counts[r];
  *total = off[c->nranks];
  if (off[c->nranks] > out_cap)
    return kacc_fail(c0, KACC_ERANGE, "gathered pods %llu exceed out_cap %llu", (unsigned long long)off[c->nranks],
                     (unsigned long long)out_cap);
  // 2. every local shard packs its pods at its global position
  for (size_t d = 0; d < nd; ++d) {
    const int f = c->dev_first[d];
    uint64_t base = off[c->rank0 + static_cast<int>(d)];
    hipStream_t sf = shard_stream(c, streams, f);
    KACC_HIP(c0, hipSetDevice(c->shards[f]->device));
    for (int s = f; s < f + c->dev_count[d]; ++s) {
      if (first) first[s] = base;
      if (n_pods[s]) {
        if (!pod_slot[s]) return kacc_fail(c0, KACC_EINVAL, "shard %d: NULL pod_slot", s);
        hipStream_t ss = shard_stream(c, streams, s);
        (void)hipGetLastError();
        pod_pack(c->shards[s], n_pods[s], pod_slot[s], base, out_energy[f], out_power[f], ss);
        KACC_HIP(c0, hipGetLastError());
        if (ss != sf) {
          KACC_HIP(c0, hipEventRecord(c->events[s], ss));
          KACC_HIP(c0, hipStreamWaitEvent(sf, c->events[s], 0));
        }
      }
      base += n_pods[s];
    }
  }
  // 3. all-gather-v: one in-place broadcast per rank, its exact block
  KACC_NCCL(c0, rccl().GroupStart());
  for (int r = 0; r < c->nranks; ++r) {
    if (!counts[r]) continue;
    for (size_t d = 0; d < nd; ++d) {
      const int f = c->dev_first[d];
      hipStream_t sf = shard_stream(c, streams, f);
      uint64_t *e = out_energy[f] + off[r] * Z;
      double *p = out_power[f] + off[r] * Z;
      ncclResult_t rr = rccl().Broadcast(e, e, counts[r] * Z, ncclUint64, r, c->comms[d], sf);
      if (rr == ncclSuccess) rr = rccl().Broadcast(p, p, counts[r] * Z, ncclFloat64, r, c->comms[d], sf);
      if (rr != ncclSuccess) {
        (void)rccl().GroupEnd();
        return nccl_fail(c0, rr, "ncclBroadcast(pods)");
      }
    }
  }
  KACC_NCCL(c0, rccl().GroupEnd());
  return local_broadcast(c, streams, out_energy, off[c->nranks] * Z, out_power, off[c->nranks] * Z);
}

}  // extern "C"
