// TEST INFRASTRUCTURE ONLY — a loopback stand-in for the eleven RCCL entry
// points libkepler_accel binds (kacc_cluster.hip), for N ranks that are N
// processes on ONE GPU.  RCCL itself refuses that ("Duplicate GPU detected",
// its init checks every rank's bus id), and the GPU box has one GPU, so the
// nranks > 1 logic of the library — ncclCommInitRank with real peers, the
// cross-rank all-reduce of kacc_allreduce_sums / kacc_allreduce_namespaces, the
// count all-gather and the per-rank broadcasts of kacc_gather_pods — runs
// against this file instead, loaded through KACC_RCCL_PATH.
//
// Semantics are NCCL's for the calls the library makes (sum of u64 / i64 / f64,
// in-place or not; all-gather by rank; broadcast from a root), executed eagerly
// on the host: a collective synchronises its stream, copies the rank's buffer
// into a POSIX shared-memory segment named by the unique id, meets the other
// ranks at a barrier, combines in RANK order (for two ranks a + b, the order
// RCCL's ring gives too; f64 addition of two terms commutes), and copies the
// result back on the stream.  Calls inside ncclGroupStart/End run in issue order
// (every rank issues the same sequence).  Buffers larger than the segment's
// per-rank slot are moved in pieces.  Every barrier gives up after
// KACC_LOOPBACK_TIMEOUT_S (default 60) seconds with ncclSystemError, so a lost
// peer fails the test instead of hanging it.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

constexpr size_t kSlotBytes = 16u << 20;  // per-rank staging slot
constexpr int kMaxRanks = 16;
constexpr char kTag[] = "kacc-loopback:";

struct Header {
  std::atomic<uint32_t> arrived;
  std::atomic<uint32_t> generation;
  std::atomic<uint32_t> attached;
  std::atomic<uint32_t> detached;
};
static_assert(std::atomic<uint32_t>::is_always_lock_free, "cross-process atomics");

}  // namespace

struct ncclComm {
  int nranks = 0, rank = 0;
  std::string name;
  void *base = nullptr;
  size_t bytes = 0;
  Header *hdr() const { return static_cast<Header *>(base); }
  char *slot(int r) const { return static_cast<char *>(base) + 4096 + static_cast<size_t>(r) * kSlotBytes; }
};

namespace {

double timeout_s() {
  const char *e = std::getenv("KACC_LOOPBACK_TIMEOUT_S");
  return e && *e ? std::atof(e) : 60.0;
}

double now_s() {
  timespec t{};
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

// Sense-counting barrier over the segment: the last rank to arrive bumps the
// generation; the others wait for it (bounded).
ncclResult_t barrier(ncclComm *c) {
  Header *h = c->hdr();
  const uint32_t gen = h->generation.load(std::memory_order_acquire);
  if (h->arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == static_cast<uint32_t>(c->nranks)) {
    h->arrived.store(0, std::memory_order_relaxed);
    h->generation.fetch_add(1, std::memory_order_acq_rel);
    return ncclSuccess;
  }
  const double deadline = now_s() + timeout_s();
  while (h->generation.load(std::memory_order_acquire) == gen) {
    if (now_s() > deadline) {
      std::fprintf(stderr, "loopback_rccl: rank %d of %d: barrier timed out\n", c->rank, c->nranks);
      return ncclSystemError;
    }
    usleep(50);
  }
  return ncclSuccess;
}

size_t type_bytes(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
  }
}

#define LB_HIP(call)                                                                   \
  do {                                                                                 \
    if ((call) != hipSuccess) {                                                        \
      std::fprintf(stderr, "loopback_rccl: %s failed\n", #call);                       \
      return ncclUnhandledCudaError;                                                   \
    }                                                                                  \
  } while (0)

template <typename T>
void add_into(T *acc, const T *x, size_t n) {
  for (size_t i = 0; i < n; ++i) acc[i] = acc[i] + x[i];
}

}  // namespace

extern "C" {

ncclResult_t ncclGetVersion(int *version) {
  if (!version) return ncclInvalidArgument;
  *version = NCCL_VERSION_CODE;
  return ncclSuccess;
}

const char *ncclGetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess: return "no error (loopback)";
    case ncclUnhandledCudaError: return "HIP call failed (loopback)";
    case ncclSystemError: return "system error: shared memory or a lost peer (loopback)";
    case ncclInvalidArgument: return "invalid argument (loopback)";
    case ncclInvalidUsage: return "invalid usage (loopback)";
    default: return "error (loopback)";
  }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId *id) {
  if (!id) return ncclInvalidArgument;
  std::memset(id, 0, sizeof(*id));
  timespec t{};
  clock_gettime(CLOCK_REALTIME, &t);
  std::snprintf(id->internal, sizeof(id->internal), "%s/kacc_lb_%d_%ld_%ld", kTag, static_cast<int>(getpid()),
                static_cast<long>(t.tv_sec), static_cast<long>(t.tv_nsec));
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t *out, int nranks, ncclUniqueId id, int rank) {
  if (!out || nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  if (std::strncmp(id.internal, kTag, sizeof(kTag) - 1) != 0) return ncclInvalidUsage;
  auto *c = new ncclComm;
  c->nranks = nranks;
  c->rank = rank;
  c->name.assign(id.internal + sizeof(kTag) - 1, strnlen(id.internal + sizeof(kTag) - 1, 100));
  c->bytes = 4096 + static_cast<size_t>(nranks) * kSlotBytes;
  const int fd = shm_open(c->name.c_str(), O_CREAT | O_RDWR, 0600);
  if (fd < 0 || ftruncate(fd, static_cast<off_t>(c->bytes)) != 0) {
    if (fd >= 0) close(fd);
    delete c;
    return ncclSystemError;
  }
  c->base = mmap(nullptr, c->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (c->base == MAP_FAILED) {
    delete c;
    return ncclSystemError;
  }
  c->hdr()->attached.fetch_add(1);
  const ncclResult_t r = barrier(c);  // every rank attached before any collective
  if (r != ncclSuccess) {
    munmap(c->base, c->bytes);
    shm_unlink(c->name.c_str());
    delete c;
    return r;
  }
  *out = c;
  return ncclSuccess;
}

ncclResult_t ncclCommInitAll(ncclComm_t *comms, int ndev, const int *) {
  // one process per rank only: several devices in one process would need
  // asynchronous collectives, which this eager loopback does not have
  if (!comms || ndev != 1) return ncclInvalidUsage;
  ncclUniqueId id;
  ncclGetUniqueId(&id);
  return ncclCommInitRank(comms, 1, id, 0);
}

ncclResult_t ncclCommDestroy(ncclComm_t c) {
  if (!c) return ncclInvalidArgument;
  (void)barrier(c);
  const bool last = c->hdr()->detached.fetch_add(1) + 1 == static_cast<uint32_t>(c->nranks);
  munmap(c->base, c->bytes);
  if (last) shm_unlink(c->name.c_str());
  delete c;
  return ncclSuccess;
}

ncclResult_t ncclGroupStart() { return ncclSuccess; }
ncclResult_t ncclGroupEnd() { return ncclSuccess; }

ncclResult_t ncclAllReduce(const void *send, void *recv, size_t count, ncclDataType_t dt, ncclRedOp_t op,
                           ncclComm_t c, hipStream_t stream) {
  const size_t tb = type_bytes(dt);
  if (!c || !tb || op != ncclSum) return ncclInvalidArgument;
  LB_HIP(hipStreamSynchronize(stream));
  const size_t per = kSlotBytes / tb;
  std::vector<char> acc(std::min(count, per) * tb);
  for (size_t first = 0; first < count; first += per) {
    const size_t n = std::min(per, count - first);
    LB_HIP(hipMemcpyAsync(c->slot(c->rank), static_cast<const char *>(send) + first * tb, n * tb,
                          hipMemcpyDeviceToHost, stream));
    LB_HIP(hipStreamSynchronize(stream));
    ncclResult_t r = barrier(c);
    if (r != ncclSuccess) return r;
    std::memcpy(acc.data(), c->slot(0), n * tb);  // rank order: ((r0 + r1) + r2) ...
    for (int k = 1; k < c->nranks; ++k) {
      if (dt == ncclFloat64)
        add_into(reinterpret_cast<double *>(acc.data()), reinterpret_cast<const double *>(c->slot(k)), n);
      else if (dt == ncclFloat32)
        add_into(reinterpret_cast<float *>(acc.data()), reinterpret_cast<const float *>(c->slot(k)), n);
      else if (tb == 8)
        add_into(reinterpret_cast<uint64_t *>(acc.data()), reinterpret_cast<const uint64_t *>(c->slot(k)), n);
      else if (tb == 4)
        add_into(reinterpret_cast<uint32_t *>(acc.data()), reinterpret_cast<const uint32_t *>(c->slot(k)), n);
      else
        add_into(reinterpret_cast<uint8_t *>(acc.data()), reinterpret_cast<const uint8_t *>(c->slot(k)), n);
    }
    if ((r = barrier(c)) != ncclSuccess) return r;  // every rank has read every slot
    LB_HIP(hipMemcpyAsync(static_cast<char *>(recv) + first * tb, acc.data(), n * tb, hipMemcpyHostToDevice, stream));
    LB_HIP(hipStreamSynchronize(stream));
  }
  return ncclSuccess;
}

ncclResult_t ncclAllGather(const void *send, void *recv, size_t count, ncclDataType_t dt, ncclComm_t c,
                           hipStream_t stream) {
  const size_t tb = type_bytes(dt);
  if (!c || !tb) return ncclInvalidArgument;
  LB_HIP(hipStreamSynchronize(stream));
  const size_t per = kSlotBytes / tb;
  for (size_t first = 0; first < count; first += per) {
    const size_t n = std::min(per, count - first);
    LB_HIP(hipMemcpyAsync(c->slot(c->rank), static_cast<const char *>(send) + first * tb, n * tb,
                          hipMemcpyDeviceToHost, stream));
    LB_HIP(hipStreamSynchronize(stream));
    ncclResult_t r = barrier(c);
    if (r != ncclSuccess) return r;
    std::vector<char> all(static_cast<size_t>(c->nranks) * n * tb);
    for (int k = 0; k < c->nranks; ++k) std::memcpy(all.data() + k * n * tb, c->slot(k), n * tb);
    if ((r = barrier(c)) != ncclSuccess) return r;
    for (int k = 0; k < c->nranks; ++k)
      LB_HIP(hipMemcpyAsync(static_cast<char *>(recv) + (k * count + first) * tb, all.data() + k * n * tb, n * tb,
                            hipMemcpyHostToDevice, stream));
    LB_HIP(hipStreamSynchronize(stream));
  }
  return ncclSuccess;
}

ncclResult_t ncclBroadcast(const void *send, void *recv, size_t count, ncclDataType_t dt, int root, ncclComm_t c,
                           hipStream_t stream) {
  const size_t tb = type_bytes(dt);
  if (!c || !tb || root < 0 || root >= c->nranks) return ncclInvalidArgument;
  LB_HIP(hipStreamSynchronize(stream));
  const size_t per = kSlotBytes / tb;
  std::vector<char> buf(std::min(count, per) * tb);
  for (size_t first = 0; first < count; first += per) {
    const size_t n = std::min(per, count - first);
    if (c->rank == root) {
      LB_HIP(hipMemcpyAsync(c->slot(root), static_cast<const char *>(send) + first * tb, n * tb,
                            hipMemcpyDeviceToHost, stream));
      LB_HIP(hipStreamSynchronize(stream));
    }
    ncclResult_t r = barrier(c);
    if (r != ncclSuccess) return r;
    std::memcpy(buf.data(), c->slot(root), n * tb);
    if ((r = barrier(c)) != ncclSuccess) return r;
    LB_HIP(hipMemcpyAsync(static_cast<char *>(recv) + first * tb, buf.data(), n * tb, hipMemcpyHostToDevice, stream));
    LB_HIP(hipStreamSynchronize(stream));
  }
  return ncclSuccess;
}

}  // extern "C"
