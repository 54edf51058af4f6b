// Internal host-side definitions shared by the engine's translation units
// (kacc_engine.hip: interval path, kacc_join.hip: slot join + terminated
// tracker).  Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <string>
#include <utility>
#include <vector>

#include "../../include/kepler_accel.h"

namespace kacc {
struct ChunkItem;
}

struct kacc_ctx {
  int device = 0;
  kacc_config cfg{};
  hipStream_t stream = nullptr;
  hipStream_t copy_stream = nullptr;  // pinned-batch H2D (overlaps the previous interval's kernel)
  void *tables[KACC_T_COUNT] = {};
  uint64_t counts[KACC_T_COUNT] = {};
  uint32_t *d_err = nullptr;
  uint32_t *d_ctr = nullptr;  // [0,1] chunk list length / head, [2] deferred pods
  kacc::ChunkItem *d_items = nullptr;
  // cluster node totals past kColSplitFrom nodes: [5 * KACC_MAX_ZONES][col_split_cap] column
  // partials and [5 * KACC_MAX_ZONES] arrival counts (zero between launches)
  uint64_t *d_colpart = nullptr;
  uint32_t *d_colarrived = nullptr;
  uint32_t item_cap = 0;
  uint2 *d_defer = nullptr;
  uint32_t defer_cap = 0;
  kacc_interval *d_batches = nullptr;  // fused kacc_run_intervals: descriptors on the device
  kacc_interval *h_batches = nullptr;  //   and their pinned staging copy
  uint32_t batch_cap = 0;
  hipEvent_t batch_copied = nullptr;
  uint32_t live_nodes = 0;  // n_nodes of the last interval run: the nodes the cluster totals sum
  hipEvent_t time_start = nullptr, time_stop = nullptr;  // kacc_time_next_launch (one call)
  std::string err;
};

struct kacc_batch {
  kacc_shape cap{};                 // capacities of every interval + the interval count
  std::vector<kacc_interval> host;  // [intervals] the caller's views (pinned host pointers)
  std::vector<kacc_interval> dev;   // [intervals] the same arrays on the device
  std::vector<kacc_interval> orig;  // [intervals] the views as allocated (pointers are fixed)
  std::vector<void *> allocs;       // pinned host buffers
  std::vector<void *> dev_allocs;   // device buffers
  hipEvent_t copied = nullptr;  // H2D of the last submit done (copy stream)
  hipEvent_t done = nullptr;    // the last submit's kernels + error word copy done
  uint32_t *h_err = nullptr;    // pinned: device error word after the last submit
  bool submitted = false;
};

// Elements [first, first + count) of table t as a dense array (device, async on
// `stream`): derived power tables are derived, the pod tables (stored as [Sq][2Z]
// energy | power records) gathered, the others copied; and the inverse scatter
// into a pod table (kacc_engine.hip).
extern "C" int kacc_internal_dense_range(kacc_ctx *ctx, int t, uint64_t first, uint64_t count, void *out,
                                         void *stream);
extern "C" int kacc_internal_pod_scatter(kacc_ctx *ctx, int t, uint64_t first, uint64_t count, const void *in,
                                         void *stream);

// kacc_time_next_launch: while a LaunchTiming scope is alive on this thread,
// KACC_LAUNCH attaches the scope's start event to the first kernel it launches
// and its stop event to every one (the last recording wins), through the
// dispatch packets (hipExtLaunchKernelGGL); otherwise a plain launch.
namespace kacc {
struct LaunchTiming {
  hipEvent_t start = nullptr, stop = nullptr;
};
inline LaunchTiming *&launch_timing() {
  static thread_local LaunchTiming *t = nullptr;
  return t;
}
// Takes the context's pending events for the duration of one entry point.
class TimingScope {
 public:
  explicit TimingScope(kacc_ctx *ctx) {
    if (ctx && (ctx->time_start || ctx->time_stop)) {
      t_.start = ctx->time_start;
      t_.stop = ctx->time_stop;
      ctx->time_start = ctx->time_stop = nullptr;
      launch_timing() = &t_;
      on_ = true;
    }
  }
  ~TimingScope() {
    if (on_) launch_timing() = nullptr;
  }
  TimingScope(const TimingScope &) = delete;
  TimingScope &operator=(const TimingScope &) = delete;

 private:
  LaunchTiming t_;
  bool on_ = false;
};
}  // namespace kacc

#define KACC_LAUNCH(kernel, grid, block, shmem, stream, ...)                                             \
  do {                                                                                                    \
    kacc::LaunchTiming *kacc_lt_ = kacc::launch_timing();                                                 \
    if (kacc_lt_) {                                                                                       \
      hipExtLaunchKernelGGL(kernel, grid, block, shmem, stream, kacc_lt_->start, kacc_lt_->stop, 0,       \
                            __VA_ARGS__);                                                                 \
      kacc_lt_->start = nullptr;                                                                          \
    } else {                                                                                              \
      hipLaunchKernelGGL(kernel, grid, block, shmem, stream, __VA_ARGS__);                                \
    }                                                                                                     \
  } while (0)

// Slot map of one workload kind (kacc_join.hip).
struct kacc_slotmap {
  kacc_ctx *ctx = nullptr;  // for errors and the default stream while the context lives
  int device = 0;           // destroy must not touch ctx (it may be gone already)
  kacc_kind kind = KACC_KIND_PROC;
  uint32_t n_nodes = 0;
  uint32_t total_slots = 0;  // slot_off[n_nodes]
  uint64_t buckets = 0;
  uint32_t *d_slot_off = nullptr;
  uint64_t *d_hoff = nullptr;
  bool has_big = false;         // some node's table exceeds the LDS size
  bool uniform = false;         // every node's table has kLdsBuckets buckets: hoff[n] = n kLdsBuckets
  uint32_t policy = 0;          // KACC_JOIN_* bits (kacc_slotmap_set_policy)
  int fmt = 0;                  // PID small-table format, fixed at reset (the join variant
                                // launched then): 0 8-B buckets, 1 6-B buckets, 2 slot-keyed
                                // (kJSK); a join in another format fails
  uint64_t *d_ent = nullptr;    // packed entries (PIDs) or keys (64-bit IDs)
  uint32_t *d_slots = nullptr;  // 64-bit IDs only
};

// Namespace partial sums (kacc_namespace_totals' order) and, when node_energy
// is non-NULL, the context's cluster node totals (node_energy [2Z], node_power
// [3Z]), in ONE launch on `stream` (kacc_engine.hip; used by kacc_cluster.hip).
extern "C" int kacc_internal_cluster_partials(kacc_ctx *ctx, uint32_t n_ns, const uint32_t *off,
                                              const uint32_t *slots, uint64_t *out_energy, double *out_power,
                                              uint64_t *node_energy, double *node_power, void *stream);

// The same from an interval's exports (kacc_interval.pod_export / node_export):
// namespace k sums the export rows rows[off[k] .. off[k+1]) (< n_pods); with
// from_exports the node totals sum the export's n_nodes rows (n_nodes 0: zeros,
// node_export may be NULL), else the tables' live nodes, as above.
extern "C" int kacc_internal_export_partials(kacc_ctx *ctx, uint32_t n_ns, const uint32_t *off, const uint32_t *rows,
                                             const uint64_t *pod_export, uint64_t n_pods,
                                             const uint64_t *node_export, uint64_t n_nodes, int from_exports,
                                             uint64_t *out_energy,
                                             double *out_power, uint64_t *node_energy, double *node_power,
                                             void *stream);

// Records the message on ctx (or the thread's create error when ctx is NULL)
// and returns code.
int kacc_fail(kacc_ctx *ctx, int code, const char *fmt, ...) __attribute__((format(printf, 3, 4)));

#define KACC_HIP(ctx, call)                                                                   \
  do {                                                                                        \
    hipError_t e_ = (call);                                                                   \
    if (e_ != hipSuccess)                                                                     \
      return kacc_fail((ctx), e_ == hipErrorOutOfMemory ? KACC_ENOMEM : KACC_EHIP, "%s: %s", \
                       #call, hipGetErrorString(e_));                                         \
  } while (0)
