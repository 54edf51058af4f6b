#!/usr/bin/env python3
"""Benchmark: Kepler power attribution on MI355X (BASELINE.json metric).

One *step* = one collection interval (PowerMonitor.calculatePower,
internal/monitor/monitor.go:399-431) over the whole fleet shard of a GPU:
node split + segmented CPU-time sums + process/container/VM/pod attribution
(one kacc_run_interval launch) followed by the cluster namespace totals
(kacc_namespace_totals, then an RCCL all-reduce across GPUs when N > 1).

Workload: BASELINE config 3 — a 10k-node fleet of 2k processes per node, Z = 4
RAPL zones (package/core/uncore/dram), ~1.6k container processes / 200
containers / 71 pods / 20 VMs per node, synthetic inputs (kepler_amd/fleet.py)
resident in HBM before timing.  Scaling is STRONG (the north star's "10k-node x
2k-process fleet interval" at 1/2/4/8 GPUs): the fixed fleet is cut into N node
ranges by shard.plan_node_ranges (balanced process rows) and every rank
generates and owns only its range (node snapshots are independent), so N GPUs
share one 20M-row interval.  At N > 1 a weak-scaling line (a full 10k-node shard
per GPU) is added as `weak_scaling`; `--scaling weak` makes it the headline.
`--shard-of W` runs rank 0's shard of a W-way split on one GPU (the per-GPU step
of a W-GPU run).  Only the cluster totals cross GPUs: per-namespace and cluster
node totals, all-reduced by the library's own RCCL communicator
(kacc_cluster_join; every step's partial sums by kacc_cluster_partials, then one
kacc_allreduce_sums per --allreduce-every steps on the comm stream — the C ABI a
cgo caller uses; at N = 1 the same calls run with a one-rank communicator).  torch.distributed
(gloo) is only the control plane: rank-0 unique-id broadcast, barriers,
max-over-ranks timing.

Prints ONE JSON line on rank 0.  Launch with N > 1 as
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
      --master-addr 127.0.0.1 --master-port P bench.py --gpus N
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
# --totals auto: the partial sums ride in the next interval's launch up to this many nodes per GPU
# (the launch's tail is then short of work and a second launch per step is a tenth of the step);
# past it the export stores cost more than the launch they save
FUSED_MAX_NODES = 2048
METRIC = "process attributions/sec + achieved HBM GB/s, 10k-node fleet, 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=3, choices=[1, 2, 3, 4, 5],
                    help="BASELINE config; 4 = a 100k-node fleet split over the ranks; "
                         "1 = a fleet of config-1 nodes (500 procs, Z=2; 40k per GPU)")
    ap.add_argument("--nodes", type=int, default=None, help="override nodes per GPU")
    ap.add_argument("--distinct", type=int, default=4, help="distinct process-input sets cycled")
    ap.add_argument("--intervals", type=int, default=1,
                    help="intervals per step, issued by one kacc_run_intervals call (config 5: 60)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-nodes", type=int, default=100)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--node-order", action="store_true", help="launch heaviest nodes first")
    ap.add_argument("--fragment", type=float, default=0.0,
                    help="process slots on a random subset of each node's slot range of (1+F) x rows, "
                         "with node_proc_span (the slot join's steady state under churn)")
    ap.add_argument("--cpu-runs", type=int, default=0, help="CPU baseline: timed runs (0 = as many as fit)")
    ap.add_argument("--frag-line", type=float, default=0.02,
                    help="N = 1: also time this workload under three slot layouts on the same box (pristine "
                         "without / with node_proc_span, F fragmented) and report them as `slot_layouts` (0 = off)")
    ap.add_argument("--no-pipeline-line", dest="pipeline_line", action="store_false",
                    help="N = 1, config 3: skip the join -> tracker -> interval line (`pipeline`)")
    ap.add_argument("--no-host-line", dest="host_line", action="store_false",
                    help="N = 1, config 3: skip the end-to-end pinned-batch line (`host_path`)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="N > 1: strong = the config's fixed fleet (config 3: 10k nodes) cut into N node ranges "
                         "(the north star's 8-GPU target); weak = N x the fleet, a full shard per GPU")
    ap.add_argument("--shard-of", type=int, default=1,
                    help="N = 1 only: run rank 0's shard of a W-way split of the fleet on this GPU (the per-GPU "
                         "step of a W-GPU strong-scaling run, without the cross-GPU all-reduce)")
    ap.add_argument("--no-weak-line", dest="weak_line", action="store_false",
                    help="N > 1, strong scaling: skip the extra weak-scaling measurement (`weak_scaling`)")
    ap.add_argument("--totals", choices=["auto", "fused", "tables", "exports", "tables+writes"], default="auto",
                    help="auto (default): fused when this GPU's shard has <= FUSED_MAX_NODES nodes (one interval per "
                         "step), else tables — the measured crossover (profiles/r05/sums_ab: 1/8 shard fused 54.1 vs "
                         "56.3 us per step, 1/4 shard equal, config 3 fused 391 vs 375 us).  "
                         "tables: cluster totals from the state tables, partial sums on the compute stream and the RCCL "
                         "all-reduce on the comm stream (kacc_allreduce_namespaces, the default: measured fastest), "
                         "or from the interval's exports with everything on the comm stream (kacc_allreduce_exports: "
                         "the export stores cost 26 us and the concurrent partial sums slow the next interval more "
                         "than they save at config 3, profiles/r03/exports_ablation); tables+writes = the export "
                         "stores alone (ablation); fused = each interval writes its exports in namespace order "
                         "(pod_export_pos) and its launch also computes the previous interval's partial sums "
                         "(kacc_run_interval_sums: one launch per step; the region's last step's sums by "
                         "kacc_run_export_sums inside the timed region)")
    ap.add_argument("--sums-order", choices=["ns", "rows"], default="ns",
                    help="--totals fused: pod exports written in namespace order (pod_export_pos; the sums read "
                         "contiguous records) or in batch order (the sums gather them through ns_pod_row)")
    ap.add_argument("--allreduce-every", type=int, default=8,
                    help="tables mode: the cluster totals of this many consecutive steps are all-reduced by ONE "
                         "kacc_allreduce_sums (each step's partial sums have their own rows; SURVEY 5: one "
                         "all-reduce per K intervals), so the compute stream carries one handoff event per group "
                         "(each costs ~6.5 us of stream gap, profiles/r03/handoff); 1 = every step")
    ap.add_argument("--handoff-event", choices=["device", "torch"], default="device",
                    help="--comm-wait always: the emulated handoff event is the library's (timing disabled, "
                         "device-scope release) or a default torch event (system-scope release; ablation)")
    ap.add_argument("--comm-wait", choices=["auto", "always"], default="auto",
                    help="auto: cross-stream packets only where the library issues them (N > 1: an event on the "
                         "compute stream after the partial sums, waited for by the comm stream's all-reduce); "
                         "always: at one rank, record the same timing-free event on the compute stream and make "
                         "the comm stream wait for it every step (the N > 1 handoff without RCCL, ablation)")
    ap.add_argument("--step-events", choices=["separate", "inline", "markers"], default="separate",
                    help="how the kernels are timed with HIP events: separate = the timed region has NO event "
                         "packet between its kernels (value, ms_per_step) and a second timed pass over the same "
                         "number of steps right after it carries a start/stop pair on the dispatch packets of each "
                         "step's interval and totals launches (kacc_time_next_launch) -> kernel_ms, "
                         "totals_compute_ms; inline = those launch events inside the timed region; markers = "
                         "hipEventRecord markers around them inside the timed region (round 2).  Every event "
                         "packet costs a stream gap: ~9 us per step, profiles/r03/events")
    ap.add_argument("--slot-nodes", choices=["stable", "write"], default="stable",
                    help="stable: KACC_F_STABLE_SLOT_NODES (a process slot keeps its node; only NEW rows store "
                         "it); write: every row stores its node (ablation)")
    ap.add_argument("--totals-probe", choices=["both", "ns", "nodes"], default="both",
                    help="ablation: only the namespace sums (ns) or only the cluster node totals (nodes) per step")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def host_cpu():
    """CPU model and core counts of this host (report them beside the CPU baseline)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        usable = os.cpu_count()
    return dict(model=model, nproc=os.cpu_count(), usable=usable)


def cpu_share():
    """Host threads this job may use and where that number comes from.  A GPU box grants each
    one-GPU job a share of its host (OMP_NUM_THREADS, set by the box: 16 of the 256 hardware
    threads; the rest belong to the other GPUs' jobs), else a cgroup CPU quota, else the
    affinity mask (usable cores)."""
    usable = host_cpu()["usable"] or 1
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return min(usable, int(env)), "OMP_NUM_THREADS (the box's CPU share for this job)"
    for path, parse_q in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                          ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            with open(path) as f:
                txt = f.read().strip()
            if parse_q:
                q, per = parse_q(txt)
            else:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                    q, per = txt, f.read().strip()
            if q not in ("max", "-1"):
                return max(1, min(usable, -(-int(q) // int(per)))), f"cgroup CPU quota ({path})"
        except (OSError, ValueError):
            pass
    return usable, "affinity mask (usable cores)"


def _median_rate(run, rows, budget_s, min_runs=5, max_runs=0):
    """Warm-up call, then timed calls until the budget (>= min_runs); rows / median seconds."""
    run(-1)  # warm-up (untimed)
    times = []
    t_end = time.perf_counter() + budget_s
    k = 0
    while len(times) < min_runs or (time.perf_counter() < t_end and (not max_runs or len(times) < max_runs)):
        t0 = time.perf_counter()
        run(k)
        times.append(time.perf_counter() - t0)
        k += 1
    med = float(np.median(times))
    return dict(value=rows / med, runs=len(times), median_s=med, min_s=float(np.min(times)),
                max_s=float(np.max(times)), seconds=float(np.sum(times)))


def cpu_baseline(layout, intervals, node_steps, n_nodes, seconds, max_runs=0):
    """The C++ restatement of the Go path on this host's cores (steady_clock-style timing of
    the attribution call only; warm-up, then the median of >= 5 runs of one interval each).

    gofaithful: Go's data structures (string-keyed maps, per-object zone maps), 1 thread —
    the reference attributes on one goroutine; soa: the flat-array oracle, 1 thread;
    soa_mt: the flat-array oracle over node ranges on the host's usable cores."""
    from kepler_amd import fleet
    from oracle.oracle import GoFaithful, Oracle

    nodes = np.arange(min(n_nodes, layout.n_nodes))
    subs = [fleet.subset_interval(a, nodes, layout.zones) for a in intervals]
    _, sizes, _ = subs[0]
    caps = dict(nodes=sizes["n_nodes"], proc_slots=sizes["n_procs"], ctr_slots=sizes["n_ctrs"],
                vm_slots=sizes["n_vms"], pod_slots=sizes["n_pods"])
    zidx = (nodes[:, None] * layout.zones + np.arange(layout.zones)).reshape(-1)

    def batch(k):  # interval k >= 0 of the sample: distinct process inputs + fresh node counters
        k = max(k, 0)
        a = dict(subs[1 + k % (len(subs) - 1)][0])
        na = node_steps[k % len(node_steps)]
        for key in ("node_ts_ns", "node_usage_ratio", "node_status"):
            a[key] = np.ascontiguousarray(na[key][nodes])
        a["zone_energy"] = np.ascontiguousarray(na["zone_energy"][zidx])
        return a

    out = {}
    for name, cls, budget in (("gofaithful", GoFaithful, seconds), ("soa", Oracle, min(seconds, 5.0))):
        o = cls(layout.zones, **caps)
        o.interval(subs[0][0], sizes)  # first read (untimed, as on the GPU)
        pre = [batch(k) for k in range(8)]
        out[name] = _median_rate(lambda k: o.interval(pre[max(k, 0) % 8], sizes), sizes["n_procs"], budget,
                                 max_runs=max_runs)
    # the flat-array port on every host thread this job may use (node ranges per thread), on a
    # node sample of >= 10x the 1-thread one and >= 40 nodes per thread: the strongest CPU
    # number this repo can produce
    threads, share_source = cpu_share()
    nodes_mt = np.arange(min(max(10 * n_nodes, 40 * threads), layout.n_nodes))
    subs_mt = [fleet.subset_interval(a, nodes_mt, layout.zones) for a in intervals[:3]]
    _, sizes_mt, _ = subs_mt[0]
    o = Oracle(layout.zones, nodes=sizes_mt["n_nodes"], proc_slots=sizes_mt["n_procs"],
               ctr_slots=sizes_mt["n_ctrs"], vm_slots=sizes_mt["n_vms"], pod_slots=sizes_mt["n_pods"])
    o.interval_mt(subs_mt[0][0], sizes_mt, threads)
    out["soa_mt"] = _median_rate(lambda k: o.interval_mt(subs_mt[1 + max(k, 0) % 2][0], sizes_mt, threads),
                                 sizes_mt["n_procs"], 5.0, max_runs=max_runs)
    out["soa_mt"].update(threads=threads, procs=sizes_mt["n_procs"], share_source=share_source)
    return out, sizes


def exchange_unique_id(rank, world, make_id):
    """Rank 0's RCCL unique id, handed to every rank over the torch.distributed control group."""
    uid = make_id() if rank == 0 else None
    if world > 1:
        import torch.distributed as dist

        box = [uid]
        dist.broadcast_object_list(box, src=0)
        uid = box[0]
    return uid


def slot_layout_lines(args, frag, K, steps, bytes_per_interval, steady_intervals=40, rounds=3):
    """Same-box kernel time per interval (HIP events on the launch stream around back-to-back
    launches, median over `rounds` interleaved rounds of `steps`) of this config under four
    process-slot layouts, all on ONE engine context (contexts of one box differ by up to 12 %:
    table placement, profiles/r02/placement/): pristine slots (slot = row) without and with
    node_proc_span; the layout the slot join itself produces in production — kacc_slot_join
    with KACC_JOIN_REUSE_TERMINATED over `steady_intervals` intervals of /proc-shaped churn
    (fleet.ProcChurn, 2 % per interval), its spans given; and a synthetic one (each node's rows
    on a random subset of (1+frag) x rows slots in random row order).  Same rows, same
    algorithmic bytes."""
    import torch

    from kepler_amd import accel, fleet
    from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device

    _, _, layout = fleet.config_shard(args.config, 1, 0, bench_nodes(args.config, 1, args.nodes))
    sizes = layout.sizes()
    N, P = layout.n_nodes, sizes["n_procs"]
    off = layout.proc_off.astype(np.int64)
    rows = np.diff(off)
    node_of_row = np.repeat(np.arange(N), rows)
    local = np.arange(P) - off[node_of_row]
    slot_off = np.r_[0, np.cumsum(np.ceil(rows * (1 + max(frag, 0.05))).astype(np.int64) + 8)].astype(np.uint32)
    caps = layout.capacities()
    caps["proc_slots"] = int(slot_off[-1])
    acc = accel.Accel(layout.zones, **caps)
    stream = current_stream_handle()

    # the production layout: the slot join's own output after steady_intervals of churn
    sm = accel.SlotMap(acc, accel.KACC_KIND_PROC, slot_off)
    sm.set_policy(accel.KACC_JOIN_REUSE_TERMINATED)
    churn = fleet.ProcChurn(layout, churn=0.02)
    d_off = torch.from_numpy(layout.proc_off.view(np.int32)).cuda()
    d_out = torch.zeros(P, dtype=torch.int32, device="cuda")
    tk = torch.zeros(int(slot_off[-1]), dtype=torch.int64, device="cuda")
    ts = torch.zeros(int(slot_off[-1]), dtype=torch.int32, device="cuda")
    cnt = torch.zeros(N, dtype=torch.int32, device="cuda")
    d_span = torch.zeros(2 * N, dtype=torch.int32, device="cuda")
    for _ in range(steady_intervals + 1):
        d_keys = torch.from_numpy(churn.next_keys().view(np.int32)).cuda()
        sm.join(P, d_off.data_ptr(), d_keys.data_ptr(), 0, d_out.data_ptr(), tk.data_ptr(), ts.data_ptr(),
                cnt.data_ptr(), stream, d_span.data_ptr())
    acc.sync(stream)
    steady = d_out.cpu().numpy().view(np.uint32).copy()
    steady_span = d_span.cpu().numpy().view(np.uint32).copy()
    sm.close()
    del d_keys, d_out, tk, ts, cnt, d_span

    pristine = (slot_off[node_of_row].astype(np.int64) + local).astype(np.uint32)
    pristine_span = np.stack([slot_off[:-1], slot_off[:-1] + rows.astype(np.uint32) - 1], 1).reshape(-1)
    flay = fleet.config_layout(args.config, nodes=N, fragment_slots=frag)
    assert np.array_equal(flay.proc_off, layout.proc_off)
    fcap = (rows * (1.0 + frag)).astype(np.int64) + 1
    fslot = (slot_off[node_of_row].astype(np.int64) + flay.proc_slot.astype(np.int64)
             - np.repeat(np.r_[0, np.cumsum(fcap)[:-1]], rows)).astype(np.uint32)
    fspan = np.zeros(2 * N, dtype=np.uint32)
    if P:
        nz = rows > 0
        fspan[0::2][nz] = np.minimum.reduceat(fslot.astype(np.int64), off[:-1][nz])
        fspan[1::2][nz] = np.maximum.reduceat(fslot.astype(np.int64), off[:-1][nz])
        fspan[0::2][~nz] = 1

    sim = fleet.FleetSim(layout, seed=fleet.SEED)
    statics = to_device(layout.static_arrays())
    flags = layout.fast_flag() | accel.KACC_F_NODE_SLOT_RANGES | accel.KACC_F_STABLE_SLOT_NODES
    prime = sim.next_interval()
    prime["proc_slot"] = pristine
    tp = dict(statics)
    tp.update(to_device(prime))
    acc.run_interval(interval_from_tensors(tp, sizes), stream)
    full = [sim.next_interval() for _ in range(2)]
    keys_iv = ("proc_cpu_delta", "ctr_slot", "vm_slot", "pod_slot", "node_ts_ns", "node_usage_ratio",
               "node_status", "zone_energy", "zone_max")
    dev_full = [to_device({n: f[n] for n in keys_iv}) for f in full]

    def layout_ivs(proc_slot, span):
        base = dict(statics)
        base.update(to_device({"proc_slot": proc_slot}))
        if span is not None:
            base.update(to_device({"node_proc_span": span}))
        ivs = []
        for k in range((steps + 1) * K):
            t = dict(base)
            t.update(dev_full[k % 2])
            t.update(to_device({n: a for n, a in sim.next_node_inputs().items()
                                if n in ("node_ts_ns", "node_usage_ratio", "node_status", "zone_energy", "zone_max")}))
            ivs.append((interval_from_tensors(t, sizes, flags), t))
        return ivs

    cases = {"pristine_no_span": layout_ivs(pristine, None), "pristine_span": layout_ivs(pristine, pristine_span),
             "join_steady_state_span": layout_ivs(steady, steady_span),
             f"fragmented_{frag:g}_span": layout_ivs(fslot, fspan)}
    times = {n: [] for n in cases}
    for _ in range(rounds):
        for name, ivs in cases.items():
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps + 1)]
            for i in range(steps + 1):  # back to back, as the headline's steps (sustained clocks)
                ev[i][0].record()
                if K == 1:
                    acc.run_interval(ivs[i][0], stream)
                else:
                    acc.run_intervals([x[0] for x in ivs[i * K:(i + 1) * K]], stream)
                ev[i][1].record()
            torch.cuda.synchronize()
            times[name] += [a.elapsed_time(b) / K for a, b in ev[1:]]
    acc.sync(stream)
    acc.close()
    out = {}
    for name, ms in times.items():
        k_ms = float(np.median(ms))
        achieved = bytes_per_interval / (k_ms * 1e-3) / 1e9
        out[name] = {"kernel_ms": k_ms, "achieved_GBps": achieved, "frac": achieved / HBM_PEAK_GBPS}
    ps = out["pristine_no_span"]["kernel_ms"]
    out["join_steady_state_over_pristine"] = out["join_steady_state_span"]["kernel_ms"] / ps
    out["fragmented_over_pristine"] = out[f"fragmented_{frag:g}_span"]["kernel_ms"] / ps
    out["join_steady_state"] = {
        "policy": "KACC_JOIN_REUSE_TERMINATED", "intervals": steady_intervals, "churn": 0.02,
        "span_over_rows": float(np.mean((steady_span[1::2].astype(np.int64) - steady_span[0::2] + 1)[rows > 0]
                                        / rows[rows > 0])),
    }
    out["note"] = ("one context, interleaved rounds, same rows / algorithmic bytes; join_steady_state = the slot "
                   "words and spans kacc_slot_join returns after /proc-shaped churn (newcomers listed last in "
                   "their container, fleet.ProcChurn); fragmented = synthetic random subset of (1+F) x rows slots "
                   "in random row order")
    return out


def pipeline_line(args, steps=10, warm=8):
    """The production interval at N = 1: kacc_slot_join (KACC_JOIN_REUSE_TERMINATED) on
    /proc-shaped churn (fleet.ProcChurn, 2 % per interval) -> the terminated trackers
    (top 500 per node, 10 J, cleared every other interval: config.go:210-211,
    process.go:80-99) -> the interval kernel on the join's slot words and spans, one
    stream, HIP events around the three; keys already on the device.  Reported beside
    the headline, never as `value`."""
    import torch

    from kepler_amd import accel, fleet
    from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device

    _, _, layout = fleet.config_shard(args.config, 1, 0, bench_nodes(args.config, 1, args.nodes))
    sizes = layout.sizes()
    N, P = layout.n_nodes, sizes["n_procs"]
    rows = np.diff(layout.proc_off.astype(np.int64))
    slot_off = np.r_[0, np.cumsum(np.ceil(rows * 1.05).astype(np.int64) + 8)].astype(np.uint32)
    caps = layout.capacities()
    caps["proc_slots"] = int(slot_off[-1])
    acc = accel.Accel(layout.zones, **caps)
    stream = current_stream_handle()
    sm = accel.SlotMap(acc, accel.KACC_KIND_PROC, slot_off)
    sm.set_policy(accel.KACC_JOIN_REUSE_TERMINATED)
    tr = accel.Tracker(acc, accel.KACC_KIND_PROC, 500, zone=0, min_energy=10 * 10**6)
    churn = fleet.ProcChurn(layout, churn=0.02)
    n_iv = warm + 3 * steps  # warm-up, the split pass, the sequence pass, the join-only pass
    keys = [torch.from_numpy(churn.next_keys().view(np.int32)).cuda() for _ in range(n_iv)]
    sim = fleet.FleetSim(layout, seed=fleet.SEED)
    statics = to_device(layout.static_arrays())
    cap = int(slot_off[-1])
    d_slot = torch.zeros(P, dtype=torch.int32, device="cuda")
    tk = torch.zeros(cap, dtype=torch.int64, device="cuda")
    ts = torch.zeros(cap, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(N, dtype=torch.int32, device="cuda")
    span = torch.zeros(2 * N, dtype=torch.int32, device="cuda")
    full = [to_device({n: a for n, a in sim.next_interval().items() if n != "proc_slot"}) for _ in range(2)]
    ivs = []
    for k in range(n_iv):
        t = dict(statics)
        t.update(full[k % 2])
        t.update(to_device({n: a for n, a in sim.next_node_inputs().items()
                            if n in ("node_ts_ns", "node_usage_ratio", "node_status", "zone_energy", "zone_max")}))
        t["proc_slot"] = d_slot  # the join writes the batch's slot words in place
        t["node_proc_span"] = span
        ivs.append((interval_from_tensors(t, sizes, layout.fast_flag() | accel.KACC_F_NODE_SLOT_RANGES
                                          | accel.KACC_F_STABLE_SLOT_NODES), t))
    def interval(k):
        sm.join(P, ivs[k][1]["proc_off"].data_ptr(), keys[k].data_ptr(), 0, d_slot.data_ptr(), tk.data_ptr(),
                ts.data_ptr(), cnt.data_ptr(), stream, span.data_ptr())
        yield
        if k % 2:
            tr.clear(stream)
        tr.add(sm, tk.data_ptr(), ts.data_ptr(), cnt.data_ptr(), stream)
        yield
        acc.run_interval(ivs[k][0], stream)
        yield

    tj, tt, ti, tall = [], [], [], []
    for k in range(warm + steps):  # warm-up, then the split: events around each kernel
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record()
        for i, _ in enumerate(interval(k)):
            ev[i + 1].record()
        if k >= warm:
            ev[3].synchronize()
            tj.append(ev[0].elapsed_time(ev[1]))
            tt.append(ev[1].elapsed_time(ev[2]))
            ti.append(ev[2].elapsed_time(ev[3]))
            tall.append(ev[0].elapsed_time(ev[3]))
    # the production sequence: `steps` intervals back to back, no event packet between their
    # kernels (each costs a stream gap): one event pair around the run
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(warm + steps, warm + 2 * steps):
        for _ in interval(k):
            pass
    e1.record()
    e1.synchronize()
    seq_ms = e0.elapsed_time(e1) / steps
    # the join alone, `steps` joins of the continuing churn back to back (one event pair)
    j0, j1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    j0.record()
    for k in range(warm + 2 * steps, warm + 3 * steps):
        sm.join(P, ivs[k][1]["proc_off"].data_ptr(), keys[k].data_ptr(), 0, d_slot.data_ptr(), tk.data_ptr(),
                ts.data_ptr(), cnt.data_ptr(), stream, span.data_ptr())
    j1.record()
    j1.synchronize()
    join_seq_ms = j0.elapsed_time(j1) / steps
    acc.sync(stream)
    n_term = int(cnt.sum().item())
    tr.close()
    sm.close()
    acc.close()
    return {"ms_per_interval": seq_ms, "proc_attr_per_s": P / (seq_ms * 1e-3),
            "ms_per_interval_split": float(np.mean(tall)),
            "join_ms": float(np.mean(tj)), "tracker_ms": float(np.mean(tt)), "interval_ms": float(np.mean(ti)),
            "join_ms_back_to_back": join_seq_ms,
            "terminated_last_interval": n_term, "intervals": steps,
            "note": "kacc_slot_join (reuse policy) -> kacc_tracker_add -> kacc_run_interval on one stream, "
                    "keys of fleet.ProcChurn (2 % /proc-shaped churn) resident on the device; ms_per_interval: "
                    "`intervals` intervals back to back with one event pair around them; join_ms / tracker_ms / "
                    "interval_ms and ms_per_interval_split: a pass with events between the kernels (each event "
                    "packet adds a stream gap); join_ms_back_to_back: `intervals` more joins of the same churn "
                    "back to back, one event pair around them"}


def host_path_line(args, steps=10):
    """End-to-end, PCIe-inclusive: what a Go caller of calculatePower (monitor.go:399-431) sees
    per interval through the cgo boundary.  The packer's output sits in two pinned batches
    (kacc_batch_alloc); each interval is kacc_batch_submit (host layout check, H2D of the
    interval's inputs on the context's copy stream, the interval kernel after an event) and
    kacc_batch_wait, two batches in flight (submit B, wait A, ...) so one interval's copies
    overlap the previous one's kernel.  Trusted: KACC_F_TRUSTED_LAYOUT (slots from
    kacc_slot_join, no host check; the device range checks stay).  Beside it the PCIe ceiling:
    a pinned -> device copy of the same bytes.  Reported beside the headline, never as `value`."""
    import torch

    from kepler_amd import accel, fleet

    _, _, layout = fleet.config_shard(args.config, 1, 0, bench_nodes(args.config, 1, args.nodes))
    sizes = layout.sizes()
    sim = fleet.FleetSim(layout, seed=fleet.SEED)
    acc = accel.Accel(layout.zones, **layout.capacities())
    ivs = [sim.next_interval() for _ in range(5)]
    batches = [accel.HostBatch.alloc(acc, **sizes) for _ in range(2)]
    nbytes = int(sum(v.nbytes for k, v in ivs[0].items() if k in accel.INTERVAL_ARRAYS and v is not None))
    try:
        batches[0].fill(ivs[0])  # first read (monitor.go:326-330), untimed
        batches[0].submit()
        batches[0].wait()

        def pipelined(k):
            t0 = time.perf_counter()
            batches[0].submit()
            for i in range(1, k):
                batches[i % 2].submit()
                batches[(i - 1) % 2].wait()
            batches[(k - 1) % 2].wait()
            return (time.perf_counter() - t0) / k

        res = {}
        for name, flags, first in (("checked", 0, 1), ("trusted", accel.KACC_F_TRUSTED_LAYOUT, 3)):
            for b, a in zip(batches, ivs[first:first + 2]):
                b.fill(a, flags)
            pipelined(4)
            res[name] = float(np.median([pipelined(steps) for _ in range(3)]))
        src = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
        dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        cps = []
        for _ in range(6):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            dst.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
            cps.append(time.perf_counter() - t0)
        t_copy = float(np.median(cps[1:]))
        del src, dst
    finally:
        for b in batches:
            b.free()
        acc.close()
    P, N = sizes["n_procs"], sizes["n_nodes"]
    tp = res["trusted"]
    return {"label": "END-TO-END (PCIe-inclusive; pinned host batches -> H2D -> interval kernel), not `value`",
            "proc_attr_per_s": P / tp, "node_snapshots_per_s": N / tp, "ms_per_interval": tp * 1e3,
            "checked_ms_per_interval": res["checked"] * 1e3, "checked_proc_attr_per_s": P / res["checked"],
            "h2d_bytes_per_interval": nbytes,
            "pcie_copy_ms": t_copy * 1e3, "pcie_copy_GBps": nbytes / t_copy / 1e9,
            "frac_of_pcie_copy": t_copy / tp, "batches_in_flight": 2, "intervals": steps,
            "note": "kacc_batch_submit / kacc_batch_wait, two pinned batches in flight; value: "
                    "KACC_F_TRUSTED_LAYOUT (slots from kacc_slot_join), checked: with the host layout check; "
                    "pcie_copy: torch pinned -> device copy of the same bytes (the ceiling)"}


def scrape_line(acc, n_procs, Z, reps=10):
    """What a per-interval scrape of every process's Usage.Power costs on the device: the
    P x Z derived powers (kacc_table_read of KACC_T_PROC_POWER: the slot's ratio x its node's
    ActivePower behind the process.go:124 guard) written to a dense device array, after the
    timed region, on the snapshot it left.  Bytes: ratio 8 + node 4 per slot in, 8 per power
    out (the node tables, N x Z, stay in cache)."""
    import torch

    from kepler_amd.torch_batch import current_stream_handle

    n = n_procs * Z
    out = torch.empty(max(n, 1), dtype=torch.float64, device="cuda")
    s = current_stream_handle()
    acc.read("proc_power", out.data_ptr(), 0, n, s)  # warm-up
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        acc.read("proc_power", out.data_ptr(), 0, n, s)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    nbytes = n_procs * 12 + n * 8
    gbps = nbytes / ms / 1e6
    return {"powers": n, "processes": n_procs, "zones": Z, "ms": ms, "bytes": nbytes, "GBps": gbps,
            "frac_of_spec": gbps / 8000.0, "reps": reps,
            "note": "kacc_table_read(KACC_T_PROC_POWER) into a dense device array after the timed region "
                    "(HIP events around reps back-to-back reads); not part of value"}


def _pack(arrays):
    """One contiguous byte image of named arrays (16-B aligned segments): {name: (offset, dtype, n)}."""
    off, layout = 0, {}
    for name, a in arrays.items():
        a = np.ascontiguousarray(a)
        layout[name] = (off, a.dtype, a.size)
        off += (a.nbytes + 15) // 16 * 16
    img = np.zeros(max(off, 16), dtype=np.uint8)
    for name, a in arrays.items():
        o, _, _ = layout[name]
        img[o:o + a.nbytes] = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
    return img, layout


def host_path_ticks_line(args, steps=10, nbuf=3, mode="full"):
    """End-to-end with the CPU-tick input format (kepler_accel.h "CPU-tick input format"): per
    interval ONE pinned host image crosses PCIe — node readings and CSR, per process row its PID
    (4 B, for the device slot join) and its tick increment (2 B; 1 % escapes as int64), the
    aggregates' CSR ends and slot words — then, on the device, kacc_slot_join (PIDs -> slot words,
    KACC_JOIN_REUSE_TERMINATED) -> kacc_ticks_delta (Go's CPUTimeDelta from the tick map) ->
    kacc_run_interval.  Three staging buffers: the copies (copy stream) run back to back while
    the kernels (compute stream) follow them — with two, a copy waited for the interval two back
    and the path ran at 3.39 ms against a 2.62 ms copy; with three (or four) 2.71 ms
    (profiles/r05/r05m, tools/bench_host_ticks.py).  Reported beside the headline, never as
    `value`."""
    import ctypes

    import torch

    from kepler_amd import accel, fleet
    from kepler_amd.torch_batch import interval_from_tensors

    _, _, layout = fleet.config_shard(args.config, 1, 0, bench_nodes(args.config, 1, args.nodes))
    sizes = layout.sizes()
    N, P = layout.n_nodes, sizes["n_procs"]
    rows = np.diff(layout.proc_off.astype(np.int64))
    slot_off = np.r_[0, np.cumsum(np.ceil(rows * 1.05).astype(np.int64) + 8)].astype(np.uint32)
    caps = layout.capacities()
    caps["proc_slots"] = int(slot_off[-1])
    acc = accel.Accel(layout.zones, **caps)
    sm = accel.SlotMap(acc, accel.KACC_KIND_PROC, slot_off)
    sm.set_policy(accel.KACC_JOIN_REUSE_TERMINATED)
    tm = accel.TickMap(acc)
    sim = fleet.FleetSim(layout, seed=fleet.SEED)
    churn = fleet.ProcChurn(layout, churn=0.02)
    rng = np.random.default_rng(5)
    statics = layout.static_arrays()
    imgs = []
    for k in range(nbuf):
        node = sim.next_node_inputs()
        keys = churn.next_keys()
        dt = rng.integers(0, 3000, size=P).astype(np.uint16)
        esc = np.flatnonzero(rng.random(P) < 0.01).astype(np.uint32)
        dt[esc] = accel.KACC_TICKS_ESCAPED
        arrays = dict(node_ts_ns=node["node_ts_ns"], node_usage_ratio=node["node_usage_ratio"],
                      node_status=node["node_status"], zone_energy=node["zone_energy"], zone_max=node["zone_max"],
                      proc_off=statics["proc_off"], ctr_off=statics["ctr_off"], vm_off=statics["vm_off"],
                      pod_off=statics["pod_off"], pid=keys, dticks=dt,
                      esc_off=np.searchsorted(esc, layout.proc_off.astype(np.int64)).astype(np.uint32),
                      esc_row=esc, esc_ticks=rng.integers(1 << 16, 1 << 40, size=esc.size).astype(np.int64),
                      ctr_proc_end=statics["ctr_proc_end"], ctr_slot=layout.ctr_slot,
                      vm_proc_end=statics["vm_proc_end"], vm_slot=layout.vm_slot,
                      pod_ctr_end=statics["pod_ctr_end"], pod_slot=layout.pod_slot)
        imgs.append(_pack(arrays))
    nbytes = max(im.nbytes for im, _ in imgs)
    host = [torch.from_numpy(im).pin_memory() for im, _ in imgs]
    dev = [torch.empty(nbytes, dtype=torch.uint8, device="cuda") for _ in range(nbuf)]
    d_slot = torch.zeros(P, dtype=torch.int32, device="cuda")
    d_delta = torch.zeros(P, dtype=torch.float64, device="cuda")
    cap = int(slot_off[-1])
    tk = torch.zeros(cap, dtype=torch.int64, device="cuda")
    ts = torch.zeros(cap, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(N, dtype=torch.int32, device="cuda")
    span = torch.zeros(2 * N, dtype=torch.int32, device="cuda")
    tdt = {np.dtype(np.uint32): torch.int32, np.dtype(np.uint64): torch.int64, np.dtype(np.int64): torch.int64,
           np.dtype(np.float64): torch.float64, np.dtype(np.uint16): torch.int16, np.dtype(np.int32): torch.int32}

    def views(b, lay):
        return {n: dev[b][o:o + cnt_ * dt_.itemsize].view(tdt[dt_]) for n, (o, dt_, cnt_) in lay.items()}

    descs = []
    for b in range(nbuf):
        v = views(b, imgs[b][1])
        t = {n: v[n] for n in ("node_ts_ns", "node_usage_ratio", "node_status", "zone_energy", "zone_max",
                               "proc_off", "ctr_off", "vm_off", "pod_off", "ctr_proc_end", "ctr_slot",
                               "vm_proc_end", "vm_slot", "pod_ctr_end", "pod_slot")}
        t.update(proc_cpu_delta=d_delta, proc_slot=d_slot, node_proc_span=span)
        iv = interval_from_tensors(t, sizes, layout.fast_flag() | accel.KACC_F_NODE_SLOT_RANGES
                                   | accel.KACC_F_STABLE_SLOT_NODES)
        tks = accel.KaccTicks(N, P, int(v["esc_row"].numel()), 0, v["proc_off"].data_ptr(),
                              v["node_status"].data_ptr(), d_slot.data_ptr(), v["dticks"].data_ptr(),
                              v["esc_off"].data_ptr(), v["esc_row"].data_ptr(), v["esc_ticks"].data_ptr(),
                              d_delta.data_ptr())
        descs.append((iv, tks, v, t))
    compute = torch.cuda.current_stream()
    copy = torch.cuda.Stream()
    cs = compute.cuda_stream
    copied = [torch.cuda.Event() for _ in range(nbuf)]
    done = [torch.cuda.Event() for _ in range(nbuf)]
    used = [False] * nbuf

    def one(i):
        b = i % nbuf
        if mode != "compute":  # mode: "copy" / "compute" time one side alone (diagnostics)
            if used[b]:
                copy.wait_event(done[b])  # staging b is free once interval i - nbuf has run
            with torch.cuda.stream(copy):
                dev[b][:imgs[b][0].nbytes].copy_(host[b], non_blocking=True)
            copied[b].record(copy)
            if mode == "copy":
                done[b].record(copy)
                used[b] = True
                return
            compute.wait_event(copied[b])
        iv, tks, v, _ = descs[b]
        sm.join(P, v["proc_off"].data_ptr(), v["pid"].data_ptr(), v["node_status"].data_ptr(), d_slot.data_ptr(),
                tk.data_ptr(), ts.data_ptr(), cnt.data_ptr(), cs, span.data_ptr())
        tm.delta(tks, cs)
        acc.run_interval(iv, cs)
        done[b].record(compute)
        used[b] = True

    try:
        if mode == "compute":  # the images resident once
            for b in range(nbuf):
                dev[b][:imgs[b][0].nbytes].copy_(host[b])
        for i in range(4):  # first read + warm-up
            one(i)
        torch.cuda.synchronize()
        acc.sync(cs)
        walls = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(steps):
                one(i)
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) / steps)
        acc.sync(cs)
        tp = float(np.median(walls))
        src = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
        dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        cps = []
        for _ in range(6):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            dst.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
            cps.append(time.perf_counter() - t0)
        t_copy = float(np.median(cps[1:]))
        del src, dst
    finally:
        tm.close()
        sm.close()
        acc.close()
    n_esc = int(descs[0][2]["esc_row"].numel())
    return {"label": "END-TO-END (PCIe-inclusive; CPU-tick format: PIDs + 2-B tick increments -> H2D -> device "
                     "slot join -> kacc_ticks_delta -> interval kernel), not `value`",
            "proc_attr_per_s": P / tp, "node_snapshots_per_s": N / tp, "ms_per_interval": tp * 1e3,
            "h2d_bytes_per_interval": nbytes, "bytes_per_process_row": nbytes / P, "escapes": n_esc,
            "pcie_copy_ms": t_copy * 1e3, "pcie_copy_GBps": nbytes / t_copy / 1e9,
            "frac_of_pcie_copy": t_copy / tp, "buffers_in_flight": nbuf, "mode": mode, "intervals": steps,
            "note": "one pinned image per interval (node readings + CSR, PID u32 + tick increment u16 per "
                    f"process, 1 % int64 escapes, aggregate CSR ends + slot words); copy stream / compute stream "
                    f"overlap, {nbuf} staging buffers; the join's churn is fleet.ProcChurn (2 %)"}


def bench_nodes(config, world, nodes=None, scaling="strong"):
    """Fleet size of a config at `world` GPUs.  Strong scaling (the north star's "10k-node x
    2k-process fleet interval" at 1/2/4/8 GPUs): one fixed fleet cut into `world` node ranges.
    Weak scaling: a fixed shard per GPU, `world` times the fleet.  Config 4 is always its
    100k-node fleet split over the GPUs."""
    if config == 4:
        return nodes or 100_000
    per = nodes or {1: 40000, 2: 1000, 3: 10000, 5: 1000}[config]
    return per if scaling == "strong" else per * world


class Workload:
    """One rank's node shard of a fleet, its per-step interval descriptors (inputs resident in
    HBM), the engine context, the cluster (RCCL) and the namespace CSR."""

    def __init__(self, args, total_nodes, split, shard_rank, rank, world, local, K, uid_fn):
        import torch

        from kepler_amd import accel, fleet
        from kepler_amd.torch_batch import interval_from_tensors, to_device

        t0 = time.time()
        self.lo, self.hi, layout = fleet.config_shard(args.config, split, shard_rank, total_nodes,
                                                      fragment_slots=args.fragment)
        self.layout = layout
        self.sizes = sizes = layout.sizes()
        self.Z = Z = layout.zones
        self.K = K
        sim = fleet.FleetSim(layout, seed=fleet.SEED + self.lo)
        n_steps = total_steps(args)
        n_ivs = n_steps * K  # every interval has its own node counters / clocks
        n_distinct = max(1, min(args.distinct, n_ivs))
        self.prime = sim.next_interval()  # first read (monitor.go:326-330), untimed
        self.full = [sim.next_interval() for _ in range(n_distinct)]
        self.node_steps = [self.full[k] if k < n_distinct else sim.next_node_inputs() for k in range(n_ivs)]
        log(rank, f"[bench] rank 0 nodes [{self.lo}, {self.hi}) of {total_nodes} (split {split}): {sizes} Z={Z}, "
                  f"inputs in {time.time() - t0:.1f}s")
        self.acc = accel.Accel(Z, **layout.capacities(), device=local)
        self.cluster = accel.Cluster.join(self.acc, exchange_unique_id(rank, world, uid_fn), world, rank)
        statics = to_device(layout.static_arrays())
        if args.fragment > 0:  # the slot join's per-node spans: rows moved in slot order
            statics.update(to_device({"node_proc_span": layout.proc_span()}))
        dev_full = [to_device({k: a[k] for k in ("proc_cpu_delta", "proc_slot", "ctr_slot", "vm_slot", "pod_slot")})
                    for a in self.full]
        node_keys = ("node_ts_ns", "node_usage_ratio", "node_status", "zone_energy", "zone_max")
        dev_nodes = [to_device({k: a[k] for k in node_keys}) for a in self.node_steps]
        order = to_device({"o": layout.node_order_heaviest_first()})["o"] if args.node_order else None

        def make(k):
            t = dict(statics)
            t.update(dev_full[k % n_distinct])
            t.update(dev_nodes[k])
            if order is not None:
                t["node_order"] = order
            return t

        self.iv_tensors = [make(k) for k in range(n_ivs)]
        # cluster-total exports (kacc_interval.pod_export / node_export) of each step's last
        # interval, double-buffered by step parity: step k's totals are reduced on the comm
        # stream while step k+1 runs (kacc_allreduce_exports)
        self.exports = args.totals == "exports"
        # --totals fused: interval k's launch also sums interval k-1's exports (kacc_run_interval_sums)
        self.fused_sums = args.totals == "fused"
        if self.fused_sums and K != 1:
            raise SystemExit("--totals fused: one interval per step (K = 1)")
        self.pex = [torch.zeros(max(sizes["n_pods"], 1) * 2 * Z, dtype=torch.int64, device="cuda") for _ in range(2)]
        self.nex = [torch.zeros(max(sizes["n_nodes"], 1) * 5 * Z, dtype=torch.int64, device="cuda") for _ in range(2)]
        ns_off, ns_slot = layout.namespace_csr()
        _, ns_row = layout.namespace_csr_rows()
        ns_pos = np.zeros(max(sizes["n_pods"], 1), dtype=np.uint32)  # pod row -> its place in namespace order
        ns_pos[ns_row] = np.arange(len(ns_row), dtype=np.uint32)
        self.ns_t = to_device({"off": ns_off, "slot": ns_slot, "row": ns_row, "pos": ns_pos})
        if args.totals != "tables":  # "tables+writes": the exports are written, the totals come from the tables
            # (an ablation: the cost of the export stores alone)
            for st in range(n_steps):
                t = self.iv_tensors[st * K + K - 1]
                t["pod_export"], t["node_export"] = self.pex[st % 2], self.nex[st % 2]
                if self.fused_sums and args.sums_order == "ns":  # the partial sums stream contiguous records
                    t["pod_export_pos"] = self.ns_t["pos"]
        # node-private slots (each node owns its slot range for the whole run): kacc_run_intervals
        # runs K > 1 fast-node intervals as one launch
        # (KACC_F_STABLE_SLOT_NODES: a slot stays with its node; only NEW rows write their node)
        self.flags = (layout.fast_flag() | accel.KACC_F_NODE_SLOT_RANGES
                      | (accel.KACC_F_STABLE_SLOT_NODES if args.slot_nodes == "stable" else 0))
        self.ivs = [interval_from_tensors(t, sizes, self.flags) for t in self.iv_tensors]
        self.iv_arrays = [(accel.KaccInterval * K)(*self.ivs[k * K:(k + 1) * K]) for k in range(n_steps)]
        self.n_ns = len(ns_off) - 1
        # cluster totals.  Tables mode: step k's partial sums go to row k of tot_e / tot_p
        # ([namespaces Z | node totals 2Z] u64, [namespaces Z | node totals 3Z] f64; 640 KB per
        # step at config 3), and every --allreduce-every steps ONE kacc_allreduce_sums reduces
        # those rows on the comm stream while the next intervals run: one compute-to-comm
        # handoff (an event packet on the compute stream, ~6.5 us of stream gap,
        # profiles/r03/handoff) per group instead of per step, and the compute stream never
        # waits for an all-reduce.  The exports ablation keeps two buffers per step parity and
        # waits for step k-2's all-reduce.
        self.n_bufs = 2 if self.exports else n_steps
        nsz = self.n_ns * Z
        self.tot_e = torch.zeros(n_steps, nsz + 2 * Z, dtype=torch.int64, device="cuda")
        self.tot_p = torch.zeros(n_steps, nsz + 3 * Z, dtype=torch.float64, device="cuda")
        if self.exports:
            self.ns_e = [torch.zeros(nsz, dtype=torch.int64, device="cuda") for _ in range(2)]
            self.ns_p = [torch.zeros(nsz, dtype=torch.float64, device="cuda") for _ in range(2)]
            self.nd_e = [torch.zeros(2 * Z, dtype=torch.int64, device="cuda") for _ in range(2)]
            self.nd_p = [torch.zeros(3 * Z, dtype=torch.float64, device="cuda") for _ in range(2)]
        else:
            self.ns_e = [self.tot_e[k, :nsz] for k in range(n_steps)]
            self.ns_p = [self.tot_p[k, :nsz] for k in range(n_steps)]
            self.nd_e = [self.tot_e[k, nsz:] for k in range(n_steps)]
            self.nd_p = [self.tot_p[k, nsz:] for k in range(n_steps)]

    def close(self):
        self.cluster.close()
        self.acc.close()


def allreduce_groups(first, n, group):
    """The all-reduce groups of the n consecutive steps first .. first + n - 1 (tables mode): at
    most `group` steps each, and the region's last step alone, so that what is left to reduce
    after the region's last interval is one step's rows.  [(first_step, last_step), ...] in
    order, covering every step exactly once."""
    out, k0, last = [], first, first + n - 1
    for k in range(first, first + n):
        if k - k0 + 1 >= max(1, group) or k >= last - 1:
            out.append((k0, k))
            k0 = k + 1
    return out


def total_steps(args):
    """Warm-up steps, the timed steps and (--step-events separate) the kernel-timing pass: every
    step has its own node counters / clocks (monotonic, as a node's RAPL readings)."""
    return args.warmup + args.steps * (2 if args.step_events == "separate" else 1)


def measure(args, w, rank, world, stream, comm_stream):
    """W untimed warm-up steps, then exactly `steps` steps bracketed by barrier + synchronize;
    returns (max wall seconds over ranks, per-interval kernel ms of the launch stream).  A step =
    K intervals (one kacc_run_intervals call) + the cluster totals (partial sums on the compute
    stream, the RCCL all-reduce on the comm stream overlapping the next step).  The host side of
    a step is a handful of C calls with prebuilt arguments: at a 1/8 shard a step is ~60 us of
    GPU work, so the issue path must stay far below that."""
    import ctypes

    import torch
    import torch.distributed as dist

    from kepler_amd import accel

    lib = accel.load()
    K = w.K
    acc, cl = w.acc, w.cluster
    cstream = ctypes.c_void_p(stream)
    P = lambda vals: (ctypes.c_void_p * 1)(*[ctypes.c_void_p(v) for v in vals])  # noqa: E731
    U = lambda v: (ctypes.c_uint32 * 1)(v)  # noqa: E731
    if w.exports:  # everything after the interval on the comm stream, from the step's exports
        ns_args = [(P([w.ns_t["off"].data_ptr()]), P([w.ns_t["row"].data_ptr()]), U(w.sizes["n_pods"]),
                    P([w.pex[b].data_ptr()]), U(w.sizes["n_nodes"]), P([w.nex[b].data_ptr()]),
                    P([w.ns_e[b].data_ptr()]), P([w.ns_p[b].data_ptr()]), P([w.nd_e[b].data_ptr()]),
                    P([w.nd_p[b].data_ptr()]), P([stream]), P([comm_stream.cuda_stream])) for b in range(2)]
        reduce_fn = lib.kacc_allreduce_exports
    elif w.fused_sums:  # step k's partial sums inside step k + 1's launch, into step k's rows
        no_nodes = args.totals_probe == "ns"
        xsums = []
        for k in range(w.n_bufs):
            x = accel.KaccExportSums()
            x.n_ns = 0 if args.totals_probe == "nodes" else w.n_ns
            x.n_pods, x.n_nodes = w.sizes["n_pods"], w.sizes["n_nodes"]
            x.ns_ordered = 1 if args.sums_order == "ns" else 0
            x.ns_pod_off = w.ns_t["off"].data_ptr()
            x.ns_pod_row = None if x.ns_ordered else w.ns_t["row"].data_ptr()
            x.pod_export, x.node_export = w.pex[k % 2].data_ptr(), None if no_nodes else w.nex[k % 2].data_ptr()
            x.out_energy, x.out_power = w.ns_e[k].data_ptr(), w.ns_p[k].data_ptr()
            x.out_node_energy = None if no_nodes else w.nd_e[k].data_ptr()
            x.out_node_power = None if no_nodes else w.nd_p[k].data_ptr()
            xsums.append(x)
        ns_args, reduce_fn = None, None
    else:  # partial sums from the state tables on the compute stream (kacc_cluster_partials); the
        # all-reduce of a group of steps' rows on the comm stream (kacc_allreduce_sums, flush())
        no_nodes = args.totals_probe == "ns"
        ns_args = [(P([w.ns_t["off"].data_ptr()]), P([w.ns_t["slot"].data_ptr()]), P([w.ns_e[b].data_ptr()]),
                    P([w.ns_p[b].data_ptr()]), None if no_nodes else P([w.nd_e[b].data_ptr()]),
                    None if no_nodes else P([w.nd_p[b].data_ptr()]), P([stream])) for b in range(w.n_bufs)]
        reduce_fn = lib.kacc_cluster_partials
    done = [torch.cuda.Event() for _ in range(w.n_bufs)]
    used = [False] * w.n_bufs
    compute = torch.cuda.current_stream()
    # one rank, one shard: the library enqueues nothing on the comm stream
    comm = world > 1 or w.exports
    handoff = world == 1 and args.comm_wait == "always"
    # --comm-wait always: the emulated handoff event, timing-free with a device-scope release
    # (--handoff-event device) or a default torch event (torch: system-scope release)
    handoff_ev = None
    if not handoff:
        pass
    elif args.handoff_event == "torch":
        handoff_ev = torch.cuda.Event()
    else:
        handoff_ev = ctypes.c_void_p()
        if lib.hipEventCreateWithFlags(ctypes.byref(handoff_ev), ctypes.c_uint(0x2 | 0x40000000)) != 0:
            raise RuntimeError("hipEventCreateWithFlags failed")
    group = max(1, args.allreduce_every)
    ne_row, np_row = w.tot_e.shape[1], w.tot_p.shape[1]
    group_of = {}  # last step of a group -> its first step (allreduce_groups of each region)

    def plan(first, n):
        group_of.clear()
        group_of.update({k1: k0 for k0, k1 in allreduce_groups(first, n, group)})

    def flush(k0, last):
        """Tables mode: ONE all-reduce of the rows of steps k0 .. last (contiguous)."""
        m = last - k0 + 1
        if handoff:  # one rank: the library reduces nothing; the handoff it would issue
            if args.handoff_event == "torch":
                handoff_ev.record(compute)
                comm_stream.wait_event(handoff_ev)
            else:
                lib.hipEventRecord(handoff_ev, ctypes.c_void_p(stream))
                lib.hipStreamWaitEvent(ctypes.c_void_p(comm_stream.cuda_stream), handoff_ev, ctypes.c_uint(0))
        rc = lib.kacc_allreduce_sums(cl.handle, P([w.tot_e[k0].data_ptr()]), m * ne_row,
                                     P([w.tot_p[k0].data_ptr()]), m * np_row, P([stream]),
                                     P([comm_stream.cuda_stream]))
        if rc != accel.KACC_OK:
            cl._check(rc)

    time_next = lib.kacc_time_next_launch
    region = [0]  # first step of the running region (fused: its first step has no previous sums)

    def step_fused(k, ev=None, markers=False):
        """--totals fused: interval k and, in the same launch, step k - 1's partial sums (from its
        namespace-ordered exports) into step k - 1's rows; a group whose last step is k - 1 is then
        complete and its all-reduce is issued."""
        prev = ctypes.byref(xsums[k - 1]) if k > region[0] else None
        if ev is not None:
            if markers:
                ev[0].record()
            else:
                time_next(acc.ctx, ev[0], ev[1])
        rc = lib.kacc_run_interval_sums(acc.ctx, w.iv_arrays[k], prev, cstream)
        if rc != accel.KACC_OK:
            acc._check(rc)
        if ev is not None and markers:
            ev[1].record()
        if k > region[0] and (k - 1) in group_of:
            flush(group_of[k - 1], k - 1)

    def finish_fused(last):
        """The region's last step's partial sums (one launch), then its group's all-reduce."""
        rc = lib.kacc_run_export_sums(acc.ctx, ctypes.byref(xsums[last]), cstream)
        if rc != accel.KACC_OK:
            acc._check(rc)
        if last in group_of:
            flush(group_of[last], last)

    def step(k, ev=None, markers=False):
        if w.fused_sums:
            return step_fused(k, ev, markers)
        b = k % w.n_bufs
        if used[b] and comm and w.exports:  # exports ablation: wait for step k-2's all-reduce (its buffers are reused)
            compute.wait_event(done[b])
        if ev is not None:
            if markers:
                ev[0].record()
            else:  # start / stop on the interval's kernels' dispatch packets
                time_next(acc.ctx, ev[0], ev[1])
        rc = lib.kacc_run_intervals(acc.ctx, w.iv_arrays[k], K, cstream)
        if rc != accel.KACC_OK:
            acc._check(rc)
        if ev is not None:
            if markers:
                ev[1].record()
            else:  # the totals' partial-sum kernel (compute stream)
                time_next(acc.ctx, ev[2], ev[3])
        rc = reduce_fn(cl.handle, 0 if args.totals_probe == "nodes" else w.n_ns, *ns_args[b])
        if rc != accel.KACC_OK:
            cl._check(rc)
        if ev is not None and markers:
            ev[2].record()  # the compute stream's part of the totals (partial sums, tables mode)
        if not w.exports and k in group_of:
            flush(group_of[k], k)
        if comm and w.exports:
            done[b].record(comm_stream)
        used[b] = True

    def timed(first, evs=None, markers=False):
        """`steps` steps from step index `first`, bracketed by barrier + synchronize: wall seconds."""
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        plan(first, args.steps)
        region[0] = first
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(first + i, evs[i] if evs else None, markers)
        if w.fused_sums:
            finish_fused(first + args.steps - 1)
        torch.cuda.synchronize()  # every all-reduce of the timed steps is inside the timed region
        if world > 1:
            dist.barrier()
        wall = time.perf_counter() - t0
        acc.sync(stream)  # surfaces any device-detected range error
        return wall

    plan(0, args.warmup)
    region[0] = 0
    for k in range(args.warmup):
        step(k)
    if w.fused_sums and args.warmup:
        finish_fused(args.warmup - 1)
    acc.sync(stream)
    torch.cuda.synchronize()
    tevs = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(4)) for _ in range(args.steps)]
    markers = args.step_events == "markers"
    if not markers:  # torch creates an event on its first record; the library re-records it
        for ev in tevs:
            for e in ev:
                e.record()
        torch.cuda.synchronize()
    hev = tevs if markers else [tuple(ctypes.c_void_p(e.cuda_event) for e in ev) for ev in tevs]
    if args.step_events == "separate":
        wall = timed(args.warmup)  # the timed region: kernels and totals only
        wall_ev = timed(args.warmup + args.steps, hev)  # kernel timing: the same steps with launch events
    else:
        wall = wall_ev = timed(args.warmup, hev, markers)
    if w.fused_sums:  # one launch per step: interval + the previous step's sums (no totals launch)
        kernel_ms = [a.elapsed_time(b) / K for a, b, _, _ in tevs]
        totals_ms = []
    elif markers:  # interval, then interval end -> partial sums end
        kernel_ms = [a.elapsed_time(b) / K for a, b, _, _ in tevs]
        totals_ms = [b.elapsed_time(c) for _, b, c, _ in tevs]
    else:  # kernels only: interval start -> end, partial sums start -> end
        kernel_ms = [a.elapsed_time(b) / K for a, b, _, _ in tevs]
        totals_ms = [c.elapsed_time(d) for _, _, c, d in tevs]
    if isinstance(handoff_ev, ctypes.c_void_p):  # the raw device-scope handoff event (ablation)
        torch.cuda.synchronize()
        lib.hipEventDestroy(handoff_ev)
    wall_t = torch.tensor([wall, wall_ev], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(wall_t, op=dist.ReduceOp.MAX)
    return float(wall_t[0].item()), kernel_ms, totals_ms, float(wall_t[1].item())


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.shard_of > 1 and world > 1:
        raise SystemExit("--shard-of emulates one rank's shard on ONE GPU (world 1 only)")
    scaling = "strong" if args.config == 4 else args.scaling

    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local)
    # an explicit stream: the engine launches on it and the HIP events below
    # time exactly that stream (a NULL handle would mean the context's stream)
    torch.cuda.set_stream(torch.cuda.Stream())
    comm_stream = torch.cuda.Stream()  # the cluster all-reduce overlaps the next interval
    if world > 1:  # control plane only (unique id, barriers, max over ranks); data path: RCCL
        dist.init_process_group("gloo")

    from kepler_amd import accel
    from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device

    t_setup = time.time()
    total_nodes = bench_nodes(args.config, world, args.nodes, scaling)
    split = world * args.shard_of
    K = max(1, args.intervals)
    totals_arg = args.totals

    def pick_totals(nodes_per_gpu):  # the shard's node count (plan_node_ranges balances processes)
        if totals_arg == "auto":
            args.totals = "fused" if K == 1 and nodes_per_gpu <= FUSED_MAX_NODES else "tables"

    pick_totals(-(-total_nodes // split))
    w = Workload(args, total_nodes, split, rank, rank, world, local, K, accel.Cluster.unique_id)
    stream = current_stream_handle()
    assert stream != 0
    layout, sizes, Z = w.layout, w.sizes, w.Z
    prime_t = to_device(w.prime)
    w.acc.run_interval(interval_from_tensors(prime_t, sizes), stream)
    w.acc.sync(stream)
    del prime_t
    log(rank, f"[bench] setup {time.time() - t_setup:.1f}s")
    wall_max, kernel_ms, totals_ms, wall_ev = measure(args, w, rank, world, stream, comm_stream)

    # same-box reference for the roofline: a 1.28 GB device-to-device copy
    src = torch.empty(160 * 1024 * 1024, dtype=torch.float64, device="cuda")
    dst = torch.empty_like(src)
    cps = []
    for _ in range(5):
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0.record()
        dst.copy_(src)
        c1.record()
        c1.synchronize()
        cps.append(c0.elapsed_time(c1))
    copy_gbps = 2 * src.numel() * 8 / (float(np.median(cps[1:])) * 1e-3) / 1e9
    del src, dst

    procs_t = torch.tensor([sizes["n_procs"], sizes["n_nodes"]], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(procs_t)
    total_procs, total_nodes_done = (float(x) for x in procs_t.tolist())

    # roofline numerator per interval: the K-interval one-launch path reads the engine state
    # once and carries it on chip, so its algorithmic bytes are fewer (kacc_intervals_bytes)
    fused = accel.fused_intervals(w.flags, K, args.node_order, Z, exports=args.totals != "tables")
    bytes_per_launch = accel.intervals_bytes(Z, sizes["n_nodes"], sizes["n_procs"], sizes["n_ctrs"], sizes["n_vms"],
                                             sizes["n_pods"], K, fused, w.flags) / K
    sums_bytes = export_sums_bytes(Z, sizes["n_nodes"], sizes["n_pods"], w.n_ns) if w.fused_sums else 0
    # the timed region's first launch carries no earlier step's sums (its last step's sums run
    # as a launch of their own, untimed): steps - 1 of the `steps` timed launches move them
    bytes_per_launch += sums_bytes * (args.steps - 1) / args.steps
    k_avg_ms = float(np.mean(kernel_ms))
    achieved = bytes_per_launch / (k_avg_ms * 1e-3) / 1e9

    traffic, traffic_source = pmc_traffic(args, sizes, K, fused, w.fused_sums)
    rccl_version, rccl_path = accel.Cluster.rccl()
    emulated = args.shard_of > 1
    result = {
        "metric": METRIC,
        "value": total_procs * K * args.steps / wall_max,
        "unit": "proc-attr/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall_max * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f64+u64",
        "data": "synthetic (kepler_amd/fleet.py, seed 0x4B45504C; inputs resident in HBM)",
        "config": {
            "workload": f"config{args.config}: {total_nodes}-node fleet"
                        + (f" split {split} ways (plan_node_ranges), {sizes['n_nodes']} nodes x "
                           f"{sizes['n_procs'] // max(sizes['n_nodes'], 1)} procs on this GPU" if split > 1 else
                           f" x {sizes['n_procs'] // max(sizes['n_nodes'], 1)} procs")
                        + f", Z={Z}"
                        + (f", {K} intervals per step (kacc_run_intervals)" if K > 1 else "")
                        + (f", fragmented slots ({args.fragment:g}, node_proc_span)" if args.fragment else "")
                        + (f" [EMULATED: rank 0's shard of a {split}-GPU split, run on one GPU]" if emulated else ""),
            "intervals_per_step": K,
            "fleet_nodes": total_nodes,
            "nodes_per_gpu": sizes["n_nodes"],
            "procs_per_gpu": sizes["n_procs"],
            "containers_per_gpu": sizes["n_ctrs"],
            "vms_per_gpu": sizes["n_vms"],
            "pods_per_gpu": sizes["n_pods"],
            "zones": Z,
            "namespaces": w.n_ns,
            "fragment_slots": args.fragment,
            "shard_of": args.shard_of,
            "cluster_totals": ("kacc_allreduce_exports (interval exports; partial sums + RCCL on the comm stream)"
                               if args.totals == "exports" else
                               f"kacc_run_interval_sums: step k's launch = interval k + step k-1's partial sums "
                               f"(namespace-ordered exports, pod_export_pos); the region's last sums by "
                               f"kacc_run_export_sums; one kacc_allreduce_sums per {max(1, args.allreduce_every)} "
                               f"steps (comm stream)" if w.fused_sums else
                               f"kacc_cluster_partials every step (from the tables, compute stream) + one "
                               f"kacc_allreduce_sums per {max(1, args.allreduce_every)} steps (comm stream)"),
            "allreduce_every": None if args.totals == "exports" else max(1, args.allreduce_every),
            "parallelism": f"node-sharded x{world} (shard.plan_node_ranges); namespace + cluster node "
                           f"totals all-reduced over RCCL inside libkepler_accel",
        },
        "node_snapshots_per_s": total_nodes_done * K * args.steps / wall_max,
        "kernel_ms": k_avg_ms,
        "kernel_ms_steps": [round(x, 5) for x in kernel_ms],
        "step_minus_kernel_ms": wall_max * 1e3 / args.steps - k_avg_ms * K,
        # the partial-sum kernel (launch) / interval end -> its end; fused: inside kernel_ms
        "totals_compute_ms": float(np.mean(totals_ms)) if totals_ms else None,
        "kernel_timing": {
            "step_events": args.step_events,
            "ms_per_step_timing_pass": wall_ev * 1e3 / args.steps,
            "note": ("timed region without event packets; kernel_ms / totals_compute_ms from HIP events on the "
                     "dispatch packets of the interval and totals launches (kacc_time_next_launch, the launch "
                     "stream) over a second timed pass of the same number of steps right after it"
                     if args.step_events == "separate" else
                     "HIP events inside the timed region (" + args.step_events + ")"),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS,
            "traffic": traffic,
            "traffic_source": traffic_source,
            "bytes_per_interval": bytes_per_launch,
            "bytes_per_interval_unfused": accel.interval_bytes(Z, sizes["n_nodes"], sizes["n_procs"], sizes["n_ctrs"],
                                                               sizes["n_vms"], sizes["n_pods"], w.flags),
            "kernel": kernel_name(w.flags, K, fused, Z, w.fused_sums),
            "export_sums_bytes": sums_bytes,
            "same_box_copy_GBps": copy_gbps,
            "frac_of_copy": achieved / copy_gbps,
        },
        "rccl": {"version": rccl_version, "path": rccl_path},
        "cpu_baseline": None,
    }
    if emulated:
        result["note"] = (f"one GPU running rank 0's shard of the {split}-way split: the per-GPU step of an "
                          f"{split}-GPU strong-scaling run without the cross-GPU all-reduce (one-rank communicator)")

    if rank == 0 and world == 1 and not args.no_cpu_baseline and not emulated:
        res, cs_ = cpu_baseline(layout, [w.prime] + w.full, w.node_steps, args.cpu_nodes, args.cpu_seconds,
                                max_runs=args.cpu_runs)
        gf = res["gofaithful"]
        hc = host_cpu()
        result["cpu_baseline"] = {
            "value": gf["value"],
            "unit": "proc-attr/s",
            "cores": 1,
            "kind": "port",
            "sample": f"C++ restatement of the Go path with Go's data structures (oracle/kor_gf_interval: "
                      f"string-keyed maps, per-object zone maps), 1 thread, first {cs_['n_nodes']} nodes of the "
                      f"same fleet ({cs_['n_procs']} procs, Z={Z}) per run: median of {gf['runs']} timed runs "
                      f"after a warm-up ({gf['seconds']:.1f} s)",
            "cpu_model": hc["model"],
            "nproc": hc["nproc"],
            "usable_cores": hc["usable"],
            "median_s": gf["median_s"],
            "runs": gf["runs"],
            "soa_port_1thread": res["soa"]["value"],
            "soa_port_threads": {"value": res["soa_mt"]["value"], "threads": res["soa_mt"]["threads"],
                                 "threads_source": res["soa_mt"]["share_source"],
                                 "usable_cores": hc["usable"],
                                 "runs": res["soa_mt"]["runs"],
                                 "sample": f"{res['soa_mt']['procs']} procs per run, median of "
                                           f"{res['soa_mt']['runs']} runs",
                                 "note": "the flat-array C++ port over node ranges, one host thread per CPU this "
                                         "job may use (threads_source); usable_cores is the whole host's "
                                         "affinity mask, shared with the other GPUs' jobs"},
        }
        result["cpu_baseline"]["gpu_over_cpu"] = result["value"] / gf["value"]
    if world == 1:
        try:
            result["scrape_powers"] = scrape_line(w.acc, w.sizes["n_procs"], Z)
        except Exception as e:  # a secondary line: report, never lose the headline
            result["scrape_powers"] = {"error": repr(e)}
        sp = result["scrape_powers"]
        if "ms" in sp:  # beside `value`: the same steps with every interval's process powers scraped
            step_ms = result["ms_per_step"] + K * sp["ms"]
            extra = {"value_with_scrape": total_procs * K / (step_ms * 1e-3),
                     "value_note": "value: intervals attributed, process Usage.Power derived on read (not "
                                   "materialised); value_with_scrape: the same steps plus one kacc_table_read of "
                                   "every process power per interval (scrape_powers.ms each)"}
            items = list(result.items())
            at = [k for k, _ in items].index("value") + 1
            result.clear()
            result.update(items[:at] + list(extra.items()) + items[at:])
    w.close()
    del w

    if world > 1 and scaling == "strong" and args.weak_line and args.config in (1, 2, 3, 5):
        # extra key: every rank a full shard of its own (weak scaling), the same timed loop
        pick_totals(bench_nodes(args.config, world, args.nodes, "weak") // world)
        wk = Workload(args, bench_nodes(args.config, world, args.nodes, "weak"), world, rank, rank, world, local, K,
                      accel.Cluster.unique_id)
        prime_t = to_device(wk.prime)
        wk.acc.run_interval(interval_from_tensors(prime_t, wk.sizes), stream)
        wk.acc.sync(stream)
        del prime_t
        wwall, wkms, _, _ = measure(args, wk, rank, world, stream, comm_stream)
        wp = torch.tensor([wk.sizes["n_procs"]], dtype=torch.float64)
        dist.all_reduce(wp)
        result["weak_scaling"] = {"value": float(wp.item()) * K * args.steps / wwall, "unit": "proc-attr/s",
                                  "totals": args.totals,
                                  "ms_per_step": wwall * 1e3 / args.steps, "kernel_ms": float(np.mean(wkms)),
                                  "nodes_per_gpu": wk.sizes["n_nodes"],
                                  "fleet_nodes": bench_nodes(args.config, world, args.nodes, "weak")}
        wk.close()
        del wk

    if world == 1 and args.frag_line > 0 and args.fragment == 0 and args.config in (1, 2, 3) and not emulated:
        try:
            result["slot_layouts"] = slot_layout_lines(args, args.frag_line, K, min(args.steps, 10),
                                                       bytes_per_launch)
        except Exception as e:  # a secondary line: report, never lose the headline
            result["slot_layouts"] = {"error": repr(e)}
        sl_ = result["slot_layouts"]
        if "join_steady_state_span" in sl_:  # the headline kernel on the layout production runs on
            result["production_layout"] = {
                "kernel_ms": sl_["join_steady_state_span"]["kernel_ms"],
                "frac": sl_["join_steady_state_span"]["frac"],
                "over_pristine": sl_["join_steady_state_over_pristine"],
                "note": "the same kernel and algorithmic bytes on the slot words and spans kacc_slot_join "
                        "(KACC_JOIN_REUSE_TERMINATED) returns after 40 intervals of 2 % /proc-shaped churn, "
                        "timed on one context beside pristine slots (slot_layouts)"}

    if world == 1 and args.pipeline_line and args.fragment == 0 and args.config == 3 and K == 1 and not emulated:
        try:
            result["pipeline"] = pipeline_line(args)
        except Exception as e:  # a secondary line: report, never lose the headline
            result["pipeline"] = {"error": repr(e)}

    if world == 1 and args.host_line and args.fragment == 0 and args.config == 3 and K == 1 and not emulated:
        try:
            result["host_path"] = host_path_line(args)
        except Exception as e:  # a secondary line: report, never lose the headline
            result["host_path"] = {"error": repr(e)}
        try:
            result["host_path_ticks"] = host_path_ticks_line(args)
        except Exception as e:  # a secondary line: report, never lose the headline
            result["host_path_ticks"] = {"error": repr(e)}

    if rank == 0:
        line = json.dumps(result)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.destroy_process_group()


def export_sums_bytes(Z, n_nodes, n_pods, n_ns):
    """Algorithmic bytes --totals fused adds to a launch: the interval's exports
    written (pod records 16Z B in namespace order, node rows 40Z B) and the previous
    interval's read by the sums blocks (the same records, the namespace offsets), plus the
    partial-sum outputs (16Z B per namespace, 40Z B of node totals)."""
    exports = n_pods * 16 * Z + n_nodes * 40 * Z
    return 2 * exports + 4 * (n_ns + 1) + n_ns * 16 * Z + 40 * Z


def kernel_name(flags, K, fused, Z, sums=False):
    from kepler_amd import accel

    if sums and not flags & accel.KACC_F_SMALL_NODES:
        return (f"kacc::interval_sums_kernel<{Z},0> (one launch per step: the interval, its exports in namespace "
                f"order, and the previous interval's cluster partial sums in the tail blocks; achieved counts "
                f"export_sums_bytes too)")
    if fused:
        return (f"kacc::intervals_carry_kernel<{Z},0,{256 if flags & accel.KACC_F_MEDIUM_NODES else 512}>"
                f" ({K} intervals in one launch, state carried on chip; "
                f"achieved = kacc_intervals_bytes(carried) / K per interval)")
    if flags & accel.KACC_F_SMALL_NODES:
        return (f"kacc::small_kernel<{Z}> (one launch per step, one wavefront per node: every node "
                f"fits KACC_F_SMALL_NODES)")
    if flags & accel.KACC_F_FAST_NODES:
        return f"kacc::interval_kernel<{Z},0> (one launch per step: every node fits the fast path, KACC_F_FAST_NODES)"
    return (f"kacc::interval_kernel<{Z},0> + chunk_kernel<{Z},0> + pod_kernel<{Z},0> (big nodes "
            f"chunked; HIP events bracket all three launches of the step)")


def lib_sha256():
    import hashlib

    from kepler_amd import accel

    with open(accel.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def pmc_traffic(args, sizes, K, fused, sums=False):
    """roofline.traffic: HBM bytes per interval from profiles/pmc_traffic.json (rocprofv3 --pmc
    FETCH_SIZE x 2 + WRITE_SIZE, tools/pmc_summary.py) ONLY when that entry was measured on this
    very build (sha256 of libkepler_accel.so) and these sizes; otherwise null, with the reason."""
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    key = (f"config{args.config}" + (f"_frag{args.fragment:g}" if args.fragment else "")
           + (f"_k{K}" if fused else "") + ("_sums" if sums else ""))
    if not os.path.exists(pmc_path):
        return None, "no profiles/pmc_traffic.json"
    with open(pmc_path) as f:
        ent = json.load(f).get(key)
    if not ent:
        return None, f"no PMC entry {key}"
    if ent.get("n_procs") != sizes["n_procs"]:
        return None, f"PMC entry {key} is for {ent.get('n_procs')} procs, not {sizes['n_procs']}"
    sha = lib_sha256()
    if ent.get("lib_sha256") != sha:
        return None, (f"PMC entry {key} was measured on build {str(ent.get('lib_sha256'))[:16]}, not this build "
                      f"{sha[:16]}: no counters of this build")
    return ent.get("hbm_bytes_per_interval", ent.get("hbm_bytes_per_launch")), ent.get("source")


if __name__ == "__main__":
    main()
