#!/usr/bin/env python3
"""Benchmark: Kepler power attribution on MI355X (BASELINE.json metric).

One *step* = one collection interval (PowerMonitor.calculatePower,
internal/monitor/monitor.go:399-431) over the whole fleet shard of a GPU:
node split + segmented CPU-time sums + process/container/VM/pod attribution
(one kacc_run_interval launch) followed by the cluster namespace totals
(kacc_namespace_totals, then an RCCL all-reduce across GPUs when N > 1).

Workload: BASELINE config 3 per GPU — 10k nodes x 2k processes, Z = 4 RAPL
zones (package/core/uncore/dram), ~1.6k container processes / 200 containers /
71 pods / 20 VMs per node, synthetic inputs (kepler_amd/fleet.py) resident in
HBM before timing.  Scaling is weak: every rank owns its own 10k-node shard
(node snapshots are independent), so N GPUs process N x 20M process rows per
interval; only the namespace totals cross GPUs.

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
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def cpu_baseline(layout, intervals, node_steps, n_nodes, seconds):
    """Go-faithful oracle (C++ restatement with Go's data structures), 1 thread."""
    from kepler_amd import fleet
    from oracle.oracle import GoFaithful, Oracle

    nodes = np.arange(min(n_nodes, layout.n_nodes))
    subs = [fleet.subset_interval(a, nodes, layout.zones) for a in intervals]
    _, sizes, _ = subs[0]
    caps = dict(nodes=sizes["n_nodes"], proc_slots=sizes["n_procs"], ctr_slots=sizes["n_ctrs"],
                vm_slots=sizes["n_vms"], pod_slots=sizes["n_pods"])
    out = {}
    for name, cls in (("gofaithful", GoFaithful), ("soa", Oracle)):
        o = cls(layout.zones, **caps)
        o.interval(subs[0][0], sizes)  # first read (untimed, as on the GPU)
        done, t_run, k = 0, 0.0, 0
        budget = seconds if name == "gofaithful" else min(seconds, 5.0)
        while t_run < budget:
            a = dict(subs[1 + k % (len(subs) - 1)][0])
            na = node_steps[k % len(node_steps)]
            for key in ("node_ts_ns", "node_usage_ratio", "node_status"):
                a[key] = np.ascontiguousarray(na[key][nodes])
            zidx = (nodes[:, None] * layout.zones + np.arange(layout.zones)).reshape(-1)
            a["zone_energy"] = np.ascontiguousarray(na["zone_energy"][zidx])
            t0 = time.perf_counter()
            o.interval(a, sizes)
            t_run += time.perf_counter() - t0
            done += sizes["n_procs"]
            k += 1
        out[name] = dict(value=done / t_run, intervals=k, seconds=t_run)
    # the flat-array port on the host's cores (node ranges per thread), on a
    # 10x larger node sample: the strongest CPU number this repo can produce
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))))
    nodes_mt = np.arange(min(10 * n_nodes, layout.n_nodes))
    subs_mt = [fleet.subset_interval(a, nodes_mt, layout.zones) for a in intervals[:3]]
    _, sizes_mt, _ = subs_mt[0]
    o = Oracle(layout.zones, nodes=sizes_mt["n_nodes"], proc_slots=sizes_mt["n_procs"],
               ctr_slots=sizes_mt["n_ctrs"], vm_slots=sizes_mt["n_vms"], pod_slots=sizes_mt["n_pods"])
    o.interval_mt(subs_mt[0][0], sizes_mt, threads)
    done, t_run, k = 0, 0.0, 0
    while t_run < 5.0:
        a = subs_mt[1 + k % 2][0]
        t0 = time.perf_counter()
        o.interval_mt(a, sizes_mt, threads)
        t_run += time.perf_counter() - t0
        done += sizes_mt["n_procs"]
        k += 1
    out["soa_mt"] = dict(value=done / t_run, threads=threads, intervals=k, procs=sizes_mt["n_procs"])
    return out, sizes


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    # rehearsal of the N > 1 logic on a one-GPU box (never the driver's runs):
    # KACC_BENCH_BACKEND=gloo KACC_BENCH_DEVICE=0 puts every rank on one device
    backend = os.environ.get("KACC_BENCH_BACKEND", "nccl")
    dev = int(os.environ.get("KACC_BENCH_DEVICE", local))
    torch.cuda.set_device(dev)
    # an explicit stream: the engine launches on it and the HIP events below
    # time exactly that stream (a NULL handle would mean the context's stream)
    torch.cuda.set_stream(torch.cuda.Stream())
    if world > 1:
        if backend == "nccl":  # RCCL over xGMI
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)

    from kepler_amd import accel, fleet
    from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device

    t_setup = time.time()
    nodes = args.nodes or {1: 40000, 2: 1000, 3: 10000, 4: -(-100000 // world), 5: 1000}[args.config]
    layout = fleet.config_layout(args.config, seed=fleet.SEED + 7919 * rank, nodes=nodes)
    sim = fleet.FleetSim(layout, seed=fleet.SEED + 7919 * rank)
    Z = layout.zones
    sizes = layout.sizes()
    log(rank, f"[bench] layout {sizes} Z={Z} built in {time.time() - t_setup:.1f}s")

    K = max(1, args.intervals)
    n_steps = args.warmup + args.steps
    n_ivs = n_steps * K  # every interval has its own node counters / clocks
    n_distinct = max(1, min(args.distinct, n_ivs))
    prime = sim.next_interval()  # first read (monitor.go:326-330), untimed
    full = [sim.next_interval() for _ in range(n_distinct)]
    node_steps = [full[k] if k < n_distinct else sim.next_node_inputs() for k in range(n_ivs)]
    log(rank, f"[bench] inputs generated in {time.time() - t_setup:.1f}s")

    acc = accel.Accel(Z, **layout.capacities(), device=dev)
    stream = current_stream_handle()
    assert stream != 0
    statics = to_device(layout.static_arrays())
    dev_full = [to_device({k: a[k] for k in ("proc_cpu_delta", "proc_slot", "ctr_slot", "vm_slot", "pod_slot")})
                for a in full]
    node_keys = ("node_ts_ns", "node_usage_ratio", "node_status", "zone_energy", "zone_max")
    dev_nodes = [to_device({k: a[k] for k in node_keys}) for a in node_steps]
    order = to_device({"o": layout.node_order_heaviest_first()})["o"] if args.node_order else None

    def make(k):
        t = dict(statics)
        t.update(dev_full[k % n_distinct])
        t.update(dev_nodes[k])
        if order is not None:
            t["node_order"] = order
        return t

    iv_tensors = [make(k) for k in range(n_ivs)]
    ivs = [interval_from_tensors(t, sizes, layout.fast_flag()) for t in iv_tensors]
    prime_t = to_device(prime)
    acc.run_interval(interval_from_tensors(prime_t, sizes), stream)
    acc.sync(stream)
    del prime_t

    ns_off, ns_slot = layout.namespace_csr()
    ns_t = to_device({"off": ns_off, "slot": ns_slot})
    n_ns = len(ns_off) - 1
    # namespace totals double-buffered: step k's RCCL all-reduce (async, on the
    # process group's stream) overlaps step k+1's interval kernel; buffer k % 2
    # is rewritten only after the all-reduce of step k-2 has been waited for.
    ns_e = [torch.zeros(n_ns * Z, dtype=torch.int64, device="cuda") for _ in range(2)]
    ns_p = [torch.zeros(n_ns * Z, dtype=torch.float64, device="cuda") for _ in range(2)]
    pending = [None, None]

    def step(k, ev=None):
        if ev is not None:
            ev[0].record()
        if K == 1:
            acc.run_interval(ivs[k], stream)
        else:  # K consecutive intervals, back to back from C
            acc.run_intervals(ivs[k * K:(k + 1) * K], stream)
        if ev is not None:
            ev[1].record()
        b = k % 2
        if pending[b] is not None:  # stream-level wait (no host sync)
            for w in pending[b]:
                w.wait()
            pending[b] = None
        acc.namespace_totals(n_ns, ns_t["off"].data_ptr(), ns_t["slot"].data_ptr(), ns_e[b].data_ptr(),
                             ns_p[b].data_ptr(), stream)
        if world > 1:  # cluster-wide namespace totals over xGMI (RCCL): u64 sum is exact
            pending[b] = [dist.all_reduce(ns_e[b], async_op=True), dist.all_reduce(ns_p[b], async_op=True)]

    def drain():
        for b in range(2):
            if pending[b] is not None:
                for w in pending[b]:
                    w.wait()
                pending[b] = None

    for k in range(args.warmup):
        step(k)
    drain()
    acc.sync(stream)
    torch.cuda.synchronize()
    log(rank, f"[bench] warmup done, setup {time.time() - t_setup:.1f}s")

    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i, events[i])
    drain()  # every all-reduce of the timed steps is inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    acc.sync(stream)  # surfaces any device-detected range error
    kernel_ms = [a.elapsed_time(b) / K for a, b in events]  # per interval

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

    wall_t = torch.tensor([wall], dtype=torch.float64, device="cuda")
    procs_t = torch.tensor([sizes["n_procs"], sizes["n_nodes"]], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(wall_t, op=dist.ReduceOp.MAX)
        dist.all_reduce(procs_t)
    wall_max = float(wall_t.item())
    total_procs, total_nodes = (float(x) for x in procs_t.tolist())

    bytes_per_launch = accel.interval_bytes(Z, sizes["n_nodes"], sizes["n_procs"], sizes["n_ctrs"],
                                            sizes["n_vms"], sizes["n_pods"])
    k_avg_ms = float(np.mean(kernel_ms))
    achieved = bytes_per_launch / (k_avg_ms * 1e-3) / 1e9

    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            pmc = json.load(f)
        ent = pmc.get(f"config{args.config}")
        if ent and ent.get("n_procs") == sizes["n_procs"]:
            traffic = ent.get("hbm_bytes_per_launch")

    result = {
        "metric": METRIC,
        "value": total_procs * K * args.steps / wall_max,
        "unit": "proc-attr/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall_max * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "strong" if args.config == 4 else "weak",
        "vs_baseline": None,
        "dtype": "f64+u64",
        "data": "synthetic (kepler_amd/fleet.py, seed 0x4B45504C; inputs resident in HBM)",
        "config": {
            "workload": f"config{args.config}: {sizes['n_nodes']} nodes x "
                        f"{sizes['n_procs'] // max(sizes['n_nodes'], 1)} procs, Z={Z} per GPU"
                        + (f", {K} intervals per step (kacc_run_intervals)" if K > 1 else ""),
            "intervals_per_step": K,
            "nodes_per_gpu": sizes["n_nodes"],
            "procs_per_gpu": sizes["n_procs"],
            "containers_per_gpu": sizes["n_ctrs"],
            "vms_per_gpu": sizes["n_vms"],
            "pods_per_gpu": sizes["n_pods"],
            "zones": Z,
            "namespaces": n_ns,
            "parallelism": f"node-sharded x{world} (namespace totals all-reduced over "
                           f"{'RCCL' if backend == 'nccl' else backend})",
        },
        "node_snapshots_per_s": total_nodes * K * args.steps / wall_max,
        "kernel_ms": k_avg_ms,
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS,
            "traffic": traffic,
            "bytes_per_launch": bytes_per_launch,
            "kernel": (f"kacc::small_kernel<{Z}> (one launch per step, one wavefront per node: every node "
                       f"fits KACC_F_SMALL_NODES)" if layout.fast_flag() & accel.KACC_F_SMALL_NODES else
                       f"kacc::interval_kernel<{Z},0> (one launch per step: every node fits the fast path, "
                       f"KACC_F_FAST_NODES)" if layout.fast_flag() else
                       f"kacc::interval_kernel<{Z},0> + chunk_kernel<{Z},0> + pod_kernel<{Z},0> (big nodes "
                       f"chunked; HIP events bracket all three launches of the step)"),
            "same_box_copy_GBps": copy_gbps,
            "frac_of_copy": achieved / copy_gbps,
        },
        "cpu_baseline": None,
    }

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res, cs = cpu_baseline(layout, [prime] + full, node_steps, args.cpu_nodes, args.cpu_seconds)
        gf = res["gofaithful"]
        result["cpu_baseline"] = {
            "value": gf["value"],
            "unit": "proc-attr/s",
            "cores": 1,
            "kind": "port",
            "sample": f"go-faithful C++ restatement of the Go path (oracle/kor_gf_interval: string-keyed "
                      f"maps, per-object zone maps), first {cs['n_nodes']} nodes of the same fleet "
                      f"({cs['n_procs']} procs, Z={Z}), {gf['intervals']} intervals in {gf['seconds']:.1f}s",
            "soa_port_1thread": res["soa"]["value"],
            "soa_port_threads": {"value": res["soa_mt"]["value"], "threads": res["soa_mt"]["threads"],
                                 "sample": f"{res['soa_mt']['procs']} procs, {res['soa_mt']['intervals']} intervals"},
        }
        result["cpu_baseline"]["gpu_over_cpu"] = result["value"] / gf["value"]

    if rank == 0:
        line = json.dumps(result)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    acc.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
