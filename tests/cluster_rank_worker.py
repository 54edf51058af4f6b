"""One rank of the nranks > 1 cluster test (tests/test_gpu_cluster_ranks.py) — MI355X only.

Every rank is its own process on the box's one GPU, as bench.py --gpus N runs one process
per GPU: it owns its node shard of a fleet (shard.plan_node_ranges), runs the intervals on
its own engine context, joins the cluster through kacc_cluster_unique_id (rank 0, handed
over a file) + kacc_cluster_join(nranks, rank), and then calls the library's cross-rank
entry points:
  * kacc_allreduce_namespaces (namespace + cluster node totals, comm stream),
  * kacc_cluster_partials per interval into rows + ONE kacc_allreduce_sums,
  * kacc_gather_pods (count all-gather, then one broadcast per rank).
The results go to <out>/rank<r>.npz for the parent test to check against the unsharded
oracle.  The collectives are RCCL's entry points from the file KACC_RCCL_PATH names (the
loopback stand-in, tests/c/loopback_rccl.cpp) or the system RCCL.

  python tests/cluster_rank_worker.py RANK NRANKS OUTDIR
"""

import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# the fleet every rank cuts (the parent builds the same one for its oracle)
FLEET = dict(n_nodes=48, procs_per_node=[2000, 300, 0, 1, 4096, 700, 12000, 64] * 6, zones=4, seed=47,
             n_namespaces=7, vm_frac=0.03, procs_per_vm=2, shuffle_slots=True)
SIM = dict(seed=47, churn=0.04, read_error_frac=0.05)
INTERVALS = 4


def main():
    rank, nranks, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    import torch

    from kepler_amd import accel, fleet, shard
    from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device

    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    kw = dict(FLEET)
    L = fleet.make_layout(kw.pop("n_nodes"), kw.pop("procs_per_node"), kw.pop("zones"), **kw)
    lo, hi, sl = shard.shard(L, nranks)[rank]
    Z, n_ns = L.zones, L.n_namespaces
    acc = accel.Accel(Z, **sl.capacities())
    sim = fleet.FleetSim(L, **SIM)
    s = current_stream_handle()
    comm = torch.cuda.Stream()

    # the unique id: rank 0's, handed to the others over a file (bench.py: torch.distributed)
    uid_path = os.path.join(out, "uid.bin")
    if rank == 0:
        uid = accel.Cluster.unique_id()
        with open(uid_path + ".tmp", "wb") as f:
            f.write(uid)
        os.rename(uid_path + ".tmp", uid_path)
    else:
        deadline = time.time() + 120
        while not os.path.exists(uid_path):
            if time.time() > deadline:
                raise SystemExit("rank %d: no unique id from rank 0" % rank)
            time.sleep(0.05)
        with open(uid_path, "rb") as f:
            uid = f.read()
    cl = accel.Cluster.join(acc, uid, nranks, rank)
    info = cl.info()

    off, slots = sl.namespace_csr()
    csr = to_device({"o": off, "s": slots})
    ne_row, np_row = n_ns * Z + 2 * Z, n_ns * Z + 3 * Z
    te = torch.zeros(INTERVALS, ne_row, dtype=torch.int64, device="cuda")
    tp = torch.zeros(INTERVALS, np_row, dtype=torch.float64, device="cuda")
    keep = []
    for k in range(INTERVALS):
        a = sim.next_interval()
        sub, sizes, _ = fleet.subset_interval(a, np.arange(lo, hi), Z)
        t = to_device(sub)
        keep.append(t)
        acc.run_interval(interval_from_tensors(t, sizes, sl.fast_flag()), s)
        # this interval's partial sums into its own row (no collective yet)
        cl.partials(n_ns, [csr["o"].data_ptr()], [csr["s"].data_ptr()], [te[k].data_ptr()], [tp[k].data_ptr()],
                    [te[k, n_ns * Z:].data_ptr()], [tp[k, n_ns * Z:].data_ptr()], streams=[s])
    # ONE all-reduce of every interval's rows (one collective per K intervals)
    cl.allreduce_sums([te.data_ptr()], INTERVALS * ne_row, [tp.data_ptr()], INTERVALS * np_row, streams=[s],
                      comm_streams=[comm.cuda_stream])
    # the last interval's totals through the one-call entry point
    oe = torch.zeros(n_ns * Z, dtype=torch.int64, device="cuda")
    op = torch.zeros(n_ns * Z, dtype=torch.float64, device="cuda")
    ne = torch.zeros(2 * Z, dtype=torch.int64, device="cuda")
    npw = torch.zeros(3 * Z, dtype=torch.float64, device="cuda")
    cl.allreduce_namespaces(n_ns, [csr["o"].data_ptr()], [csr["s"].data_ptr()], [oe.data_ptr()], [op.data_ptr()],
                            [ne.data_ptr()], [npw.data_ptr()], streams=[s], comm_streams=[comm.cuda_stream])
    # every pod of the cluster in (rank, pod) order
    pslot = to_device({"s": sl.pod_slot})["s"]
    ge = torch.zeros(max(L.n_pods, 1) * Z, dtype=torch.int64, device="cuda")
    gp = torch.zeros(max(L.n_pods, 1) * Z, dtype=torch.float64, device="cuda")
    total, first = cl.gather_pods([sl.n_pods], [pslot.data_ptr()], L.n_pods, [ge.data_ptr()], [gp.data_ptr()],
                                  streams=[s])
    torch.cuda.synchronize()
    acc.sync(s)
    np.savez(os.path.join(out, f"rank{rank}.npz"), info=np.array(info), lo=lo, hi=hi,
             te=te.cpu().numpy().view(np.uint64), tp=tp.cpu().numpy(),
             oe=oe.cpu().numpy().view(np.uint64), op=op.cpu().numpy(),
             ne=ne.cpu().numpy().view(np.uint64), npw=npw.cpu().numpy(),
             ge=ge.cpu().numpy().view(np.uint64), gp=gp.cpu().numpy(), total=total, first=np.array(first),
             rccl=np.array(str(accel.Cluster.rccl())))
    cl.close()
    acc.close()
    print(f"rank {rank} of {nranks}: ok ({info})", flush=True)


if __name__ == "__main__":
    main()
