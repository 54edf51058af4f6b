"""Multi-process path on CPU: node-sharded ranks + all-reduced namespace totals (gloo, world 2).

The GPU run uses one process per GPU and RCCL; the sharding plan and the
reduction are the same code paths, exercised here with the oracle standing in
for the engine on each rank (no GPU in this container).
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kepler_amd import fleet, shard
    from oracle.oracle import Oracle

    L = fleet.make_layout(24, [300, 2000, 5, 0, 700, 64] * 4, 4, seed=31, n_namespaces=6, shuffle_slots=True)
    sim = fleet.FleetSim(L, seed=31, churn=0.05, read_error_frac=0.05)
    lo, hi, sl = shard.shard(L, world)[rank]
    o = Oracle(L.zones, **sl.capacities())
    for _ in range(3):
        a = sim.next_interval()  # every rank replays the same fleet inputs
        sub, sizes, _ = fleet.subset_interval(a, np.arange(lo, hi), L.zones)
        o.interval(sub, sizes)
    e, p = o.namespace_totals(*sl.namespace_csr())
    te = torch.from_numpy(e.view(np.int64).copy())
    tp = torch.from_numpy(p.copy())
    dist.all_reduce(te)  # two's-complement int64 sum == modular u64 sum
    dist.all_reduce(tp)
    if rank == 0:
        np.save(os.path.join(out_dir, "e.npy"), te.numpy().view(np.uint64))
        np.save(os.path.join(out_dir, "p.npy"), tp.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_namespace_totals(tmp_path, oracle_lib):
    from kepler_amd import fleet
    from oracle.oracle import Oracle

    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    L = fleet.make_layout(24, [300, 2000, 5, 0, 700, 64] * 4, 4, seed=31, n_namespaces=6, shuffle_slots=True)
    sim = fleet.FleetSim(L, seed=31, churn=0.05, read_error_frac=0.05)
    o = Oracle(L.zones, **L.capacities())
    for _ in range(3):
        o.interval(sim.next_interval(), L.sizes())
    e_full, p_full = o.namespace_totals(*L.namespace_csr())
    np.testing.assert_array_equal(np.load(tmp_path / "e.npy"), e_full)
    np.testing.assert_allclose(np.load(tmp_path / "p.npy"), p_full, rtol=1e-12)


def _bench_worker(rank, world, port, out_dir):
    """bench.py's N > 1 control logic on gloo: the rank-0 unique id reaches every rank,
    and every rank generates only its plan_node_ranges cut of the fleet."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from kepler_amd import fleet

    uid = bench.exchange_unique_id(rank, world, lambda: bytes(range(128)))
    res = {}
    for config in (3, 4, 5):
        total = bench.bench_nodes(config, world, nodes=60 if config != 4 else 90)
        lo, hi, L = fleet.config_shard(config, world, rank, total)
        assert L.n_namespaces == total  # every shard indexes the whole fleet's namespaces
        res[config] = (lo, hi, L.n_nodes, L.n_procs, total)
    np.save(os.path.join(out_dir, f"r{rank}.npy"), np.array([uid == bytes(range(128))] +
                                                            [x for c in (3, 4, 5) for x in res[c]], dtype=np.int64))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_control_plane_two_ranks(tmp_path):
    from kepler_amd import fleet, shard

    world = 2
    mp.start_processes(_bench_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    rows = [np.load(tmp_path / f"r{r}.npy") for r in range(world)]
    assert all(r[0] == 1 for r in rows)  # both ranks hold rank 0's id
    for j, config in enumerate((3, 4, 5)):
        got = [r[1 + 5 * j: 6 + 5 * j] for r in rows]
        total = got[0][4]
        b = shard.plan_node_ranges(fleet.config_procs_per_node(config, int(total)), world)
        for r in range(world):
            lo, hi, n_nodes, n_procs, _ = got[r]
            assert (lo, hi) == (b[r], b[r + 1]) and n_nodes == hi - lo
            assert n_procs == fleet.config_procs_per_node(config, int(total))[lo:hi].sum()
        assert got[0][0] == 0 and got[-1][1] == total  # the ranks tile the fleet
    # strong scaling by default (one fixed fleet cut N ways); weak = N x the fleet
    assert rows[0][1 + 4] == 60 and rows[0][6 + 4] == 90 and rows[0][11 + 4] == 60
    import bench

    assert bench.bench_nodes(3, 2, 60, "weak") == 120 and bench.bench_nodes(4, 2, 90, "weak") == 90


def test_bench_allreduce_groups():
    """bench.py's schedule of the grouped cluster all-reduce (kacc_allreduce_sums over K steps'
    rows): every step of a region in exactly one group, in order, contiguous, at most `group`
    steps each, and the region's last step alone (one step's rows left after its last interval).
    Every rank derives the same schedule from its arguments, so the collectives match."""
    import bench

    assert bench.allreduce_groups(0, 20, 8) == [(0, 7), (8, 15), (16, 18), (19, 19)]
    assert bench.allreduce_groups(23, 20, 8) == [(23, 30), (31, 38), (39, 41), (42, 42)]
    assert bench.allreduce_groups(0, 3, 8) == [(0, 1), (2, 2)]
    assert bench.allreduce_groups(5, 1, 8) == [(5, 5)]
    assert bench.allreduce_groups(0, 0, 8) == []
    assert bench.allreduce_groups(0, 4, 1) == [(0, 0), (1, 1), (2, 2), (3, 3)]
    for first, n, g in [(0, 20, 8), (3, 50, 7), (0, 17, 16), (9, 2, 3), (0, 64, 0)]:
        gs = bench.allreduce_groups(first, n, g)
        assert [k for a, b in gs for k in range(a, b + 1)] == list(range(first, first + n))
        assert all(b - a + 1 <= max(1, g) for a, b in gs) and gs[-1][0] == gs[-1][1]
