"""Device multi-socket AggregatedZone (kacc_zone_agg_*) against the oracle — MI355X only.

Integer work: bit-exact.  The reference's own energy_zone_test.go cases
(kat_cases.json "aggregated") run through the kernel, then random fleets with
counter wraps, zero MaxEnergy sub-zones and read errors, then the aggregated
counters feed the interval kernel end to end.
"""

import numpy as np
import pytest
import torch

from kat_runner import load_kats
from kepler_amd import accel, fleet
from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device
from oracle.oracle import Oracle, OracleZoneAgg

pytestmark = pytest.mark.gpu
KATS = load_kats()


@pytest.fixture(scope="module", autouse=True)
def gpu_ready():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    accel.load()
    torch.cuda.set_stream(torch.cuda.Stream())


def dev(a, dt):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=dt).view({np.uint64: np.int64, np.uint32: np.int32}[dt])).cuda()


class GpuAgg:
    def __init__(self, acc, n_nodes, sockets, sub_max):
        self.acc, self.N, self.Z = acc, n_nodes, acc.zones
        self.z = accel.ZoneAgg(acc, n_nodes, sockets, sub_max)
        self.e = torch.zeros(n_nodes * self.Z, dtype=torch.int64, device="cuda")
        self.m = torch.zeros(n_nodes * self.Z, dtype=torch.int64, device="cuda")
        self.st = torch.zeros(n_nodes, dtype=torch.int32, device="cuda")

    def read(self, readings, sub_status=None, sync=True, zero_status=True):
        r = dev(readings, np.uint64)
        s = None if sub_status is None else dev(sub_status, np.uint32)
        if zero_status:
            self.st.zero_()
        h = current_stream_handle()
        self.z.read(r.data_ptr(), 0 if s is None else s.data_ptr(), self.e.data_ptr(), self.m.data_ptr(),
                    self.st.data_ptr(), h)
        if not sync:
            return r, s
        self.acc.sync(h)
        return (self.e.cpu().numpy().view(np.uint64), self.m.cpu().numpy().view(np.uint64),
                self.st.cpu().numpy().view(np.uint32))


@pytest.mark.parametrize("case", KATS["aggregated"], ids=lambda c: c["name"])
def test_aggregated_zone_kat_on_device(case):
    acc = accel.Accel(1, nodes=1, proc_slots=1, ctr_slots=1, vm_slots=1, pod_slots=1)
    g = GpuAgg(acc, 1, len(case["max"]), np.array(case["max"], dtype=np.uint64))
    for reads, want in zip(case["reads"], case["expect"]):
        e, m, st = g.read(np.array(reads, dtype=np.uint64))
        assert int(e[0]) == want and int(m[0]) == case["agg_max"] and st[0] == 0


@pytest.mark.parametrize("N,Z,S", [(64, 4, 2), (300, 2, 4), (5, 8, 1)])
def test_aggregated_zone_fleet_bit_exact(N, Z, S):
    rng = np.random.default_rng(N * 10 + S)
    sub_max = rng.integers(10**6, 10**9, size=N * Z * S).astype(np.uint64)
    sub_max[rng.random(sub_max.size) < 0.05] = 0  # invalid MaxEnergy: underflow kept
    acc = accel.Accel(Z, nodes=N, proc_slots=1, ctr_slots=1, vm_slots=1, pod_slots=1)
    g, o = GpuAgg(acc, N, S, sub_max), OracleZoneAgg(N, Z, S, sub_max)
    cnt = (rng.random(sub_max.size) * np.maximum(sub_max, 1)).astype(np.uint64)
    for it in range(8):
        step = rng.integers(0, 4 * 10**8, size=cnt.size).astype(np.uint64)
        cnt = np.where(sub_max > 0, (cnt + step) % np.maximum(sub_max, 1), cnt + step).astype(np.uint64)
        if it == 5:
            cnt[::7] = cnt[::7] // 2  # backward readings
        st = (rng.random(cnt.size) < 0.02).astype(np.uint32) if it >= 2 else None
        ge, gm, gs = g.read(cnt, st)
        oe, om, os_ = o.read(cnt, st)
        np.testing.assert_array_equal(gm, om)
        np.testing.assert_array_equal(gs, os_, err_msg=f"read {it}")
        ok = np.repeat(os_ == 0, Z)  # a failed zone's output is undefined; its node is skipped
        failed = np.zeros(N * Z, bool)
        if st is not None:
            failed = st.reshape(N * Z, S).any(axis=1)
        np.testing.assert_array_equal(ge[~failed], oe[~failed], err_msg=f"read {it}")
        assert ok.shape == ge.shape


def test_aggregated_zones_feed_interval():
    """Two-socket fleet: zone aggregation -> interval kernel == oracle aggregation -> oracle interval."""
    S = 2
    layout = fleet.make_layout(24, [900, 40, 0, 1500] * 6, 4, seed=41)
    N, Z = layout.n_nodes, layout.zones
    caps = layout.capacities()
    sub_max = np.full(N * Z * S, fleet.MAX_ENERGY_FAKE, dtype=np.uint64)  # fast wraps
    acc = accel.Accel(Z, **caps)
    g, o = GpuAgg(acc, N, S, sub_max), OracleZoneAgg(N, Z, S, sub_max)
    ora = Oracle(Z, **caps)
    sim = fleet.FleetSim(layout, seed=41, churn=0.03)
    rng = np.random.default_rng(41)
    cnt = rng.integers(0, fleet.MAX_ENERGY_FAKE, size=N * Z * S).astype(np.uint64)
    s = current_stream_handle()
    for it in range(4):
        a = sim.next_interval()
        cnt = (cnt + rng.integers(0, 3 * 10**5, size=cnt.size).astype(np.uint64)) % np.uint64(fleet.MAX_ENERGY_FAKE)
        st = (rng.random(cnt.size) < 0.01).astype(np.uint32) if it else None
        oe, om, ons = o.read(cnt, st)
        a_ora = dict(a, zone_energy=oe, zone_max=om, node_status=ons)
        t = to_device(a)
        g.read(cnt, st, sync=False)
        t["zone_energy"], t["zone_max"], t["node_status"] = g.e, g.m, g.st  # the batch's zone inputs
        acc.run_interval(interval_from_tensors(t, layout.sizes(), layout.fast_flag()), s)
        acc.sync(s)
        ora.interval(a_ora, layout.sizes())
        for name, _ in accel.TABLES:
            np.testing.assert_array_equal(acc.download(name), ora.state[name], err_msg=f"interval {it} {name}")


def test_read_error_bit_set_and_cleared_every_read():
    """node_status passed unchanged every interval (INTEGRATION.md's loop): the read-error
    bit follows each read — a node fails only the intervals whose reads failed (monitor.go:
    328-335) — and the caller's other status bits are kept."""
    N, Z, S = 6, 2, 2
    sub_max = np.full(N * Z * S, 10**9, dtype=np.uint64)
    acc = accel.Accel(Z, nodes=N, proc_slots=1, ctr_slots=1, vm_slots=1, pod_slots=1)
    g, o = GpuAgg(acc, N, S, sub_max), OracleZoneAgg(N, Z, S, sub_max)
    g.st.copy_(torch.tensor([0, 4, 0, 4, 0, 0], dtype=torch.int32))  # an unrelated caller bit
    cnt = np.arange(N * Z * S, dtype=np.uint64) * 1000
    for it, bad_nodes in enumerate([[], [1, 2], [2], [], [5]]):
        cnt = cnt + np.uint64(777)
        st = np.zeros(N * Z * S, np.uint32)
        for n in bad_nodes:
            st[n * Z * S + S] = 1  # node n, zone 1, socket 0
        ge, _, gs = g.read(cnt, st, zero_status=False)
        oe, _, os_ = o.read(cnt, st)
        want = np.array([4 if n in (1, 3) else 0 for n in range(N)], np.uint32) | os_
        np.testing.assert_array_equal(gs, want, err_msg=f"read {it}")
        good = np.repeat(os_ == 0, Z)
        np.testing.assert_array_equal(ge[good], oe[good], err_msg=f"read {it}")
