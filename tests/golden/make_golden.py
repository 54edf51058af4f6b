"""Generate tests/golden fixtures (committed data; re-run to regenerate).

kat_cases.json — known-answer tests transcribed from the reference's own Go
tests (sthaha/kepler @ 2025-08-24).  Each case restates one Go test scenario
as engine batches (one collection interval per entry) plus the values the Go
test asserts, with file:line.  Go mocks that inject a previous snapshot are
expressed as slot-table uploads; a mocked node snapshot built by
createNodeSnapshot(zones, t, r) (mock_utils.go:149-170: activeEnergy =
r·100 J, ActivePower = r·50 W) is reproduced by a 100 J counter delta over
2 s at usage ratio r; a mocked ProcessTotalCPUTimeDelta is passed with
KACC_F_NODE_CPU_DELTA_GIVEN.

golden_fleet.npz — a small synthetic fleet (8 nodes, Z=2, fake-meter
MaxEnergy 1e6 µJ so counters wrap every interval, 4 intervals, 5 % churn,
one read error) with the inputs and the oracle's expected state after every
interval.  It freezes the oracle's output so a later change to either side
is caught.

Usage: python tests/golden/make_golden.py
"""

from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

J = 1_000_000  # µJ per J (device/energy.go:16-20)
W = 1_000_000  # µW per W (device/energy.go:43-47)
S = 1_000_000_000  # ns per s
NEW = 0x80000000
T0 = 1_752_148_800 * S  # 2025-07-10 12:00:00 UTC as a monotonic origin


def node_batch(zones, energy, maxes, ts, ratio, procs=(), ctrs=(), vms=(), pods=(),
               node_delta=None, status=0):
    """One-node batch.  procs: [(delta, slotword)] in layout order;
    ctrs/vms: [(n_rows, slotword)], pods: [(n_ctrs, slotword)]."""
    p = len(procs)
    ctr_end, acc = [], 0
    for n_rows, _ in ctrs:
        acc += n_rows
        ctr_end.append(acc)
    vm_end = []
    for n_rows, _ in vms:
        acc += n_rows
        vm_end.append(acc)
    assert acc <= p
    pod_end, cacc = [], 0
    for n_c, _ in pods:
        cacc += n_c
        pod_end.append(cacc)
    assert cacc <= len(ctrs)
    arrays = dict(
        node_ts_ns=[ts], node_usage_ratio=[ratio], node_status=[status],
        zone_energy=list(energy), zone_max=list(maxes),
        proc_off=[0, p], ctr_off=[0, len(ctrs)], vm_off=[0, len(vms)], pod_off=[0, len(pods)],
        proc_cpu_delta=[float(d) for d, _ in procs], proc_slot=[w for _, w in procs],
        ctr_proc_end=ctr_end, ctr_slot=[w for _, w in ctrs],
        vm_proc_end=vm_end, vm_slot=[w for _, w in vms],
        pod_ctr_end=pod_end, pod_slot=[w for _, w in pods],
    )
    flags = 0
    if node_delta is not None:
        arrays["node_cpu_delta"] = [float(node_delta)]
        flags = 1
    return dict(arrays=arrays, flags=flags)


def eq(table, index, value):
    return dict(kind="eq", table=table, index=index, value=value)


def near(table, index, value, tol):
    return dict(kind="near", table=table, index=index, value=value, tol=tol)


# --- CreateTestResources (mock_utils.go:227-391) as engine rows ---------------
# layout order: container-1 {123, 1231}, container-2 {456}, VM procs 1001, 1002,
# then regular 789.  Slots: 123→0, 1231→1, 456→2, 1001→3, 1002→4, 789→5;
# container-1→0 (pod-id-1 → pod 0), container-2→1; vm-1→0, vm-2→1.
FIX_FRAC = [0.3, 0.1, 0.20, 0.20, 0.05, 0.15]  # 123, 1231, 456, 1001, 1002, 789


def fixture_rows(node_delta, new_procs=(), new_ctrs=(), new_vms=(), new_pods=()):
    procs = [(f * node_delta, s | (NEW if s in new_procs else 0)) for s, f in enumerate(FIX_FRAC)]
    ctrs = [(2, 0 | (NEW if 0 in new_ctrs else 0)), (1, 1 | (NEW if 1 in new_ctrs else 0))]
    vms = [(1, 0 | (NEW if 0 in new_vms else 0)), (1, 1 | (NEW if 1 in new_vms else 0))]
    pods = [(1, 0 | (NEW if 0 in new_pods else 0))]
    return dict(procs=procs, ctrs=ctrs, vms=vms, pods=pods)


ALL6 = set(range(6))


def cases():
    out = []

    # -- node.go:87-98 calculateEnergyDelta table (node_test.go:282-345) ------
    table = [  # name, current, previous, max, expected
        ("Normal", 25 * J, 20 * J, 100 * J, 5 * J),
        ("Wrap around", 10 * J, 90 * J, 100 * J, 20 * J),
        ("Zero values", 0, 0, 100 * J, 0),
        ("Max value is zero", 10 * J, 20 * J, 0, 0),
        ("Negative diff but max is negative", 2 * J, 8 * J, 10 * J, 4 * J),
        ("Current equals max", 100 * J, 90 * J, 100 * J, 10 * J),
        ("Previous equals max", 10 * J, 100 * J, 100 * J, 10 * J),
        ("Exact wrap", 0, 100 * J, 100 * J, 0),
    ]
    n = len(table)

    def fleet(energies, maxes, ts, ratio):
        arrays = dict(
            node_ts_ns=[ts] * n, node_usage_ratio=[ratio] * n, node_status=[0] * n,
            zone_energy=energies, zone_max=maxes,
            proc_off=[0] * (n + 1), ctr_off=[0] * (n + 1), vm_off=[0] * (n + 1),
            pod_off=[0] * (n + 1), proc_cpu_delta=[], proc_slot=[], ctr_proc_end=[],
            ctr_slot=[], vm_proc_end=[], vm_slot=[], pod_ctr_end=[], pod_slot=[])
        return dict(arrays=arrays, flags=0)

    maxes = [t[3] for t in table]
    i0 = fleet([t[2] for t in table], maxes, T0, 0.0)
    i1 = fleet([t[1] for t in table], maxes, T0 + 1 * S, 0.0)
    # ratio 0: activeEnergy 0, so IdleEnergyTotal = previous + delta and Power = delta/1s
    i1["expect"] = [eq("node_idle_total", k, t[2] + t[4]) for k, t in enumerate(table)]
    i1["expect"] += [eq("node_power", k, float(t[4])) for k, t in enumerate(table)]
    i1["expect"] += [eq("node_energy_total", k, t[1]) for k, t in enumerate(table)]
    out.append(dict(name="calculateEnergyDelta", ref="internal/monitor/node_test.go:282-345",
                    zones=1, capacities=dict(nodes=n, proc_slots=1, ctr_slots=1, vm_slots=1, pod_slots=1),
                    scalar=[dict(fn="calculate_energy_delta", args=[t[1], t[2], t[3]], value=t[4], name=t[0])
                            for t in table],
                    intervals=[i0, i1]))

    # -- TestNodePowerCollection (node_test.go:25-207) ------------------------
    mx = [200 * J, 150 * J]
    seq = [  # (Δt s, pkg J, core J, expected pkg W, core W)
        (0, 20, 10, 0, 0),
        (1, 70, 35, 50, 25),
        (3, 145, 80, 25, 15),
        (10, 25, 110, 8, 3),  # pkg 145+80 wraps at 200 -> 25
    ]
    ivs, t = [], T0
    for k, (dt, pe, ce, pw, cw) in enumerate(seq):
        t += dt * S
        b = node_batch(2, [pe * J, ce * J], mx, t, 0.5, node_delta=100.0)
        b["expect"] = [eq("node_energy_total", 0, pe * J), eq("node_energy_total", 1, ce * J),
                       near("node_power", 0, pw * W, 0.001 * W), near("node_power", 1, cw * W, 0.001 * W)]
        ivs.append(b)
    out.append(dict(name="TestNodePowerCollection", ref="internal/monitor/node_test.go:25-207", zones=2,
                    capacities=dict(nodes=1, proc_slots=1, ctr_slots=1, vm_slots=1, pod_slots=1),
                    intervals=ivs))

    # -- TestNodeActiveEnergyCounterBehavior (node_test.go:349-521) ----------
    seq = [(0, 100, 0.4, 40, 40, 60), (2, 150, 0.4, 20, 60, 90), (3, 210, 0.4, 24, 84, 126),
           (1, 250, 0.8, 32, 116, 134)]
    ivs, t = [], T0
    for dt, e, r, act, at, it in seq:
        t += dt * S
        b = node_batch(1, [e * J], [1000 * J], t, r, node_delta=80.0)
        b["expect"] = [eq("node_active_energy", 0, act * J), eq("node_active_total", 0, at * J),
                       eq("node_idle_total", 0, it * J)]
        ivs.append(b)
    out.append(dict(name="TestNodeActiveEnergyCounterBehavior", ref="internal/monitor/node_test.go:349-521",
                    zones=1, capacities=dict(nodes=1, proc_slots=1, ctr_slots=1, vm_slots=1, pod_slots=1),
                    intervals=ivs))

    # -- TestNodeActiveEnergyTotalAccumulation (node_test.go:523-665) --------
    seq = [(100, 60, 60, 40), (150, 30, 90, 60), (190, 24, 114, 76), (220, 18, 132, 88)]
    ivs, t = [], T0
    for e, act, at, it in seq:
        t += 1 * S
        b = node_batch(1, [e * J], [1000 * J], t, 0.6, node_delta=100.0)
        b["expect"] = [eq("node_active_energy", 0, act * J), eq("node_active_total", 0, at * J),
                       eq("node_idle_total", 0, it * J)]
        ivs.append(b)
    ivs[-1]["expect_sum_tables"] = [dict(tables=["node_active_total", "node_idle_total"], index=0,
                                         value=220 * J)]
    out.append(dict(name="TestNodeActiveEnergyTotalAccumulation", ref="internal/monitor/node_test.go:523-665",
                    zones=1, capacities=dict(nodes=1, proc_slots=1, ctr_slots=1, vm_slots=1, pod_slots=1),
                    intervals=ivs))

    zones2 = [1000 * J, 500 * J]  # CreateTestZones (mock_utils.go:142-146)
    cap6 = dict(nodes=1, proc_slots=6, ctr_slots=2, vm_slots=2, pod_slots=1)

    def two_reads(ratio, rows1, delta_j=100, node_delta=None, upload=None, expect=None):
        # interval 0: first read; interval 1: +2 s, +delta_j J -> createNodeSnapshot(., r)
        first = node_batch(2, [100 * J, 100 * J], zones2, T0, ratio, **rows1, node_delta=node_delta)
        second = node_batch(2, [(100 + delta_j) * J, (100 + delta_j) * J], zones2, T0 + 2 * S, ratio,
                            **rows1, node_delta=node_delta)
        second["upload"] = upload or []
        second["expect"] = expect or []
        return [first, second]

    # -- process_power_test.go:87-166 calculateProcessPower ------------------
    rows = fixture_rows(200.0, new_procs=ALL6 - {0})
    exp = []
    for z in range(2):
        exp += [near("proc_power", 0 * 2 + z, 7.5 * W, 0.01), near("proc_energy", 0 * 2 + z, 40 * J, 0.01),
                near("proc_power", 2 * 2 + z, 5 * W, 0.01), near("proc_power", 5 * 2 + z, 3.75 * W, 0.01)]
    out.append(dict(name="calculateProcessPower", ref="internal/monitor/process_power_test.go:87-166",
                    zones=2, capacities=cap6,
                    intervals=two_reads(0.5, rows, upload=[dict(table="proc_energy", first=0,
                                                                values=[25 * J, 25 * J])], expect=exp)))

    # -- process_power_test.go:168-209 zero node power -------------------------
    rows = fixture_rows(200.0)
    exp = [eq("proc_energy", k, 0) for k in range(12)] + [eq("proc_power", k, 0.0) for k in range(12)]
    out.append(dict(name="calculateProcessPower with zero node power",
                    ref="internal/monitor/process_power_test.go:168-209", zones=2, capacities=cap6,
                    intervals=two_reads(0.5, rows, delta_j=0, expect=exp)))

    # -- process_power_test.go:234-274 zero CPU time delta ---------------------
    rows1 = dict(procs=[(0.0, 0 | NEW)])
    exp = [eq("proc_energy", z, 0) for z in range(2)] + [eq("proc_power", z, 0.0) for z in range(2)]
    out.append(dict(name="zero CPU time delta", ref="internal/monitor/process_power_test.go:234-274",
                    zones=2, capacities=dict(nodes=1, proc_slots=1, ctr_slots=1, vm_slots=1, pod_slots=1),
                    intervals=two_reads(0.5, rows1, node_delta=200.0, expect=exp)))

    # -- process_power_test.go:276-343 new zone missing in previous snapshot ---
    rows1 = dict(procs=[(50.0, 0)])
    exp = [eq("node_active_energy", 0, 60 * J), eq("node_active_energy", 1, 60 * J),
           eq("node_active_power", 0, 30.0 * W), eq("node_active_power", 1, 30.0 * W),
           eq("proc_energy", 0, 25 * J), eq("proc_energy", 1, 15 * J),
           eq("proc_power", 0, 7.5 * W), eq("proc_power", 1, 7.5 * W)]
    out.append(dict(name="new zone missing in previous snapshot",
                    ref="internal/monitor/process_power_test.go:276-343", zones=2,
                    capacities=dict(nodes=1, proc_slots=1, ctr_slots=1, vm_slots=1, pod_slots=1),
                    intervals=two_reads(0.6, rows1, node_delta=200.0,
                                        upload=[dict(table="proc_energy", first=0, values=[10 * J, 0])],
                                        expect=exp)))

    # -- process_power_test.go:348-415 power conservation ----------------------
    rows1 = dict(procs=[(25.0, 0 | NEW), (35.0, 1 | NEW), (40.0, 2 | NEW)])
    exp = [dict(kind="sum_near_table", table="proc_power", indices=[0 + z, 2 + z, 4 + z],
                other="node_active_power", other_index=z, tol=1.0) for z in range(2)]
    out.append(dict(name="TestProcessPowerConsistency", ref="internal/monitor/process_power_test.go:348-415",
                    zones=2, capacities=dict(nodes=1, proc_slots=3, ctr_slots=1, vm_slots=1, pod_slots=1),
                    intervals=two_reads(0.5, rows1, expect=exp)))

    # -- container_power_test.go:79-149 calculateContainerPower ---------------
    rows = fixture_rows(200.0, new_procs=ALL6, new_ctrs={1}, new_vms={0, 1}, new_pods={0})
    exp = []
    for z in range(2):
        exp += [near("ctr_power", 0 * 2 + z, 10 * W, 0.01), near("ctr_energy", 0 * 2 + z, 45 * J, 0.01),
                near("ctr_power", 1 * 2 + z, 5 * W, 0.01)]
    exp += [eq("ctr_cpu_delta", 0, 80.0), eq("ctr_cpu_delta", 1, 40.0)]
    out.append(dict(name="calculateContainerPower", ref="internal/monitor/container_power_test.go:79-149",
                    zones=2, capacities=cap6,
                    intervals=two_reads(0.5, rows, upload=[dict(table="ctr_energy", first=0,
                                                                values=[25 * J, 25 * J])], expect=exp)))

    # -- container_power_test.go:240-282 exact container power conservation ----
    rows1 = dict(procs=[(30.0, 0 | NEW), (35.0, 1 | NEW), (35.0, 2 | NEW)],
                 ctrs=[(1, 0 | NEW), (1, 1 | NEW), (1, 2 | NEW)])
    exp = [dict(kind="sum_eq_table", table="ctr_power", indices=[0 + z, 2 + z, 4 + z],
                other="node_active_power", other_index=z, scale=0.5) for z in range(2)]
    out.append(dict(name="container power conservation", ref="internal/monitor/container_power_test.go:240-282",
                    zones=2, capacities=dict(nodes=1, proc_slots=3, ctr_slots=3, vm_slots=1, pod_slots=1),
                    intervals=two_reads(0.5, rows1, node_delta=200.0, expect=exp)))

    # -- vm_test.go:80-152 calculateVMPower (CreateTestVMs vm_test.go:579-605) -
    rows1 = dict(procs=[(60.0, 0 | NEW), (40.0, 1 | NEW)], vms=[(1, 0), (1, 1 | NEW)])
    exp = []
    for z in range(2):
        exp += [near("vm_power", 0 * 2 + z, 7.5 * W, 0.01), near("vm_energy", 0 * 2 + z, 45 * J, 0.01),
                eq("vm_power", 1 * 2 + z, 5.0 * W), eq("vm_energy", 1 * 2 + z, 10 * J)]
    out.append(dict(name="calculateVMPower", ref="internal/monitor/vm_test.go:80-152", zones=2,
                    capacities=dict(nodes=1, proc_slots=2, ctr_slots=1, vm_slots=2, pod_slots=1),
                    intervals=two_reads(0.5, rows1, node_delta=200.0,
                                        upload=[dict(table="vm_energy", first=0, values=[30 * J, 30 * J])],
                                        expect=exp)))

    # -- vm_test.go:259-322 VM missing zone in previous snapshot ---------------
    rows1 = dict(procs=[(60.0, 0 | NEW)], vms=[(1, 0)])
    exp = [eq("vm_energy", 0, 33 * J), eq("vm_energy", 1, 18 * J),
           eq("vm_power", 0, 9.0 * W), eq("vm_power", 1, 9.0 * W)]
    out.append(dict(name="VM missing zone in previous snapshot", ref="internal/monitor/vm_test.go:259-322",
                    zones=2, capacities=dict(nodes=1, proc_slots=1, ctr_slots=1, vm_slots=1, pod_slots=1),
                    intervals=two_reads(0.6, rows1, node_delta=200.0,
                                        upload=[dict(table="vm_energy", first=0, values=[15 * J, 0])],
                                        expect=exp)))

    # -- pod_power_test.go:86-142 calculatePodPower ---------------------------
    rows = fixture_rows(200.0, new_procs=ALL6, new_ctrs={0, 1}, new_vms={0, 1}, new_pods={0})
    exp = []
    for z in range(2):
        exp += [eq("pod_power", z, 10.0 * W), eq("pod_energy", z, 20 * J)]
        exp += [dict(kind="le_table", table="pod_power", index=z, other="node_active_power", other_index=z)]
    exp += [eq("pod_cpu_delta", 0, 80.0)]
    out.append(dict(name="calculatePodPower", ref="internal/monitor/pod_power_test.go:86-142", zones=2,
                    capacities=cap6, intervals=two_reads(0.5, rows, expect=exp)))

    # -- monitor_snapshot_integration_test.go:80-273 (3 Snapshot() calls) -----
    ivs = []
    for k, (e, act_t, idle_t, proc_sum) in enumerate([(100, 60, 40, 0), (150, 90, 60, 30), (200, 120, 80, 60)]):
        new = ALL6 if k == 0 else set()
        rows = fixture_rows(2000.0, new_procs=new, new_ctrs=new and {0, 1}, new_vms=new and {0, 1},
                            new_pods=new and {0})
        b = node_batch(1, [e * J], [1000 * J], T0 + 5 * k * S, 0.6, **rows)
        b["expect"] = [eq("node_active_total", 0, act_t * J), eq("node_idle_total", 0, idle_t * J),
                       dict(kind="sum_eq", table="proc_energy", indices=list(range(6)), value=proc_sum * J)]
        if k == 0:
            b["expect"].append(eq("node_power", 0, 0.0))
        else:
            b["expect"] += [
                dict(kind="sum_eq_table", table="proc_power", indices=list(range(6)),
                     other="node_active_power", other_index=0, scale=1.0),
                dict(kind="ratio_eq_table", table="node_active_power", index=0, other="node_power",
                     other_index=0, scale=0.6),
                dict(kind="diff_eq_table", table="node_idle_power", index=0, a="node_power",
                     b="node_active_power"),
            ]
        ivs.append(b)
    out.append(dict(name="TestIntegration_Monitor_Snapshot",
                    ref="internal/monitor/monitor_snapshot_integration_test.go:80-273", zones=1,
                    capacities=cap6, intervals=ivs))

    # -- read error keeps the previous snapshot (node.go:39-44, monitor.go:328-335)
    rows = fixture_rows(200.0)
    i0 = node_batch(1, [100 * J], [1000 * J], T0, 0.5, **rows)
    i1 = node_batch(1, [150 * J], [1000 * J], T0 + 5 * S, 0.5, **rows, status=1)
    i1["expect"] = [eq("node_energy_total", 0, 100 * J), eq("node_status", 0, 2), eq("node_ts", 0, T0)]
    i2 = node_batch(1, [200 * J], [1000 * J], T0 + 10 * S, 0.5, **rows)
    # the delta spans both intervals: 100 J over 10 s -> 10 W, active 50 J
    i2["expect"] = [eq("node_power", 0, 10.0 * W), eq("node_active_energy", 0, 50 * J),
                    eq("node_status", 0, 0)]
    out.append(dict(name="zone read error keeps previous snapshot",
                    ref="internal/monitor/node.go:39-44; monitor.go:328-335", zones=1, capacities=cap6,
                    intervals=[i0, i1, i2]))
    return out


# -- device/energy_zone_test.go aggregated-zone KATs (oracle scalar checks) ---
AGG_CASES = [
    dict(name="BasicAggregation", ref="internal/device/energy_zone_test.go:66-80", max=[1000, 1000],
         reads=[[100, 200]], expect=[300], agg_max=2000),
    dict(name="FirstReadingCorrectness", ref="internal/device/energy_zone_test.go:93-117", max=[1000],
         reads=[[100], [100], [150]], expect=[100, 100, 150], agg_max=1000),
    dict(name="MultiZoneWrap", ref="internal/device/energy_zone_test.go:121-139", max=[1000, 1000],
         reads=[[900, 800], [100, 850]], expect=[1700, 1950], agg_max=2000),
    dict(name="MultipleWraps", ref="internal/device/energy_zone_test.go:141-165", max=[1000],
         reads=[[900], [100], [50]], expect=[900, 100, 50], agg_max=1000),
    dict(name="BackwardReading", ref="internal/device/energy_zone_test.go:167-184", max=[1000],
         reads=[[500], [400]], expect=[500, 400], agg_max=1000),
    dict(name="ZeroMaxEnergyHandling", ref="internal/device/energy_zone_test.go:186-199", max=[0, 0],
         reads=[[100, 200]], expect=[300], agg_max=0),
    dict(name="MaxEnergyOverflow", ref="internal/device/energy_zone.go:57-67", max=[2**64 - 10, 100],
         reads=[[1, 1]], expect=[2], agg_max=2**64 - 1),
]


def golden_fleet(path):
    from kepler_amd import fleet
    from oracle.oracle import Oracle

    L = fleet.make_layout(8, [300, 500, 64, 700, 1, 0, 257, 513], 2, seed=7, procs_per_vm=2,
                          vm_frac=0.02, shuffle_slots=True)
    sim = fleet.FleetSim(L, seed=7, max_energy=fleet.MAX_ENERGY_FAKE, churn=0.05, zero_ratio_frac=0.1)
    o = Oracle(L.zones, **L.capacities())
    data = {}
    for k in range(4):
        a = sim.next_interval()
        if k == 2:
            a["node_status"] = a["node_status"].copy()
            a["node_status"][3] = 1  # one zone read error
        o.interval(a, L.sizes())
        for name, v in a.items():
            data[f"in{k}/{name}"] = np.asarray(v)
        for name, v in o.state.t.items():
            data[f"out{k}/{name}"] = v.copy()
    for name, v in L.capacities().items():
        data[f"cap/{name}"] = np.array(v)
    for name, v in L.sizes().items():
        data[f"size/{name}"] = np.array(v)
    data["zones"] = np.array(L.zones)
    np.savez_compressed(path, **data)


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "kat_cases.json"), "w") as f:
        json.dump(dict(cases=cases(), aggregated=AGG_CASES), f, indent=1)
    golden_fleet(os.path.join(here, "golden_fleet.npz"))
    print("wrote", here)


if __name__ == "__main__":
    main()
