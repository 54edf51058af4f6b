"""Packer -> slot join -> interval -> unpack, end to end on the device — MI355X only.

Informer-shaped records (per node, running processes in /proc order, with
process churn: PIDs end and new ones start; containers / VMs / pods appear
and disappear with their processes) go through kacc_pack on the host, the
four kacc_slot_join maps and kacc_run_interval on the device, and
kacc_unpack back to per-record / per-aggregate results.  The oracle runs the
same records through the Python packer restatement, the CPU slot joins and
the CPU interval; every unpacked value must match bit for bit.
"""

import numpy as np
import pytest
import torch

from kepler_amd import accel, fleet
from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device
from oracle.oracle import Oracle, OracleSlotMap
from oracle.pack_ref import pack_ref

pytestmark = pytest.mark.gpu
E = accel.KACC_KEY_EMPTY


@pytest.fixture(scope="module", autouse=True)
def gpu_ready():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    accel.load()
    torch.cuda.set_stream(torch.cuda.Stream())


class Informer:
    """A fleet of nodes whose /proc listing changes every interval."""

    def __init__(self, rows, seed):
        self.rng = np.random.default_rng(seed)
        self.nodes = []
        self.next_pid = 300
        for n, r in enumerate(rows):
            self.nodes.append([self._new(n) for _ in range(r)])

    def _new(self, n):
        rng = self.rng
        self.next_pid += int(rng.integers(1, 4))
        t = int(rng.choice([0, 1, 1, 1, 2]))
        c = int(n * 1000 + rng.integers(0, 30)) if t == 1 else 0
        v = int(n * 1000 + rng.integers(0, 3)) + 10**6 if t == 2 else 0
        pod = E if (c % 6 == 0) else (c // 3) + 10**8
        return dict(pid=self.next_pid, type=t, ctr=c, vm=v, pod=pod if t == 1 else E, ns=int(pod % 5) if t == 1 else 0,
                    total=0.0)

    def refresh(self, churn):
        rng = self.rng
        for n, procs in enumerate(self.nodes):
            keep = [p for p in procs if rng.random() >= churn]
            born = [self._new(n) for _ in range(len(procs) - len(keep) + int(rng.integers(0, 3)))]
            self.nodes[n] = keep + born  # new PIDs list after the old ones (ascending)
        recs = [p for procs in self.nodes for p in procs]
        for p in recs:  # CPUTotalTime grows; the informer's delta (informer.go:518)
            ticks = 0 if rng.random() < 0.3 else int(rng.integers(1, 5000))
            new_total = p["total"] + ticks / 100.0
            p["delta"], p["total"] = new_total - p["total"], new_total
        rec_off = np.r_[0, np.cumsum([len(p) for p in self.nodes])].astype(np.uint32)
        col = lambda k, dt: np.array([p[k] for p in recs], dtype=dt)  # noqa: E731
        return dict(rec_off=rec_off, pid=col("pid", np.uint32), cpu_delta=col("delta", np.float64),
                    ptype=col("type", np.uint8), ctr_key=col("ctr", np.uint64), vm_key=col("vm", np.uint64),
                    pod_key=col("pod", np.uint64), pod_ns=col("ns", np.uint32))


def _slot_off(counts, extra):
    return np.r_[0, np.cumsum(counts + extra)].astype(np.uint32)


@pytest.mark.parametrize("zones", [4, 2])
def test_pack_join_interval_unpack_bit_exact(zones):
    rows = [300, 0, 1200, 45, 2000, 7, 600, 90]
    inf = Informer(rows, seed=zones)
    N = len(rows)
    cap = np.array(rows) * 2 + 64
    offs = {"proc": _slot_off(cap, 0), "ctr": _slot_off(np.full(N, 40), 0), "vm": _slot_off(np.full(N, 8), 0),
            "pod": _slot_off(np.full(N, 24), 0)}
    caps = dict(nodes=N, proc_slots=int(offs["proc"][-1]), ctr_slots=int(offs["ctr"][-1]),
                vm_slots=int(offs["vm"][-1]), pod_slots=int(offs["pod"][-1]))
    acc = accel.Accel(zones, **caps)
    ora = Oracle(zones, **caps)
    kinds = {"proc": accel.KACC_KIND_PROC, "ctr": accel.KACC_KIND_CTR, "vm": accel.KACC_KIND_VM,
             "pod": accel.KACC_KIND_POD}
    smaps = {k: accel.SlotMap(acc, kinds[k], offs[k]) for k in kinds}
    omaps = {k: OracleSlotMap(offs[k]) for k in kinds}
    node_sim = fleet.FleetSim(fleet.make_layout(N, 1, zones, seed=3), seed=3)
    s = current_stream_handle()
    for it in range(4):
        r = inf.refresh(churn=0.05 if it else 0.0)
        p = accel.pack(threads=3, **r)
        want = pack_ref(r["rec_off"], r["pid"], r["cpu_delta"], r["ptype"], r["ctr_key"], r["vm_key"],
                        r["pod_key"], r["pod_ns"])
        for k, v in want.items():  # the host packer == its restatement
            np.testing.assert_array_equal(p[k], v, err_msg=k)
        sizes = {k: p[k] for k in ("n_nodes", "n_procs", "n_ctrs", "n_vms", "n_pods")}
        nd = node_sim.next_node_inputs()
        batch = dict(nd, **{k: p[k] for k in ("proc_off", "ctr_off", "vm_off", "pod_off", "proc_cpu_delta",
                                              "ctr_proc_end", "vm_proc_end", "pod_ctr_end")})
        # device: joins write the slot words into the batch, then the interval
        t = to_device(batch)
        keys = {"proc": p["proc_key"], "ctr": p["ctr_key"], "vm": p["vm_key"], "pod": p["pod_key"]}
        row_off = {"proc": "proc_off", "ctr": "ctr_off", "vm": "vm_off", "pod": "pod_off"}
        a_ora = dict(batch)
        for k in kinds:
            n_rows = int(p[row_off[k]][-1])
            kd = to_device({"k": keys[k].astype(np.uint32) if k == "proc" else keys[k]})["k"]
            slot = torch.zeros(max(n_rows, 1), dtype=torch.int32, device="cuda")
            tot = int(offs[k][-1])
            tk = torch.zeros(tot, dtype=torch.int64, device="cuda")
            ts = torch.zeros(tot, dtype=torch.int32, device="cuda")
            tc = torch.zeros(N, dtype=torch.int32, device="cuda")
            span = torch.zeros(2 * N, dtype=torch.int32, device="cuda") if k == "proc" else None
            smaps[k].join(n_rows, t[row_off[k]].data_ptr(), kd.data_ptr(), t["node_status"].data_ptr(),
                          slot.data_ptr(), tk.data_ptr(), ts.data_ptr(), tc.data_ptr(), s,
                          span.data_ptr() if span is not None else 0)
            t[f"{k}_slot"] = slot[:n_rows]
            if span is not None:
                t["node_proc_span"] = span
            rc, oslot, _, _, _ = omaps[k].join(p[row_off[k]], keys[k], batch["node_status"])
            assert rc == 0, k
            a_ora[f"{k}_slot"] = oslot
        acc.run_interval(interval_from_tensors(t, sizes, 0), s)
        acc.sync(s)
        for k in kinds:  # the device join == the CPU join
            np.testing.assert_array_equal(t[f"{k}_slot"].cpu().numpy().view(np.uint32), a_ora[f"{k}_slot"],
                                          err_msg=f"interval {it} {k} slots")
        ora.interval(a_ora, sizes)
        # unpack: processes in input-record order, aggregates in batch (key) order
        st = ora.state
        for k in kinds:
            n = int(p[row_off[k]][-1])
            if not n:
                continue
            oe = torch.zeros(n * zones, dtype=torch.int64, device="cuda")
            op = torch.zeros(n * zones, dtype=torch.float64, device="cuda")
            dest = to_device({"d": p["row_record"]})["d"] if k == "proc" else None
            acc.unpack(kinds[k], n, t[f"{k}_slot"].data_ptr(), dest.data_ptr() if dest is not None else 0,
                       oe.data_ptr(), op.data_ptr(), s)
            acc.sync(s)
            sl = (a_ora[f"{k}_slot"] & np.uint32(accel.KACC_SLOT_MASK)).astype(np.int64)
            we = st[f"{k}_energy"].reshape(-1, zones)[sl]
            wp = st[f"{k}_power"].reshape(-1, zones)[sl]
            if k == "proc":  # row r -> record row_record[r]
                inv = np.empty(n, np.int64)
                inv[p["row_record"]] = np.arange(n)
                we, wp = we[inv], wp[inv]
            np.testing.assert_array_equal(oe.cpu().numpy().view(np.uint64).reshape(-1, zones), we,
                                          err_msg=f"interval {it} {k} energy")
            np.testing.assert_array_equal(op.cpu().numpy().reshape(-1, zones).view(np.uint64), wp.view(np.uint64),
                                          err_msg=f"interval {it} {k} power")
    for m in smaps.values():
        m.close()
    acc.close()
