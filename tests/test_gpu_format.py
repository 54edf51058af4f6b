"""Device exposition formatting (kacc_format_values) against oracle/gofmt.py — MI355X only.

Text is compared byte for byte: energy tables as Joules(), power tables as
Watts(), over edge values (0, 1 J, exact powers of ten, u64 extremes, NaN,
±Inf, -0, subnormals, DBL_MAX, halfway-looking decimals) and 1M random bit
patterns / realistic attribution values.
"""

import math

import numpy as np
import pytest
import torch

from kepler_amd import accel
from oracle.gofmt import joules, watts, write_float

pytestmark = pytest.mark.gpu
W = accel.KACC_FMT_WIDTH


@pytest.fixture(scope="module", autouse=True)
def gpu_ready():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    accel.load()
    torch.cuda.set_stream(torch.cuda.Stream())


def device_text(acc, table, n):
    from kepler_amd.torch_batch import current_stream_handle

    out = torch.zeros(n * W, dtype=torch.uint8, device="cuda")
    ln = torch.zeros(n, dtype=torch.uint8, device="cuda")
    s = current_stream_handle()
    acc.format_values(table, 0, n, out.data_ptr(), ln.data_ptr(), s)
    acc.sync(s)
    buf = out.cpu().numpy().reshape(n, W)
    lens = ln.cpu().numpy()
    return [bytes(buf[i, : lens[i]]).decode() for i in range(n)]


def edge_energies():
    v = [0, 1, 2, 5, 999_999, 10**6, 10**6 + 1, 1_500_000, 10**12, 10**15, 123_456_789_012, 2**53, 2**53 + 1,
         2**63, 2**64 - 1, 2**64 - 1024, 10**19, 7 * 10**18 + 3]
    v += [10**k for k in range(20)] + [10**k - 1 for k in range(1, 20)]
    # the integer fast path's boundary (write_joules: e < 10^15 µJ) and trailing zeros
    v += [10**15 - 1, 10**15 + 1, 10**15 - 10, 999_999_999_999_990, 2**49, 2**50 - 1, 120_000, 3_000_000,
          4_500_000_000, 10**14 + 1, 987_654_321_000_000]
    v += [d * 10**k for d in (1, 7, 25, 123) for k in range(14)]
    return np.array(v, dtype=np.uint64)


def edge_powers():
    v = [0.0, -0.0, 1e6, -1e6, 1.0, -1.0, float("nan"), float("inf"), float("-inf"), 5e-324, 2.2250738585072014e-308,
         1.7976931348623157e308, -1.7976931348623157e308, 0.5, 1.5e6, 123456.0, 9.999999e12, 1e-10, 2.5e-5,
         3.0e5 / 7, 1e23, 9007199254740993.0, 0.1, 0.2, 0.30000000000000004]
    v += [10.0 ** k for k in range(-30, 30)] + [5.0 * 10.0 ** k for k in range(-20, 20)]
    return np.array(v, dtype=np.float64)


def test_format_edges():
    e, p = edge_energies(), edge_powers()
    n = max(e.size, p.size)
    # power values through the stored power table (process / container / VM power is derived)
    acc = accel.Accel(1, nodes=1, proc_slots=n, ctr_slots=1, vm_slots=1, pod_slots=n)
    acc.upload("proc_energy", np.resize(e, n))
    acc.upload("pod_power", np.resize(p, n))
    got_e, got_p = device_text(acc, "proc_energy", n), device_text(acc, "pod_power", n)
    for i in range(n):
        ev, pv = int(np.resize(e, n)[i]), float(np.resize(p, n)[i])
        assert got_e[i] == write_float(joules(ev)), (ev, got_e[i])
        want_p = write_float(watts(pv))
        assert got_p[i] == want_p, (pv, got_p[i], want_p)


@pytest.mark.parametrize("kind", ["bits", "realistic"])
def test_format_random(kind):
    rng = np.random.default_rng(17 if kind == "bits" else 18)
    n = 1 << 20
    if kind == "bits":  # any double; energies over the whole u64 range
        p = rng.integers(-2**63, 2**63 - 1, size=n, dtype=np.int64).view(np.float64)
        e = rng.integers(0, 2**64 - 1, size=n, dtype=np.uint64, endpoint=True)
    else:  # attribution-like: µJ totals and µW powers
        e = (rng.lognormal(18, 4, size=n)).astype(np.uint64)
        p = rng.lognormal(12, 3, size=n) * rng.choice([1.0, 1.0, 1.0, 0.0], size=n)
    acc = accel.Accel(1, nodes=1, proc_slots=n, ctr_slots=1, vm_slots=1, pod_slots=n)
    acc.upload("proc_energy", e)
    acc.upload("pod_power", p)
    got_e, got_p = device_text(acc, "proc_energy", n), device_text(acc, "pod_power", n)
    bad = []
    for i in range(n):
        we = write_float(joules(int(e[i])))
        if got_e[i] != we:
            bad.append(("E", int(e[i]), got_e[i], we))
        wp = write_float(watts(float(p[i])))
        if got_p[i] != wp and not (math.isnan(p[i]) and got_p[i] == "NaN"):
            bad.append(("P", float(p[i]), got_p[i], wp))
        if len(bad) > 10:
            break
    assert not bad, bad[:10]


@pytest.mark.parametrize("table,metric", [
    ("proc_energy", "kepler_process_cpu_joules_total"),
    ("pod_power", "kepler_pod_cpu_watts"),
])
def test_format_lines_byte_exact(table, metric):
    """kacc_format_lines: NAME{LABELS,zone="ZONE"} VALUE lines, byte for byte against
    oracle/gofmt.sample_line, with escaped label values, a row permutation, a
    zone subset in a caller-chosen order and a sizing call first."""
    from kepler_amd.torch_batch import current_stream_handle
    from oracle.gofmt import label_pairs, sample_line

    rng = np.random.default_rng(17)
    Z, slots, first, count = 4, 700, 37, 600
    acc = accel.Accel(Z, nodes=1, proc_slots=slots, ctr_slots=1, vm_slots=1, pod_slots=slots)
    if table.endswith("energy"):
        vals = rng.integers(0, 2**40, size=slots * Z, dtype=np.uint64)
        vals[:8] = [0, 10**6, 1, 2**64 - 1, 123, 10**12, 5 * 10**5, 10**19]
    else:
        vals = rng.random(slots * Z) * 10.0 ** rng.integers(-3, 9, size=slots * Z)
        vals[:6] = [0.0, 1e6, -1e6, float("nan"), float("inf"), 1e-300]
    acc.upload(table, vals)
    alphabet = ['a', 'Z', '0', '/', '-', '"', '\\', '\n', 'é', ' ', '{', '=']
    rows = []
    for r in range(count):
        comm = "".join(rng.choice(alphabet, size=int(rng.integers(0, 12))))
        rows.append(label_pairs([("pid", str(1000 + r)), ("comm", comm), ("container_id", ""),
                                 ("exe", "/usr/bin/" + comm), ("state", "running"), ("type", "regular"),
                                 ("vm_id", "")]).encode())
    label_off = np.r_[0, np.cumsum([len(x) for x in rows])].astype(np.uint64)
    d_labels = torch.from_numpy(np.frombuffer(b"".join(rows), dtype=np.uint8).copy()).cuda()
    d_loff = torch.from_numpy(label_off.view(np.int64)).cuda()
    order = rng.permutation(count).astype(np.uint32)
    d_order = torch.from_numpy(order.view(np.int32)).cuda()
    zone_order, zone_names = [3, 0, 2], ["dram", "package", "uncore"]
    n_lines = count * len(zone_order)
    d_line_off = torch.zeros(n_lines + 1, dtype=torch.int64, device="cuda")
    s = current_stream_handle()
    args = (table, metric, first, count, zone_names, d_labels.data_ptr(), d_loff.data_ptr(), d_line_off.data_ptr())
    total = acc.format_lines(*args, zone_order=zone_order, row_order_ptr=d_order.data_ptr(), stream=s)
    with pytest.raises(accel.AccelError):  # too small a buffer: KACC_ERANGE, nothing written
        small = torch.zeros(16, dtype=torch.uint8, device="cuda")
        acc.format_lines(*args, out_ptr=small.data_ptr(), out_cap=16, zone_order=zone_order,
                         row_order_ptr=d_order.data_ptr(), stream=s)
    out = torch.zeros(total, dtype=torch.uint8, device="cuda")
    assert acc.format_lines(*args, out_ptr=out.data_ptr(), out_cap=total, zone_order=zone_order,
                            row_order_ptr=d_order.data_ptr(), stream=s) == total
    acc.sync(s)
    conv = (lambda v: joules(int(v))) if table.endswith("energy") else (lambda v: watts(float(v)))
    want = []
    for i in range(count):
        r = int(order[i])
        labels = rows[r].decode()
        for z, zn in zip(zone_order, zone_names):
            want.append(sample_line(metric, labels, zn, conv(vals[(first + r) * Z + z])))
    want = "".join(want).encode()
    got = bytes(out.cpu().numpy())
    assert len(got) == len(want)
    assert got == want
    offs = d_line_off.cpu().numpy()
    assert offs[-1] == total and np.all(np.diff(offs) > 0)
    acc.close()


def test_format_lines_hipcub_fault_regression_multi_tile_past_4gib():
    """Regression guard for the round-1 fault (hipcub's scan faulted at 80M lines;
    the scan is now the library's own reduce-then-scan): 16M lines = 3,907 scan tiles of
    4,096 (> 256 tiles: the multi-level scan_tile_prefix path) and 5.0 GB of text, so line
    offsets cross 4 GiB.  line_off is strictly increasing, its last entry is the sizing pass's
    total, and sampled lines (tile edges, the 4 GiB crossing, random) match
    oracle/gofmt.sample_line byte for byte."""
    from kepler_amd.torch_batch import current_stream_handle
    from oracle.gofmt import sample_line

    Z, count, L = 4, 4_000_000, 260
    metric = "kepler_process_cpu_joules_total"
    zone_names = ["package", "core", "uncore", "dram"]
    rng = np.random.default_rng(23)
    acc = accel.Accel(Z, nodes=1, proc_slots=count, ctr_slots=1, vm_slots=1, pod_slots=1)
    # finite energies over the whole u64 range (lognormal's tail is clipped below 2^64, so no
    # inf / NaN reaches the cast): µJ values from 1 to ~1.8e19
    vals = np.minimum(rng.lognormal(20, 5, size=count * Z), 1.8e19).astype(np.uint64)
    acc.upload("proc_energy", vals)
    # fixed-width label pairs: pid="00001234",comm="xxxx...x" (L bytes per row)
    head = b'comm="'
    body = np.frombuffer((head + b"w" * (L - len(head) - len(b'",pid="00000000"')) + b'",pid="00000000"'), np.uint8)
    labels = np.tile(body, (count, 1))
    digits = np.array([(np.arange(count) // 10 ** k) % 10 for k in range(7, -1, -1)], dtype=np.uint8).T + ord("0")
    labels[:, L - 9:L - 1] = digits
    d_labels = torch.from_numpy(labels.reshape(-1)).cuda()
    label_off = (np.arange(count + 1, dtype=np.int64) * L)
    d_loff = torch.from_numpy(label_off).cuda()
    n_lines = count * Z
    d_line_off = torch.zeros(n_lines + 1, dtype=torch.int64, device="cuda")
    s = current_stream_handle()
    args = ("proc_energy", metric, 0, count, zone_names, d_labels.data_ptr(), d_loff.data_ptr(),
            d_line_off.data_ptr())
    total = acc.format_lines(*args, stream=s)
    assert total > 2**32 and n_lines > 256 * 4096
    out = torch.empty(total, dtype=torch.uint8, device="cuda")
    assert acc.format_lines(*args, out_ptr=out.data_ptr(), out_cap=total, stream=s) == total
    acc.sync(s)
    offs = d_line_off.cpu().numpy()
    assert offs[0] == 0 and offs[-1] == total
    assert np.all(np.diff(offs) > 0)
    cross = int(np.searchsorted(offs, 2**32, side="right")) - 1  # the line holding byte 2^32
    picks = {0, 1, n_lines - 1, cross - 1, cross, cross + 1}
    for t in (4096, 4096 * 256, 4096 * 257, 4096 * 1000):  # scan tile edges
        picks |= {t - 1, t, t + 1}
    picks |= set(rng.integers(0, n_lines, size=400).tolist())
    for i in sorted(p for p in picks if 0 <= p < n_lines):
        r, z = divmod(i, Z)
        got = bytes(out[int(offs[i]):int(offs[i + 1])].cpu().numpy())
        want = sample_line(metric, bytes(labels[r]).decode(), zone_names[z], joules(int(vals[r * Z + z]))).encode()
        assert got == want, (i, got[:120], want[:120])
    del out
    acc.close()


def test_format_derived_process_power():
    """KACC_T_PROC_POWER is derived on read (ratio x the node's ActivePower, kacc_derive.hpp):
    format_values and format_lines of it == the downloaded (derived) values written as Go
    writes them, after real intervals (guarded zones, NaN / Inf ratios of adversarial nodes)."""
    from kepler_amd import fleet
    from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device
    from oracle.gofmt import sample_line

    L = fleet.make_layout(24, [300, 2000, 1, 0, 700, 64] * 4, 4, seed=8)
    acc = accel.Accel(L.zones, **L.capacities())
    sim = fleet.FleetSim(L, seed=8, adversarial=0.2, zero_ratio_frac=0.1)
    s = current_stream_handle()
    for _ in range(3):
        t = to_device(sim.next_interval())
        acc.run_interval(interval_from_tensors(t, L.sizes(), L.fast_flag()), s)
    acc.sync(s)
    with pytest.raises(accel.AccelError):  # no device storage
        acc.device_ptr("proc_power")
    with pytest.raises(accel.AccelError):  # not uploadable
        acc.upload("proc_power", np.zeros(4), 0)
    for tname in ("ctr_power", "vm_power"):  # containers and VMs are derived the same way
        cp = acc.download(tname)
        gc = device_text(acc, tname, cp.size)
        for i in range(0, cp.size, 3):
            want = write_float(watts(float(cp[i])))
            assert gc[i] == want or (math.isnan(cp[i]) and gc[i] == "NaN"), (tname, i, cp[i], gc[i], want)
    pp = acc.download("proc_power")
    n = pp.size
    got = device_text(acc, "proc_power", n)
    for i in range(n):
        want = write_float(watts(float(pp[i])))
        assert got[i] == want or (math.isnan(pp[i]) and got[i] == "NaN"), (i, pp[i], got[i], want)
    # a range not starting at 0 (the derived range is materialised from `first`)
    first, cnt = 1000 * L.zones + 3, 5000
    d_out = torch.zeros(cnt * accel.KACC_FMT_WIDTH, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(cnt, dtype=torch.uint8, device="cuda")
    acc.format_values("proc_power", first, cnt, d_out.data_ptr(), d_len.data_ptr(), s)
    acc.sync(s)
    raw, ln = d_out.cpu().numpy().reshape(cnt, -1), d_len.cpu().numpy()
    for i in range(0, cnt, 7):
        assert bytes(raw[i, :ln[i]]).decode() == got[first + i]
    # whole lines over a slot range of the derived table, a zone subset
    Z, rows0, rows = L.zones, 17, 4000
    label = 'comm="x",pid="1"'
    labels = np.frombuffer((label * rows).encode(), np.uint8)
    d_labels = torch.from_numpy(labels.copy()).cuda()
    d_loff = torch.from_numpy(np.arange(rows + 1, dtype=np.int64) * len(label)).cuda()
    zn, zo = ["package", "dram"], [0, 3]
    d_line_off = torch.zeros(rows * 2 + 1, dtype=torch.int64, device="cuda")
    args = ("proc_power", "kepler_process_cpu_watts", rows0, rows, zn, d_labels.data_ptr(), d_loff.data_ptr(),
            d_line_off.data_ptr())
    total = acc.format_lines(*args, zone_order=zo, stream=s)
    out = torch.empty(total, dtype=torch.uint8, device="cuda")
    acc.format_lines(*args, out_ptr=out.data_ptr(), out_cap=total, zone_order=zo, stream=s)
    acc.sync(s)
    text = bytes(out.cpu().numpy()).decode()
    want = "".join(sample_line("kepler_process_cpu_watts", label, zn[j], watts(float(pp[(rows0 + r) * Z + zo[j]])))
                   for r in range(rows) for j in range(2))
    assert text == want
    acc.close()


def _parse_exposition(text):
    """Sample lines of the text format -> [(name, {label: value}, float)] (label values
    unescaped: \\\\, \\" and \\n, expfmt's escapes)."""
    out = []
    for line in text.splitlines():
        name, rest = line.split("{", 1)
        labels, i = {}, 0
        while rest[i] != "}":
            eq = rest.index("=", i)
            key = rest[i:eq]
            assert rest[eq + 1] == '"', line
            j, val = eq + 2, []
            while rest[j] != '"':
                if rest[j] == "\\":
                    val.append({"\\": "\\", '"': '"', "n": "\n"}[rest[j + 1]])
                    j += 2
                else:
                    val.append(rest[j])
                    j += 1
            labels[key] = "".join(val)
            i = j + 1
            if rest[i] == ",":
                i += 1
        assert rest[i + 1] == " ", line
        out.append((name, labels, float(rest[i + 2:])))
    return out


def test_format_collector_fixture_snapshot():
    """The reference exporter test's snapshot (power_collector_test.go:184-272, transcribed in
    tests/golden/collector_snapshot.json) held in the engine's tables and written by the
    device: kacc_format_lines for the node families (one call per zone, whose path label sorts
    before zone) and the four workload families, kacc_format_values for the usage ratio.  The
    text is parsed back and checked as the reference test checks its registry: the 16 family
    names (:307-328), the node joules / watts / active / idle values per zone path and the zone
    names and paths (:342-418), and each workload family's labels and value (:437-483).
    kepler_process_cpu_seconds_total is CPUTotalTime from the Go informer (not an engine
    table): its line is the Go side's, written here with oracle/gofmt.  Every device line is
    also byte-compared with oracle/gofmt.sample_line."""
    import json
    import os

    from kepler_amd.torch_batch import current_stream_handle
    from oracle.gofmt import joules, label_pairs, sample_line, watts

    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "collector_snapshot.json")))
    node_name, zones, nd = fx["node_name"], fx["zones"], fx["node"]
    Z = len(zones)
    acc = accel.Accel(Z, nodes=1, proc_slots=1, ctr_slots=1, vm_slots=1, pod_slots=1)
    # the node x zone tables; activeEnergy and ProcessTotalCPUTimeDelta pass the derive guard
    # (process.go:124) and ActivePower is the snapshot's, so ratio x ActivePower = the usage's power
    acc.upload("node_energy_total", np.array(nd["energy_total"], dtype=np.uint64))
    acc.upload("node_active_total", np.array(nd["active_energy_total"], dtype=np.uint64))
    acc.upload("node_idle_total", np.array(nd["idle_energy_total"], dtype=np.uint64))
    acc.upload("node_active_energy", np.array(nd["active_energy_total"], dtype=np.uint64))
    acc.upload("node_power", np.array(nd["power"], dtype=np.float64))
    acc.upload("node_active_power", np.array(nd["active_power"], dtype=np.float64))
    acc.upload("node_idle_power", np.array(nd["idle_power"], dtype=np.float64))
    acc.upload("node_usage_ratio", np.array([nd["usage_ratio"]], dtype=np.float64))
    acc.upload("node_cpu_delta", np.array([1.0]))
    zi = {z["name"]: i for i, z in enumerate(zones)}
    wl = fx["workloads"]
    for kind in ("proc", "ctr", "vm", "pod"):
        u = wl[{"proc": "process", "ctr": "container", "vm": "vm", "pod": "pod"}[kind]]["usage"]
        e = np.zeros(Z, dtype=np.uint64)
        e[zi[u["zone"]]] = u["energy_total"]
        acc.upload(f"{kind}_energy", e)
        if kind == "pod":  # stored
            p = np.zeros(Z)
            p[zi[u["zone"]]] = u["power"]
            acc.upload("pod_power", p)
        else:  # derived: ratio x the node's ActivePower of the zone
            acc.upload(f"{kind}_ratio", np.array([u["power"] / nd["active_power"][zi[u["zone"]]]]))
            acc.upload(f"{kind}_node", np.array([0], dtype=np.uint32))
    s = current_stream_handle()

    def lines(table, metric, label_text, zone_names, zone_order):
        d_labels = torch.from_numpy(np.frombuffer(label_text.encode(), np.uint8).copy()).cuda()
        d_loff = torch.tensor([0, len(label_text.encode())], dtype=torch.int64, device="cuda")
        d_line_off = torch.zeros(len(zone_names) + 1, dtype=torch.int64, device="cuda")
        args = (table, metric, 0, 1, zone_names, d_labels.data_ptr(), d_loff.data_ptr(), d_line_off.data_ptr())
        total = acc.format_lines(*args, zone_order=zone_order, stream=s)
        out = torch.zeros(total, dtype=torch.uint8, device="cuda")
        acc.format_lines(*args, out_ptr=out.data_ptr(), out_cap=total, zone_order=zone_order, stream=s)
        acc.sync(s)
        return bytes(out.cpu().numpy()).decode()

    text, want = [], []
    node_tables = [("kepler_node_cpu_joules_total", "node_energy_total"), ("kepler_node_cpu_watts", "node_power"),
                   ("kepler_node_cpu_active_joules_total", "node_active_total"),
                   ("kepler_node_cpu_idle_joules_total", "node_idle_total"),
                   ("kepler_node_cpu_active_watts", "node_active_power"),
                   ("kepler_node_cpu_idle_watts", "node_idle_power")]
    for metric, table in node_tables:  # labels {zone, path} + node_name (power_collector.go:111-121)
        for z, zone in enumerate(zones):
            lab = label_pairs([("node_name", node_name), ("path", zone["path"])])
            text.append(lines(table, metric, lab, [zone["name"]], [z]))
            v = nd[table.replace("node_", "").replace("active_total", "active_energy_total")
                   .replace("idle_total", "idle_energy_total")][z]
            want.append(sample_line(metric, lab, zone["name"], joules(int(v)) if "joules" in metric else watts(v)))
    # usage ratio: no zone label (power_collector.go:123-126); the value from the device
    d_out = torch.zeros(W, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(1, dtype=torch.uint8, device="cuda")
    acc.format_values("node_usage_ratio", 0, 1, d_out.data_ptr(), d_len.data_ptr(), s)
    acc.sync(s)
    ratio_text = bytes(d_out.cpu().numpy()[: int(d_len.item())]).decode()
    assert ratio_text == write_float(nd["usage_ratio"])
    text.append(f'kepler_node_cpu_usage_ratio{{node_name="{node_name}"}} {ratio_text}\n')
    want.append(text[-1])
    p, c, v, q = wl["process"], wl["container"], wl["vm"], wl["pod"]
    fams = [  # label sets of power_collector.go:128-139 (state "running": :226-241), zone spliced last
        ("proc", "kepler_process_cpu", [("pid", p["pid"]), ("comm", p["comm"]), ("exe", p["exe"]),
                                        ("type", p["type"]), ("state", "running"), ("container_id", p["container_id"]),
                                        ("vm_id", p["vm_id"]), ("node_name", node_name)], p["usage"]),
        ("ctr", "kepler_container_cpu", [("container_id", c["id"]), ("container_name", c["name"]),
                                         ("runtime", c["runtime"]), ("state", "running"), ("pod_id", c["pod_id"]),
                                         ("node_name", node_name)], c["usage"]),
        ("vm", "kepler_vm_cpu", [("vm_id", v["id"]), ("vm_name", v["name"]), ("hypervisor", v["hypervisor"]),
                                 ("state", "running"), ("node_name", node_name)], v["usage"]),
        ("pod", "kepler_pod_cpu", [("pod_id", q["id"]), ("pod_name", q["name"]), ("pod_namespace", q["namespace"]),
                                   ("state", "running"), ("node_name", node_name)], q["usage"]),
    ]
    for kind, prefix, pairs, u in fams:
        lab = label_pairs(pairs)
        for suffix, table, conv in (("_joules_total", f"{kind}_energy", lambda x: joules(int(x))),
                                    ("_watts", f"{kind}_power", watts)):
            text.append(lines(table, prefix + suffix, lab, [u["zone"]], [zi[u["zone"]]]))
            want.append(sample_line(prefix + suffix, lab, u["zone"],
                                    conv(u["energy_total"] if suffix == "_joules_total" else u["power"])))
    # the Go side's line (CPUTotalTime is the informer's, power_collector.go:315-321)
    secs = label_pairs([("pid", p["pid"]), ("comm", p["comm"]), ("exe", p["exe"]), ("type", p["type"]),
                        ("container_id", p["container_id"]), ("vm_id", p["vm_id"]), ("node_name", node_name)])
    text.append(f"kepler_process_cpu_seconds_total{{{secs}}} {write_float(p['cpu_total_time'])}\n")
    want.append(text[-1])
    assert "".join(text) == "".join(want)  # byte-exact against the restated expfmt
    samples = _parse_exposition("".join(text))
    assert sorted({n for n, _, _ in samples}) == sorted(fx["expected_metric_names"])  # :307-328
    node_js = [(lb, val) for n, lb, val in samples if n == "kepler_node_cpu_joules_total"]
    assert sorted({lb["zone"] for lb, _ in node_js}) == sorted(fx["expected_zone_names"])  # :419-432
    assert sorted({lb["path"] for lb, _ in node_js}) == sorted(fx["expected_zone_paths"])
    for chk in fx["node_checks"]:  # :342-418
        got = [val for n, lb, val in samples if n == chk["metric"] and lb.get("path") == chk["path"]]
        assert got == [chk["value"]], chk
        assert all(lb["node_name"] == node_name for n, lb, _ in samples if n == chk["metric"])
    for chk in fx["label_checks"]:  # :437-483
        for metric, value in zip(chk["metrics"], chk["values"]):
            hits = [val for n, lb, val in samples
                    if n == metric and all(lb.get(k) == x for k, x in chk["labels"].items())]
            assert hits == [value], (metric, chk["labels"], hits)
    acc.close()
