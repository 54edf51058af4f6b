"""kacc_table_read (device-side scrape of a snapshot) — MI355X only.

Every table, read into device memory after two intervals, equals kacc_table_download of the same
logical range bit for bit: derived process / container / VM powers (ratio x the node's
ActivePower behind the process.go:124-142 guard), the pod tables gathered out of their records,
plain copies of the rest; sub-ranges and range errors as the download's.
"""

import numpy as np
import pytest
import torch

from kepler_amd import accel, fleet
from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu_ready():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    accel.load()
    torch.cuda.set_stream(torch.cuda.Stream())


_TORCH = {np.dtype(np.uint64): torch.int64, np.dtype(np.int64): torch.int64, np.dtype(np.float64): torch.float64,
          np.dtype(np.uint32): torch.int32, np.dtype(np.int32): torch.int32}


@pytest.mark.parametrize("zones", [2, 4])
def test_table_read_equals_download(zones):
    L = fleet.make_layout(12, [700, 2000, 3, 0, 64, 1500] * 2, zones, seed=5, n_namespaces=4, vm_frac=0.05)
    acc = accel.Accel(zones, **L.capacities())
    sim = fleet.FleetSim(L, seed=5, read_error_frac=0.1, churn=0.03)
    s = current_stream_handle()
    keep = []
    for _ in range(2):
        t = to_device(sim.next_interval())
        acc.run_interval(interval_from_tensors(t, L.sizes(), L.fast_flag()), s)
        keep.append(t)
    acc.sync(s)
    for name, dt in accel.TABLES:
        eb, total = acc.table_info(name)
        if total == 0:
            continue
        want = acc.download(name)
        buf = torch.full((total,), -1, dtype=_TORCH[np.dtype(dt)], device="cuda")
        acc.read(name, buf.data_ptr(), stream=s)
        acc.sync(s)
        got = buf.cpu().numpy().view(want.dtype)
        np.testing.assert_array_equal(got.view(np.uint8), want.view(np.uint8), err_msg=name)
        # a sub-range lands at the start of dev_dst
        lo, n = total // 3, max(total // 4, 1)
        sub = torch.zeros((n,), dtype=buf.dtype, device="cuda")
        acc.read(name, sub.data_ptr(), first=lo, count=n, stream=s)
        acc.sync(s)
        np.testing.assert_array_equal(sub.cpu().numpy().view(want.dtype).view(np.uint8),
                                      want[lo:lo + n].view(np.uint8), err_msg=f"{name}[{lo}:+{n}]")
    power = acc.download("proc_power")
    assert np.count_nonzero(power) > 0  # the derive produced real powers
    with pytest.raises(accel.AccelError):
        acc.read("proc_power", buf.data_ptr(), first=1, count=acc.table_info("proc_power")[1], stream=s)
    acc.close()
