"""BASELINE config 2 at its real size — MI355X only.

fleet.config_layout(2): 1,000 nodes x 1,000 processes (1M rows, Z = 2), the grid and
residency the config's own launch has (1,000 node workgroups), with 2 % churn, 2 % read
errors and fake-meter counters that wrap (MaxEnergy 1e6 µJ, fake_cpu_power_meter.go).
Every table bit-exact against the oracle: one interval per kacc_run_interval call (each
compared), and 12 intervals in ONE kacc_run_intervals call (the one-launch carry path the
config's 60-interval bench line takes).
"""

import pytest
import torch

from kepler_amd import accel, fleet
from kepler_amd.torch_batch import current_stream_handle, interval_from_tensors, to_device
from table_check import assert_tables_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu_ready():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    accel.load()
    torch.cuda.set_stream(torch.cuda.Stream())


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode", ["per_interval", "one_call_x12"])
def test_config2_full_size_bit_exact(mode):
    from oracle.oracle import Oracle

    layout = fleet.config_layout(2)
    sizes = layout.sizes()
    assert sizes["n_nodes"] == 1000 and sizes["n_procs"] == 1_000_000 and layout.zones == 2
    sim = fleet.FleetSim(layout, seed=22, churn=0.02, read_error_frac=0.02, max_energy=fleet.MAX_ENERGY_FAKE)
    acc = accel.Accel(layout.zones, **layout.capacities())
    ora = Oracle(layout.zones, **layout.capacities())
    s = current_stream_handle()
    flags = layout.fast_flag()
    first = sim.next_interval()
    acc.run_interval(interval_from_tensors(to_device(first), sizes, flags), s)
    ora.interval(first, sizes)
    if mode == "per_interval":
        for it in range(4):
            a = sim.next_interval()
            acc.run_interval(interval_from_tensors(to_device(a), sizes, flags), s)
            acc.sync(s)
            ora.interval(a, sizes)
            assert_tables_equal(acc.download, ora.state, f"config 2, interval {it + 1}")
    else:
        ivs = [sim.next_interval() for _ in range(12)]
        statics = to_device(layout.static_arrays())
        dev = []
        for a in ivs:
            t = to_device({k: v for k, v in a.items() if k not in statics})
            t.update(statics)
            dev.append(t)
        acc.run_intervals([interval_from_tensors(t, sizes, flags) for t in dev], s)
        acc.sync(s)
        for a in ivs:
            ora.interval(a, sizes)
        assert_tables_equal(acc.download, ora.state, "config 2, 12 intervals in one call")
    acc.close()
