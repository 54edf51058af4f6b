"""BASELINE config 5 at its real size — MI355X only.

fleet.config_layout(5): 1,000 heavy-tailed nodes of 10k-50k processes (18M rows, Z = 4), the
bench's workload.  A first read, then 3 intervals in ONE kacc_run_intervals call over one
layout (the chunk items generated once and reused), with churn, read errors and counter
wraparound: every table bit-exact against the oracle over every node (the shape test in
test_gpu_parity.py runs 7 such nodes for 60 intervals; this one the full fleet).
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
def test_config5_full_size_bit_exact():
    from oracle.oracle import Oracle

    layout = fleet.config_layout(5)
    sizes = layout.sizes()
    assert sizes["n_nodes"] == 1000 and sizes["n_procs"] > 10_000_000
    assert layout.fast_flag() == 0  # big nodes: the chunked path
    sim = fleet.FleetSim(layout, seed=5, churn=0.02, read_error_frac=0.02, max_energy=fleet.MAX_ENERGY_FAKE)
    acc = accel.Accel(layout.zones, **layout.capacities())
    ora = Oracle(layout.zones, **layout.capacities())
    s = current_stream_handle()
    first = sim.next_interval()
    acc.run_intervals([interval_from_tensors(to_device(first), sizes)], s)
    ora.interval(first, sizes)
    ivs = [sim.next_interval() for _ in range(3)]
    statics = to_device(layout.static_arrays())
    dev = []
    for a in ivs:
        t = to_device({k: v for k, v in a.items() if k not in statics})
        t.update(statics)
        dev.append(t)
    acc.run_intervals([interval_from_tensors(t, sizes) for t in dev], s)
    acc.sync(s)
    for a in ivs:
        ora.interval(a, sizes)
    assert_tables_equal(acc.download, ora.state, "config 5")
    acc.close()
