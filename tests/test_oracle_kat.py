"""The oracle against the reference's own known-answer tests (CPU)."""

import numpy as np
import pytest

from kat_runner import load_golden_fleet, load_kats, run_case

KATS = load_kats()


class OracleBackend:
    def __init__(self, zones, caps):
        from oracle.oracle import Oracle

        self.o = Oracle(zones, **caps)

    def upload(self, table, first, values):
        t = self.o.state[table]
        t[first:first + len(values)] = values

    def interval(self, arrays, sizes, flags):
        self.o.interval(arrays, sizes, flags)

    def table(self, name):
        return self.o.state[name]


class GoFaithfulBackend(OracleBackend):
    def __init__(self, zones, caps):
        from oracle.oracle import GoFaithful

        self.o = GoFaithful(zones, **caps)

    def upload(self, table, first, values):
        pytest.skip("go-faithful baseline keeps its previous snapshot in maps")


@pytest.mark.parametrize("case", KATS["cases"], ids=[c["name"] for c in KATS["cases"]])
def test_oracle_kat(case, oracle_lib):
    run_case(case, OracleBackend)


@pytest.mark.parametrize("case", [c for c in KATS["cases"] if not any(iv.get("upload") for iv in c["intervals"])],
                         ids=lambda c: c["name"])
def test_gofaithful_kat(case, oracle_lib):
    run_case(case, GoFaithfulBackend)


def test_energy_delta_scalar(oracle_lib):
    from oracle.oracle import calculate_energy_delta

    case = next(c for c in KATS["cases"] if c["name"] == "calculateEnergyDelta")
    for s in case["scalar"]:
        assert calculate_energy_delta(*s["args"]) == s["value"], s["name"]


@pytest.mark.parametrize("case", KATS["aggregated"], ids=lambda c: c["name"])
def test_aggregated_zone_kat(case, oracle_lib):
    from oracle.oracle import AggregatedZone

    az = AggregatedZone(case["max"])
    assert az.max == case["agg_max"]
    for reads, want in zip(case["reads"], case["expect"]):
        assert az.energy(reads) == want


def test_go_conversions(oracle_lib):
    from oracle.oracle import go_duration_seconds, go_f64_to_u64

    # float64 -> uint64 on amd64: truncation, and the >= 2^63 branch
    assert go_f64_to_u64(59999999.99999999) == 59999999
    assert go_f64_to_u64(0.6 * 100_000_000) == 60_000_000
    assert go_f64_to_u64(2.0**63) == 2**63
    assert go_f64_to_u64(2.0**63 + 4096) == 2**63 + 4096
    assert go_f64_to_u64(-1.5) == 2**64 - 1  # int64(-1.5) = -1 reinterpreted
    assert go_f64_to_u64(-0.5) == 0
    assert go_f64_to_u64(float("nan")) == 2**63
    assert go_f64_to_u64(2.0**64) == 2**63
    # time.Duration.Seconds()
    assert go_duration_seconds(5_000_000_000) == 5.0
    assert go_duration_seconds(1_500_000_001) == 1.0 + 500_000_001 / 1e9
    assert go_duration_seconds(-2_500_000_000) == -2.0 + -500_000_000 / 1e9


def test_golden_fleet_reproduces(oracle_lib):
    """The oracle still produces the frozen golden_fleet outputs bit for bit."""
    from oracle.oracle import Oracle

    zones, caps, sizes, intervals = load_golden_fleet()
    o = Oracle(zones, **caps)
    for k, (ins, outs) in enumerate(intervals):
        o.interval(ins, sizes)
        for name, want in outs.items():
            np.testing.assert_array_equal(o.state[name], want, err_msg=f"interval {k} {name}")


def test_aggregated_zone_read_error_keeps_earlier_subzones(oracle_lib):
    """energy_zone.go:104-108: Energy() returns at the first failing sub-zone;
    the sub-zones before it have their last reading updated, the aggregate not."""
    from oracle.oracle import OracleZoneAgg

    z = OracleZoneAgg(1, 1, 2, [1000, 1000])
    e, mx, ns = z.read([100, 200])
    assert e[0] == 300 and mx[0] == 2000 and ns[0] == 0
    e, _, ns = z.read([150, 999], sub_status=[0, 1])  # sub-zone 1 fails
    assert ns[0] == 1
    e, _, ns = z.read([170, 260])  # sub-zone 0: 150 -> 170 (+20); sub-zone 1: 200 -> 260 (+60)
    assert ns[0] == 0 and e[0] == 380
    e, _, ns = z.read([180, 999], sub_status=[1, 0])  # sub-zone 0 fails first: nothing updated
    assert ns[0] == 1
    e, _, _ = z.read([190, 270])  # 170 -> 190 (+20), 260 -> 270 (+10)
    assert e[0] == 410
