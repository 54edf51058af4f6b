"""Exposition number formatting oracle (oracle/gofmt.py) — CPU.

Pins the restatement of Go's strconv.FormatFloat(f, 'g', -1, 64) and expfmt
writeFloat to outputs Go is documented / known to produce (the formatting
lives in the Go standard library and prometheus/common, neither of which is
in the reference; the reference's own collector tests compare float values,
not text): %e from exponent 6 on (process_start_time_seconds 1.6983e+09), two
exponent digits at least, shortest round-trip digits, writeFloat's spelled-out
specials.
"""

import math
import struct

import numpy as np
import pytest

from oracle.gofmt import go_g, joules, watts, write_float

KNOWN = [
    (1e6, "1e+06"), (1234567.5, "1.2345675e+06"), (123456.0, "123456"), (999999.0, "999999"),
    (9999999.0, "9.999999e+06"), (100000.0, "100000"), (0.0001, "0.0001"), (0.00001, "1e-05"),
    (0.000123, "0.000123"), (0.0000123, "1.23e-05"), (1e21, "1e+21"), (1e100, "1e+100"),
    (5e-324, "5e-324"), (1.7976931348623157e308, "1.7976931348623157e+308"), (0.1, "0.1"),
    (0.3, "0.3"), (0.1 + 0.2, "0.30000000000000004"), (2.0 ** 63, "9.223372036854776e+18"),
    (12345.678, "12345.678"), (-2.5, "-2.5"), (1.6983e9, "1.6983e+09"), (1.5, "1.5"),
]


@pytest.mark.parametrize("x,want", KNOWN, ids=[w for _, w in KNOWN])
def test_go_g_known(x, want):
    assert go_g(x) == want


def test_write_float_specials():
    assert write_float(1.0) == "1" and write_float(0.0) == "0" and write_float(-0.0) == "0"
    assert write_float(-1.0) == "-1" and write_float(float("nan")) == "NaN"
    assert write_float(float("inf")) == "+Inf" and write_float(float("-inf")) == "-Inf"


def test_units():
    assert joules(1_500_000) == 1.5 and watts(2.5e6) == 2.5
    assert write_float(joules(10**6)) == "1"  # Joules() of 1 J is exactly 1


def test_round_trip_and_shortest():
    rng = np.random.default_rng(3)
    for b in rng.integers(0, 2**63, size=20000, dtype=np.int64).tolist():
        x = struct.unpack("<d", struct.pack("<q", b))[0]
        if not math.isfinite(x) or x in (0.0, 1.0, -1.0):
            continue
        s = write_float(x)
        assert float(s) == x, (x, s)
        mant = s.split("e")[0].replace(".", "").replace("-", "").lstrip("0")
        assert len(mant) <= 17


def test_sample_line_layout_and_escaping():
    """expfmt text: label pairs sorted by name (client_golang MakeLabelPairs),
    label values escaped (backslash, double quote, newline), zone last."""
    from oracle.gofmt import escape_label_value, label_pairs, sample_line

    assert escape_label_value('a"b\\c\nd') == 'a\\"b\\\\c\\nd'
    # node_name is the descriptors' const label (power_collector.go:17, :63-95), merged and sorted
    labels = label_pairs([("pid", "42"), ("comm", 'sh "x"'), ("vm_id", ""), ("container_id", "c1"),
                          ("exe", "/bin/sh"), ("state", "running"), ("type", "container"), ("node_name", "n7")])
    assert labels == ('comm="sh \\"x\\"",container_id="c1",exe="/bin/sh",node_name="n7",pid="42",'
                      'state="running",type="container",vm_id=""')
    assert sample_line("kepler_process_cpu_joules_total", labels, "package", joules(1_500_000)) == (
        'kepler_process_cpu_joules_total{' + labels + ',zone="package"} 1.5\n')
    assert sample_line("kepler_pod_cpu_watts", 'pod_id="p"', "dram", watts(0.0)).endswith('zone="dram"} 0\n')
    # "zone" sorts after every other label name of the workload families
    # (power_collector.go:128-139, plus the node_name const label)
    for names in (["comm", "container_id", "exe", "pid", "state", "type", "vm_id"],
                  ["container_id", "container_name", "pod_id", "runtime", "state"],
                  ["hypervisor", "state", "vm_id", "vm_name"], ["pod_id", "pod_name", "pod_namespace", "state"]):
        assert sorted(names + ["node_name", "zone"])[-1] == "zone"
