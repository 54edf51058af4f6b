"""ORACLE — TEST INFRASTRUCTURE ONLY.

Restatement of the Prometheus text exposition's number formatting for the
attribution values, to check kacc_format_values:

* prometheus/common v0.62.0 (go.mod:68, via client_golang v1.22.0, go.mod:13;
  neither is vendored in the reference): expfmt writeFloat writes 1 -> "1",
  0 -> "0" (also -0), -1 -> "-1", NaN -> "NaN", +Inf -> "+Inf", -Inf -> "-Inf",
  anything else with strconv.AppendFloat(f, 'g', -1, 64);
* Go 1.23 strconv (toolchain go1.23.3, go.mod:5), 'g' with precision -1: the
  shortest digit string that round-trips; %e form ("d.ddde±XX", at least two
  exponent digits) when the decimal exponent is < -4 or >= 6 (precision 6 is
  used for the decision in shortest mode), else %f form;
* device/energy.go:30-32 Joules() = float64(e) / 1e6, :57-59 Watts() = p / 1e6.

Python's repr() yields the same shortest round-trip digits; the layout rules
above are applied to them here.
"""

from __future__ import annotations

import math
from decimal import Decimal


def shortest(x: float):
    """(digits str, dp) with value = 0.digits x 10^dp, x finite and nonzero."""
    sign, digs, exp = Decimal(repr(abs(x))).as_tuple()
    s = "".join(map(str, digs)).lstrip("0")
    trail = len(s) - len(s.rstrip("0"))
    s = s.rstrip("0")
    exp += trail
    return s, len(s) + exp


def go_g(x: float) -> str:
    """strconv.FormatFloat(x, 'g', -1, 64)."""
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "+Inf" if x > 0 else "-Inf"
    if x == 0:
        return "-0" if math.copysign(1.0, x) < 0 else "0"
    neg = x < 0
    d, dp = shortest(x)
    nd = len(d)
    e = dp - 1
    out = "-" if neg else ""
    if e < -4 or e >= 6:  # fmtE with nd-1 fraction digits
        out += d[0]
        if nd > 1:
            out += "." + d[1:]
        out += "e" + ("-" if e < 0 else "+")
        a = abs(e)
        out += f"{a:02d}"
        return out
    # fmtF with max(nd - dp, 0) fraction digits
    if dp > 0:
        out += d[:dp] + "0" * max(dp - nd, 0)
    else:
        out += "0"
    frac = max(nd - dp, 0)
    if frac:
        out += "." + "".join(d[dp + i] if 0 <= dp + i < nd else "0" for i in range(frac))
    return out


def write_float(f: float) -> str:
    """expfmt writeFloat (prometheus/common v0.62.0 text_create.go)."""
    if f == 1:
        return "1"
    if f == 0:
        return "0"
    if f == -1:
        return "-1"
    if math.isnan(f):
        return "NaN"
    if math.isinf(f):
        return "+Inf" if f > 0 else "-Inf"
    return go_g(f)


def joules(e: int) -> float:
    return float(e) / 1e6


def watts(p: float) -> float:
    return p / 1e6


def escape_label_value(v: str) -> str:
    """expfmt text format label-value escaping: backslash, double quote, newline."""
    return v.replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n")


def label_pairs(pairs) -> str:
    """`name="value",...` in label-name order (client_golang MakeLabelPairs sorts by name)."""
    return ",".join(f'{k}="{escape_label_value(v)}"' for k, v in sorted(pairs))


def sample_line(metric: str, labels: str, zone: str, value: float) -> str:
    """One expfmt text line of a Kepler workload metric; "zone" sorts after every
    other label of the process / container / VM / pod families."""
    return f'{metric}{{{labels},zone="{escape_label_value(zone)}"}} {write_float(value)}\n'
