"""Generate tests/golden/collector_snapshot.json (committed data; re-run to regenerate).

The snapshot and the assertions of the reference's exporter test
TestPowerCollector (internal/exporter/prometheus/collector/power_collector_test.go
@ 2025-08-24), transcribed as data: the node zones and their sysfs paths
(:181-182), the node usage of both zones (:184-215), one running process,
container, VM and pod with package-zone energy and power (:217-272), the node
name (:287), the metric family names the test expects (:307-328), the node
values it checks per zone path (:342-418) and each workload family's label set
and value (:437-483).  Values are in the engine's units: µJ (device.Joule =
1e6, energy.go:16-20) and µW (device.Watt = 1e6, energy.go:43-47); the expected
values are Joules() / Watts() (energy.go:30-32, 57-59) as the test computes them.

Usage: python tests/golden/make_collector_fixture.py
"""

from __future__ import annotations

import json
import os

J = 1_000_000
W = 1_000_000
SRC = "internal/exporter/prometheus/collector/power_collector_test.go"


def fixture():
    pkg_abs, pkg_delta, pkg_power = 12300 * J, 123 * J, 12 * W      # :184-186
    dram_abs, dram_delta, dram_power = 2340 * J, 234 * J, 2 * W     # :188-190
    zones = [  # :181-182 (NewMockRaplZone name, index, path)
        {"name": "package", "path": "/sys/class/powercap/intel-rapl/intel-rapl:0"},
        {"name": "dram", "path": "/sys/class/powercap/intel-rapl/intel-rapl:0:1"},
    ]
    node = {  # :193-215 — Energy halves are u64 integer division, Power halves f64 division
        "usage_ratio": 0.5,
        "energy_total": [pkg_abs, dram_abs],
        "active_energy_total": [pkg_delta // 2, dram_delta // 2],
        "idle_energy_total": [pkg_delta // 2, dram_delta // 2],
        "power": [pkg_power, dram_power],
        "active_power": [pkg_power / 2, dram_power / 2],
        "idle_power": [pkg_power / 2, dram_power / 2],
    }
    usage = {"zone": "package", "energy_total": 100 * J, "power": 5 * W}  # every workload, :225-229 ...
    workloads = {
        "process": {"pid": "123", "comm": "test-process", "exe": "/usr/bin/123", "type": "regular",
                    "cpu_total_time": 100.0, "container_id": "", "vm_id": "", "usage": usage},   # :217-233
        "container": {"id": "abcd-efgh", "name": "test-container", "runtime": "podman", "pod_id": "",
                      "usage": usage},                                                         # :235-247
        "vm": {"id": "abcd-efgh", "name": "test-vm", "hypervisor": "kvm", "usage": usage},    # :249-260
        "pod": {"id": "test-pod", "name": "test-pod", "namespace": "default", "usage": usage},  # :262-272
    }
    names = [  # :307-328
        "kepler_node_cpu_joules_total", "kepler_node_cpu_watts", "kepler_node_cpu_usage_ratio",
        "kepler_node_cpu_active_joules_total", "kepler_node_cpu_idle_joules_total",
        "kepler_node_cpu_active_watts", "kepler_node_cpu_idle_watts",
        "kepler_process_cpu_joules_total", "kepler_process_cpu_watts", "kepler_process_cpu_seconds_total",
        "kepler_container_cpu_joules_total", "kepler_container_cpu_watts",
        "kepler_vm_cpu_joules_total", "kepler_vm_cpu_watts",
        "kepler_pod_cpu_joules_total", "kepler_pod_cpu_watts",
    ]
    node_checks = [  # :342-418: {metric, path} -> value; node_name on every sample
        {"metric": "kepler_node_cpu_joules_total", "path": zones[0]["path"], "value": pkg_abs / J, "line": "354-356"},
        {"metric": "kepler_node_cpu_joules_total", "path": zones[1]["path"], "value": dram_abs / J, "line": "357-359"},
        {"metric": "kepler_node_cpu_watts", "path": zones[0]["path"], "value": pkg_power / W, "line": "374-376"},
        {"metric": "kepler_node_cpu_watts", "path": zones[1]["path"], "value": dram_power / W, "line": "377-379"},
        {"metric": "kepler_node_cpu_active_watts", "path": zones[0]["path"], "value": (pkg_power / 2) / W,
         "line": "395-398"},
        {"metric": "kepler_node_cpu_idle_watts", "path": zones[0]["path"], "value": (pkg_power / 2) / W,
         "line": "411-414"},
    ]
    label_checks = [  # :437-483 (assertMetricLabelValues: these labels match, then the value)
        {"metrics": ["kepler_process_cpu_joules_total", "kepler_process_cpu_watts"], "values": [100.0, 5.0],
         "labels": {"node_name": "test-node", "pid": "123", "comm": "test-process", "exe": "/usr/bin/123",
                    "type": "regular", "zone": "package"}, "line": "437-448"},
        {"metrics": ["kepler_container_cpu_joules_total", "kepler_container_cpu_watts"], "values": [100.0, 5.0],
         "labels": {"node_name": "test-node", "container_id": "abcd-efgh", "container_name": "test-container",
                    "runtime": "podman", "zone": "package"}, "line": "450-460"},
        {"metrics": ["kepler_vm_cpu_joules_total", "kepler_vm_cpu_watts"], "values": [100.0, 5.0],
         "labels": {"node_name": "test-node", "vm_id": "abcd-efgh", "vm_name": "test-vm", "hypervisor": "kvm",
                    "zone": "package"}, "line": "462-472"},
        {"metrics": ["kepler_pod_cpu_joules_total", "kepler_pod_cpu_watts"], "values": [100.0, 5.0],
         "labels": {"node_name": "test-node", "pod_id": "test-pod", "pod_name": "test-pod",
                    "pod_namespace": "default", "zone": "package"}, "line": "474-484"},
    ]
    return {"source": SRC, "node_name": "test-node", "zones": zones, "node": node, "workloads": workloads,
            "expected_metric_names": names, "expected_zone_names": ["package", "dram"],
            "expected_zone_paths": [z["path"] for z in zones], "node_checks": node_checks,
            "label_checks": label_checks}


def main():
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "collector_snapshot.json")
    with open(path, "w") as f:
        json.dump(fixture(), f, indent=1)
        f.write("\n")
    print("wrote", path)


if __name__ == "__main__":
    main()
