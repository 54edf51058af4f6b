"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product.

Independent pure-Python restatement of the host packer (kacc_pack), written in
the informer's own shape (internal/resource/informer.go): per node, walk the
running processes in /proc listing order (refreshProcesses :182-205),
collect containers and VMs by first appearance (refreshContainers :223-249,
refreshVMs :251-273), look up each container's pod (refreshPods :275-326,
ContainersNoPod last), then lay the rows out as kepler_accel.h requires.
"""

from __future__ import annotations

import numpy as np

REGULAR, CONTAINER, VM = 0, 1, 2
NO_POD = 0xFFFFFFFFFFFFFFFF


def pack_ref(rec_off, pid, cpu_delta, ptype, ctr_key, vm_key, pod_key=None, pod_ns=None) -> dict:
    out = {k: [] for k in ("proc_cpu_delta", "proc_key", "row_record", "ctr_proc_end", "ctr_key", "vm_proc_end",
                           "vm_key", "pod_ctr_end", "pod_key", "pod_ns")}
    offs = {k: [0] for k in ("proc_off", "ctr_off", "vm_off", "pod_off")}
    for n in range(len(rec_off) - 1):
        recs = range(int(rec_off[n]), int(rec_off[n + 1]))
        containers = {}  # container key -> [record indices] (dict keeps first appearance order)
        ctr_pod = {}
        vms = {}
        rest = []
        for r in recs:  # /proc listing order
            t = int(ptype[r])
            if t == CONTAINER:
                k = int(ctr_key[r])
                if k not in containers:
                    containers[k] = []
                    ctr_pod[k] = (int(pod_key[r]) if pod_key is not None else NO_POD,
                                  int(pod_ns[r]) if pod_ns is not None else 0)
                containers[k].append(r)
            elif t == VM:
                vms.setdefault(int(vm_key[r]), []).append(r)
            else:
                rest.append(r)
        pods = {}  # pod key -> [container keys], first appearance
        no_pod = []
        for k in containers:  # one fixed order of the running-containers map
            pk, ns = ctr_pod[k]
            if pk >= 0xFFFFFFFFFFFFFFFE:
                no_pod.append(k)
            else:
                pods.setdefault(pk, (ns, []))[1].append(k)
        ctr_order = [k for pk in pods for k in pods[pk][1]] + no_pod
        base = offs["proc_off"][-1]
        row = base
        rows = []
        for k in ctr_order:
            rows += containers[k]
            row += len(containers[k])
            out["ctr_proc_end"].append(row)
            out["ctr_key"].append(k)
        for k, rr in vms.items():
            rows += rr
            row += len(rr)
            out["vm_proc_end"].append(row)
            out["vm_key"].append(k)
        rows += rest
        cend = offs["ctr_off"][-1]
        for pk, (ns, ks) in pods.items():
            cend += len(ks)
            out["pod_ctr_end"].append(cend)
            out["pod_key"].append(pk)
            out["pod_ns"].append(ns)
        for r in rows:
            out["proc_cpu_delta"].append(float(cpu_delta[r]))
            out["proc_key"].append(int(pid[r]))
            out["row_record"].append(r)
        offs["proc_off"].append(base + len(rows))
        offs["ctr_off"].append(offs["ctr_off"][-1] + len(ctr_order))
        offs["vm_off"].append(offs["vm_off"][-1] + len(vms))
        offs["pod_off"].append(offs["pod_off"][-1] + len(pods))
    dt = dict(proc_cpu_delta=np.float64, ctr_key=np.uint64, vm_key=np.uint64, pod_key=np.uint64)
    res = {k: np.array(v, dtype=dt.get(k, np.uint32)) for k, v in out.items()}
    res.update({k: np.array(v, dtype=np.uint32) for k, v in offs.items()})
    return res
