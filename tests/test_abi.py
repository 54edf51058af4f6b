"""The C-ABI library: loads, exports every declared symbol, struct layout (CPU)."""

import ctypes
import os
import re
import subprocess

import pytest

from kepler_amd import accel

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "kepler_accel.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kacc_[a-z_0-9]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(accel.LIB_PATH):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "kepler_amd", "csrc")], check=True)
    return accel.load()


def test_exports_every_declared_symbol(lib):
    decl = declared_functions()
    assert sorted(accel.EXPORTS) == decl
    for name in decl:
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", accel.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (kacc_\w+)", out))
    assert set(decl) <= exported


def test_rccl_is_loaded_lazily_and_reported(lib):
    """RCCL is not a link-time dependency (single-GPU users and the C client need no
    librccl); kacc_cluster_rccl names the RCCL the collectives would run with."""
    out = subprocess.run(["readelf", "-d", accel.LIB_PATH], capture_output=True, text=True).stdout
    needed = re.findall(r"\(NEEDED\)\s+Shared library: \[([^\]]+)\]", out)
    assert needed and not any("rccl" in n for n in needed), needed
    version, path = accel.Cluster.rccl()
    assert version // 10000 == 2, version  # NCCL_MAJOR of the headers the library was built with
    assert os.path.exists(path), path


def test_abi_version(lib):
    assert lib.kacc_abi_version() == accel.KACC_ABI_VERSION


def test_struct_layout_matches_header(tmp_path):
    c = tmp_path / "layout.c"
    fields = ["n_nodes", "flags"] + accel.INTERVAL_ARRAYS + accel.INTERVAL_OUTPUTS
    body = "\n".join(f'printf("%zu\\n", offsetof(kacc_interval, {f}));' for f in fields)
    c.write_text(f"""
#include <stddef.h>
#include <stdio.h>
#include "kepler_accel.h"
int main(void) {{
  printf("%zu\\n%zu\\n", sizeof(kacc_interval), sizeof(kacc_config));
  printf("%zu\\n", offsetof(kacc_config, nodes));
  {body}
  return 0;
}}""")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)], check=True)
    vals = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    assert vals[0] == ctypes.sizeof(accel.KaccInterval)
    assert vals[1] == ctypes.sizeof(accel.KaccConfig)
    assert vals[2] == accel.KaccConfig.nodes.offset
    for f, off in zip(fields, vals[3:]):
        assert getattr(accel.KaccInterval, f).offset == off, f


def test_export_sums_layout_matches_header(tmp_path):
    """kacc_export_sums (ABI 5): the ctypes twin's size and every field offset."""
    c = tmp_path / "xs.c"
    fields = [f for f, _ in accel.KaccExportSums._fields_]
    body = "\n".join(f'printf("%zu\\n", offsetof(kacc_export_sums, {f}));' for f in fields)
    c.write_text(f"""
#include <stddef.h>
#include <stdio.h>
#include "kepler_accel.h"
int main(void) {{
  printf("%zu\\n", sizeof(kacc_export_sums));
  {body}
  return 0;
}}""")
    exe = tmp_path / "xs"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)], check=True)
    vals = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    assert vals[0] == ctypes.sizeof(accel.KaccExportSums)
    for f, off in zip(fields, vals[1:]):
        assert getattr(accel.KaccExportSums, f).offset == off, f


def test_interval_bytes_formula(lib):
    # node 76+96Z, proc 24+16Z (Δ 8 + slot 4 + prev 8Z in; totals 8Z + ratio 8 +
    # node 4 out: the power is derived, ABI 3), ctr 44+16Z, vm 28+16Z (ratio + node stored
    # for those too), pod 32+24Z (pod power stored)
    z = 4
    assert accel.interval_bytes(z, 1, 0, 0, 0, 0) == 76 + 96 * z
    assert accel.interval_bytes(z, 0, 1, 0, 0, 0) == 24 + 16 * z
    assert accel.interval_bytes(z, 0, 0, 1, 1, 1) == (44 + 28 + 32) + (16 + 16 + 24) * z
    n, p, c, v, q = 10_000, 20_000_000, 1_975_000, 200_000, 711_000
    assert accel.interval_bytes(z, n, p, c, v, q) == n * 460 + p * 88 + c * 108 + v * 92 + q * 128
    # KACC_F_STABLE_SLOT_NODES: a process row's node is not rewritten (4 B)
    stable = accel.KACC_F_STABLE_SLOT_NODES
    assert accel.interval_bytes(z, 0, 1, 0, 0, 0, stable) == 20 + 16 * z
    assert accel.interval_bytes(z, n, p, c, v, q, stable) == accel.interval_bytes(z, n, p, c, v, q) - 4 * p
    assert accel.intervals_bytes(z, n, p, c, v, q, 3, False, stable) == 3 * accel.interval_bytes(z, n, p, c, v, q, stable)


def test_create_error_visible_from_another_thread(lib):
    """kacc_create's error is process-wide: a cgo caller's next C call may land on
    another OS thread (goroutine migration) and must still see the message."""
    import threading

    cfg = accel.KaccConfig(99, 0, 1, 1, 1, 1, 1)  # zones out of range
    rc = []
    t = threading.Thread(target=lambda: rc.append(lib.kacc_create(0, ctypes.byref(cfg), ctypes.byref(ctypes.c_void_p()))))
    t.start()
    t.join()
    assert rc == [accel.KACC_EINVAL]
    assert "zones must be" in accel.last_error(None)
    buf = ctypes.create_string_buffer(8)
    full = lib.kacc_last_error_copy(None, buf, len(buf))
    assert full > 7 and len(buf.value) == 7  # truncated, NUL-terminated


def test_create_multi_bad_arguments(lib):
    """kacc_create_multi rejects non-contiguous shards of one device before creating anything."""
    cfg = (accel.KaccConfig * 3)(*[accel.KaccConfig(2, 0, 1, 1, 1, 1, 1)] * 3)
    devs = (ctypes.c_int * 3)(0, 1, 0)
    ctxs = (ctypes.c_void_p * 3)()
    h = ctypes.c_void_p()
    assert lib.kacc_create_multi(devs, 3, cfg, ctypes.byref(h), ctxs) == accel.KACC_EINVAL
    assert "not contiguous" in accel.last_error(None)
    assert lib.kacc_allreduce_namespaces(None, 0, None, None, None, None, None, None, None, None) == accel.KACC_EINVAL


def test_struct_layout_shape(tmp_path):
    c = tmp_path / "shape.c"
    c.write_text("""
#include <stddef.h>
#include <stdio.h>
#include "kepler_accel.h"
int main(void) { printf("%zu %zu\\n", sizeof(kacc_shape), offsetof(kacc_shape, intervals)); return 0; }""")
    exe = tmp_path / "shape"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)], check=True)
    size, off = (int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split())
    assert size == ctypes.sizeof(accel.KaccShape) and off == accel.KaccShape.intervals.offset


def test_bad_arguments_do_not_crash(lib):
    cfg = accel.KaccConfig(0, 0, 1, 1, 1, 1, 1)  # zones = 0 is invalid
    h = ctypes.c_void_p()
    assert lib.kacc_create(0, ctypes.byref(cfg), ctypes.byref(h)) == accel.KACC_EINVAL
    assert b"zones" in lib.kacc_last_error(None)
    assert lib.kacc_reset(None) == accel.KACC_EINVAL
    assert lib.kacc_run_interval(None, None, None) == accel.KACC_EINVAL


def test_loopback_collectives_export_what_the_engine_binds():
    """tests/c/loopback_rccl.cpp (the two-rank cluster test's stand-in for RCCL, loaded via
    KACC_RCCL_PATH) exports every entry point kacc_cluster.hip dlsym()s."""
    import ctypes
    import re

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-s", "-C", os.path.join(root, "tests", "c")], check=True)
    lib = ctypes.CDLL(os.path.join(root, "tests", "c", "build", "libkacc_loopback_rccl.so"))
    with open(os.path.join(root, "kepler_amd", "csrc", "kacc_cluster.hip")) as f:
        names = re.findall(r'sym\(r\.\w+, "(nccl\w+)"\)', f.read())
    assert len(names) == 11
    for n in names:
        assert hasattr(lib, n), n
    v = ctypes.c_int()
    assert lib.ncclGetVersion(ctypes.byref(v)) == 0 and v.value // 10000 == 2
