"""The C ABI from a plain C99 program (what a cgo binding compiles against).

CPU: the header compiles as strict C99 and the program links against the
library.  GPU: the program runs two intervals through the pinned batch path
and checks the reference-style known answers itself.
"""

import os
import subprocess

import pytest

from kepler_amd import accel

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c", "abi_client.c")


def build(out):
    if not os.path.exists(accel.LIB_PATH):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "kepler_amd", "csrc")], check=True)
    libdir = os.path.dirname(accel.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic", "-I", os.path.join(ROOT, "include"),
                    SRC, "-o", out, "-L", libdir, "-lkepler_accel", f"-Wl,-rpath,{libdir}"], check=True)


def test_c_client_compiles_and_links(tmp_path):
    build(str(tmp_path / "abi_client"))


@pytest.mark.gpu
def test_c_client_runs_on_gpu(tmp_path):
    exe = str(tmp_path / "abi_client")
    build(exe)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "abi_client ok" in r.stdout
