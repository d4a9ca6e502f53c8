"""The C++ facade (include/beast_amd/*.hpp) compiles against the C ABI and
links with libbeast_pmd.so; on a GPU the impl_base<true>-style round trip
(tests/cpp/facade_roundtrip.cpp) passes, on a CPU-only host it reports the
missing engine instead of falling back."""
import os
import subprocess

import pytest

from beast_amd import build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "facade_roundtrip.cpp")
OUT = os.path.join(ROOT, "tests", "cpp", "_build", "facade_roundtrip")


def _build():
    build.build()
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    libdir = os.path.dirname(build.LIB)
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-I", os.path.join(ROOT, "include"), SRC, "-o", OUT,
                    "-L", libdir, "-lbeast_pmd", f"-Wl,-rpath,{libdir}", "-L/opt/rocm/lib", "-lamdhip64",
                    "-Wl,-rpath,/opt/rocm/lib"], check=True)
    return OUT


def test_facade_compiles_and_links():
    assert os.path.exists(_build())


@pytest.mark.gpu
def test_facade_roundtrip_on_gpu():
    r = subprocess.run([_build()], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("ok") == 4
