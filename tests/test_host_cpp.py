"""Build and run the C++ host-mirror tests (tests/cpp/test_host.cpp) against
include/sva.hpp + libsva.so."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "stereovisionarray_amd")


@pytest.fixture(scope="module")
def binary(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("cpp") / "test_host")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I",
                    os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "cpp", "test_host.cpp"),
                    "-L", LIBDIR, "-lsva", f"-Wl,-rpath,{LIBDIR}", "-o", out], check=True)
    return out


def test_host_cpu(binary):
    r = subprocess.run([binary, "cpu"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_host_gpu(binary):
    r = subprocess.run([binary, "gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
