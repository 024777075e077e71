"""examples/camera_stereo_vision.cpp -- the reference's main() flow on the
engine through include/sva.hpp -- compiles as plain C++ and (GPU) runs to OK."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "stereovisionarray_amd")


@pytest.fixture(scope="module")
def example(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("ex") / "camera_stereo_vision")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I",
                    os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "examples", "camera_stereo_vision.cpp"), "-L", LIBDIR,
                    "-lsva", f"-Wl,-rpath,{LIBDIR}", "-o", out], check=True)
    return out


def test_example_builds(example):
    assert os.path.exists(example)


@pytest.mark.gpu
def test_example_runs(example):
    r = subprocess.run([example, "640", "480"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr
