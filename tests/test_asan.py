"""Host sanitizer build: the CPU oracle and the
C++ host mirror's CPU tests (include/sva.hpp: pair tables, getGroups,
bresenham, Camera, OpenCV-YAML I/O) compiled with ASan + UBSan
(`make -C oracle asan`) and run; any out-of-bounds access, leak or undefined
behaviour fails the test."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN = os.path.join(ROOT, "oracle", "_asan")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", OMP_NUM_THREADS="4")


def _build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)


def test_oracle_under_asan_ubsan():
    _build()
    r = subprocess.run([os.path.join(ASAN, "oracle_asan")], capture_output=True, text=True,
                       env=ENV, timeout=600)
    assert r.returncode == 0 and "asan driver ok" in r.stdout, r.stdout + r.stderr


def test_host_mirror_under_asan_ubsan():
    _build()
    r = subprocess.run([os.path.join(ASAN, "test_host_asan"), "cpu"], capture_output=True,
                       text=True, env=ENV, timeout=300)
    assert r.returncode == 0 and "0 failure(s)" in r.stdout, r.stdout + r.stderr
