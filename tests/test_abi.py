"""C-ABI boundary checks that need no GPU: the library loads, exports every
symbol include/sva.h declares, the header compiles as C and C++, and the
product path refuses to run (no CPU fallback) when no device is visible."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sva.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sva_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_expected_set(sva):
    assert declared_functions() == sorted(sva.EXPORTED)


def test_every_declared_symbol_exported(sva):
    out = subprocess.run(["nm", "-D", "--defined-only", sva.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (sva_[a-z0-9_]+)", out))
    missing = set(declared_functions()) - exported
    assert not missing, missing


@pytest.mark.parametrize("lang,compiler", [("c", "gcc"), ("c++", "g++")])
def test_header_compiles(tmp_path, lang, compiler):
    src = tmp_path / ("t.c" if lang == "c" else "t.cpp")
    src.write_text('#include "sva.h"\nint main(void){sva_sgm_params p; '
                   'sva_sgm_params_default(&p); return p.D == 128 ? 0 : 1;}\n')
    subprocess.run([compiler, "-std=c11" if lang == "c" else "-std=c++17", "-Wall", "-Werror",
                    "-fsyntax-only", "-I", os.path.join(ROOT, "include"), str(src)], check=True)


def test_defaults_and_strings(sva):
    p = sva.default_params()
    assert (p.D, p.dmin, p.dir, p.dir_y, p.P1, p.P2, p.subpixel, p.lr_check, p.invalid) == \
        (128, 0, -1, 0, 10, 120, 0, 0, 0xFFFF)
    assert sva.lib.sva_abi_version() == 4
    assert sva.lib.sva_status_string(sva.SVA_ERR_NO_DEVICE) == b"no usable HIP device"


def test_no_cpu_fallback_without_device(sva):
    if sva.device_count() > 0:
        pytest.skip("a HIP device is visible; covered by the gpu suite")
    with pytest.raises(sva.SvaError) as e:
        sva.Context(0)
    assert e.value.status == sva.SVA_ERR_NO_DEVICE


def test_null_context_is_rejected(sva):
    assert sva.lib.sva_synchronize(None) == sva.SVA_ERR_INVALID_ARG
    assert sva.lib.sva_destroy(None) == sva.SVA_ERR_INVALID_ARG
