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
    assert sva.lib.sva_abi_version() == 6 == sva.ABI_VERSION
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


def test_tile_stage_sizes_checked_without_device(sva):
    """the tile stages take byte sizes; a buffer smaller
    than its plane is SVA_ERR_INVALID_ARG before any device work.
    sva_tile_check is the entry points' own size test (sva_api.cpp
    check_tile_buffers), callable without a device."""
    W, H, D = 1920, 1080, 128
    lay = sva.tile_layout(W, H, D)
    assert (lay.seg, lay.nsx, lay.nsy) == (8, 240, 135)
    nv = lay.diag_volumes
    assert nv in (0, 2, 4)          # 0: the strip route (D <= 128)
    assert lay.cost_bytes == W * H * D and lay.diag_bytes == nv * W * H * D
    assert lay.hckpt_bytes == 2 * H * 240 * D and lay.vckpt_bytes == (6 - nv) * 135 * W * D
    full = [lay.cost_bytes, lay.diag_bytes, lay.hckpt_bytes, lay.vckpt_bytes]
    assert sva.lib.sva_tile_check(W, H, D, *full) == sva.SVA_OK
    for i in range(4):
        if full[i] == 0:            # no diagonal volume on the strip route
            continue
        short = list(full)
        short[i] -= 1
        assert sva.lib.sva_tile_check(W, H, D, *short) == sva.SVA_ERR_INVALID_ARG, i
    # ragged sizes: the planes round the segments up
    lay2 = sva.tile_layout(17, 9, 256)
    assert (lay2.seg, lay2.nsx, lay2.nsy) == (8, 3, 2)
    assert sva.lib.sva_tile_check(17, 9, 256, lay2.cost_bytes, lay2.diag_bytes,
                                  lay2.hckpt_bytes, lay2.vckpt_bytes) == sva.SVA_OK
    # non-native D and a null context are argument errors too
    assert sva.lib.sva_tile_check(W, H, 100, *full) == sva.SVA_ERR_INVALID_ARG
    assert sva.lib.sva_paths_tile_d(None, None, 0, W, H, None, None, 0, None, 0, None, 0) == \
        sva.SVA_ERR_INVALID_ARG
