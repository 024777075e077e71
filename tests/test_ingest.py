"""Ingestion host plumbing: sorted folder listing and
grayscale decode (CPU); the GPU resize is in tests/test_ingest_gpu.py."""
import os

import numpy as np
import pytest

from stereovisionarray_amd import ingest


def test_image_paths_sorted_and_filtered(tmp_path):
    for n in ["b.png", "a.PNG", "c.txt", "10.png", "2.png"]:
        (tmp_path / n).write_bytes(b"x")
    (tmp_path / "sub.png").mkdir()
    got = [os.path.basename(p) for p in ingest.image_paths(str(tmp_path))]
    assert got == ["10.png", "2.png", "a.PNG", "b.png"]


def test_load_gray_decodes_luma(tmp_path):
    PIL = pytest.importorskip("PIL.Image")
    rgb = np.zeros((4, 6, 3), np.uint8)
    rgb[..., 0] = 200
    rgb[..., 1] = 100
    rgb[..., 2] = 50
    p = tmp_path / "x.png"
    PIL.fromarray(rgb).save(p)
    g = ingest.load_gray(str(p))
    assert g.shape == (4, 6) and g.dtype == np.uint8
    # ITU-R 601-2 luma: 200*.299 + 100*.587 + 50*.114 = 124.2 -> 124
    assert (g == 124).all()
