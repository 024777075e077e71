"""Ingestion: the reference's image loading
(CameraStereoVision.cpp:13-19): list a folder (getImagesPathsFromFolder,
functions.cpp:240-250), decode each file as 8-bit grayscale (imread
IMREAD_GRAYSCALE), halve it (resize 0.5 INTER_LINEAR).

Host plumbing only: the listing is sorted by file name (the reference's
std::filesystem::directory_iterator order is unspecified); decoding uses
Pillow, whose RGB->L conversion is ITU-R 601-2 luma
(L = R*299/1000 + G*587/1000 + B*114/1000, rounded), while OpenCV's
IMREAD_GRAYSCALE may differ by one grey level (OpenCV absent: parity
unpinned).  The resize runs on the GPU (libsva.so sva_resize_half).
"""
from __future__ import annotations

import os

import numpy as np

IMAGE_EXTENSIONS = (".png", ".jpg", ".jpeg", ".bmp", ".tif", ".tiff", ".pgm", ".ppm", ".pnm")


def image_paths(folder: str) -> list[str]:
    """getImagesPathsFromFolder (functions.cpp:240-250), sorted by name;
    only regular files with an image extension."""
    out = []
    for name in sorted(os.listdir(folder)):
        p = os.path.join(folder, name)
        if os.path.isfile(p) and name.lower().endswith(IMAGE_EXTENSIONS):
            out.append(p)
    return out


def load_gray(path: str) -> np.ndarray:
    """imread(path, IMREAD_GRAYSCALE) via Pillow (host decode)."""
    from PIL import Image
    with Image.open(path) as im:
        return np.ascontiguousarray(np.asarray(im.convert("L"), dtype=np.uint8))


def load_folder(ctx, folder: str, half: bool = True) -> list[np.ndarray]:
    """CameraStereoVision.cpp:13-19: every image of `folder`, grayscale,
    halved on the GPU (ctx: stereovisionarray_amd.Context)."""
    imgs = [load_gray(p) for p in image_paths(folder)]
    return [ctx.resize_half(i) for i in imgs] if half else imgs
