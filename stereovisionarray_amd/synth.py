"""Synthetic stereo inputs: uniform u8 texture from MT19937 and
a matched image shifted by a piecewise-constant disparity field.

There is no dataset in this image (the reference's Renders2/ and Images/ are
not shipped, reference .gitignore:8-14); every test and bench uses these.
"""
from __future__ import annotations

import numpy as np


def texture(H: int, W: int, seed: int) -> np.ndarray:
    return np.random.RandomState(seed).randint(0, 256, size=(H, W)).astype(np.uint8)


def stripe_disparity(W: int, dmin: int, D: int, stripes: int = 16, step: int = 8) -> np.ndarray:
    """Disparity per column of the matched image: stripe i gets dmin + step*i
    (clamped into [dmin, dmin + D - 1])."""
    idx = (np.arange(W) * stripes) // max(W, 1)
    return np.minimum(dmin + step * idx, dmin + D - 1).astype(np.int64)


def stereo_pair(H: int, W: int, D: int, dmin: int = 0, dir: int = -1, seed: int = 1,
                stripes: int = 16, step: int = 8):
    """Reference image L and matched image R with R(x + dir*d(x), y) = L(x, y)
    where d is piecewise constant; returns (L, R, d_of_right_column)."""
    L = texture(H, W, seed)
    d = stripe_disparity(W, dmin, D, stripes, step)
    xr = np.arange(W)
    src = np.clip(xr - dir * d, 0, W - 1)
    R = L[:, src]
    return np.ascontiguousarray(L), np.ascontiguousarray(R), d


def reference_array(pixel_size: float, f: float = 0.05):
    """The reference's 5x5 camera grid (CameraStereoVision.cpp:34-39):
    pitch 0.05 m, z = -0.75, index = 5*y + x."""
    cams = []
    for y in range(5):
        for x in range(5):
            cams.append((f, (-0.1 + x * 0.05, -0.1 + y * 0.05, -0.75), pixel_size))
    return cams
