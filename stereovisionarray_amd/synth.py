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


def step_offset(s, bx: int, by: int):
    """(dx, dy) of match distance s along the integer baseline direction
    (bx, by): s along the major axis, round_half_up(s*m/M) along the minor one
    (DESIGN.md §2.2).  Works elementwise on integer arrays."""
    s = np.asarray(s, dtype=np.int64)
    ax, ay = abs(bx), abs(by)
    M, m = max(ax, ay), min(ax, ay)
    minor = (2 * s * m + M) // (2 * M)
    mx, my = (s, minor) if ax >= ay else (minor, s)
    return np.sign(bx) * mx, np.sign(by) * my


def stereo_pair2(H: int, W: int, D: int, dmin: int = 0, sx: int = 0, sy: int = -1,
                 seed: int = 1, stripes: int = 16, step: int = 8):
    """Array-pair matching step: R(q) = L(q - off(d(q))) with
    off = step_offset(d, sx, sy) and d piecewise constant in stripes along an
    axis across the step; returns (L, R, d_of_R)."""
    L = texture(H, W, seed)
    if sy != 0:
        d = stripe_disparity(W, dmin, D, stripes, step)[None, :].repeat(H, 0)
    else:
        d = stripe_disparity(H, dmin, D, stripes, step)[:, None].repeat(W, 1)
    yy, xx = np.mgrid[0:H, 0:W]
    ox, oy = step_offset(d, sx, sy)
    R = L[np.clip(yy - oy, 0, H - 1), np.clip(xx - ox, 0, W - 1)]
    return np.ascontiguousarray(L), np.ascontiguousarray(R), d


def reference_array(pixel_size: float, f: float = 0.05):
    """The reference's 5x5 camera grid (CameraStereoVision.cpp:34-39):
    pitch 0.05 m, z = -0.75, index = 5*y + x."""
    cams = []
    for y in range(5):
        for x in range(5):
            cams.append((f, (-0.1 + x * 0.05, -0.1 + y * 0.05, -0.75), pixel_size))
    return cams


def array_grid(rows: int = 2, cols: int = 4):
    """Camera grid positions (gx, gy) in grid units, index = cols*gy + gx
    (the reference's row-major numbering, CameraStereoVision.cpp:34-39)."""
    return [(gx, gy) for gy in range(rows) for gx in range(cols)]


def array_pairs(n_cams: int):
    """All pairwise baselines (i, j), i < j, grouped by reference camera i so
    each camera's maps are contiguous for the fusion."""
    return [(i, j) for i in range(n_cams) for j in range(i + 1, n_cams)]


def pair_step(gi, gj):
    """Match step of pair (ref i, other j): a scene point at q in camera i
    appears at q - (gj - gi) * delta in camera j, so the step is -(gj - gi)
    reduced by the gcd of its components.  Returns
    (sx, sy, k): k = |major component| of the baseline in grid units, so the
    disparity along the major axis is k * delta."""
    bx, by = int(gj[0] - gi[0]), int(gj[1] - gi[1])
    g = int(np.gcd(abs(bx), abs(by)))
    k = max(abs(bx), abs(by))
    return -bx // g, -by // g, k


def array_views(H: int, W: int, grid, delta, seed: int = 1):
    """Synthetic array views: camera at grid position (gx, gy) sees
    I(x, y) = T(x + gx * delta(x, y), y + gy * delta(x, y)) (backward warp of one
    texture T by the per-grid-unit disparity field delta, edge-clamped)."""
    T = texture(H, W, seed)
    yy, xx = np.mgrid[0:H, 0:W]
    views = []
    for gx, gy in grid:
        views.append(np.ascontiguousarray(
            T[np.clip(yy + gy * delta, 0, H - 1), np.clip(xx + gx * delta, 0, W - 1)]))
    return views


def array_delta(H: int, W: int, dmax: int, stripes: int = 12):
    """Per-grid-unit disparity field for array_views: vertical stripes of
    constant disparity 4 .. dmax (piecewise fronto-parallel planes)."""
    idx = (np.arange(W) * stripes) // max(W, 1)
    row = 4 + (idx * (dmax - 4)) // max(stripes - 1, 1)
    return np.repeat(row[None, :], H, 0).astype(np.int64)
