"""Seeded random sweep of the Mode S frame route against the CPU oracle.

The other GPU suites pick their sizes by hand: tile edges, native and padded
D, penalty extremes, 2-D steps.  This one draws 40 frames from a fixed
generator so that the combinations nobody picked get exercised too: frame
sizes off every tile and segment boundary (the 16 x 8 tiles and 8-pixel
checkpoint segments of DESIGN.md §4.9, the 128-pixel census+cost tiles of
§4.2), any D in 1..256 (§4.7), dmin, both 1-D step signs, the full penalty
range of include/sva.h (0 <= P1, P2 <= 193), sub-pixel on and off.  Every
disparity must equal oracle.sgm bit for bit (SURVEY.md §8a
A10-A13); sub-pixel values within 1e-5 px (§2.4).  The draw is part of the
test: the same 40 cases run every time.
"""
import numpy as np
import pytest

from stereovisionarray_amd import synth

pytestmark = pytest.mark.gpu

SUB_TOL = 1e-5


def _cases(n=40, seed=20261017):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        if rng.random() < 0.5:                           # native widths half the time
            D = int(rng.choice([64, 128, 192, 256]))
        else:
            D = int(rng.integers(1, 257))
        W = int(rng.integers(9, 420))
        H = int(rng.integers(7, 150))
        dmin = int(rng.integers(0, 40))
        d = int(rng.choice([-1, 1]))
        P1 = int(rng.integers(0, 70))
        P2 = int(rng.integers(P1, 194)) if rng.random() < 0.8 else int(rng.integers(0, 194))
        sub = bool(rng.random() < 0.7)
        out.append((i, W, H, D, dmin, d, P1, P2, sub))
    return out


@pytest.mark.parametrize("case", _cases(), ids=lambda c: "r%02d_%dx%d_D%d" % c[:4])
def test_random_frame(ctx, sva, oracle, case):
    i, W, H, D, dmin, d, P1, P2, want_sub = case
    L, R, _ = synth.stereo_pair(H, W, max(D, 2), dmin, d, seed=1000 + i,
                                stripes=int(1 + i % 7), step=max(1, D // 6))
    p = sva.default_params(D=D, dmin=dmin, dir=d, P1=P1, P2=P2, subpixel=int(want_sub))
    disp, sub = ctx.disparity_sgm(L, R, p)
    od, osub = oracle.sgm(L, R, D, dmin, d, P1, P2, subpixel=want_sub)
    bad = int((disp != od).sum())
    assert bad == 0, f"{bad} of {W * H} pixels differ (W={W} H={H} D={D} dmin={dmin} dir={d} " \
                     f"P1={P1} P2={P2})"
    assert int(disp.max()) < dmin + D and int(disp.min()) >= dmin
    if want_sub:
        assert np.max(np.abs(sub - osub)) <= SUB_TOL


def _cases_2d(n=16, seed=20261018):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        sx, sy = 0, 0
        while sx == 0 and sy == 0:
            sx, sy = int(rng.integers(-3, 4)), int(rng.integers(-3, 4))
        D = int(rng.choice([64, 128, int(rng.integers(1, 257))]))
        W, H = int(rng.integers(9, 260)), int(rng.integers(7, 200))
        dmin = int(rng.integers(0, 12))
        P1 = int(rng.integers(0, 60))
        P2 = int(rng.integers(P1, 194))
        out.append((i, W, H, D, dmin, sx, sy, P1, P2))
    return out


@pytest.mark.parametrize("case", _cases_2d(), ids=lambda c: "r%02d_%dx%d_D%d" % c[:4])
def test_random_frame_2d_step(ctx, sva, oracle, case):
    """Array pairs: a random integer step (sx, sy) on the
    camera grid, matched through hamming_cost2_kernel."""
    i, W, H, D, dmin, sx, sy, P1, P2 = case
    L, R, _ = synth.stereo_pair2(H, W, max(D, 2), dmin, sx, sy, seed=2000 + i,
                                 stripes=int(1 + i % 5), step=max(1, D // 5))
    p = sva.default_params(D=D, dmin=dmin, dir=sx, dir_y=sy, P1=P1, P2=P2, subpixel=1)
    disp, sub = ctx.disparity_sgm(L, R, p)
    od, osub = oracle.sgm2(L, R, D, dmin, sx, sy, P1, P2, subpixel=True)
    bad = int((disp != od).sum())
    assert bad == 0, f"{bad} of {W * H} pixels differ (W={W} H={H} D={D} dmin={dmin} " \
                     f"step=({sx},{sy}) P1={P1} P2={P2})"
    assert np.max(np.abs(sub - osub)) <= SUB_TOL
