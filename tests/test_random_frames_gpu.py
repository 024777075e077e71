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


def _cases_ref(n=32, seed=20261019):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        W, H = int(rng.integers(48, 480)), int(rng.integers(40, 360))
        ref = int(rng.integers(0, 25))
        oth = ref
        while oth == ref:
            oth = int(rng.integers(0, 25))
        k = int(rng.integers(1, min(33, min(W, H) // 3)))
        # keep the single-threaded oracle to a second or two: W*H pixels x
        # ~W/4 candidates x (2k)^2 absolute differences
        while W * H * (W // 4) * 4 * k * k > 8e9 and min(W, H) > 48:
            W, H = W * 3 // 4, H * 3 // 4
        k = min(k, min(W, H) // 3)
        masked = bool(rng.random() < 0.4)
        shift = int(rng.integers(0, 24))
        out.append((i, W, H, ref, oth, k, masked, shift))
    return out


@pytest.mark.parametrize("case", _cases_ref(), ids=lambda c: "r%02d_%dx%d_%d-%d_k%d" % c[:6])
def test_random_mode_r(ctx, sva, oracle, case):
    """Mode R, the reference's own path (CameraStereoVision.cpp:44-95): any
    camera pair of the 5x5 rig (Low and High Bresenham lines, both signs,
    long baselines), any window 1 <= k <= 32, with and without a mask;
    valid, the u8-wrapped and the u16 maps bit-exact vs the oracle."""
    i, W, H, ref, oth, k, masked, shift = case
    ps = 0.036 / W
    grid = synth.reference_array(ps)
    cr, co = sva.Camera.make(*grid[ref]), sva.Camera.make(*grid[oth])
    ocr, oco = oracle.OCamera.make(*grid[ref]), oracle.OCamera.make(*grid[oth])
    a = synth.texture(H, W, 3000 + i)
    b = np.roll(a, shift, axis=int(i % 2))
    mask = None
    if masked:
        mask = (synth.texture(H, W, 4000 + i) > 96).astype(np.uint8) * 255
    d8, d16, valid = ctx.disparity_ref(a, b, cr, co, k=k, mask=mask)
    o8, o16, ovalid, _ = oracle.ref_pair(a, b, ocr, oco, k=k, mask=mask)
    assert np.array_equal(valid, ovalid), f"{int((valid != ovalid).sum())} valid flags differ"
    assert np.array_equal(d16, o16) and np.array_equal(d8, o8)
