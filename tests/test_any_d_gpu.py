"""Any disparity count D in 1..256 on the GPU (VERDICT r02 "missing" #5 /
"next" #8).

The reference's own per-pixel candidate counts are 45-49 at 640 px and
134-145 at 1080p (CameraStereoVision.cpp:60-73), none of
them a native kernel width.  A frame with such a D runs at the next native
width Dp in {64, 128, 192, 256}: the cost kernels write 255 at d >= D, which
never wins a neighbour term or the row minimum of the recurrence, the WTA
masks d >= D, and the horizontal checkpoints restart padded disparities at
255.  Every result must equal the CPU oracle run at the caller's D, bit for
bit (sub-pixel within 1e-5 px, the tolerance of DESIGN.md §2.4).
"""
import numpy as np
import pytest

from stereovisionarray_amd import synth

from checks import assert_sub_close

pytestmark = pytest.mark.gpu

SUB_TOL = 1e-5


@pytest.mark.parametrize("D", [1, 2, 16, 33, 48, 63, 65, 96, 127, 144, 160, 191, 200, 255])
@pytest.mark.parametrize("dir", [-1, 1])
def test_any_d_pipeline(ctx, sva, oracle, D, dir):
    """1-D steps: D < 128 takes the census + cost kernels, D > 128 the fused
    census+cost kernel; widths off the 128-pixel tile, sub-pixel on."""
    W, H, dmin = 203, 61, 3
    L, R, _ = synth.stereo_pair(H, W, max(D, 2), dmin, dir, seed=D + 7 * (dir + 1), stripes=5,
                                step=max(1, D // 6))
    p = sva.default_params(D=D, dmin=dmin, dir=dir, subpixel=1)
    disp, sub = ctx.disparity_sgm(L, R, p)
    od, osub = oracle.sgm(L, R, D, dmin, dir, subpixel=True)
    assert np.array_equal(disp, od), f"D={D}: {int((disp != od).sum())} pixels differ"
    assert np.max(np.abs(sub - osub)) <= SUB_TOL
    assert disp.max() < dmin + D


@pytest.mark.parametrize("D,P1,P2", [(48, 0, 0), (48, 193, 193), (100, 1, 193), (150, 30, 60),
                                     (250, 193, 10)])
def test_any_d_penalties(ctx, sva, oracle, D, P1, P2):
    """The padding argument needs m + P2 <= 255 <= A_pad + P1: the extremes
    of the penalty range, P1 = P2 = 193 included."""
    W, H = 150, 70
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=D + P1, stripes=4, step=max(1, D // 5))
    p = sva.default_params(D=D, dir=-1, P1=P1, P2=P2, subpixel=1)
    disp, sub = ctx.disparity_sgm(L, R, p)
    od, osub = oracle.sgm(L, R, D, 0, -1, P1, P2, subpixel=True)
    assert np.array_equal(disp, od)
    assert np.max(np.abs(sub - osub)) <= SUB_TOL


@pytest.mark.parametrize("D,sx,sy", [(48, 0, -1), (96, -1, -1), (80, 2, -1), (144, 1, 1),
                                     (200, -1, 3)])
def test_any_d_2d_steps(ctx, sva, oracle, D, sx, sy):
    """Array pairs on 2-D steps (hamming_cost2_kernel pads the same way)."""
    W, H = 97, 230
    L, R, _ = synth.stereo_pair2(H, W, D, 0, sx, sy, seed=D + sx, stripes=4,
                                 step=max(1, D // 5))
    p = sva.default_params(D=D, dir=sx, dir_y=sy, subpixel=1)
    disp, sub = ctx.disparity_sgm(L, R, p)
    od, osub = oracle.sgm2(L, R, D, 0, sx, sy, subpixel=True)
    assert np.array_equal(disp, od)
    assert np.max(np.abs(sub - osub)) <= SUB_TOL


@pytest.mark.parametrize("D,dir", [(45, -1), (140, 1)])
def test_any_d_lr_check(ctx, sva, oracle, D, dir):
    W, H = 180, 64
    L, R, _ = synth.stereo_pair(H, W, D, 2, dir, seed=D, stripes=6, step=max(1, D // 7))
    p = sva.default_params(D=D, dmin=2, dir=dir, lr_check=1, lr_max_diff=1, subpixel=1)
    disp, sub = ctx.disparity_sgm(L, R, p)
    dl, osub = oracle.sgm(L, R, D, 2, dir, subpixel=True)
    dr, _ = oracle.sgm(R, L, D, 2, -dir, subpixel=False)
    exp = oracle.lr_check(dl, dr, dir, 1, 0xFFFF)
    assert np.array_equal(disp, exp)
    assert_sub_close(sub, oracle.lr_sub(exp, osub, 0xFFFF))


def test_stage_entry_points_stay_native(ctx, sva, torch_dev):
    """The stage entry points read and write [..][D] volumes, so they keep the
    native widths; the whole-frame entry points take any D <= 256."""
    import torch
    W, H = 32, 16
    C = torch.zeros((H, W, 64), dtype=torch.uint8, device=torch_dev)
    L8 = torch.zeros((8, H, W, 64), dtype=torch.uint8, device=torch_dev)
    with pytest.raises(sva.SvaError) as e:
        ctx.paths_d(C.data_ptr(), W, H, sva.default_params(D=48), L8.data_ptr())
    assert e.value.status == sva.SVA_ERR_UNSUPPORTED
    for bad in (0, 257, 1000):
        with pytest.raises(sva.SvaError):
            ctx.disparity_sgm(np.zeros((H, W), np.uint8), np.zeros((H, W), np.uint8),
                              sva.default_params(D=bad))


@pytest.mark.slow
def test_any_d_1080p_d144(ctx, sva, oracle):
    """A full 1920x1080 frame at D = 144 (the reference's 1080p candidate
    count class), padded to 192, bit-exact vs the threaded oracle."""
    W, H, D = 1920, 1080, 144
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=11)
    p = sva.default_params(D=D, dir=-1, subpixel=1)
    disp, sub = ctx.disparity_sgm(L, R, p)
    od, osub = oracle.sgm(L, R, D, 0, -1, subpixel=True, threads=16)
    assert np.array_equal(disp, od)
    assert np.max(np.abs(sub - osub)) <= SUB_TOL
