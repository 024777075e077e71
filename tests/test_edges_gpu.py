"""Edge cases of the Mode S pipeline vs the oracle (empty and
ragged inputs, maximum sizes): images smaller than the census window, D
larger than the image, one-pixel-wide/-high images, ragged widths around the
workgroup tiles, large dmin, and every D the kernels are built for.
All bit-exact (integer stages)."""
import numpy as np
import pytest

from stereovisionarray_amd import synth

pytestmark = pytest.mark.gpu

SIZES = [(1, 1), (2, 3), (9, 7), (8, 6), (17, 5), (5, 40), (63, 33), (65, 31), (129, 3),
         (1, 70), (70, 1),
         # around the tile pipeline's 16 x 8 tiles and 8-pixel checkpoint segments
         (16, 8), (15, 9), (31, 17), (48, 24), (23, 16), (8, 1), (1, 8)]


@pytest.mark.parametrize("W,H", SIZES)
@pytest.mark.parametrize("D", [64, 128, 192, 256])
def test_tiny_and_ragged(ctx, sva, oracle, W, H, D):
    L = synth.texture(H, W, W * 7 + H)
    R = synth.texture(H, W, W * 7 + H + 1)
    p = sva.default_params(D=D, dir=-1, subpixel=1)
    disp, sub = ctx.disparity_sgm(L, R, p)
    od, osub = oracle.sgm(L, R, D, 0, -1, subpixel=True, threads=4)
    assert np.array_equal(disp, od)
    assert np.max(np.abs(sub - osub)) <= 1e-5


@pytest.mark.parametrize("sx,sy", [(0, -1), (1, 1), (-2, 1)])
@pytest.mark.parametrize("W,H", [(1, 1), (3, 40), (40, 3), (33, 33)])
def test_tiny_2d_steps(ctx, sva, oracle, W, H, sx, sy):
    L = synth.texture(H, W, 11)
    R = synth.texture(H, W, 12)
    p = sva.default_params(D=64, dir=sx, dir_y=sy)
    disp, _ = ctx.disparity_sgm(L, R, p)
    od, _ = oracle.sgm2(L, R, 64, 0, sx, sy, subpixel=False)
    assert np.array_equal(disp, od)


def test_large_dmin(ctx, sva, oracle):
    W, H, D, dmin = 400, 40, 128, 300     # most candidates leave the image
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=5)
    p = sva.default_params(D=D, dmin=dmin, dir=-1)
    disp, _ = ctx.disparity_sgm(L, R, p)
    od, _ = oracle.sgm(L, R, D, dmin, -1, subpixel=False, threads=4)
    assert np.array_equal(disp, od)
    assert disp.min() >= dmin


def test_constant_images(ctx, sva, oracle):
    """All census words 0, all costs 0 inside: every disparity ties ->
    first minimum (dmin) everywhere except where the 62 border costs bite."""
    W, H, D = 200, 50, 64
    L = np.full((H, W), 77, np.uint8)
    disp, _ = ctx.disparity_sgm(L, L, sva.default_params(D=D))
    od, _ = oracle.sgm(L, L, D, 0, -1, subpixel=False, threads=4)
    assert np.array_equal(disp, od)


def test_rejects_bad_arguments(ctx, sva):
    L = np.zeros((8, 8), np.uint8)
    for kw in (dict(D=0), dict(D=64, dmin=-1), dict(D=64, dir=0, dir_y=0), dict(D=64, dir=300),
               dict(D=64, dmin=65500), dict(D=64, P1=-1)):
        with pytest.raises(sva.SvaError):
            ctx.disparity_sgm(L, L, sva.default_params(**kw))


def test_rejects_unsupported_shapes(ctx, sva):
    """shapes the kernels cannot launch are refused before any
    workspace is allocated: H > 65535 (gridDim.y of the L/R check) and
    W*H*D >= 2^32 (32-bit path-volume offsets)."""
    tall = np.zeros((65536, 1), np.uint8)
    with pytest.raises(sva.SvaError) as e:
        ctx.disparity_sgm(tall, tall, sva.default_params(D=64))
    assert e.value.status == sva.SVA_ERR_UNSUPPORTED
    wide = np.zeros((1024, 16384), np.uint8)           # 16384*1024*256 = 2^32
    with pytest.raises(sva.SvaError) as e:
        ctx.disparity_sgm(wide, wide, sva.default_params(D=256))
    assert e.value.status == sva.SVA_ERR_UNSUPPORTED
