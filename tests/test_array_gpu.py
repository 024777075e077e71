"""Array extensions of Mode S (DESIGN.md §2.2 2-D step, §2.5 2-D L/R check,
§2.6 depth fusion; SURVEY.md §8e, BASELINE config 4): HIP vs the CPU oracle.

Bars: cost / disparity / L/R-checked maps bit-exact; fused depth bit-exact in
f64 (the same IEEE mul/div/mean on both sides, no contraction) and the
per-pixel valid-map counts exact.  Parity vs the reference is unpinned (the
reference has no 2-D matcher and no fusion: its loop keeps the last pair,
CameraStereoVision.cpp:55).
"""
import numpy as np
import pytest
import torch

from stereovisionarray_amd import synth

from checks import assert_sub_close

pytestmark = pytest.mark.gpu

SUB_TOL = 1e-5
STEPS_2D = [(0, -1), (0, 1), (-1, -1), (1, 1), (1, -1), (-1, 1), (2, -1), (-1, 3), (-3, -2),
            (2, 0), (2, 2), (-4, 2)]


def dev(a, d):
    return torch.from_numpy(np.ascontiguousarray(a)).to(d)


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def run_sync(ctx):
    ctx.synchronize()
    torch.cuda.synchronize()


@pytest.mark.parametrize("D", [64, 128, 192, 256])
@pytest.mark.parametrize("sx,sy", STEPS_2D)
@pytest.mark.parametrize("dmin", [0, 9])
def test_cost2(ctx, sva, oracle, torch_dev, D, sx, sy, dmin):
    W, H = 71, 290  # taller than D so every disparity has in-image matches
    L, R, _ = synth.stereo_pair2(H, W, D, dmin, sx, sy, seed=D + 3 * sx + sy)
    cl, cr = oracle.census(L), oracle.census(R)
    C = torch.zeros((H, W, D), dtype=torch.uint8, device=torch_dev)
    p = sva.default_params(D=D, dmin=dmin, dir=sx, dir_y=sy)
    d_cl, d_cr = dev(cl.view(np.int64), torch_dev), dev(cr.view(np.int64), torch_dev)
    ctx.cost_d(d_cl.data_ptr(), d_cr.data_ptr(), W, H, p, C.data_ptr())
    run_sync(ctx)
    exp = oracle.cost2(cl, cr, D, dmin, sx, sy)
    got = host(C)
    assert np.array_equal(got, exp)
    assert (exp == 62).any() and (exp < 62).any()


@pytest.mark.parametrize("W,H,D,dmin,sx,sy", [
    (120, 160, 64, 0, 0, -1), (97, 200, 64, 5, 0, 1), (150, 150, 64, 0, -1, -1),
    (130, 260, 128, 2, 1, -1), (300, 300, 256, 0, -1, 1), (200, 180, 64, 0, -2, -1),
    (170, 190, 128, 1, 1, 3),
])
def test_full_pipeline_2d(ctx, sva, oracle, W, H, D, dmin, sx, sy):
    L, R, _ = synth.stereo_pair2(H, W, D, dmin, sx, sy, seed=W + H)
    p = sva.default_params(D=D, dmin=dmin, dir=sx, dir_y=sy, subpixel=1)
    disp, sub = ctx.disparity_sgm(L, R, p)
    od, osub = oracle.sgm2(L, R, D, dmin, sx, sy, subpixel=True)
    assert np.array_equal(disp, od)
    assert np.max(np.abs(sub - osub)) <= SUB_TOL


@pytest.mark.parametrize("sx,sy", [(0, -1), (-1, -1), (2, 1), (-1, 3)])
def test_cost2_large(ctx, sva, oracle, torch_dev, sx, sy):
    """Many sheared tiles / bands and a large dmin (offset table > D)."""
    W, H, D, dmin = 333, 517, 128, 40
    L, R, _ = synth.stereo_pair2(H, W, D, dmin, sx, sy, seed=7)
    cl, cr = oracle.census(L), oracle.census(R)
    C = torch.zeros((H, W, D), dtype=torch.uint8, device=torch_dev)
    p = sva.default_params(D=D, dmin=dmin, dir=sx, dir_y=sy)
    d_cl, d_cr = dev(cl.view(np.int64), torch_dev), dev(cr.view(np.int64), torch_dev)
    ctx.cost_d(d_cl.data_ptr(), d_cr.data_ptr(), W, H, p, C.data_ptr())
    run_sync(ctx)
    assert np.array_equal(host(C), oracle.cost2(cl, cr, D, dmin, sx, sy))


def test_vertical_shift_exact(ctx, sva):
    """KAT: R(x, y - d0) = L(x, y) (camera below the reference, sy = -1):
    every interior pixel far enough from the top returns d0."""
    W, H, D, d0 = 96, 240, 64, 17
    L = synth.texture(H, W, 21)
    R = np.zeros_like(L)
    R[: H - d0] = L[d0:]
    R[H - d0:] = synth.texture(d0, W, 22)
    disp, _ = ctx.disparity_sgm(L, R, sva.default_params(D=D, dir=0, dir_y=-1))
    assert (disp[d0 + 40: H - 40, 8:-8] == d0).all()


@pytest.mark.parametrize("sx,sy", [(0, -1), (-1, -1), (1, 1), (-2, 1)])
def test_lr_check_2d(ctx, sva, oracle, sx, sy):
    W, H, D = 110, 180, 64
    L, R, _ = synth.stereo_pair2(H, W, D, 0, sx, sy, seed=5, stripes=6, step=9)
    p = sva.default_params(D=D, dir=sx, dir_y=sy, lr_check=1, lr_max_diff=1, subpixel=1)
    disp, sub = ctx.disparity_sgm(L, R, p)
    dl, osub = oracle.sgm2(L, R, D, 0, sx, sy, subpixel=True)
    dr, _ = oracle.sgm2(R, L, D, 0, -sx, -sy, subpixel=False)
    exp = oracle.lr_check2(dl, dr, sx, sy, 1, 0xFFFF)
    assert np.array_equal(disp, exp)
    assert (disp == 0xFFFF).any() and (disp != 0xFFFF).any()
    assert_sub_close(sub, oracle.lr_sub(exp, osub, 0xFFFF))


def _fuse_inputs(n, H, W, seed):
    rng = np.random.default_rng(seed)
    d = rng.integers(0, 200, size=(n, H, W)).astype(np.uint16)
    d[rng.random((n, H, W)) < 0.2] = 0xFFFF          # L/R-rejected pixels
    d[:, :2, :3] = 0xFFFF                            # no valid map at all
    d[:, 3, :] = 40                                  # ties across maps
    b = rng.choice([0.05, 0.1, 0.05 * np.sqrt(2.0), 0.15], size=n)
    return d, b


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 8, 9, 16, 17, 32])
def test_fuse_depth(ctx, oracle, n):
    H, W = 37, 129
    d, b = _fuse_inputs(n, H, W, n)
    f, ps = 0.05, 2e-5
    got, gn = ctx.fuse_depth(d, b, f, ps)
    exp, en = oracle.fuse_depth(d, b, f, ps)
    assert np.array_equal(gn, en)
    assert np.array_equal(got.view(np.uint64), exp.view(np.uint64))
    assert (got[:2, :3] == 0).all()


def test_fuse_depth_device_buffers(ctx, oracle, torch_dev):
    n, H, W = 8, 300, 257
    d, b = _fuse_inputs(n, H, W, 99)
    dd = dev(d.view(np.int16), torch_dev)
    depth = torch.zeros((H, W), dtype=torch.float64, device=torch_dev)
    nv = torch.zeros((H, W), dtype=torch.uint8, device=torch_dev)
    ctx.fuse_depth_d(dd.data_ptr(), n, W, H, b, 0.05, 2e-5, 0xFFFF, depth.data_ptr(),
                     nv.data_ptr())
    run_sync(ctx)
    exp, en = oracle.fuse_depth(d, b, 0.05, 2e-5)
    assert np.array_equal(host(nv), en)
    assert np.array_equal(host(depth).view(np.uint64), exp.view(np.uint64))


def test_fuse_custom_invalid_and_limits(ctx, sva, oracle):
    d, b = _fuse_inputs(3, 8, 8, 1)
    got, _ = ctx.fuse_depth(d, b, 0.05, 2e-5, invalid=40)
    exp, _ = oracle.fuse_depth(d, b, 0.05, 2e-5, invalid=40)
    assert np.array_equal(got.view(np.uint64), exp.view(np.uint64))
    with pytest.raises(sva.SvaError) as e:
        ctx.fuse_depth(np.zeros((33, 4, 4), np.uint16), [0.05] * 33, 0.05, 2e-5)
    assert e.value.status == sva.SVA_ERR_UNSUPPORTED


def test_array_depth_end_to_end(ctx, sva, oracle):
    """Config-4 shape in miniature: one reference view matched against a
    right, a lower and a diagonal neighbour with a constant true disparity;
    the fused depth is b*f/(d0*ps) on the interior."""
    W, H, D, d0 = 160, 160, 64, 12
    f, ps, pitch = 0.05, 2e-5, 0.05
    L = synth.texture(H, W, 31)
    maps, bases = [], []
    for sx, sy in [(-1, 0), (0, -1), (-1, -1)]:
        yy, xx = np.mgrid[0:H, 0:W]
        R = L[np.clip(yy - sy * d0, 0, H - 1), np.clip(xx - sx * d0, 0, W - 1)]
        disp, _ = ctx.disparity_sgm(L, R, sva.default_params(D=D, dir=sx, dir_y=sy))
        maps.append(disp)
        bases.append(pitch)
    depth, nv = ctx.fuse_depth(np.stack(maps), bases, f, ps)
    exp, _ = oracle.fuse_depth(np.stack(maps), bases, f, ps)
    assert np.array_equal(depth.view(np.uint64), exp.view(np.uint64))
    inner = depth[d0 + 30: H - 30, d0 + 30: W - 30]
    assert np.allclose(inner, pitch * f / (d0 * ps))
    assert (nv[d0 + 30: H - 30, d0 + 30: W - 30] == 3).all()
