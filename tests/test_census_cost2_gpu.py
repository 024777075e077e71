"""The 2-D array-step census+cost kernel (census_cost2.hip, DESIGN.md §4.2b,
reached through sva_census_cost_d and every sva_disparity_sgm* frame with a
supported 2-D step) vs the CPU oracle's census -> cost2, bit-exact.

Supported: steps whose primitive form has |dir_y| = 1 and |dir| <= 3 (the
rig baselines of getCameraPairs, functions.cpp:148-213, and of BASELINE
config 4's 2x4 grid).  The cases cover the kernel's tiling edges: widths and
heights off its 8-line x 64-row workgroup, images narrower than a line's
shear, windows at every border, dmin past the image, pitched images, every
native D, non-primitive steps, and a full 1080p frame against the census-word
route (sva_census_d x2 -> sva_cost_d).  Unsupported steps are refused.
"""
import numpy as np
import pytest
import torch

from stereovisionarray_amd import synth

pytestmark = pytest.mark.gpu

STEPS = [(0, 1), (0, -1), (1, 1), (-1, -1), (1, -1), (-1, 1), (2, 1), (-2, -1), (2, -1),
         (3, 1), (-3, 1), (3, -1), (-3, -1), (4, -2), (0, 2)]


def dev(a, d):
    return torch.from_numpy(np.ascontiguousarray(a)).to(d)


def cost2_gpu(ctx, sva, L, R, D, dmin, sx, sy, torch_dev, pitch=None):
    H, W = L.shape
    pitch = W if pitch is None else pitch
    Lp = np.zeros((H, pitch), np.uint8)
    Rp = np.zeros((H, pitch), np.uint8)
    Lp[:, :W], Rp[:, :W] = L, R
    Lp[:, W:], Rp[:, W:] = 251, 3          # pitch padding must never be read as pixels
    dL, dR = dev(Lp, torch_dev), dev(Rp, torch_dev)
    C = torch.full((H, W, D), 0xAA, dtype=torch.uint8, device=torch_dev)
    p = sva.default_params(D=D, dmin=dmin, dir=sx, dir_y=sy)
    ctx.census_cost_d(dL.data_ptr(), dR.data_ptr(), W, H, pitch, p, C.data_ptr())
    ctx.synchronize()
    torch.cuda.synchronize()
    return C.cpu().numpy()


def want(oracle, L, R, D, dmin, sx, sy):
    return oracle.cost2(oracle.census(L), oracle.census(R), D, dmin, sx, sy)


@pytest.mark.parametrize("D", [64, 128, 192, 256])
@pytest.mark.parametrize("sx,sy", STEPS)
@pytest.mark.parametrize("dmin", [0, 9])
def test_census_cost2_vs_oracle(ctx, sva, oracle, torch_dev, D, sx, sy, dmin):
    W, H = 71, 290          # taller than D: every disparity has in-image matches
    L, R, _ = synth.stereo_pair2(H, W, D, dmin, sx, sy, seed=D + 3 * sx + sy)
    L[::5, ::3] = 128
    R[::5, ::3] = 128       # equal neighbours: the census '<' stays strict
    got = cost2_gpu(ctx, sva, L, R, D, dmin, sx, sy, torch_dev)
    exp = want(oracle, L, R, D, dmin, sx, sy)
    assert np.array_equal(got, exp)
    assert (exp == 62).any() and (exp < 62).any()


@pytest.mark.parametrize("W,H", [(1, 1), (9, 7), (8, 3), (5, 70), (63, 64), (65, 65), (130, 129),
                                 (300, 41)])
@pytest.mark.parametrize("sx,sy", [(0, 1), (-1, -1), (2, -1), (-3, 1)])
def test_census_cost2_shapes(ctx, sva, oracle, torch_dev, W, H, sx, sy):
    D = 64
    L = synth.texture(H, W, W * 7 + H)
    R = synth.texture(H, W, W * 11 + H + 1)
    got = cost2_gpu(ctx, sva, L, R, D, 0, sx, sy, torch_dev)
    assert np.array_equal(got, want(oracle, L, R, D, 0, sx, sy))


@pytest.mark.parametrize("dmin", [150, 700])
@pytest.mark.parametrize("sx,sy", [(0, -1), (1, 1), (-2, 1), (3, -1)])
def test_census_cost2_far_dmin(ctx, sva, oracle, torch_dev, dmin, sx, sy):
    # matched pixels partly or wholly outside the image (62)
    W, H, D = 120, 140, 128
    L = synth.texture(H, W, 1)
    R = synth.texture(H, W, 2)
    got = cost2_gpu(ctx, sva, L, R, D, dmin, sx, sy, torch_dev)
    assert np.array_equal(got, want(oracle, L, R, D, dmin, sx, sy))


def test_census_cost2_pitched(ctx, sva, oracle, torch_dev):
    W, H, D = 250, 130, 128
    L, R, _ = synth.stereo_pair2(H, W, D, 0, -1, 1, seed=5)
    got = cost2_gpu(ctx, sva, L, R, D, 0, -1, 1, torch_dev, pitch=320)
    assert np.array_equal(got, want(oracle, L, R, D, 0, -1, 1))


@pytest.mark.parametrize("D,sx,sy,dmin", [(128, 0, -1, 0), (128, -1, -1, 0), (128, 1, -1, 3),
                                          (128, 3, -1, 0), (64, -2, -1, 5), (192, 0, 1, 0),
                                          (256, -1, 1, 0)])
def test_census_cost2_matches_census_word_route_1080p(ctx, sva, torch_dev, D, sx, sy, dmin):
    """The same bytes as the census-word route (census x2 -> cost2) on a full
    1080p frame: 240-272 line groups x 17 row chunks, every border."""
    W, H = 1920, 1080
    L, R, _ = synth.stereo_pair2(H, W, D, dmin, sx, sy, seed=1)
    dL, dR = dev(L, torch_dev), dev(R, torch_dev)
    p = sva.default_params(D=D, dmin=dmin, dir=sx, dir_y=sy)
    cl = torch.zeros((H, W), dtype=torch.int64, device=torch_dev)
    cr = torch.zeros((H, W), dtype=torch.int64, device=torch_dev)
    C1 = torch.zeros((H, W, D), dtype=torch.uint8, device=torch_dev)
    C2 = torch.ones((H, W, D), dtype=torch.uint8, device=torch_dev)
    ctx.census_d(dL.data_ptr(), W, H, W, cl.data_ptr())
    ctx.census_d(dR.data_ptr(), W, H, W, cr.data_ptr())
    ctx.cost_d(cl.data_ptr(), cr.data_ptr(), W, H, p, C1.data_ptr())
    ctx.census_cost_d(dL.data_ptr(), dR.data_ptr(), W, H, W, p, C2.data_ptr())
    ctx.synchronize()
    torch.cuda.synchronize()
    assert torch.equal(C1, C2)


@pytest.mark.parametrize("sx,sy", [(1, 2), (2, 3), (4, 1), (-1, 3)])
def test_census_cost2_refuses_other_steps(ctx, sva, torch_dev, sx, sy):
    W, H = 64, 16
    img = torch.zeros((H, W), dtype=torch.uint8, device=torch_dev)
    C = torch.zeros((H, W, 64), dtype=torch.uint8, device=torch_dev)
    p = sva.default_params(D=64, dir=sx, dir_y=sy)
    with pytest.raises(sva.SvaError) as e:
        ctx.census_cost_d(img.data_ptr(), img.data_ptr(), W, H, W, p, C.data_ptr())
    assert e.value.status == sva.SVA_ERR_UNSUPPORTED


@pytest.mark.parametrize("W,H,D,dmin,sx,sy", [
    (120, 160, 64, 0, 0, -1), (150, 150, 64, 0, -1, -1), (130, 260, 128, 2, 1, -1),
    (300, 300, 256, 0, -1, 1), (200, 180, 64, 0, -2, -1), (190, 140, 100, 3, 3, 1),
])
def test_frames_through_census_cost2(ctx, sva, oracle, W, H, D, dmin, sx, sy):
    """sva_disparity_sgm on a supported 2-D step runs census_cost2 -> paths ->
    wta_hv (D = 100 padded to 128 as well)."""
    L, R, _ = synth.stereo_pair2(H, W, D, dmin, sx, sy, seed=W + H)
    p = sva.default_params(D=D, dmin=dmin, dir=sx, dir_y=sy, subpixel=1)
    disp, sub = ctx.disparity_sgm(L, R, p)
    od, osub = oracle.sgm2(L, R, D, dmin, sx, sy, subpixel=True)
    assert np.array_equal(disp, od)
    assert np.max(np.abs(sub - osub)) <= 1e-5
