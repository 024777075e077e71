"""Mode S parity: every HIP stage vs the CPU oracle, through the C-ABI.

Integer stages (census words, cost volume, every path volume, S, disparity)
must be bit-exact.  Sub-pixel (f32 parabola) tolerance: |GPU - CPU| <= 1e-5 px
(both sides evaluate the same IEEE expression; observed 0).
Parity vs the reference itself is unpinned (Census/SGM do not exist in the
reference).
"""
import numpy as np
import pytest
import torch

from stereovisionarray_amd import synth

from checks import assert_sub_close

pytestmark = pytest.mark.gpu

SUB_TOL = 1e-5


def dev(a, d):
    return torch.from_numpy(np.ascontiguousarray(a)).to(d)


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def run_sync(ctx):
    ctx.synchronize()
    torch.cuda.synchronize()


@pytest.mark.parametrize("W,H", [(9, 7), (64, 48), (161, 97), (640, 480)])
def test_census(ctx, oracle, torch_dev, W, H):
    img = synth.texture(H, W, W * 31 + H)
    img[::7, ::5] = 128  # equal-valued neighbours: '<' must stay strict
    d_img = dev(img, torch_dev)
    out = torch.zeros((H, W), dtype=torch.int64, device=torch_dev)
    ctx.census_d(d_img.data_ptr(), W, H, W, out.data_ptr())
    run_sync(ctx)
    got = host(out).view(np.uint64)
    assert np.array_equal(got, oracle.census(img))


def test_census_pitched(ctx, oracle, torch_dev):
    W, H, pitch = 100, 40, 128
    big = synth.texture(H, pitch, 5)
    d_img = dev(big, torch_dev)
    out = torch.zeros((H, W), dtype=torch.int64, device=torch_dev)
    ctx.census_d(d_img.data_ptr(), W, H, pitch, out.data_ptr())
    run_sync(ctx)
    assert np.array_equal(host(out).view(np.uint64), oracle.census(big[:, :W]))


@pytest.mark.parametrize("D", [64, 128, 192, 256])
@pytest.mark.parametrize("dir,dmin", [(-1, 0), (1, 0), (1, 7), (-1, 13)])
def test_cost(ctx, sva, oracle, torch_dev, D, dir, dmin):
    W, H = 203, 11
    L, R, _ = synth.stereo_pair(H, W, D, dmin, dir, seed=D + dmin)
    cl, cr = oracle.census(L), oracle.census(R)
    C = torch.zeros((H, W, D), dtype=torch.uint8, device=torch_dev)
    p = sva.default_params(D=D, dmin=dmin, dir=dir)
    d_cl, d_cr = dev(cl.view(np.int64), torch_dev), dev(cr.view(np.int64), torch_dev)
    ctx.cost_d(d_cl.data_ptr(), d_cr.data_ptr(), W, H, p, C.data_ptr())
    run_sync(ctx)
    assert np.array_equal(host(C), oracle.cost(cl, cr, D, dmin, dir))


def _paths(ctx, sva, torch_dev, C, P1=10, P2=120):
    H, W, D = C.shape
    L8 = torch.zeros((8, H, W, D), dtype=torch.uint8, device=torch_dev)
    p = sva.default_params(D=D, P1=P1, P2=P2)
    d_C = dev(C, torch_dev)
    ctx.paths_d(d_C.data_ptr(), W, H, p, L8.data_ptr())
    run_sync(ctx)
    return host(L8)


@pytest.mark.parametrize("D", [64, 128, 192, 256])
@pytest.mark.parametrize("W,H", [(37, 23), (23, 61), (130, 41)])
def test_paths_each_direction(ctx, sva, oracle, torch_dev, D, W, H):
    """All 8 directions, incl. tall images (H > W: diagonal lines wrap more
    than once in x) and sizes that leave partial 16-line blocks."""
    rng = np.random.RandomState(D * 1000 + W)
    C = rng.randint(0, 63, size=(H, W, D)).astype(np.uint8)
    L8 = _paths(ctx, sva, torch_dev, C)
    for r in range(8):
        exp = oracle.path(C, r)
        assert np.array_equal(L8[r], exp), f"direction {r} {oracle.direction(r)}"


@pytest.mark.parametrize("P1,P2", [(0, 0), (10, 120), (3, 7), (50, 20), (193, 193)])
def test_paths_penalties(ctx, sva, oracle, torch_dev, P1, P2):
    H, W, D = 19, 29, 64
    rng = np.random.RandomState(P1 * 7 + P2)
    C = rng.randint(0, 63, size=(H, W, D)).astype(np.uint8)
    L8 = _paths(ctx, sva, torch_dev, C, P1, P2)
    for r in range(8):
        assert np.array_equal(L8[r], oracle.path(C, r, P1, P2)), f"direction {r}"


def test_paths_constant_cost(ctx, sva, oracle, torch_dev):
    """KAT: constant cost c everywhere -> every L equals c (min term is 0)."""
    H, W, D = 17, 33, 128
    C = np.full((H, W, D), 9, np.uint8)
    L8 = _paths(ctx, sva, torch_dev, C)
    assert (L8 == 9).all()


@pytest.mark.parametrize("D", [64, 256])
def test_aggregate_sum(ctx, sva, oracle, torch_dev, D):
    H, W = 31, 45
    rng = np.random.RandomState(D)
    C = rng.randint(0, 63, size=(H, W, D)).astype(np.uint8)
    S = torch.zeros((H, W, D), dtype=torch.int16, device=torch_dev)
    d_C = dev(C, torch_dev)
    ctx.aggregate_d(d_C.data_ptr(), W, H, sva.default_params(D=D), S.data_ptr())
    run_sync(ctx)
    assert np.array_equal(host(S).view(np.uint16), oracle.aggregate(C))


@pytest.mark.parametrize("D", [64, 128, 192, 256])
def test_wta_first_minimum(ctx, sva, oracle, torch_dev, D):
    """S drawn from a tiny range so most pixels have tied minima: the lowest
    d must win (CameraStereoVision.cpp:85 first-min rule)."""
    H, W = 13, 57
    rng = np.random.RandomState(D + 1)
    S = rng.randint(3, 6, size=(H, W, D)).astype(np.uint16)
    S[0, 0, :] = 5
    S[0, 1, D - 1] = 0  # minimum at the last disparity (no parabola)
    S[0, 2, 0] = 0      # minimum at the first disparity
    dmin = 11
    d = torch.zeros((H, W), dtype=torch.int16, device=torch_dev)
    s = torch.zeros((H, W), dtype=torch.float32, device=torch_dev)
    p = sva.default_params(D=D, dmin=dmin, subpixel=1)
    d_S = dev(S.view(np.int16), torch_dev)
    ctx.wta_d(d_S.data_ptr(), W, H, p, d.data_ptr(), s.data_ptr())
    run_sync(ctx)
    od, osub = oracle.wta(S, dmin)
    assert np.array_equal(host(d).view(np.uint16), od)
    assert np.max(np.abs(host(s) - osub)) <= SUB_TOL


@pytest.mark.parametrize("W,H,D,dmin,dir", [
    (160, 120, 64, 0, -1), (97, 61, 128, 3, 1), (256, 64, 192, 0, -1), (300, 70, 256, 5, 1),
    (640, 480, 64, 44, 1),
])
def test_full_pipeline(ctx, sva, oracle, W, H, D, dmin, dir):
    L, R, _ = synth.stereo_pair(H, W, D, dmin, dir, seed=W + D)
    p = sva.default_params(D=D, dmin=dmin, dir=dir, subpixel=1)
    disp, sub = ctx.disparity_sgm(L, R, p)
    od, osub = oracle.sgm(L, R, D, dmin, dir, subpixel=True, threads=8)
    assert np.array_equal(disp, od)
    assert np.max(np.abs(sub - osub)) <= SUB_TOL


def test_full_pipeline_device_buffers(ctx, sva, oracle, torch_dev):
    W, H, D = 200, 90, 128
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=3)
    pitch = 256
    Lp = np.zeros((H, pitch), np.uint8); Lp[:, :W] = L
    Rp = np.zeros((H, pitch), np.uint8); Rp[:, :W] = R
    dL, dR = dev(Lp, torch_dev), dev(Rp, torch_dev)
    disp = torch.zeros((H, W), dtype=torch.int16, device=torch_dev)
    p = sva.default_params(D=D)
    ctx.disparity_sgm_d(dL.data_ptr(), dR.data_ptr(), W, H, pitch, p, disp.data_ptr())
    run_sync(ctx)
    od, _ = oracle.sgm(L, R, D, 0, -1, subpixel=False, threads=8)
    assert np.array_equal(host(disp).view(np.uint16), od)


# 1-D steps run the census+cost kernel at every D (D = 64 since round 4) for
# both matching roles (the right-reference pass swaps the images, not census maps)
@pytest.mark.parametrize("D,dir,dmin", [(64, -1, 0), (128, -1, 0), (128, 1, 3), (192, -1, 2)])
def test_lr_check(ctx, sva, oracle, D, dir, dmin):
    W, H = 300, 60
    L, R, _ = synth.stereo_pair(H, W, D, dmin, dir, seed=11, stripes=6, step=9)
    p = sva.default_params(D=D, dmin=dmin, dir=dir, lr_check=1, lr_max_diff=1, invalid=0xFFFF,
                           subpixel=1)
    disp, sub = ctx.disparity_sgm(L, R, p)
    dl, osub = oracle.sgm(L, R, D, dmin, dir, subpixel=True, threads=8)
    dr, _ = oracle.sgm(R, L, D, dmin, -dir, subpixel=False, threads=8)
    exp = oracle.lr_check(dl, dr, dir, 1, 0xFFFF)
    assert np.array_equal(disp, exp)
    assert (disp == 0xFFFF).any() and (disp != 0xFFFF).any()
    assert_sub_close(sub, oracle.lr_sub(exp, osub, 0xFFFF))



def test_shifted_texture_exact(ctx, sva):
    """KAT: R(x - d0) = L(x) with a constant d0 -> Hamming cost 0 at d0 on
    every interior pixel, so WTA returns d0 there."""
    W, H, D, d0 = 320, 96, 64, 23
    L = synth.texture(H, W, 9)
    R = np.zeros_like(L)
    R[:, : W - d0] = L[:, d0:]
    R[:, W - d0:] = synth.texture(H, d0, 10)
    disp, _ = ctx.disparity_sgm(L, R, sva.default_params(D=D, dir=-1))
    inner = disp[8:-8, d0 + 40: W - 40]
    assert (inner == d0).all()


def test_rejects_unsupported(ctx, sva):
    L = np.zeros((32, 32), np.uint8)
    with pytest.raises(sva.SvaError) as e:
        ctx.disparity_sgm(L, L, sva.default_params(D=257))
    assert e.value.status == sva.SVA_ERR_UNSUPPORTED
    with pytest.raises(sva.SvaError) as e:
        ctx.disparity_sgm(L, L, sva.default_params(D=64, P2=200))
    assert e.value.status == sva.SVA_ERR_INVALID_ARG


@pytest.mark.slow
def test_full_size_1080p_d128(ctx, sva, oracle):
    """BASELINE config 2 at full size, bit-exact vs the (threaded) oracle."""
    W, H, D = 1920, 1080, 128
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=1)
    p = sva.default_params(D=D, subpixel=1)
    disp, sub = ctx.disparity_sgm(L, R, p)
    od, osub = oracle.sgm(L, R, D, 0, -1, subpixel=True, threads=16)
    assert np.array_equal(disp, od)
    assert np.max(np.abs(sub - osub)) <= SUB_TOL


@pytest.mark.slow
def test_full_size_4k_d256(ctx, sva, oracle):
    """BASELINE config 3 at full size (3840x2160, D=256, seed 2):
    bit-exact vs the threaded oracle on the default route, which is the route
    bench.py times for this workload (~9 GB of oracle buffers, ~15 s)."""
    W, H, D = 3840, 2160, 256
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=2)
    p = sva.default_params(D=D, subpixel=1)
    disp, sub = ctx.disparity_sgm(L, R, p)
    od, osub = oracle.sgm(L, R, D, 0, -1, subpixel=True, threads=16)
    assert np.array_equal(disp, od)
    assert np.max(np.abs(sub - osub)) <= SUB_TOL


@pytest.mark.slow
def test_full_size_4k_d256_properties(ctx, sva):
    """BASELINE config 3 (3840x2160, D=256): size-independent properties --
    deterministic across runs, and exact d0 on a constant-shift texture."""
    W, H, D, d0 = 3840, 2160, 256, 150
    L = synth.texture(H, W, 2)
    R = np.zeros_like(L)
    R[:, : W - d0] = L[:, d0:]
    R[:, W - d0:] = synth.texture(H, d0, 4)
    p = sva.default_params(D=D, dir=-1, subpixel=1)
    a, sa = ctx.disparity_sgm(L, R, p)          # default AUTO: the cost-volume route
    b, _ = ctx.disparity_sgm(L, R, p)
    assert np.array_equal(a, b)
    assert (a[8:-8, d0 + 64: W - 64] == d0).all()
    # sub-pixel run to run identical too, and finite where the parabola applies
    _, sb = ctx.disparity_sgm(L, R, p)
    assert np.array_equal(sa.view(np.uint32), sb.view(np.uint32))
    assert np.isfinite(sa).all()
