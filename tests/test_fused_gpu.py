"""Census-fused path kernel (sgm_fused.hip) vs the CPU oracle.

The fused kernel forms C(p,d) = popcount(CL ^ CR) in registers instead of
reading a cost volume, so its 8 path volumes must equal the oracle's
path(cost(census(L), census(R))) bit for bit.  The cases stress what is new
in it: the shared vertical/diagonal window (4 lines per wave, phantom lines
in partial waves, diagonal groups straddling the x wrap, read through the
cyclic census pad), the horizontal register window (one word enters per
step), and the outside-image mask at both image edges for both step signs,
including dmin beyond the image width.
"""
import numpy as np
import pytest
import torch

from stereovisionarray_amd import synth

from checks import assert_sub_close

pytestmark = pytest.mark.gpu


def dev(a, d):
    return torch.from_numpy(np.ascontiguousarray(a)).to(d)


def fused_volumes(ctx, sva, torch_dev, L, R, D, dmin, dir, P1=10, P2=120, pitch=None):
    H, W = L.shape
    pitch = pitch or W
    Lp = np.zeros((H, pitch), np.uint8); Lp[:, :W] = L
    Rp = np.zeros((H, pitch), np.uint8); Rp[:, :W] = R
    dL, dR = dev(Lp, torch_dev), dev(Rp, torch_dev)
    L8 = torch.full((8, H, W, D), 0xAB, dtype=torch.uint8, device=torch_dev)
    p = sva.default_params(D=D, dmin=dmin, dir=dir, P1=P1, P2=P2)
    ctx.paths_fused_d(dL.data_ptr(), dR.data_ptr(), W, H, pitch, p, L8.data_ptr())
    ctx.synchronize()
    torch.cuda.synchronize()
    return L8.cpu().numpy()


def check(ctx, sva, oracle, torch_dev, W, H, D, dmin, dir, seed, P1=10, P2=120, pitch=None):
    L, R, _ = synth.stereo_pair(H, W, D, min(dmin, 10_000), dir, seed=seed)
    got = fused_volumes(ctx, sva, torch_dev, L, R, D, dmin, dir, P1, P2, pitch)
    C = oracle.cost(oracle.census(L), oracle.census(R), D, dmin, dir)
    for r in range(8):
        exp = oracle.path(C, r, P1, P2)
        if not np.array_equal(got[r], exp):
            bad = np.argwhere(got[r] != exp)
            raise AssertionError(f"direction {r} {oracle.direction(r)}: {len(bad)} mismatches, "
                                 f"first (y,x,d) {bad[0].tolist()}")


@pytest.mark.parametrize("D", [64, 128, 192, 256])
@pytest.mark.parametrize("dir", [-1, 1])
@pytest.mark.parametrize("W,H,dmin", [(37, 23, 0), (23, 61, 3), (130, 41, 0), (203, 19, 17), (33, 40, 1), (97, 9, 0)])
def test_fused_volumes(ctx, sva, oracle, torch_dev, D, dir, W, H, dmin):
    """Ragged widths (partial waves, phantom lines), tall images (diagonal lines
    wrap in x more than once) and D > W (every pixel has outside disparities)."""
    check(ctx, sva, oracle, torch_dev, W, H, D, dmin, dir, seed=D * 7 + W + dir)


@pytest.mark.parametrize("W,H", [(1, 1), (1, 9), (2, 5), (3, 3), (4, 2), (5, 17), (17, 1)])
@pytest.mark.parametrize("dir", [-1, 1])
def test_fused_tiny(ctx, sva, oracle, torch_dev, W, H, dir):
    """Images narrower than one wave's 4 lines: the cyclic pad wraps more than
    once and most lines of the wave are phantom."""
    check(ctx, sva, oracle, torch_dev, W, H, 64, 0, dir, seed=W * 13 + H)


@pytest.mark.parametrize("dmin", [1, 63, 64, 200, 500])
@pytest.mark.parametrize("dir", [-1, 1])
def test_fused_dmin(ctx, sva, oracle, torch_dev, dmin, dir):
    """dmin near and beyond the width: windows start outside the image; with
    dmin >= W every cost is the outside value 62."""
    check(ctx, sva, oracle, torch_dev, 150, 13, 128, dmin, dir, seed=dmin)


@pytest.mark.parametrize("P1,P2", [(0, 0), (3, 7), (50, 20), (193, 193)])
def test_fused_penalties(ctx, sva, oracle, torch_dev, P1, P2):
    check(ctx, sva, oracle, torch_dev, 71, 29, 64, 2, -1, seed=P1 + P2, P1=P1, P2=P2)


def test_fused_pitched_input(ctx, sva, oracle, torch_dev):
    check(ctx, sva, oracle, torch_dev, 100, 31, 128, 0, -1, seed=5, pitch=160)


@pytest.mark.parametrize("D,dir", [(128, -1), (64, 1), (256, -1)])
def test_fused_matches_cost_volume_path(ctx, sva, torch_dev, D, dir):
    """Larger frame: the fused volumes equal the materialised path's
    (census -> cost -> sgm_paths) volumes, all 8 directions."""
    W, H = 640, 360
    L, R, _ = synth.stereo_pair(H, W, D, 0, dir, seed=D)
    got = fused_volumes(ctx, sva, torch_dev, L, R, D, 0, dir)
    dL, dR = dev(L, torch_dev), dev(R, torch_dev)
    cl = torch.zeros((H, W), dtype=torch.int64, device=torch_dev)
    cr = torch.zeros_like(cl)
    ctx.census_d(dL.data_ptr(), W, H, W, cl.data_ptr())
    ctx.census_d(dR.data_ptr(), W, H, W, cr.data_ptr())
    p = sva.default_params(D=D, dir=dir)
    C = torch.zeros((H, W, D), dtype=torch.uint8, device=torch_dev)
    ctx.cost_d(cl.data_ptr(), cr.data_ptr(), W, H, p, C.data_ptr())
    L8 = torch.zeros((8, H, W, D), dtype=torch.uint8, device=torch_dev)
    ctx.paths_d(C.data_ptr(), W, H, p, L8.data_ptr())
    ctx.synchronize()
    torch.cuda.synchronize()
    exp = L8.cpu().numpy()
    for r in range(8):
        assert np.array_equal(got[r], exp[r]), f"direction {r}"


def test_fused_rejects_2d_step(ctx, sva, torch_dev):
    L = torch.zeros((16, 16), dtype=torch.uint8, device=torch_dev)
    L8 = torch.zeros((8, 16, 16, 64), dtype=torch.uint8, device=torch_dev)
    p = sva.default_params(D=64, dir=-1, dir_y=-1)
    with pytest.raises(sva.SvaError) as e:
        ctx.paths_fused_d(L.data_ptr(), L.data_ptr(), 16, 16, 16, p, L8.data_ptr())
    assert e.value.status == sva.SVA_ERR_UNSUPPORTED


@pytest.fixture
def fused_ctx(ctx, sva):
    ctx.set_path_kernel(sva.SVA_PATH_KERNEL_FUSED)
    yield ctx
    ctx.set_path_kernel(sva.SVA_PATH_KERNEL_AUTO)


@pytest.mark.parametrize("W,H,D,dmin,dir", [
    (160, 120, 64, 0, -1), (97, 61, 128, 3, 1), (256, 64, 192, 0, -1), (300, 70, 256, 5, 1),
    (640, 480, 64, 44, 1),
])
def test_fused_pipeline(fused_ctx, sva, oracle, W, H, D, dmin, dir):
    """sva_disparity_sgm on the fused path kernel: bit-exact disparities,
    sub-pixel within the stated 1e-5 px."""
    L, R, _ = synth.stereo_pair(H, W, D, dmin, dir, seed=W + D)
    p = sva.default_params(D=D, dmin=dmin, dir=dir, subpixel=1)
    disp, sub = fused_ctx.disparity_sgm(L, R, p)
    od, osub = oracle.sgm(L, R, D, dmin, dir, subpixel=True, threads=8)
    assert np.array_equal(disp, od)
    assert np.max(np.abs(sub - osub)) <= 1e-5


# the fused route's L/R pass reuses one padded census buffer with
# swapped offsets and a flipped step (sva_api.cpp fused_paths), so it is run
# over D (incl. config 3's 256), both step signs and dmin > 0.
@pytest.mark.parametrize("D,dir,dmin", [(64, -1, 0), (128, -1, 0), (128, 1, 0), (128, -1, 7),
                                        (256, -1, 0), (256, 1, 5), (256, -1, 3)])
def test_fused_pipeline_lr_check(fused_ctx, sva, oracle, D, dir, dmin):
    """The L/R pass swaps the padded census maps' roles inside one buffer."""
    W, H = 260, 48
    L, R, _ = synth.stereo_pair(H, W, D, dmin, dir, seed=11 + D, stripes=6, step=9)
    p = sva.default_params(D=D, dmin=dmin, dir=dir, lr_check=1, lr_max_diff=1, invalid=0xFFFF,
                           subpixel=1)
    disp, sub = fused_ctx.disparity_sgm(L, R, p)
    dl, osub = oracle.sgm(L, R, D, dmin, dir, subpixel=True, threads=8)
    dr, _ = oracle.sgm(R, L, D, dmin, -dir, subpixel=False, threads=8)
    exp = oracle.lr_check(dl, dr, dir, 1, 0xFFFF)
    assert np.array_equal(disp, exp)
    assert (disp == 0xFFFF).any() and (disp != 0xFFFF).any()
    assert_sub_close(sub, oracle.lr_sub(exp, osub, 0xFFFF))


@pytest.mark.parametrize("kern", ["auto", "fused"])
@pytest.mark.parametrize("dir", [-1, 1])
def test_d256_lr_check_both_routes(ctx, sva, oracle, dir, kern):
    """D = 256 with the L/R check on the AUTO route (the cost volume, DESIGN.md
    §4.5) and on the fused route."""
    W, H, D, dmin = 300, 40, 256, 2
    L, R, _ = synth.stereo_pair(H, W, D, dmin, dir, seed=31, stripes=6, step=9)
    ctx.set_path_kernel(sva.SVA_PATH_KERNEL_AUTO if kern == "auto" else sva.SVA_PATH_KERNEL_FUSED)
    p = sva.default_params(D=D, dmin=dmin, dir=dir, lr_check=1, lr_max_diff=1, subpixel=1)
    disp, sub = ctx.disparity_sgm(L, R, p)
    dl, osub = oracle.sgm(L, R, D, dmin, dir, subpixel=True, threads=8)
    dr, _ = oracle.sgm(R, L, D, dmin, -dir, subpixel=False, threads=8)
    exp = oracle.lr_check(dl, dr, dir, 1, 0xFFFF)
    assert np.array_equal(disp, exp)
    assert_sub_close(sub, oracle.lr_sub(exp, osub, 0xFFFF))


def test_fused_pipeline_2d_step_uses_cost_volume(fused_ctx, sva, oracle):
    """Array pairs on 2-D steps keep the cost-volume kernels in fused mode."""
    A, B, _ = synth.stereo_pair2(90, 100, 64, 0, -2, -1, seed=5, stripes=4, step=8)
    d, _ = fused_ctx.disparity_sgm(A, B, sva.default_params(D=64, dir=-2, dir_y=-1))
    o, _ = oracle.sgm2(A, B, 64, 0, -2, -1, subpixel=False)
    assert np.array_equal(d, o)


@pytest.mark.slow
def test_fused_full_size_1080p_d128(fused_ctx, sva):
    """BASELINE config 2 at full size: fused and cost-volume kernels agree on
    every disparity and sub-pixel value (the cost-volume path is checked against
    the oracle at this size in test_sgm_gpu.py)."""
    W, H, D = 1920, 1080, 128
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=1)
    p = sva.default_params(D=D, subpixel=1)
    a, sa = fused_ctx.disparity_sgm(L, R, p)
    fused_ctx.set_path_kernel(sva.SVA_PATH_KERNEL_COST_VOLUME)
    b, sb = fused_ctx.disparity_sgm(L, R, p)
    fused_ctx.set_path_kernel(sva.SVA_PATH_KERNEL_FUSED)
    assert np.array_equal(a, b)
    assert np.array_equal(sa.view(np.uint32), sb.view(np.uint32))
