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
