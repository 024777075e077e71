"""The one-line-per-wave path kernel (sgm_paths_wide.hip)
against the oracle and against the 16-lane kernel, bit-exact.

sva_set_path_kernel selects the lane layout: WIDE forces one line per wave
at D = 64 / 128 / 256, COST_VOLUME forces the 16-lane layout, AUTO (the
default) takes WIDE for single frames whose 16-lane launch would not fill the
chip.  Both layouts must write the same bytes: the eight direction volumes
of sva_paths_d (each against oracle.path), the tile
pipeline's diagonal volumes and checkpoints of sva_paths_tile_d, and whole
frames against the oracle.  Shapes cover lines shorter than the prefetch
ring, one-column / one-row images (every diagonal step wraps), tall images
(diagonals wrap more than once), padded-cost bytes (255) and the penalty
extremes.
"""
import numpy as np
import pytest
import torch

from stereovisionarray_amd import synth

pytestmark = pytest.mark.gpu

NATIVE_WIDE = [64, 128, 256]


def dev(a, d):
    return torch.from_numpy(np.ascontiguousarray(a)).to(d)


@pytest.fixture()
def layout(ctx, sva):
    """Set a lane layout for one test, AUTO again afterwards."""
    def set_(kind):
        ctx.set_path_kernel(kind)
    yield set_
    ctx.set_path_kernel(sva.SVA_PATH_KERNEL_AUTO)


def paths8(ctx, sva, torch_dev, C, P1=10, P2=120):
    H, W, D = C.shape
    L8 = torch.full((8, H, W, D), 0x5A, dtype=torch.uint8, device=torch_dev)
    p = sva.default_params(D=D, P1=P1, P2=P2)
    d_C = dev(C, torch_dev)
    ctx.paths_d(d_C.data_ptr(), W, H, p, L8.data_ptr())
    ctx.synchronize()
    torch.cuda.synchronize()
    return L8.cpu().numpy()


def tiles(ctx, sva, torch_dev, C, P1=10, P2=120):
    H, W, D = C.shape
    lay = sva.tile_layout(W, H, D)
    d_C = dev(C, torch_dev)
    diag = torch.full((lay.diag_bytes,), 0xAB, dtype=torch.uint8, device=torch_dev)
    hck = torch.full((lay.hckpt_bytes,), 0xCD, dtype=torch.uint8, device=torch_dev)
    vck = torch.full((lay.vckpt_bytes,), 0xEF, dtype=torch.uint8, device=torch_dev)
    p = sva.default_params(D=D, P1=P1, P2=P2)
    ctx.paths_tile_d(d_C.data_ptr(), d_C.numel(), W, H, p, diag.data_ptr(), diag.numel(),
                     hck.data_ptr(), hck.numel(), vck.data_ptr(), vck.numel())
    ctx.synchronize()
    torch.cuda.synchronize()
    return diag.cpu().numpy(), hck.cpu().numpy(), vck.cpu().numpy()


@pytest.mark.parametrize("D", NATIVE_WIDE)
@pytest.mark.parametrize("W,H", [(1, 1), (1, 37), (37, 1), (5, 70), (70, 5), (15, 17), (64, 9),
                                 (33, 130), (130, 33)])
def test_wide_volumes_vs_oracle(ctx, sva, oracle, torch_dev, layout, D, W, H):
    layout(sva.SVA_PATH_KERNEL_WIDE)
    rng = np.random.RandomState(D + 7 * W + H)
    C = rng.randint(0, 63, size=(H, W, D)).astype(np.uint8)
    L8 = paths8(ctx, sva, torch_dev, C)
    for r in range(8):
        assert np.array_equal(L8[r], oracle.path(C, r)), f"direction {r} {oracle.direction(r)}"


@pytest.mark.parametrize("P1,P2", [(0, 0), (3, 7), (50, 20), (193, 193)])
@pytest.mark.parametrize("D", NATIVE_WIDE)
def test_wide_penalties_vs_oracle(ctx, sva, oracle, torch_dev, layout, P1, P2, D):
    layout(sva.SVA_PATH_KERNEL_WIDE)
    H, W = 19, 29
    rng = np.random.RandomState(P1 * 7 + P2 + D)
    C = rng.randint(0, 63, size=(H, W, D)).astype(np.uint8)
    L8 = paths8(ctx, sva, torch_dev, C, P1, P2)
    for r in range(8):
        assert np.array_equal(L8[r], oracle.path(C, r, P1, P2)), f"direction {r}"


@pytest.mark.parametrize("D", NATIVE_WIDE)
@pytest.mark.parametrize("W,H", [(3, 3), (17, 9), (29, 41), (97, 23), (200, 150)])
def test_wide_equals_16_lane_layout(ctx, sva, torch_dev, layout, D, W, H):
    """Eight volumes and the tile stages, both layouts, on costs that include
    the padded value 255 (a padded frame's d >= dreal)."""
    rng = np.random.RandomState(W * 31 + H + D)
    C = rng.randint(0, 63, size=(H, W, D)).astype(np.uint8)
    C[..., D - D // 5:] = 255
    out = {}
    for kind in (sva.SVA_PATH_KERNEL_WIDE, sva.SVA_PATH_KERNEL_COST_VOLUME):
        layout(kind)
        out[kind] = (paths8(ctx, sva, torch_dev, C, 10, 120), tiles(ctx, sva, torch_dev, C, 10, 120))
    a, b = out[sva.SVA_PATH_KERNEL_WIDE], out[sva.SVA_PATH_KERNEL_COST_VOLUME]
    assert np.array_equal(a[0], b[0])
    for x, y, name in zip(a[1], b[1], ("diagonal volumes", "horizontal ckpt", "vertical ckpt")):
        assert np.array_equal(x, y), name


@pytest.mark.parametrize("kind", ["WIDE", "COST_VOLUME", "AUTO"])
@pytest.mark.parametrize("W,H,D,dmin", [(640, 480, 64, 44), (160, 120, 128, 0), (97, 83, 256, 3),
                                        (200, 71, 100, 0)])
def test_frames_each_layout_vs_oracle(ctx, sva, oracle, layout, kind, W, H, D, dmin):
    """Whole frames (census + cost -> paths -> wta_hv + sub-pixel) with the
    layout forced either way and the default: BASELINE config 1's 640x480
    D=64 dmin 44, and a padded D=100."""
    layout(getattr(sva, f"SVA_PATH_KERNEL_{kind}"))
    L, R, _ = synth.stereo_pair(H, W, D, dmin, -1, seed=W + D)
    p = sva.default_params(D=D, dmin=dmin, subpixel=1)
    disp, sub = ctx.disparity_sgm(L, R, p)
    od, osub = oracle.sgm(L, R, D, dmin, -1, subpixel=True, threads=8)
    assert np.array_equal(disp, od)
    assert np.max(np.abs(sub - osub)) <= 1e-5


def test_layout_selector(ctx, sva, layout):
    for kind in (sva.SVA_PATH_KERNEL_WIDE, sva.SVA_PATH_KERNEL_COST_VOLUME,
                 sva.SVA_PATH_KERNEL_AUTO):
        layout(kind)
    with pytest.raises(sva.SvaError) as e:
        ctx.set_path_kernel(7)
    assert e.value.status == sva.SVA_ERR_INVALID_ARG
