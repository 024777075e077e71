"""The frame route's two stages (the tile pipeline)
through their ABI v6 entry points, against the CPU oracle, bit-exact:
sva_paths_tile_d writes the diagonal volumes and the checkpoints (the
oracle's L_0 / L_1 at the checkpoint columns, L_2 / L_3 at the checkpoint
rows, and in a build that recomputes the down diagonals per tile their L_4 /
L_6 rows too); sva_wta_hv_d recomputes the checkpointed directions per tile
and picks d* (sub-pixel within 1e-5 px, observed 0).  The volume / plane
layout is read from sva_tile_layout_of, so the same checks cover the product
build (diag_volumes 4) and the §4.11 experiment build (2).
Ragged widths and heights around the 16 x seg tile, every native D, five
penalty pairs.  Every entry refuses an undersized buffer with
SVA_ERR_INVALID_ARG before launching.
"""
import numpy as np
import pytest
import torch

from stereovisionarray_amd import synth

pytestmark = pytest.mark.gpu

SUB_TOL = 1e-5


def dev(a, d):
    return torch.from_numpy(np.ascontiguousarray(a)).to(d)


def run_tiles(ctx, sva, torch_dev, C, p):
    H, W, D = C.shape
    lay = sva.tile_layout(W, H, D)
    d_C = dev(C, torch_dev)
    nvol = lay.diag_volumes
    diag = torch.full((nvol, H, W, D), 0xAB, dtype=torch.uint8, device=torch_dev)
    hck = torch.full((2, H, lay.nsx, D), 0xCD, dtype=torch.uint8, device=torch_dev)
    vck = torch.full((6 - nvol, lay.nsy, W, D), 0xEF, dtype=torch.uint8, device=torch_dev)
    assert diag.numel() == lay.diag_bytes and hck.numel() == lay.hckpt_bytes
    assert vck.numel() == lay.vckpt_bytes and d_C.numel() == lay.cost_bytes
    ctx.paths_tile_d(d_C.data_ptr(), d_C.numel(), W, H, p, diag.data_ptr(), diag.numel(),
                     hck.data_ptr(), hck.numel(), vck.data_ptr(), vck.numel())
    disp = torch.zeros((H, W), dtype=torch.int16, device=torch_dev)
    sub = torch.zeros((H, W), dtype=torch.float32, device=torch_dev)
    ctx.wta_hv_d(d_C.data_ptr(), d_C.numel(), diag.data_ptr(), diag.numel(), hck.data_ptr(),
                 hck.numel(), vck.data_ptr(), vck.numel(), W, H, p, disp.data_ptr(), sub.data_ptr())
    ctx.synchronize()
    torch.cuda.synchronize()
    return (diag.cpu().numpy(), hck.cpu().numpy(), vck.cpu().numpy(),
            disp.cpu().numpy().view(np.uint16), sub.cpu().numpy(), lay)


def oracle_cost(oracle, H, W, D, dmin, seed):
    L, R, _ = synth.stereo_pair(H, W, D, dmin, -1, seed=seed, stripes=5, step=7)
    return oracle.cost(oracle.census(L), oracle.census(R), D, dmin, -1)


def check_stages(oracle, C, dmin, res, P1=10, P2=120):
    H, W, D = C.shape
    diag, hck, vck, disp, sub, lay = res
    seg = lay.seg
    vols = [oracle.path(C, r, P1, P2) for r in range(8)]
    # volumes: all four diagonals (the wta_hv route, D >= 192), none (the
    # strip route, D <= 128: all eight directions recomputed per tile,
    # DESIGN.md §4.12), or the up diagonals 5, 7 in the §4.11 experiment build
    vol_dirs = {4: [4, 5, 6, 7], 2: [5, 7], 0: []}[lay.diag_volumes]
    for slot, r in enumerate(vol_dirs):
        assert np.array_equal(diag[slot], vols[r]), f"direction {r}"
    for s in range(lay.nsx):
        if s * seg + seg < W:          # L_0 at the segment's last column
            assert np.array_equal(hck[0, :, s], vols[0][:, s * seg + seg - 1]), ("h0", s)
        if s > 0:                      # L_1 at the segment's first column
            assert np.array_equal(hck[1, :, s], vols[1][:, s * seg]), ("h1", s)
    for s in range(lay.nsy):
        if s * seg + seg < H:          # L_2 at the segment's last row
            assert np.array_equal(vck[0, s], vols[2][s * seg + seg - 1]), ("v0", s)
        if s > 0:                      # L_3 at the segment's first row
            assert np.array_equal(vck[1, s], vols[3][s * seg]), ("v1", s)
        if lay.diag_volumes <= 2 and s * seg + seg < H:   # L_4, L_6 at the last row
            assert np.array_equal(vck[2, s], vols[4][s * seg + seg - 1]), ("d4", s)
            assert np.array_equal(vck[3, s], vols[6][s * seg + seg - 1]), ("d6", s)
        if lay.diag_volumes == 0 and s > 0:                # L_5, L_7 at the first row
            assert np.array_equal(vck[4, s], vols[5][s * seg]), ("d5", s)
            assert np.array_equal(vck[5, s], vols[7][s * seg]), ("d7", s)
    S = np.zeros(C.shape, np.uint16)
    for v in vols:
        S += v
    od, osub = oracle.wta(S, dmin, True)
    assert np.array_equal(disp, od)
    assert np.max(np.abs(sub - osub)) <= SUB_TOL


@pytest.mark.parametrize("D", [64, 128, 192, 256])
@pytest.mark.parametrize("W", [1, 7, 8, 9, 16, 17, 33, 100, 257])
def test_tile_stages(ctx, sva, oracle, torch_dev, D, W):
    H, dmin = 21, 2
    C = oracle_cost(oracle, H, W, D, dmin, seed=W + D)
    p = sva.default_params(D=D, dmin=dmin, subpixel=1)
    check_stages(oracle, C, dmin, run_tiles(ctx, sva, torch_dev, C, p))


@pytest.mark.parametrize("H", [1, 7, 8, 9, 16, 17, 40])
def test_tile_stages_heights(ctx, sva, oracle, torch_dev, H):
    W, D = 45, 128
    C = oracle_cost(oracle, H, W, D, 0, seed=H)
    p = sva.default_params(D=D, subpixel=1)
    check_stages(oracle, C, 0, run_tiles(ctx, sva, torch_dev, C, p))


@pytest.mark.parametrize("P1,P2", [(0, 0), (1, 193), (10, 120), (30, 60), (193, 193)])
def test_tile_stages_penalties(ctx, sva, oracle, torch_dev, P1, P2):
    H, W, D = 17, 130, 128
    C = oracle_cost(oracle, H, W, D, 0, seed=P1 + P2)
    p = sva.default_params(D=D, P1=P1, P2=P2, subpixel=1)
    check_stages(oracle, C, 0, run_tiles(ctx, sva, torch_dev, C, p), P1, P2)


def test_tile_stages_without_subpixel(ctx, sva, oracle, torch_dev):
    H, W, D = 9, 70, 64
    C = oracle_cost(oracle, H, W, D, 0, seed=3)
    p = sva.default_params(D=D, subpixel=0)
    _, _, _, disp, sub, _ = run_tiles(ctx, sva, torch_dev, C, p)
    od, _ = oracle.wta(oracle.aggregate(C), 0, False)
    assert np.array_equal(disp, od)
    assert (sub == 0).all()            # not written


def test_undersized_buffers_refused(ctx, sva, torch_dev):
    """Each of the four planes one byte short: SVA_ERR_INVALID_ARG, and
    nothing written (the sentinel survives)."""
    H, W, D = 20, 50, 64
    lay = sva.tile_layout(W, H, D)
    C = torch.zeros(lay.cost_bytes, dtype=torch.uint8, device=torch_dev)
    diag = torch.full((lay.diag_bytes,), 7, dtype=torch.uint8, device=torch_dev)
    hck = torch.full((lay.hckpt_bytes,), 7, dtype=torch.uint8, device=torch_dev)
    vck = torch.full((lay.vckpt_bytes,), 7, dtype=torch.uint8, device=torch_dev)
    disp = torch.zeros((H, W), dtype=torch.int16, device=torch_dev)
    p = sva.default_params(D=D)
    full = [lay.cost_bytes, lay.diag_bytes, lay.hckpt_bytes, lay.vckpt_bytes]
    for i in range(4):
        if full[i] == 0:            # no diagonal volume on the strip route (D <= 128)
            continue
        sizes = list(full)
        sizes[i] -= 1
        with pytest.raises(sva.SvaError) as e:
            ctx.paths_tile_d(C.data_ptr(), sizes[0], W, H, p, diag.data_ptr(), sizes[1],
                             hck.data_ptr(), sizes[2], vck.data_ptr(), sizes[3])
        assert e.value.status == sva.SVA_ERR_INVALID_ARG
        with pytest.raises(sva.SvaError) as e:
            ctx.wta_hv_d(C.data_ptr(), sizes[0], diag.data_ptr(), sizes[1], hck.data_ptr(),
                         sizes[2], vck.data_ptr(), sizes[3], W, H, p, disp.data_ptr())
        assert e.value.status == sva.SVA_ERR_INVALID_ARG
    ctx.synchronize()
    assert int((diag != 7).sum()) == 0 and int((hck != 7).sum()) == 0
    assert int((vck != 7).sum()) == 0


@pytest.mark.parametrize("D", [64, 128, 192, 256])
def test_frame_matches_eight_volume_route(ctx, sva, torch_dev, D):
    """The frame pipeline (tile route) against the stage route that
    materialises all 8 volumes (sva_aggregate_d + sva_wta_d), same cost
    volume, at a multi-tile size: identical disparities and sub-pixel."""
    H, W = 64, 700
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=D)
    p = sva.default_params(D=D, subpixel=1)
    a, sa = ctx.disparity_sgm(L, R, p)
    dL, dR = dev(L, torch_dev), dev(R, torch_dev)
    C = torch.zeros((H, W, D), dtype=torch.uint8, device=torch_dev)
    if D >= 128:
        ctx.census_cost_d(dL.data_ptr(), dR.data_ptr(), W, H, W, p, C.data_ptr())
    else:
        cl = torch.zeros((H, W), dtype=torch.int64, device=torch_dev)
        cr = torch.zeros((H, W), dtype=torch.int64, device=torch_dev)
        ctx.census_d(dL.data_ptr(), W, H, W, cl.data_ptr())
        ctx.census_d(dR.data_ptr(), W, H, W, cr.data_ptr())
        ctx.cost_d(cl.data_ptr(), cr.data_ptr(), W, H, p, C.data_ptr())
    S = torch.zeros((H, W, D), dtype=torch.int16, device=torch_dev)
    ctx.aggregate_d(C.data_ptr(), W, H, p, S.data_ptr())
    disp = torch.zeros((H, W), dtype=torch.int16, device=torch_dev)
    sub = torch.zeros((H, W), dtype=torch.float32, device=torch_dev)
    ctx.wta_d(S.data_ptr(), W, H, p, disp.data_ptr(), sub.data_ptr())
    ctx.synchronize()
    torch.cuda.synchronize()
    assert np.array_equal(a, disp.cpu().numpy().view(np.uint16))
    assert np.array_equal(sa.view(np.uint32), sub.cpu().numpy().view(np.uint32))
