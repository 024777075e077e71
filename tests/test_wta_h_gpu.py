"""Checkpoint-mode frame pipeline: sgm_paths writes the six
vertical/diagonal volumes plus horizontal-path checkpoints, and wta_h
recomputes the two horizontal directions segment by segment before the sum
and the WTA.  Every stage against the CPU oracle, bit-exact: the six volumes,
each checkpoint (the oracle's L_0 / L_1 at the checkpoint columns), and the
disparities (sub-pixel within 1e-5 px, observed 0) on ragged widths around
the segment length (32 up to D = 128, 16 above), widths below one segment,
every D the kernels are built for and five penalty pairs.
"""
import numpy as np
import pytest
import torch

from stereovisionarray_amd import synth

pytestmark = pytest.mark.gpu

SUB_TOL = 1e-5


def dev(a, d):
    return torch.from_numpy(np.ascontiguousarray(a)).to(d)


def run_ckpt(ctx, sva, torch_dev, C, p):
    H, W, D = C.shape
    ns, seg = sva.ckpt_segments(W, D)
    d_C = dev(C, torch_dev)
    L6 = torch.full((6, H, W, D), 0xAB, dtype=torch.uint8, device=torch_dev)
    CK = torch.full((2, H, ns, D), 0xCD, dtype=torch.uint8, device=torch_dev)
    ctx.paths_ckpt_d(d_C.data_ptr(), W, H, p, L6.data_ptr(), CK.data_ptr())
    disp = torch.zeros((H, W), dtype=torch.int16, device=torch_dev)
    sub = torch.zeros((H, W), dtype=torch.float32, device=torch_dev)
    ctx.wta_h_d(d_C.data_ptr(), L6.data_ptr(), CK.data_ptr(), W, H, p, disp.data_ptr(),
                sub.data_ptr())
    ctx.synchronize()
    torch.cuda.synchronize()
    return (L6.cpu().numpy(), CK.cpu().numpy(), disp.cpu().numpy().view(np.uint16),
            sub.cpu().numpy(), ns, seg)


def oracle_cost(oracle, H, W, D, dmin, seed):
    L, R, _ = synth.stereo_pair(H, W, D, dmin, -1, seed=seed, stripes=5, step=7)
    return oracle.cost(oracle.census(L), oracle.census(R), D, dmin, -1)


@pytest.mark.parametrize("D", [64, 128, 192, 256])
@pytest.mark.parametrize("W", [1, 15, 16, 17, 31, 32, 33, 64, 100, 257])
def test_ckpt_pipeline(ctx, sva, oracle, torch_dev, D, W):
    H, dmin = 21, 2
    C = oracle_cost(oracle, H, W, D, dmin, seed=W + D)
    p = sva.default_params(D=D, dmin=dmin, subpixel=1)
    L6, CK, disp, sub, ns, seg = run_ckpt(ctx, sva, torch_dev, C, p)
    vols = [oracle.path(C, r) for r in range(8)]
    for r in range(2, 8):
        assert np.array_equal(L6[r - 2], vols[r]), f"direction {r}"
    for s in range(ns):
        if s * seg + seg < W:          # L_0 at the segment's last column
            assert np.array_equal(CK[0, :, s], vols[0][:, s * seg + seg - 1]), ("ck0", s)
        if s > 0:                      # L_1 at the segment's first column
            assert np.array_equal(CK[1, :, s], vols[1][:, s * seg]), ("ck1", s)
    S = np.zeros(C.shape, np.uint16)
    for v in vols:
        S += v
    od, osub = oracle.wta(S, dmin, True)
    assert np.array_equal(disp, od)
    assert np.max(np.abs(sub - osub)) <= SUB_TOL


@pytest.mark.parametrize("P1,P2", [(0, 0), (1, 193), (10, 120), (30, 60), (193, 193)])
def test_ckpt_pipeline_penalties(ctx, sva, oracle, torch_dev, P1, P2):
    H, W, D = 17, 130, 128
    C = oracle_cost(oracle, H, W, D, 0, seed=P1 + P2)
    p = sva.default_params(D=D, P1=P1, P2=P2, subpixel=1)
    _, _, disp, sub, _, _ = run_ckpt(ctx, sva, torch_dev, C, p)
    S = oracle.aggregate(C, P1, P2)
    od, osub = oracle.wta(S, 0, True)
    assert np.array_equal(disp, od)
    assert np.max(np.abs(sub - osub)) <= SUB_TOL


def test_ckpt_without_subpixel(ctx, sva, oracle, torch_dev):
    H, W, D = 9, 70, 64
    C = oracle_cost(oracle, H, W, D, 0, seed=3)
    p = sva.default_params(D=D, subpixel=0)
    _, _, disp, sub, _, _ = run_ckpt(ctx, sva, torch_dev, C, p)
    od, _ = oracle.wta(oracle.aggregate(C), 0, False)
    assert np.array_equal(disp, od)
    assert (sub == 0).all()            # not written


@pytest.mark.parametrize("D", [64, 128, 192, 256])
def test_frame_matches_eight_volume_route(ctx, sva, torch_dev, D):
    """The frame pipeline (checkpoint mode) against the stage route that
    materialises all 8 volumes (sva_aggregate_d + sva_wta_d), same cost
    volume, at a multi-segment size: identical disparities and sub-pixel."""
    H, W = 64, 700
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=D)
    p = sva.default_params(D=D, subpixel=1)
    ctx.set_path_kernel(sva.SVA_PATH_KERNEL_COST_VOLUME)
    try:
        a, sa = ctx.disparity_sgm(L, R, p)
    finally:
        ctx.set_path_kernel(sva.SVA_PATH_KERNEL_AUTO)
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
