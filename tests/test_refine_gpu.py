"""SURVEY.md §8f rows 1-2 on the GPU vs the CPU oracle: disparity refinement
(improveWithDisparity / shiftPerspectiveWithDisparity, functions.cpp:11-72)
and depth <-> 3-D output (shiftPerspective2, Points3DToDepthMap,
DepthMapToPoints3D, functions.cpp:74-146).

Bars: u8 maps bit-exact; f64 depth maps and 3-D points bit-exact (same
operand order, no contraction, IEEE div/sqrt on both sides); scatter
collisions resolve to the reference's loop order; untouched pixels keep the
caller's buffer.  Parity vs the reference itself is unpinned (no fixtures,
OpenCV absent)."""
import numpy as np
import pytest
import torch

from stereovisionarray_amd import synth

pytestmark = pytest.mark.gpu


def rig_pair(sva, oracle, a, b, W):
    cams = synth.reference_array(0.036 / W)
    return (sva.Camera.make(*cams[a]), sva.Camera.make(*cams[b]),
            oracle.OCamera.make(*cams[a]), oracle.OCamera.make(*cams[b]))


@pytest.mark.parametrize("b", [11, 13, 7, 17, 6, 18, 8, 16])
def test_shift_perspective(ctx, sva, oracle, b):
    W, H = 173, 91
    ci, co, oi, oo = rig_pair(sva, oracle, 12, b, W)
    rng = np.random.default_rng(b)
    disp = rng.integers(0, 60, size=(H, W)).astype(np.uint8)
    disp[rng.random((H, W)) < 0.1] = 0
    img = synth.texture(H, W, b)
    init = rng.integers(0, 256, size=(H, W)).astype(np.uint8)
    got = ctx.shift_perspective(ci, co, disp, img, init=init)
    exp = oracle.shift_perspective(oi, oo, disp, img, init=init)
    assert np.array_equal(got, exp)
    assert (got == init).any() and (got != init).any()


def _refine_case(H, W, d0, corr, seed):
    center = synth.texture(H, W, seed)
    img = np.zeros_like(center)
    img[:, d0 + corr:] = center[:, : W - d0 - corr]
    return center, img


@pytest.mark.parametrize("window", [1, 3, 4, 7, 20, 21, 33, 65])
def test_improve_with_disparity_windows(ctx, sva, oracle, window):
    W, H = 150, 110
    center = synth.texture(H, W, window)
    cams = [(12, 11), (12, 13), (12, 7), (12, 17), (12, 6)]
    pairs, opairs, imgs = [], [], []
    rng = np.random.default_rng(window)
    for i, (a, b) in enumerate(cams):
        ci, co, oi, oo = rig_pair(sva, oracle, a, b, W)
        pairs.append((ci, co)); opairs.append((oi, oo))
        imgs.append(synth.texture(H, W, 100 + i))
    disp = rng.integers(0, 40, size=(H, W)).astype(np.uint8)
    mask = (rng.random((H, W)) < 0.7).astype(np.uint8)
    init = rng.integers(0, 256, size=(H, W)).astype(np.uint8)
    got = ctx.improve_with_disparity(disp, center, imgs, pairs, window=window, mask=mask,
                                     init=init)
    st, exp = oracle.improve_with_disparity(disp, center, imgs, opairs, window=window, mask=mask,
                                            init=init)
    assert st == 0
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("W,H,window", [(37, 23, 3), (301, 77, 21), (301, 77, 33),
                                          (301, 77, 35), (130, 70, 2)])
def test_improve_padded_pitch_sparse_mask(ctx, sva, oracle, torch_dev, W, H, window):
    """Device entry point on planes with pitch > W and random bytes in the
    padding.  Cases:
    * the box kernel's strip / band edges, including images smaller than one strip;
    * k = 16, the last box size, against k = 17 on the direct kernel;
    * horizontal, vertical and diagonal steps;
    * a 2% mask, so most strips are skipped.
    The output padding stays untouched."""
    P = W + 13
    rng = np.random.default_rng(W * 1000 + window)
    center = synth.texture(H, W, 3)
    pairs, opairs, imgs = [], [], []
    for i, b in enumerate((13, 7, 18, 6)):
        ci, co, oi, oo = rig_pair(sva, oracle, 12, b, W)
        pairs.append((ci, co)); opairs.append((oi, oo))
        imgs.append(synth.texture(H, W, 60 + i))
    disp = rng.integers(0, 12, size=(H, W)).astype(np.uint8)
    mask = (rng.random((H, W)) < 0.02).astype(np.uint8)
    init = rng.integers(0, 256, size=(H, W)).astype(np.uint8)

    def padded(a):
        full = rng.integers(0, 256, size=(H, P)).astype(np.uint8)
        full[:, :W] = a
        return torch.from_numpy(full).to(torch_dev)

    dd, dc, dm = padded(disp), padded(center), padded(mask)
    di = [padded(im) for im in imgs]
    out = padded(init)
    pad_before = out[:, W:].cpu().numpy().copy()
    ctx.improve_with_disparity_d(dd.data_ptr(), dc.data_ptr(), [t.data_ptr() for t in di], pairs,
                                 W, H, P, dm.data_ptr(), window, False, out.data_ptr())
    ctx.synchronize()
    torch.cuda.synchronize()
    st, exp = oracle.improve_with_disparity(disp, center, imgs, opairs, window=window, mask=mask,
                                            init=init)
    got = out.cpu().numpy()
    assert np.array_equal(got[:, :W], exp)
    assert np.array_equal(got[:, W:], pad_before)


def test_improve_finds_known_correction(ctx, sva, oracle):
    W, H, d0 = 200, 80, 9
    center, img = _refine_case(H, W, d0, 3, 5)
    c0 = sva.Camera.make(0.05, (0.05, 0, -0.75), 1e-4)
    c1 = sva.Camera.make(0.05, (0.0, 0, -0.75), 1e-4)
    disp = np.full((H, W), d0, np.uint8)
    mask = np.zeros((H, W), np.uint8)
    mask[20:60, 40:160] = 1
    got = ctx.improve_with_disparity(disp, center, [img], [(c0, c1)], window=21, mask=mask)
    assert (got[20:60, 40:160] == d0 + 3).all()


def test_improve_strict_and_device(ctx, sva, oracle, torch_dev):
    W, H = 96, 64
    ci, co, oi, oo = rig_pair(sva, oracle, 12, 11, W)
    center = synth.texture(H, W, 1)
    img = synth.texture(H, W, 2)
    disp = np.full((H, W), 4, np.uint8)
    with pytest.raises(sva.SvaError) as e:     # full mask: border windows leave the image
        ctx.improve_with_disparity(disp, center, [img], [(ci, co)], window=21, strict=True)
    assert e.value.status == sva.SVA_ERR_INVALID_ARG
    # device entry point, non-strict, no mask: border pixels skipped
    dd, dc, di = (torch.from_numpy(a).to(torch_dev) for a in (disp, center, img))
    out = torch.full((H, W), 77, dtype=torch.uint8, device=torch_dev)
    ctx.improve_with_disparity_d(dd.data_ptr(), dc.data_ptr(), [di.data_ptr()], [(ci, co)], W, H,
                                 W, None, 21, False, out.data_ptr())
    ctx.synchronize()
    torch.cuda.synchronize()
    st, exp = oracle.improve_with_disparity(disp, center, [img], [(oi, oo)], window=21,
                                            init=np.full((H, W), 77, np.uint8))
    assert np.array_equal(out.cpu().numpy(), exp)
    assert (exp[:10] == 77).all() and (exp[20:40, 30:60] != 77).all()


def test_improve_1080p(ctx, sva, oracle):
    """Full-size refinement (the reference's 1080p, 20x20 windows, CROSS pairs
    of camera 12) bit-exact vs the oracle on a masked face-sized region."""
    W, H = 1920, 1080
    center = synth.texture(H, W, 12)
    pairs, opairs, imgs = [], [], []
    for i, b in enumerate((7, 17, 11, 13)):
        ci, co, oi, oo = rig_pair(sva, oracle, 12, b, W)
        pairs.append((ci, co)); opairs.append((oi, oo))
        imgs.append(synth.texture(H, W, 40 + i))
    rng = np.random.default_rng(0)
    disp = rng.integers(100, 160, size=(H, W)).astype(np.uint8)
    mask = np.zeros((H, W), np.uint8)
    mask[300:800, 700:1200] = 1
    got = ctx.improve_with_disparity(disp, center, imgs, pairs, window=21, mask=mask)
    st, exp = oracle.improve_with_disparity(disp, center, imgs, opairs, window=21, mask=mask)
    assert st == 0 and np.array_equal(got, exp)


@pytest.mark.parametrize("b", [11, 13, 7, 6, 18])
def test_shift_perspective2(ctx, sva, oracle, b):
    W, H = 211, 97
    ci, co, oi, oo = rig_pair(sva, oracle, 12, b, W)
    rng = np.random.default_rng(b)
    depth = rng.uniform(0.3, 3.0, size=(H, W))
    depth[rng.random((H, W)) < 0.05] = np.nan
    depth[0, :5] = np.inf
    init = rng.uniform(-1, 0, size=(H, W))
    got = ctx.shift_perspective2(ci, co, depth, init=init)
    exp = oracle.shift_perspective2(oi, oo, depth, init=init)
    assert np.array_equal(got.view(np.uint64), exp.view(np.uint64))
    assert (got == init).any()


def test_shift_perspective2_collisions(ctx, sva, oracle):
    """Many sources per target: only the reference loop's last write survives."""
    W, H = 64, 48
    ci = sva.Camera.make(0.05, (0.05, 0.02, 0), 1e-3)
    co = sva.Camera.make(0.05, (0.0, 0.0, 0), 1e-3)
    oi = oracle.OCamera.make(0.05, (0.05, 0.02, 0), 1e-3)
    oo = oracle.OCamera.make(0.05, (0.0, 0.0, 0), 1e-3)
    rng = np.random.default_rng(3)
    depth = rng.choice([0.6, 0.9, 1.3, 2.5, 5.0], size=(H, W))
    got = ctx.shift_perspective2(ci, co, depth)
    exp = oracle.shift_perspective2(oi, oo, depth)
    assert np.array_equal(got.view(np.uint64), exp.view(np.uint64))


@pytest.mark.parametrize("n", [0, 1, 1000, 200000])
def test_points_to_depth(ctx, sva, oracle, n):
    W, H = 160, 120
    cams = synth.reference_array(0.036 / W)
    cam, ocam = sva.Camera.make(*cams[12]), oracle.OCamera.make(*cams[12])
    rng = np.random.default_rng(n)
    pts = np.stack([rng.uniform(-0.2, 0.2, n), rng.uniform(-0.15, 0.15, n),
                    rng.uniform(-0.5, 1.0, n)], 1)
    if n > 10:
        pts[:5, 2] = cams[12][1][2]          # z == camera z: mult inf -> skipped
        pts[5:10] = pts[10]                  # exact duplicates: last wins
    init = np.full((H, W), -7.0)
    got = ctx.points_to_depth(pts, cam, W, H, init=init)
    exp = oracle.points_to_depth(pts, ocam, W, H, init=init)
    assert np.array_equal(got.view(np.uint64), exp.view(np.uint64))


@pytest.mark.parametrize("W,H", [(1, 1), (33, 17), (640, 480), (3840, 2160)])
def test_depth_to_points(ctx, sva, oracle, W, H):
    cams = synth.reference_array(0.036 / W)
    cam, ocam = sva.Camera.make(*cams[7]), oracle.OCamera.make(*cams[7])
    rng = np.random.default_rng(W)
    depth = rng.uniform(0.0, 0.3, size=(H, W))
    depth[rng.random((H, W)) < 0.01] = np.nan
    got = ctx.depth_to_points(depth, cam)
    exp = oracle.depth_to_points(depth, ocam)
    assert got.shape == exp.shape
    assert np.array_equal(got.view(np.uint64), exp.view(np.uint64))


def test_depth_points_round_trip(ctx, sva):
    """Points3DToDepthMap(DepthMapToPoints3D(depth)) at constant depth 1: every
    pixel becomes one point; re-projection lands on the pixel or (truncation
    of x.9999) a neighbour, and the depth it carries is r_z of the source ray,
    which differs from r_z at the landing pixel by at most ~1.6e-3 relative
    (one pixel's change of the ray angle at the frame edge)."""
    W, H = 320, 240
    cams = synth.reference_array(0.036 / W)
    cam = sva.Camera.make(*cams[12])
    pts = ctx.depth_to_points(np.ones((H, W)), cam)
    assert pts.shape[0] == W * H
    back = ctx.points_to_depth(pts, cam, W, H)
    hit = back != 0
    assert hit.mean() > 0.5
    u, v = np.meshgrid(np.arange(W) - W // 2, np.arange(H) - H // 2)
    ps, f = cams[12][2], cams[12][0]
    rz = f / np.sqrt((u * ps) ** 2 + (v * ps) ** 2 + f * f)
    assert np.allclose(back[hit], rz[hit], rtol=2e-3, atol=0)
    assert (np.abs(back[hit] - rz[hit]) == 0).mean() > 0.4
