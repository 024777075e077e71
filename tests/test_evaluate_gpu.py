"""SURVEY.md §8f row 4 evaluation on the GPU vs the CPU oracle:
resize INTER_LINEAR on f64 and the (resize(depth, ref.size()) - ref) * 50
error (CameraStereoVision.cpp:107-110,118-119) bit-exact; cv::mean(image,
mask) (functions.cpp:348-354) within rel 1e-12 (tree vs sequential f64
summation).  OpenCV absent: parity vs OpenCV itself unpinned."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sw,sh,dw,dh", [(960, 540, 640, 360), (960, 540, 480, 270),
                                         (960, 540, 1920, 1080), (960, 540, 960, 540),
                                         (97, 61, 250, 13), (1, 50, 7, 9), (50, 1, 9, 7),
                                         (640, 480, 641, 479), (3, 3, 1, 1)])
def test_resize_linear(ctx, oracle, sw, sh, dw, dh):
    src = np.random.default_rng(sw + dh).uniform(0.2, 5.0, size=(sh, sw))
    assert np.array_equal(ctx.resize_linear(src, dw, dh), oracle.resize_linear_f64(src, dw, dh))


def test_ref_error_host_and_device(ctx, oracle, torch_dev):
    rng = np.random.default_rng(3)
    depth = rng.uniform(0.3, 2.0, size=(540, 960))
    depth[rng.random(depth.shape) < 0.1] = 0.0          # unmatched pixels (depth 0)
    ref = rng.uniform(0.3, 2.0, size=(400, 700))
    exp = oracle.ref_error(depth, ref, 50.0)
    assert np.array_equal(ctx.ref_error(depth, ref, 50.0), exp)
    dd, dr = torch.from_numpy(depth).to(torch_dev), torch.from_numpy(ref).to(torch_dev)
    out = torch.zeros((400, 700), dtype=torch.float64, device=torch_dev)
    ctx.ref_error_d(dd.data_ptr(), 960, 540, dr.data_ptr(), 700, 400, 50.0, out.data_ptr())
    ctx.synchronize()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), exp)
    out2 = torch.zeros((400, 700), dtype=torch.float64, device=torch_dev)
    ctx.resize_linear_d(dd.data_ptr(), 960, 540, out2.data_ptr(), 700, 400)
    ctx.synchronize()
    torch.cuda.synchronize()
    assert np.array_equal(out2.cpu().numpy(), oracle.resize_linear_f64(depth, 700, 400))


@pytest.mark.parametrize("w,h,density", [(960, 540, 0.3), (1920, 1080, 1.0), (33, 7, 0.5),
                                         (1, 1, 1.0), (300, 200, 0.0)])
def test_masked_mean(ctx, oracle, torch_dev, w, h, density):
    rng = np.random.default_rng(w + h)
    img = rng.normal(1.0, 5.0, size=(h, w))
    mask = (rng.random((h, w)) < density).astype(np.uint8)
    exp = oracle.masked_mean(img, mask)
    got = ctx.masked_mean(img, mask)
    if exp == 0.0:
        assert got == 0.0
    else:
        assert got == pytest.approx(exp, rel=1e-12)
    assert ctx.masked_mean(img) == pytest.approx(oracle.masked_mean(img), rel=1e-12)
    di = torch.from_numpy(img).to(torch_dev)
    dm = torch.from_numpy(mask).to(torch_dev)
    torch.cuda.synchronize()
    a = ctx.masked_mean_d(di.data_ptr(), dm.data_ptr(), w, h)
    assert a == ctx.masked_mean(img, mask)              # deterministic, same tree


def test_evaluation_errors(ctx, sva):
    with pytest.raises(sva.SvaError):
        ctx.resize_linear(np.zeros((4, 4)), 0, 3)
    with pytest.raises(sva.SvaError):
        ctx.ref_error(np.zeros((4, 4)), np.zeros((0, 3)))
