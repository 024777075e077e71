"""GPU ingestion resize vs the oracle restatement of
OpenCV's exact-2x INTER_LINEAR/area path: bit-exact, including odd sizes
(partial edge blocks, half-to-even sizes), pitched device buffers and the
folder loader end to end."""
import numpy as np
import pytest
import torch

from stereovisionarray_amd import ingest, synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("W,H", [(2, 2), (3, 3), (5, 7), (7, 5), (640, 480), (1921, 1079),
                                 (1923, 1081), (3840, 2160)])
def test_resize_half(ctx, oracle, W, H):
    img = synth.texture(H, W, W + H)
    got = ctx.resize_half(img)
    exp = oracle.resize_half(img)
    assert got.shape == exp.shape
    assert np.array_equal(got, exp)


def test_resize_half_pitched_device(ctx, sva, oracle, torch_dev):
    W, H, pitch = 301, 77, 320
    big = synth.texture(H, pitch, 3)
    dw, dh = sva.resize_half_size(W, H)
    src = torch.from_numpy(big).to(torch_dev)
    dst = torch.full((dh, 160), 7, dtype=torch.uint8, device=torch_dev)
    ctx.resize_half_d(src.data_ptr(), W, H, pitch, dst.data_ptr(), 160)
    ctx.synchronize()
    torch.cuda.synchronize()
    out = dst.cpu().numpy()
    assert np.array_equal(out[:, :dw], oracle.resize_half(np.ascontiguousarray(big[:, :W])))
    assert (out[:, dw:] == 7).all()


def test_load_folder(ctx, oracle, tmp_path):
    PIL = pytest.importorskip("PIL.Image")
    for i in range(3):
        PIL.fromarray(synth.texture(60, 90, i)).save(tmp_path / f"view{i:02d}.png")
    imgs = ingest.load_folder(ctx, str(tmp_path))
    assert len(imgs) == 3
    for i, im in enumerate(imgs):
        assert np.array_equal(im, oracle.resize_half(synth.texture(60, 90, i)))
