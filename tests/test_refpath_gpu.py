"""Mode R parity: the reference's own path (CameraStereoVision.cpp:44-95) on
the GPU vs the CPU restatement (oracle/refpath_oracle.c), bit-exact.

Parity of the restatement against the reference binary is unpinned (the
reference needs OpenCV, absent here); tests/test_oracle_kat.py pins the
restatement by hand-derived known answers instead.
"""
import numpy as np
import pytest
import torch

from stereovisionarray_amd import synth

pytestmark = pytest.mark.gpu


def cams_for(sva, oracle, W, i_ref, i_oth):
    ps = 0.036 / W  # pixelSize = sensor_size / width (CameraStereoVision.cpp:30)
    grid = synth.reference_array(ps)
    return (sva.Camera.make(*grid[i_ref]), sva.Camera.make(*grid[i_oth]),
            oracle.OCamera.make(*grid[i_ref]), oracle.OCamera.make(*grid[i_oth]))


# pairs from getCameraPairs (functions.cpp:148-197): MID_LEFT, MID_TOP and the
# diagonal TO_CENTER_SMALL members, so Low and High Bresenham lines and both
# step signs are exercised.
PAIRS = [(12, 11), (12, 13), (12, 7), (12, 17), (12, 6), (12, 8), (12, 16), (12, 18)]


@pytest.mark.parametrize("W,H", [(160, 120), (640, 480), (1920, 1080), (3840, 2160), (321, 243)])
@pytest.mark.parametrize("pair", [(12, 11), (12, 7), (12, 18)])
def test_endpoints_bit_exact(ctx, sva, oracle, torch_dev, W, H, pair):
    """f64 ray geometry: every pixel's (pixel1, pixel2) and the bounds check,
    including the ~19% of 1080p pixels whose row truncates off by one."""
    cr, co, ocr, oco = cams_for(sva, oracle, W, *pair)
    k = 20
    ends = torch.zeros((H, W, 4), dtype=torch.int32, device=torch_dev)
    valid = torch.zeros((H, W), dtype=torch.uint8, device=torch_dev)
    ctx.ref_endpoints_d(W, H, cr, co, k, 0.5, 1.0, ends.data_ptr(), valid.data_ptr())
    ctx.synchronize()
    e = ends.cpu().numpy()
    v = valid.cpu().numpy()
    rng = np.random.RandomState(W + pair[1])
    ys = np.concatenate([rng.randint(k, H - k, 400), [k, H - k - 1, H // 2]])
    xs = np.concatenate([rng.randint(k, W - k, 400), [k, W - k - 1, W // 2]])
    for y, x in zip(ys, xs):
        ok, a, b = oracle.ref_endpoints(ocr, oco, W, H, k, 0.5, 1.0, int(x), int(y))
        assert tuple(e[y, x]) == (a[0], a[1], b[0], b[1]), (x, y)
        assert bool(v[y, x]) == ok, (x, y)


@pytest.mark.parametrize("pair", PAIRS)
def test_ref_path_pairs(ctx, sva, oracle, pair):
    W, H, k = 160, 120, 12
    cr, co, ocr, oco = cams_for(sva, oracle, W, *pair)
    img_ref = synth.texture(H, W, pair[1])
    img_oth = synth.texture(H, W, 100 + pair[1])
    # embed a shifted copy so the minimum is meaningful
    img_oth[:, 12:] = img_ref[:, :-12]
    d8, d16, valid = ctx.disparity_ref(img_ref, img_oth, cr, co, k=k)
    o8, o16, ovalid, n = oracle.ref_pair(img_ref, img_oth, ocr, oco, k=k)
    assert n > 0
    assert np.array_equal(valid, ovalid)
    assert np.array_equal(d8, o8)
    assert np.array_equal(d16, o16)


@pytest.mark.parametrize("pair", [(12, 11), (12, 7)])
@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 8, 13, 20, 21, 27, 28, 29, 32])
def test_ref_path_window_sizes(ctx, sva, oracle, k, pair):
    """Windows 2k x 2k incl. odd k (2k % 4 == 2: partial last dword), every
    row-count class of the plane kernel (k <= 28, one instantiation per k)
    and the per-pixel kernel above it; Low (12 -> 11) and High (12 -> 7)
    lines, i.e. both plane orders."""
    W, H = 200, 150
    cr, co, ocr, oco = cams_for(sva, oracle, W, *pair)
    a = synth.texture(H, W, k)
    b = np.roll(a, 10, axis=1 if pair[1] == 11 else 0)
    d8, d16, valid = ctx.disparity_ref(a, b, cr, co, k=k)
    o8, o16, ovalid, _ = oracle.ref_pair(a, b, ocr, oco, k=k)
    assert np.array_equal(valid, ovalid) and np.array_equal(d16, o16)


def test_ref_path_mask_and_overwrite(ctx, sva, oracle):
    """mask == 0 pixels are skipped (:53) and keep the caller's values; a
    second pair overwrites only the pixels it keeps (:55)."""
    W, H, k = 160, 120, 10
    cr, co, ocr, oco = cams_for(sva, oracle, W, 12, 11)
    _, co2, _, oco2 = cams_for(sva, oracle, W, 12, 7)
    a = synth.texture(H, W, 1)
    b = np.roll(a, 8, axis=1)
    c = np.roll(a, 8, axis=0)
    mask = np.zeros((H, W), np.uint8)
    mask[20:90, 30:140] = 255
    g8 = np.full((H, W), 77, np.uint8)
    g16 = np.full((H, W), 777, np.uint16)
    gv = np.zeros((H, W), np.uint8)
    ctx.disparity_ref(a, b, cr, co, k=k, mask=mask, disp_u8=g8, disp_u16=g16, valid=gv)
    ctx.disparity_ref(a, c, cr, co2, k=k, mask=mask, disp_u8=g8, disp_u16=g16, valid=gv)
    o8 = np.full((H, W), 77, np.uint8)
    o16 = np.full((H, W), 777, np.uint16)
    ov = np.zeros((H, W), np.uint8)
    oracle.ref_pair(a, b, ocr, oco, k=k, mask=mask, disp_u8=o8, disp_u16=o16, valid=ov)
    oracle.ref_pair(a, c, ocr, oco2, k=k, mask=mask, disp_u8=o8, disp_u16=o16, valid=ov)
    assert np.array_equal(g8, o8) and np.array_equal(g16, o16) and np.array_equal(gv, ov)
    assert (g8[mask == 0] == 77).all()


def test_ref_path_wraps_mod_256(ctx, sva, oracle):
    """1080p-class geometry: disparities above 255 wrap in the u8 map (:89)
    while the u16 map keeps them."""
    W, H, k = 1920, 64, 20
    ps = 0.036 / W
    grid = synth.reference_array(ps)
    # cameras 12 and 10 (JUMP_CROSS, functions.cpp:191) are 0.1 m apart
    cr, co = sva.Camera.make(*grid[12]), sva.Camera.make(*grid[10])
    ocr, oco = oracle.OCamera.make(*grid[12]), oracle.OCamera.make(*grid[10])
    a = synth.texture(H, W, 5)
    b = np.roll(a, 300, axis=1)
    mask = np.zeros((H, W), np.uint8)
    mask[30:34, 700:1200] = 1
    d8, d16, valid = ctx.disparity_ref(a, b, cr, co, k=k, mask=mask)
    o8, o16, ov, _ = oracle.ref_pair(a, b, ocr, oco, k=k, mask=mask)
    assert np.array_equal(valid, ov) and np.array_equal(d16, o16) and np.array_equal(d8, o8)
    assert (d16[valid == 1] > 255).any()


def test_depth(ctx, oracle, torch_dev):
    disp = np.arange(256, dtype=np.uint8).repeat(3)
    cam_distance, f, ps = 0.05, 0.05, 0.036 / 640
    d = torch.from_numpy(disp).to(torch_dev)
    out = torch.zeros(disp.size, dtype=torch.float64, device=torch_dev)
    ctx.disparity_to_depth_d(d.data_ptr(), disp.size, cam_distance, f, ps, out.data_ptr())
    ctx.synchronize()
    assert np.array_equal(out.cpu().numpy(), oracle.disp_to_depth(disp, cam_distance, f, ps))


def test_ref_path_plane_fallback_diagonal_jump(ctx, sva, oracle):
    """Pair 12 -> 0 (two grid units on the diagonal) at 1080p: per-tile offset
    boxes exceed the plane kernel's bitmap, so those tiles take the per-pixel
    fallback inside the same launch -- still bit-exact."""
    W, H, k = 1920, 1080, 20
    grid = synth.reference_array(0.036 / W)
    cr, co = sva.Camera.make(*grid[12]), sva.Camera.make(*grid[0])
    ocr, oco = oracle.OCamera.make(*grid[12]), oracle.OCamera.make(*grid[0])
    a = synth.texture(H, W, 8)
    # camera 0 sees the scene shifted by +266..+533 px on both axes here:
    # only pixels with x, y small enough keep both endpoints in the image
    b = np.roll(np.roll(a, 400, axis=0), 400, axis=1)
    mask = np.zeros((H, W), np.uint8)
    mask[100:104, 300:500] = 1
    d8, d16, valid = ctx.disparity_ref(a, b, cr, co, k=k, mask=mask)
    o8, o16, ov, n = oracle.ref_pair(a, b, ocr, oco, k=k, mask=mask)
    assert n > 0 and ov.sum() > 0
    assert np.array_equal(valid, ov) and np.array_equal(d16, o16) and np.array_equal(d8, o8)


@pytest.mark.parametrize("pair", [(12, 6), (12, 13)])
def test_ref_path_full_frame_vga(ctx, sva, oracle, pair):
    """A whole 640x480 frame (the reference's own size class, k = 20) through
    the offset-plane kernel, bit-exact vs the oracle."""
    W, H, k = 640, 480, 20
    cr, co, ocr, oco = cams_for(sva, oracle, W, *pair)
    a = synth.texture(H, W, pair[1])
    gx, gy = pair[1] % 5 - 2, pair[1] // 5 - 2
    b = np.roll(np.roll(a, -60 * gy, axis=0), -60 * gx, axis=1)
    d8, d16, valid = ctx.disparity_ref(a, b, cr, co, k=k)
    o8, o16, ov, _ = oracle.ref_pair(a, b, ocr, oco, k=k)
    assert np.array_equal(valid, ov) and np.array_equal(d16, o16) and np.array_equal(d8, o8)


# VERDICT r01 "next" #2: the offset-plane kernel's tiling, LDS bitmap and
# per-tile fallback at the headline size.  32 full-width rows spread from top
# to bottom (so every 32-row tile band is entered at a different row) keep the
# CPU restatement to a few seconds; the oracle runs over row chunks in
# threads (ctypes drops the GIL; each call writes only its own masked pixels).
MODE_R_1080P_ROWS = np.linspace(20, 1080 - 21, 32).astype(int)


def _oracle_rows(oracle, a, b, ocr, oco, k, rows, W, H, chunks=16, workers=None):
    from concurrent.futures import ThreadPoolExecutor
    o8 = np.zeros((H, W), np.uint8)
    o16 = np.zeros((H, W), np.uint16)
    ov = np.zeros((H, W), np.uint8)

    def part(rs):
        m = np.zeros((H, W), np.uint8)
        m[rs, :] = 1
        oracle.ref_pair(a, b, ocr, oco, k=k, mask=m, disp_u8=o8, disp_u16=o16, valid=ov)

    with ThreadPoolExecutor(workers or chunks) as ex:
        list(ex.map(part, np.array_split(rows, chunks)))
    return o8, o16, ov


@pytest.mark.slow
@pytest.mark.parametrize("pair", [(12, 11), (12, 7), (12, 18), (12, 6)])
def test_ref_path_1080p_row_sampled(ctx, sva, oracle, pair):
    W, H, k = 1920, 1080, 20
    cr, co, ocr, oco = cams_for(sva, oracle, W, *pair)
    a = synth.texture(H, W, 40 + pair[1])
    # the other camera sees the scene shifted by ~178 px per grid unit
    # (0.05 m * 0.05 m / 0.75 m / (0.036 / 1920) m/px) along its baseline
    gx, gy = pair[1] % 5 - 2, pair[1] // 5 - 2
    b = np.roll(np.roll(a, -178 * gy, axis=0), -178 * gx, axis=1)
    mask = np.zeros((H, W), np.uint8)
    mask[MODE_R_1080P_ROWS, :] = 1
    d8, d16, valid = ctx.disparity_ref(a, b, cr, co, k=k, mask=mask)
    o8, o16, ov = _oracle_rows(oracle, a, b, ocr, oco, k, MODE_R_1080P_ROWS, W, H)
    assert ov.sum() > 0.3 * mask.sum()
    assert np.array_equal(valid, ov)
    assert np.array_equal(d16, o16)
    assert np.array_equal(d8, o8)


# VERDICT r02 "next" #1: a WHOLE 1080p frame at k = 20 for the reference rig's
# Low (12 -> 11) and High (12 -> 7) pairs -- every tile band, every tile edge,
# no mask -- against the oracle threaded over 64 row chunks (about 250 M
# candidate SADs, ~12 s on 16 host threads per pair).
@pytest.mark.slow
@pytest.mark.parametrize("pair", [(12, 11), (12, 7)])
def test_ref_path_1080p_full_frame(ctx, sva, oracle, pair):
    W, H, k = 1920, 1080, 20
    cr, co, ocr, oco = cams_for(sva, oracle, W, *pair)
    a = synth.texture(H, W, 80 + pair[1])
    gx, gy = pair[1] % 5 - 2, pair[1] // 5 - 2
    b = np.roll(np.roll(a, -178 * gy, axis=0), -178 * gx, axis=1)
    d8, d16, valid = ctx.disparity_ref(a, b, cr, co, k=k)
    rows = np.arange(k, H - k)
    o8, o16, ov = _oracle_rows(oracle, a, b, ocr, oco, k, rows, W, H, chunks=64, workers=16)
    assert ov.sum() > 0.5 * (H - 2 * k) * (W - 2 * k)
    assert np.array_equal(valid, ov)
    assert np.array_equal(d16, o16)
    assert np.array_equal(d8, o8)
    # the synthetic shift is the true disparity on most of the frame
    assert np.mean(d16[ov == 1] == 178) > 0.75


# 4K (BASELINE config 3's size): the v3 plane kernel stages O in chunks of
# outer offsets (diagonal pairs) and splits one outer offset's inner span into
# windows (High lines, 12 -> 7); 12 full-width rows per pair.
MODE_R_4K_ROWS = np.linspace(20, 2160 - 21, 12).astype(int)


@pytest.mark.slow
@pytest.mark.parametrize("pair", [(12, 11), (12, 7), (12, 6), (12, 18)])
def test_ref_path_4k_row_sampled(ctx, sva, oracle, pair):
    W, H, k = 3840, 2160, 20
    cr, co, ocr, oco = cams_for(sva, oracle, W, *pair)
    a = synth.texture(H, W, 60 + pair[1])
    gx, gy = pair[1] % 5 - 2, pair[1] // 5 - 2
    b = np.roll(np.roll(a, -356 * gy, axis=0), -356 * gx, axis=1)
    mask = np.zeros((H, W), np.uint8)
    mask[MODE_R_4K_ROWS, :] = 1
    d8, d16, valid = ctx.disparity_ref(a, b, cr, co, k=k, mask=mask)
    o8, o16, ov = _oracle_rows(oracle, a, b, ocr, oco, k, MODE_R_4K_ROWS, W, H, chunks=12)
    assert ov.sum() > 0.3 * mask.sum()
    assert np.array_equal(valid, ov)
    assert np.array_equal(d16, o16)
    assert np.array_equal(d8, o8)


# The split plane loop (refpath.hip: a tile's inner offsets over several
# workgroups, first-minimum keys meeting by atomicMin, ref_finalize_kernel):
# the host splits every tile over 3-6 shares; SVA_DEBUG_PLANE_SPLIT
# (sva_set_debug) forces a share count so that every size and the per-pixel
# fallback run through it too.  The switch is reset afterwards.
@pytest.fixture()
def plane_split(ctx, sva):
    def set_(n):
        ctx.set_debug(sva.SVA_DEBUG_PLANE_SPLIT, n)
    yield set_
    ctx.set_debug(sva.SVA_DEBUG_PLANE_SPLIT, 0)


@pytest.mark.parametrize("shares", [1, 2, 3, 7])
@pytest.mark.parametrize("pair", [(12, 11), (12, 7), (12, 6), (12, 18)])
def test_ref_path_split_shares_vga(ctx, sva, oracle, plane_split, shares, pair):
    W, H, k = 640, 480, 20
    plane_split(shares)
    cr, co, ocr, oco = cams_for(sva, oracle, W, *pair)
    a = synth.texture(H, W, 7 + pair[1])
    gx, gy = pair[1] % 5 - 2, pair[1] // 5 - 2
    b = np.roll(np.roll(a, -60 * gy, axis=0), -60 * gx, axis=1)
    # the maps start non-zero: pixels no share matches keep their value
    d8_0 = np.full((H, W), 201, np.uint8)
    d16_0 = np.full((H, W), 40000, np.uint16)
    v_0 = np.zeros((H, W), np.uint8)
    mask = np.ones((H, W), np.uint8)
    mask[200:260, 300:380] = 0
    d8, d16, valid = ctx.disparity_ref(a, b, cr, co, k=k, mask=mask, disp_u8=d8_0.copy(),
                                       disp_u16=d16_0.copy(), valid=v_0.copy())
    o8, o16, ov, _ = oracle.ref_pair(a, b, ocr, oco, k=k, mask=mask, disp_u8=d8_0.copy(),
                                     disp_u16=d16_0.copy(), valid=v_0.copy())
    assert ov.sum() > 0
    assert np.array_equal(valid, ov) and np.array_equal(d16, o16) and np.array_equal(d8, o8)


@pytest.mark.parametrize("shares", [2, 5])
def test_ref_path_split_fallback_diagonal_jump(ctx, sva, oracle, plane_split, shares):
    """The per-pixel fallback tiles of test_ref_path_plane_fallback_diagonal_jump
    through the split route: share 0 matches them and leaves keys too."""
    plane_split(shares)
    W, H, k = 1920, 1080, 20
    grid = synth.reference_array(0.036 / W)
    cr, co = sva.Camera.make(*grid[12]), sva.Camera.make(*grid[0])
    ocr, oco = oracle.OCamera.make(*grid[12]), oracle.OCamera.make(*grid[0])
    a = synth.texture(H, W, 8)
    b = np.roll(np.roll(a, 400, axis=0), 400, axis=1)
    mask = np.zeros((H, W), np.uint8)
    mask[100:104, 300:500] = 1
    d8, d16, valid = ctx.disparity_ref(a, b, cr, co, k=k, mask=mask)
    o8, o16, ov, n = oracle.ref_pair(a, b, ocr, oco, k=k, mask=mask)
    assert n > 0 and ov.sum() > 0
    assert np.array_equal(valid, ov) and np.array_equal(d16, o16) and np.array_equal(d8, o8)


@pytest.mark.slow
@pytest.mark.parametrize("pair", [(12, 11), (12, 6)])
def test_ref_path_split_1080p_row_sampled(ctx, sva, oracle, plane_split, pair):
    plane_split(3)
    test_ref_path_1080p_row_sampled(ctx, sva, oracle, pair)


# VERDICT r05 missing #3: the reference bounds neither k nor the frame
# (CameraStereoVision.cpp:44-51, :76-85).  k > 32 runs ref_pixel_kernel (one
# wave per pixel, 2k-byte rows in 64-byte chunks plus a tail); W or H >= 4096
# runs the WIDE plane kernel, whose first-minimum keys are u64 (SAD << 32 | i).
@pytest.mark.parametrize("k", [33, 34, 40, 64])
@pytest.mark.parametrize("pair", [(12, 11), (12, 7), (12, 18)])
def test_ref_path_k_above_32(ctx, sva, oracle, k, pair):
    W, H = 640, 480
    cr, co, ocr, oco = cams_for(sva, oracle, W, *pair)
    a = synth.texture(H, W, 40 + k)
    gx, gy = pair[1] % 5 - 2, pair[1] // 5 - 2
    b = np.roll(np.roll(a, -60 * gy, axis=0), -60 * gx, axis=1)
    mask = np.zeros((H, W), np.uint8)          # a band of rows keeps the oracle in seconds
    mask[H // 2 - 4: H // 2 + 4, :] = 1
    mask[k + 1, :] = 1                         # and the first rows the window allows
    mask[H - k - 2, ::7] = 1
    d8_0 = np.full((H, W), 201, np.uint8)
    d8, d16, valid = ctx.disparity_ref(a, b, cr, co, k=k, mask=mask, disp_u8=d8_0.copy())
    o8, o16, ov, n = oracle.ref_pair(a, b, ocr, oco, k=k, mask=mask, disp_u8=d8_0.copy())
    assert n > 0 and ov.sum() > 0
    assert np.array_equal(valid, ov) and np.array_equal(d16, o16) and np.array_equal(d8, o8)


@pytest.mark.parametrize("shares", [0, 1, 3])
def test_ref_path_wide_frame_4160(ctx, sva, oracle, plane_split, shares):
    """A 4160 x 96 frame (pair 12 -> 11, k = 20): past the u32 key's 4096
    columns, through the WIDE plane kernel unsplit (1), split (3) and with the
    automatic share count (0)."""
    plane_split(shares)
    W, H, k = 4160, 96, 20
    cr, co, ocr, oco = cams_for(sva, oracle, W, 12, 11)
    a = synth.texture(H, W, 17)
    b = np.roll(a, 300, axis=1)
    d8, d16, valid = ctx.disparity_ref(a, b, cr, co, k=k)
    o8, o16, ov, n = oracle.ref_pair(a, b, ocr, oco, k=k)
    assert n > 0 and ov.sum() > 1000
    assert np.array_equal(valid, ov) and np.array_equal(d16, o16) and np.array_equal(d8, o8)


@pytest.mark.parametrize("shares", [1, 3])
def test_ref_path_wide_keys_index_past_4095(ctx, sva, oracle, plane_split, shares):
    """Lines of more than 4096 candidates whose first minimum sits at index
    > 4095: a 4600 x 64 frame, pair 12 -> 11 with t_near = 0.0745, t_far = 2
    (pixels x <= 45 keep ~4,380-point lines) and the other image rolled by
    4,300 px, so the exact match is candidate ~4,126.  The u32 key's 12-bit
    index would alias it; the WIDE key must not."""
    plane_split(shares)
    W, H, k = 4600, 64, 4
    cr, co, ocr, oco = cams_for(sva, oracle, W, 12, 11)
    a = synth.texture(H, W, 23)
    b = np.roll(a, 4300, axis=1)
    d8, d16, valid = ctx.disparity_ref(a, b, cr, co, k=k, t_near=0.0745, t_far=2.0)
    o8, o16, ov, n = oracle.ref_pair(a, b, ocr, oco, k=k, t_near=0.0745, t_far=2.0)
    assert ov.sum() > 1000 and n > 4096 * int(ov.sum())
    assert (o16[ov > 0] == 4300).mean() > 0.3      # matched at index 4300 - 174 > 4095
    assert np.array_equal(valid, ov) and np.array_equal(d16, o16) and np.array_equal(d8, o8)


def test_ref_path_limits(ctx, sva):
    """What Mode R still refuses: k < 1, a window not inside the image
    (2k >= W or H, the reference's own loop bounds), W or H > 32767."""
    W, H = 64, 48
    a = np.zeros((H, W), np.uint8)
    cr = sva.Camera.make(0.05, (0.0, 0.0, 0.0), 0.036 / W)
    co = sva.Camera.make(0.05, (-0.05, 0.0, 0.0), 0.036 / W)
    for k, status in ((0, sva.SVA_ERR_INVALID_ARG), (24, sva.SVA_ERR_INVALID_ARG)):
        with pytest.raises(sva.SvaError) as e:
            ctx.disparity_ref(a, a, cr, co, k=k)
        assert e.value.status == status
    d8, _, v = ctx.disparity_ref(a, a, cr, co, k=23)        # 2k = 46 < 48: accepted
    assert d8.shape == (H, W)


@pytest.mark.parametrize("k", [4, 13, 32])
@pytest.mark.parametrize("pair", [(12, 11), (12, 6)])
def test_ref_path_unsplit_other_k(ctx, sva, oracle, plane_split, k, pair):
    """the unsplit plane loop (direct writes, no keys) at k other
    than 20, forced through SVA_DEBUG_PLANE_SPLIT = 1."""
    plane_split(1)
    test_ref_path_window_sizes(ctx, sva, oracle, k, pair)


def test_ref_path_keys_stay_clean_across_calls(ctx, sva, oracle):
    """ref_finalize_kernel puts every key back to all-ones, so only the first
    call (or a grown buffer) memsets the key buffer: a u32-key frame, a WIDE
    (u64-key) frame, a smaller frame and the first again on one context, each
    bit-exact."""
    runs = []
    for (W, H, seed) in ((640, 480, 3), (4160, 64, 4), (320, 240, 5), (640, 480, 3)):
        cr, co, ocr, oco = cams_for(sva, oracle, W, 12, 11)
        a = synth.texture(H, W, seed)
        b = np.roll(a, W // 20, axis=1)
        d8, d16, valid = ctx.disparity_ref(a, b, cr, co, k=8)
        o8, o16, ov, _ = oracle.ref_pair(a, b, ocr, oco, k=8)
        assert ov.sum() > 0
        assert np.array_equal(valid, ov) and np.array_equal(d16, o16) and np.array_equal(d8, o8)
        runs.append(d16)
    assert np.array_equal(runs[0], runs[3])
