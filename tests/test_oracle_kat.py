"""Known-answer tests that pin the CPU oracle (no GPU needed).

The reference ships no tests or golden vectors and cannot be built here
(OpenCV absent), so the oracle is "parity unpinned" with respect to the
reference binary.  These KATs are hand-derived from the reference source
(functions.cpp:253-321, Camera.cpp:15-34, CameraStereoVision.cpp:85-89) and
from the Mode S spec; each expected value below was traced by
hand, not produced by the code under test.
"""
import math

import numpy as np
import pytest

from stereovisionarray_amd import synth


# -------------------------------------------------------------- Bresenham --
# Hand traces of plotLineLow/plotLineHigh (functions.cpp:253-297) as selected
# by bresenham(point2, point1) (:299-321) called with (pixel1, pixel2).
BRESENHAM_KAT = [
    (((0, 0), (3, 1)), [(0, 0), (1, 0), (2, 1), (3, 1)]),
    (((3, 1), (0, 0)), [(0, 0), (1, 0), (2, 1), (3, 1)]),          # emitted from lower x
    (((5, 5), (4, 9)), [(5, 5), (5, 6), (5, 7), (4, 8), (4, 9)]),  # High, xi = -1
    (((4, 9), (5, 5)), [(5, 5), (5, 6), (5, 7), (4, 8), (4, 9)]),  # emitted from lower y
    (((0, 0), (2, 2)), [(0, 0), (1, 1), (2, 2)]),                  # |dx| == |dy| -> High
    (((4, 4), (4, 4)), [(4, 4)]),                                  # single point
    (((0, 2), (4, 0)), [(0, 2), (1, 2), (2, 1), (3, 1), (4, 0)]),  # Low, yi = -1
    (((10, 10), (20, 13)), [(10, 10), (11, 10), (12, 11), (13, 11), (14, 11), (15, 11),
                            (16, 12), (17, 12), (18, 12), (19, 13), (20, 13)]),
]


@pytest.mark.parametrize("args,expected", BRESENHAM_KAT)
def test_bresenham_kat(oracle, args, expected):
    assert oracle.bresenham(*args) == expected


def test_bresenham_closed_form(oracle):
    """The GPU kernel enumerates candidate i in O(1):
    Low: (x0+i, y0 + yi*floor((2|dy|i + dx - 1)/(2dx))), High transposed.
    Check that formula against the oracle's iterative trace on many lines."""
    rng = np.random.RandomState(0)
    for _ in range(3000):
        p1 = tuple(int(v) for v in rng.randint(-40, 40, 2))
        p2 = tuple(int(v) for v in rng.randint(-40, 40, 2))
        pts = oracle.bresenham(p1, p2)
        (ax, ay), (bx, by) = p1, p2
        if abs(ay - by) < abs(ax - bx):
            x0, y0, x1, y1 = (ax, ay, bx, by) if bx > ax else (bx, by, ax, ay)
            dx, dy = x1 - x0, abs(y1 - y0)
            s = -1 if y1 < y0 else 1
            exp = [(x0 + i, y0 + s * ((2 * dy * i + dx - 1) // (2 * dx))) for i in range(dx + 1)]
        else:
            x0, y0, x1, y1 = (ax, ay, bx, by) if by > ay else (bx, by, ax, ay)
            dy, dx = y1 - y0, abs(x1 - x0)
            s = -1 if x1 < x0 else 1
            if dy == 0:
                exp = [(x0, y0)]
            else:
                exp = [(x0 + s * ((2 * dx * i + dy - 1) // (2 * dy)), y0 + i) for i in range(dy + 1)]
        assert pts == exp, (p1, p2)


# ----------------------------------------------------------------- Camera --
def test_project_truncates_toward_zero(oracle):
    # f = 0.05, pixel 0.036/640: mult = 0.05/(0.25+0.75)/5.625e-5 = 888.88..
    cam = oracle.OCamera.make(0.05, (0.0, 0.0, -0.75), 0.036 / 640)
    assert oracle.project(cam, (0.01, -0.02, 0.25)) == (8, -17)   # 8.88 -> 8, -17.77 -> -17


def test_inv_project_3_4_12(oracle):
    cam = oracle.OCamera.make(12.0, (0.0, 0.0, 0.0), 1.0)
    assert oracle.inv_project(cam, 3, 4) == (3 / 13, 4 / 13, 12 / 13)


def test_endpoints_second_restatement(oracle):
    """Independent Python restatement of CameraStereoVision.cpp:28,60-71 and
    Camera.cpp:15-33 (IEEE doubles, same operand order) vs the C oracle."""
    W, H, k = 640, 480, 20
    ps = 0.036 / W
    grid = synth.reference_array(ps)
    for (ir, io) in [(12, 11), (12, 7), (12, 18), (12, 6)]:
        f, pr, _ = grid[ir]
        _, po, _ = grid[io]
        cref = oracle.OCamera.make(*grid[ir])
        coth = oracle.OCamera.make(*grid[io])
        hx, hy = W // 2, H // 2
        for y in range(k, H - k, 37):
            for x in range(k, W - k, 29):
                v = ((x - hx) * ps, (y - hy) * ps, f)
                n = math.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])
                e = (v[0] / n, v[1] / n, v[2] / n)
                out = []
                for t in (0.5, 1.0):
                    P = [pr[i] + e[i] * t for i in range(3)]
                    mult = f / (P[2] - po[2]) / ps
                    out.append((int((P[0] - po[0]) * mult) + hx, int((P[1] - po[1]) * mult) + hy))
                ok = all(not (p[0] < k or p[1] < k or p[0] > W - k or p[1] > H - k) for p in out)
                got = oracle.ref_endpoints(cref, coth, W, H, k, 0.5, 1.0, x, y)
                assert got == (ok, out[0], out[1]), (ir, io, x, y)


def test_reference_geometry_candidate_counts(oracle):
    """with the reference rig, pair 12/11 at 640 px wide has
    45-49 candidates per pixel."""
    W, H, k = 640, 480, 20
    grid = synth.reference_array(0.036 / W)
    cref, coth = oracle.OCamera.make(*grid[12]), oracle.OCamera.make(*grid[11])
    counts = []
    for y in range(k, H - k, 23):
        for x in range(k, W - k, 19):
            ok, a, b = oracle.ref_endpoints(cref, coth, W, H, k, 0.5, 1.0, x, y)
            if ok:
                counts.append(len(oracle.bresenham(a, b)))
    assert min(counts) >= 45 and max(counts) <= 49


# -------------------------------------------------------------------- SAD --
def test_sad_kat(oracle):
    a = np.array([[0, 255], [10, 20]], np.uint8)
    b = np.array([[255, 0], [20, 10]], np.uint8)
    assert oracle.lib.svo_sad(a.ctypes.data, 2, b.ctypes.data, 2, 2, 2) == 530


def test_ref_pair_constant_images_pick_first_candidate(oracle):
    """All SADs 0 -> std::min_element returns index 0, the first emitted point
    (lowest x for a Low line) -> disparity = |first - (x,y)| truncated."""
    W, H, k = 160, 120, 6
    grid = synth.reference_array(0.036 / W)
    cref, coth = oracle.OCamera.make(*grid[12]), oracle.OCamera.make(*grid[11])
    img = np.full((H, W), 90, np.uint8)
    d8, d16, valid, _ = oracle.ref_pair(img, img, cref, coth, k=k)
    for y, x in [(40, 40), (60, 80), (100, 120)]:
        ok, a, b = oracle.ref_endpoints(cref, coth, W, H, k, 0.5, 1.0, x, y)
        assert valid[y, x] == ok
        if ok:
            first = oracle.bresenham(a, b)[0]
            assert d16[y, x] == int(math.sqrt((first[0] - x) ** 2 + (first[1] - y) ** 2))


def test_depth_kat(oracle):
    d = np.array([0, 1, 2, 255], np.uint8)
    out = oracle.disp_to_depth(d, 0.05, 0.05, 0.036 / 640)
    num = 0.05 * 0.05
    assert out[0] == 0.0
    assert out[1] == num / (1.0 * (0.036 / 640))
    assert out[3] == num / (255.0 * (0.036 / 640))


# ----------------------------------------------------------------- Census --
def _census_window_image(center=100, fill=150):
    img = np.full((7, 9), fill, np.uint8)
    img[3, 4] = center
    return img


def test_census_kat(oracle):
    img = _census_window_image()
    assert int(oracle.census(img)[3, 4]) == 0                 # nothing darker
    img[0, 0] = 50                                            # first window element
    assert int(oracle.census(img)[3, 4]) == 1 << 61
    img = _census_window_image()
    img[6, 8] = 50                                            # last window element
    assert int(oracle.census(img)[3, 4]) == 1
    img = _census_window_image()
    img[3, 3] = 50                                            # just left of centre: e = 3*8+3 = 30
    assert int(oracle.census(img)[3, 4]) == 1 << (61 - 30)
    img = _census_window_image(center=100, fill=100)          # equal is not '<'
    assert int(oracle.census(img)[3, 4]) == 0
    c = oracle.census(_census_window_image())
    assert (c[np.arange(7) != 3].sum() == 0) and c[3, :4].sum() == 0  # borders are 0


def test_cost_kat(oracle):
    cl = np.array([[0b1011, 0, 0b1111]], np.uint64)
    cr = np.array([[0b0001, 0b0110, 0]], np.uint64)
    C = oracle.cost(cl, cr, D=2, dmin=0, dir=1)
    # x=0: d0 pop(1011^0001)=2, d1 pop(1011^0110)=3; x=1: pop(0^0110)=2, pop(0^0)=0;
    # x=2: d0 pop(1111^0)=4, d1 -> column 3 outside -> 62
    assert C[0].tolist() == [[2, 3], [2, 0], [4, 62]]
    C = oracle.cost(cl, cr, D=2, dmin=1, dir=-1)
    # x=0: col -1,-2 outside; x=1: d0 col 0 -> pop(0^1)=1, d1 col -1 -> 62; x=2: col 1 -> pop(1111^0110)=2, col 0 -> pop(1111^0001)=3
    assert C[0].tolist() == [[62, 62], [1, 62], [2, 3]]


# -------------------------------------------------------------------- SGM --
C1D = np.array([[[0, 5, 9], [3, 3, 3], [9, 0, 9], [1, 1, 1]]], np.uint8)  # H=1, W=4, D=3


def test_path_1d_hand_expanded(oracle):
    """P1=2, P2=6 recurrence expanded by hand."""
    L0 = oracle.path(C1D, 0, P1=2, P2=6)   # left -> right
    assert L0[0].tolist() == [[0, 5, 9], [3, 5, 9], [9, 2, 13], [3, 1, 3]]
    L1 = oracle.path(C1D, 1, P1=2, P2=6)   # right -> left
    assert L1[0].tolist() == [[2, 5, 11], [5, 3, 5], [9, 0, 9], [1, 1, 1]]
    for r in range(2, 8):                  # H = 1: every pixel starts a path
        assert np.array_equal(oracle.path(C1D, r, P1=2, P2=6), C1D)
    S = oracle.aggregate(C1D, P1=2, P2=6)
    assert np.array_equal(S, L0.astype(np.uint16) + L1 + 6 * C1D.astype(np.uint16))


def test_path_bounds(oracle):
    rng = np.random.RandomState(1)
    C = rng.randint(0, 63, size=(9, 11, 16)).astype(np.uint8)
    for r in range(8):
        L = oracle.path(C, r).astype(int)
        assert (L >= C).all() and (L <= C.astype(int) + 120).all()
        assert (L.min(axis=2) <= C.astype(int).max(axis=2)).all()


def test_wta_kat(oracle):
    S = np.array([[[5, 3, 3, 7]]], np.uint16)
    d, s = oracle.wta(S, dmin=10)
    assert d[0, 0] == 11                 # first of the tied minima
    assert s[0, 0] == np.float32(11.5)   # a=5 b=3 c=3: (5-3)/(2*2)
    S = np.array([[[1, 3, 3, 7]]], np.uint16)
    d, s = oracle.wta(S, dmin=0)
    assert d[0, 0] == 0 and s[0, 0] == 0.0   # edge: no parabola


def test_sgm_shifted_texture(oracle):
    W, H, D, d0 = 160, 48, 32, 9
    L = synth.texture(H, W, 4)
    R = np.zeros_like(L)
    R[:, : W - d0] = L[:, d0:]
    d, _ = oracle.sgm(L, R, D, 0, -1, subpixel=False)
    assert (d[6:-6, d0 + 24: W - 24] == d0).all()


def test_sgm_threads_identical(oracle):
    L, R, _ = synth.stereo_pair(40, 90, 64, 0, -1, seed=2)
    a, sa = oracle.sgm(L, R, 64, threads=1)
    b, sb = oracle.sgm(L, R, 64, threads=4)
    assert np.array_equal(a, b) and np.array_equal(sa, sb)


def test_lr_check_kat(oracle):
    dl = np.array([[0, 2, 2, 1]], np.uint16)
    dr = np.array([[0, 3, 2, 9]], np.uint16)
    out = oracle.lr_check(dl, dr, dir=-1, max_diff=0, invalid=0xFFFF)
    # x=0: xr=0 dr=0 ok; x=1: xr=-1 outside; x=2: xr=0, dr=0 vs 2 -> reject; x=3: xr=2 dr=2 vs 1 -> reject
    assert out[0].tolist() == [0, 0xFFFF, 0xFFFF, 0xFFFF]
    out = oracle.lr_check(dl, dr, dir=-1, max_diff=2, invalid=0xFFFF)
    assert out[0].tolist() == [0, 0xFFFF, 2, 1]


def test_lr_sub_kat(oracle):
    """the f32 map is NaN exactly where the checked disparity
    is `invalid`."""
    d = np.array([[5, 0xFFFF, 7, 0xFFFF]], np.uint16)
    s = np.array([[5.25, 3.5, 6.75, 1.0]], np.float32)
    out = oracle.lr_sub(d, s, 0xFFFF)
    assert np.isnan(out[0, 1]) and np.isnan(out[0, 3])
    assert out[0, 0] == 5.25 and out[0, 2] == 6.75
    assert s[0, 1] == 3.5          # input untouched


def test_cost2_kat(oracle):
    """2-D step: hand-placed census words."""
    cl = np.zeros((4, 3), np.uint64)
    cr = np.zeros((4, 3), np.uint64)
    cl[1, 1] = 0b1011
    cr[1, 1], cr[2, 1], cr[3, 2], cr[0, 1] = 0b0001, 0b1000, 0b1011, 0b1111
    C = oracle.cost2(cl, cr, D=3, dmin=0, sx=0, sy=1)     # (1,1) -> (1,1),(1,2),(1,3)
    assert C[1, 1].tolist() == [2, 2, 3]
    C = oracle.cost2(cl, cr, D=3, dmin=0, sx=1, sy=1)     # (1,1),(2,2),(3,3)->outside
    assert C[1, 1].tolist() == [2, 3, 62]
    C = oracle.cost2(cl, cr, D=3, dmin=1, sx=0, sy=-1)    # (1,0), then outside
    assert C[1, 1].tolist() == [1, 62, 62]
    # sy = 0 is exactly the 1-D cost
    rng = np.random.default_rng(0)
    a = rng.integers(0, 1 << 62, size=(5, 40), dtype=np.int64).astype(np.uint64)
    b = rng.integers(0, 1 << 62, size=(5, 40), dtype=np.int64).astype(np.uint64)
    for dr in (-1, 1):
        assert np.array_equal(oracle.cost2(a, b, 16, 2, dr, 0), oracle.cost(a, b, 16, 2, dr))


def test_lr_check2_kat(oracle):
    dl = np.array([[0], [1], [1], [2]], np.uint16)
    dr = np.array([[5], [0], [1], [9]], np.uint16)
    # sy=-1: (x, y) -> (x, y - d); y=1 d=1 -> dr[0]=5 reject; y=2 d=1 -> dr[1]=0 ok (|1-0|<=1)
    # y=3 d=2 -> dr[1]=0 reject (2 > 1); y=0 d=0 -> dr[0]=5 reject
    out = oracle.lr_check2(dl, dr, 0, -1, 1, 0xFFFF)
    assert out[:, 0].tolist() == [0xFFFF, 0xFFFF, 1, 0xFFFF]
    out = oracle.lr_check2(dl, dr, 0, 1, 1, 0xFFFF)       # y=3 d=2 -> row 5: outside
    assert out[3, 0] == 0xFFFF


def test_fuse_depth_kat(oracle):
    """DESIGN.md §2.6 by hand: b*f/(d*ps), median, mean of the middle two."""
    f, ps = 0.05, 1e-4
    d = np.array([[[10, 0xFFFF]], [[20, 5]], [[0, 0]]], np.uint16)    # 3 maps, 1x2
    z, n = oracle.fuse_depth(d, [0.05, 0.05, 0.1], f, ps)
    # pixel 0: 2.5 and 1.25 (map 2 has d=0: skipped) -> mean 1.875
    # pixel 1: map 1 only -> 0.0025 / 5e-4 = 5
    assert z[0].tolist() == pytest.approx([1.875, 5.0], rel=1e-14) and n[0].tolist() == [2, 1]
    d = np.array([[[4]], [[8]], [[2]], [[0xFFFF]]], np.uint16)
    z, n = oracle.fuse_depth(d, [0.1, 0.1, 0.1, 0.1], 1.0, 1.0)     # 0.025, 0.0125, 0.05
    assert z[0, 0] == pytest.approx(0.025, rel=1e-14) and n[0, 0] == 3
    z, n = oracle.fuse_depth(np.full((2, 1, 1), 0xFFFF, np.uint16), [1, 1], 1.0, 1.0)
    assert z[0, 0] == 0.0 and n[0, 0] == 0


def test_step_offset_kat(oracle):
    """DESIGN.md §2.2 offsets by hand; and the synth restatement agrees."""
    assert [oracle.step_offset(s, 2, 1) for s in range(6)] == \
        [(0, 0), (1, 1), (2, 1), (3, 2), (4, 2), (5, 3)]       # round(s/2), half up
    assert [oracle.step_offset(s, -1, 3) for s in range(5)] == \
        [(0, 0), (0, 1), (-1, 2), (-1, 3), (-1, 4)]            # round(s/3)
    assert oracle.step_offset(7, 0, -1) == (0, -7)
    assert oracle.step_offset(7, -1, -1) == (-7, -7)
    assert oracle.step_offset(7, 5, 0) == (7, 0)
    for bx, by in [(2, 1), (-3, -2), (1, -4), (0, 2), (7, 7)]:
        for s in range(0, 300, 7):
            assert oracle.step_offset(s, bx, by) == tuple(int(v) for v in synth.step_offset(s, bx, by))


# ---- refinement / 3-D, hand-derived ---------------------

def _cam(oracle, f, pos, ps):
    return oracle.OCamera.make(f, pos, ps)


def test_shift_perspective_kat(oracle):
    """functions.cpp:55-77: pre = (in - out) / |in - out|; gather at
    ((int)(d*preX + x), (int)(d*preY + y)); d == 0 and out-of-range keep init."""
    c12 = _cam(oracle, 0.05, (0, 0, -0.75), 1e-4)
    c11 = _cam(oracle, 0.05, (-0.05, 0, -0.75), 1e-4)
    d = np.array([[0, 2, 1, 5]], np.uint8)
    img = np.array([[10, 20, 30, 40]], np.uint8)
    out = oracle.shift_perspective(c12, c11, d, img, init=np.full((1, 4), 7, np.uint8))
    assert out[0].tolist() == [7, 40, 40, 7]     # x=3: 3+5 outside -> untouched
    c6 = _cam(oracle, 0.05, (-0.05, -0.05, -0.75), 1e-4)   # diagonal: pre = (1/sqrt2, 1/sqrt2)
    d = np.zeros((4, 4), np.uint8); d[0, 0] = 3            # 3/sqrt2 = 2.12 -> (2, 2)
    img = np.arange(16, dtype=np.uint8).reshape(4, 4)
    assert oracle.shift_perspective(c12, c6, d, img)[0, 0] == img[2, 2]


def test_improve_with_disparity_kat(oracle):
    """functions.cpp:11-52 by construction: with disp = d0 and the paired image
    img(x) = centre(x - d0 - 2), the shifted image is centre(x - 2), so
    candidate p = 7 matches exactly and the refined disparity is d0 + 2."""
    W, H, d0 = 64, 24, 6
    center = synth.texture(H, W, 3)
    img = np.zeros_like(center)
    img[:, d0 + 2:] = center[:, : W - d0 - 2]
    c0 = _cam(oracle, 0.05, (0.05, 0, -0.75), 1e-4)   # c0 - c1 = (+0.05, 0): ddx = 1, pre = (1, 0)
    c1 = _cam(oracle, 0.05, (0.0, 0, -0.75), 1e-4)
    disp = np.full((H, W), d0, np.uint8)
    mask = np.zeros((H, W), np.uint8)
    mask[6:18, 20:40] = 1
    st, out = oracle.improve_with_disparity(disp, center, [img], [(c0, c1)], window=7, mask=mask)
    assert st == 0
    assert (out[6:18, 20:40] == d0 + 2).all() and (out[mask == 0] == 0).all()
    # disp = 0: nothing shifts (shifted stays 0), all 11 SADs tie -> first
    # candidate p = 0 -> 0 + (0 - 5) * 1 = -5 -> (uchar)(int) wraps to 251
    st, out = oracle.improve_with_disparity(np.zeros((H, W), np.uint8), center, [img],
                                            [(c0, c1)], window=7, mask=mask)
    assert (out[6:18, 20:40] == 251).all()
    # other camera at +x (c0 - c1 < 0): direction (0, 0) -> disparity unchanged
    st, out = oracle.improve_with_disparity(disp, center, [img], [(c1, c0)], window=7, mask=mask)
    assert (out[6:18, 20:40] == d0).all()
    # strict: a masked pixel whose window leaves the image fails like the ROI throw
    m2 = mask.copy(); m2[0, 0] = 1
    st, _ = oracle.improve_with_disparity(disp, center, [img], [(c0, c1)], window=7, mask=m2,
                                          strict=True)
    assert st == -1


def test_shift_perspective2_kat(oracle):
    """functions.cpp:79-103: preX = 0.05*0.05/1e-3 = 2.5 (to f64 rounding);
    depth 1 at x=0 -> +int(2.5) = 2; depth 2 at x=1 -> +int(1.25) = 1: both
    land on x=2, the later x (loop order) wins; depth < 0.5 skipped."""
    cin = _cam(oracle, 0.05, (0.05, 0, 0), 1e-3)
    cout = _cam(oracle, 0.05, (0.0, 0, 0), 1e-3)
    depth = np.array([[1.0, 2.0, 0.4, 0.0, 0.0]], np.float64)
    out = oracle.shift_perspective2(cin, cout, depth)
    assert out[0].tolist() == [0.0, 0.0, 2.0, 0.0, 0.0]


def test_points_depth_kat(oracle):
    """functions.cpp:118-146 with f = ps = 1 at the origin, 4x4 (half = 2)."""
    cam = _cam(oracle, 1.0, (0, 0, 0), 1.0)
    pts = np.array([[1, 1, 2], [-1.9, 0, 1], [0, 0, 5], [0.4, 0, 2], [0, 0, 0]], np.float64)
    d = oracle.points_to_depth(pts, cam, 4, 4)
    # (1,1,2): mult .5 -> (0,0)+2 = (2,2) z=2; (-1.9,0,1): (int)-1.9 = -1 -> (1,2);
    # (0,0,5) -> (2,2) z=5; (0.4,0,2): (int)0.2 = 0 -> (2,2) z=2 (last wins);
    # (0,0,0): z - cz = 0 -> mult inf -> 0*inf = NaN -> skipped
    assert d[2, 2] == 2.0 and d[2, 1] == 1.0 and np.count_nonzero(d) == 2
    depth = np.array([[0.0, 1.0], [0.05, 2.0]])
    p = oracle.depth_to_points(depth, cam)          # column-major: u=1 v=0, then u=1 v=1
    r = 1 / np.sqrt(2.0)
    assert p.shape == (2, 3)
    assert np.allclose(p[0], [0, -r, r], atol=0, rtol=1e-15) and p[1].tolist() == [0, 0, 2]


def test_resize_half_kat(oracle):
    """CameraStereoVision.cpp:18 (OpenCV exact-2x area path): full blocks
    (sum+2)>>2; partial edge blocks cvRound(sum/count), half to even; output
    (cvRound(W/2), cvRound(H/2))."""
    a = np.array([[1, 2, 3, 4, 5], [5, 6, 7, 8, 9], [10, 11, 12, 13, 14]], np.uint8)
    # W=5 -> cvRound(2.5) = 2, H=3 -> cvRound(1.5) = 2: the last row is partial
    # (10+11)/2 = 10.5 -> 10 (even), (12+13)/2 = 12.5 -> 12
    assert oracle.resize_half(a).tolist() == [[4, 6], [10, 12]]
    b = np.array([[0, 1, 2], [3, 4, 6]], np.uint8)   # W=3 -> 2 columns, last partial
    # (0+1+3+4+2)>>2 = 2; (2+6)/2 = 4
    assert oracle.resize_half(b).tolist() == [[2, 4]]
    c = np.array([[1, 2, 3, 4, 5, 6, 7]], np.uint8)   # H=1 -> cvRound(0.5) = 0 rows
    assert oracle.resize_half(c).shape == (0, 4)
    d = np.array([[255, 254], [255, 254]], np.uint8)  # (1018+2)>>2 = 255 (no overflow)
    assert oracle.resize_half(d).tolist() == [[255]]


def test_mode_r_planes_line_offsets(oracle):
    """tools/mode_r_planes.py (the bench's sad_planes_per_candidate report)
    forms each pixel's candidate offsets with the kernel's closed form; they
    must be the oracle's Bresenham points relative to the pixel, in order."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "mode_r_planes", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                      "tools", "mode_r_planes.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    rng = np.random.RandomState(5)
    for _ in range(2000):
        x, y = (int(v) for v in rng.randint(0, 100, 2))
        a = tuple(int(v) for v in rng.randint(-60, 160, 2))
        b = tuple(int(v) for v in rng.randint(-60, 160, 2))
        want = [(px - x, py - y) for px, py in oracle.bresenham(a, b)]
        assert m.line_offsets(x, y, a, b) == want, (x, y, a, b)
