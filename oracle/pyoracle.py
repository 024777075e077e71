"""ctypes binding of liboracle.so -- the CPU ORACLE (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker or the timed CPU baseline.  Parity status:
"parity unpinned" (see sva_oracle.h and DESIGN.md §5).
"""
from __future__ import annotations

import ctypes as ct
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


class OCamera(ct.Structure):
    _fields_ = [("f", ct.c_double), ("pos", ct.c_double * 3), ("pixel_size", ct.c_double)]

    @classmethod
    def make(cls, f, pos, pixel_size):
        c = cls()
        c.f = f
        c.pos[0], c.pos[1], c.pos[2] = pos
        c.pixel_size = pixel_size
        return c


def _load():
    if not os.path.exists(LIB_PATH):
        build()
    lib = ct.CDLL(LIB_PATH)
    vp, i32, dbl, P = ct.c_void_p, ct.c_int, ct.c_double, ct.POINTER
    sig = {
        "svo_cam_project": (None, [P(OCamera), P(dbl), P(i32)]),
        "svo_cam_inv_project": (None, [P(OCamera), i32, i32, P(dbl)]),
        "svo_bresenham": (i32, [i32, i32, i32, i32, P(i32), P(i32), i32]),
        "svo_sad": (ct.c_int64, [vp, ct.c_ssize_t, vp, ct.c_ssize_t, i32, i32]),
        "svo_ref_endpoints": (i32, [P(OCamera), P(OCamera), i32, i32, i32, dbl, dbl, i32, i32,
                                    P(i32), P(i32)]),
        "svo_ref_pair": (ct.c_int64, [vp, vp, i32, i32, ct.c_ssize_t, vp, P(OCamera), P(OCamera),
                                      i32, dbl, dbl, vp, vp, vp]),
        "svo_disp_to_depth": (None, [vp, i32, dbl, dbl, dbl, vp]),
        "svo_census": (None, [vp, i32, i32, ct.c_ssize_t, vp]),
        "svo_cost": (None, [vp, vp, i32, i32, i32, i32, i32, vp]),
        "svo_cost2": (None, [vp, vp, i32, i32, i32, i32, i32, i32, vp]),
        "svo_lr_check2": (None, [vp, vp, i32, i32, i32, i32, i32, ct.c_uint16]),
        "svo_fuse_depth": (None, [vp, i32, i32, i32, vp, dbl, dbl, ct.c_uint16, vp, vp]),
        "svo_path": (None, [vp, i32, i32, i32, i32, i32, i32, i32, vp]),
        "svo_direction": (None, [i32, P(i32), P(i32)]),
        "svo_aggregate": (None, [vp, i32, i32, i32, i32, i32, vp, i32]),
        "svo_wta": (None, [vp, i32, i32, i32, i32, vp, vp]),
        "svo_sgm": (None, [vp, vp, i32, i32, ct.c_ssize_t, i32, i32, i32, i32, i32, vp, vp, i32]),
        "svo_lr_check": (None, [vp, vp, i32, i32, i32, i32, ct.c_uint16]),
        "svo_sgm2": (None, [vp, vp, i32, i32, ct.c_ssize_t, i32, i32, i32, i32, i32, i32, vp, vp,
                            i32]),
        "svo_lr_sub": (None, [vp, vp, ct.c_size_t, ct.c_uint16]),
        "svo_step_offset": (None, [i32, i32, i32, P(i32), P(i32)]),
        "svo_shift_perspective": (None, [P(OCamera), P(OCamera), vp, vp, i32, i32,
                                         ct.c_ssize_t, vp]),
        "svo_improve_with_disparity": (i32, [vp, vp, P(vp), P(OCamera), i32, i32, i32,
                                             ct.c_ssize_t, vp, i32, i32, vp]),
        "svo_shift_perspective2": (None, [P(OCamera), P(OCamera), vp, i32, i32, vp]),
        "svo_points_to_depth": (None, [vp, ct.c_int64, P(OCamera), i32, i32, vp]),
        "svo_depth_to_points": (ct.c_int64, [vp, i32, i32, P(OCamera), vp]),
        "svo_resize_half_size": (None, [i32, i32, P(i32), P(i32)]),
        "svo_resize_half": (None, [vp, i32, i32, ct.c_ssize_t, vp, ct.c_ssize_t]),
        "svo_resize_linear_f64": (None, [vp, i32, i32, vp, i32, i32]),
        "svo_ref_error": (None, [vp, i32, i32, vp, i32, i32, ct.c_double, vp]),
        "svo_masked_mean": (ct.c_double, [vp, vp, i32, i32]),
    }
    for n, (r, a) in sig.items():
        f = getattr(lib, n)
        f.restype = r
        f.argtypes = a
    return lib


lib = _load()


def _p(a):
    return None if a is None else a.ctypes.data


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


# ------------------------------------------------------------------ Mode R --
def project(cam: OCamera, P):
    out = (ct.c_int * 2)()
    lib.svo_cam_project(ct.byref(cam), (ct.c_double * 3)(*P), out)
    return out[0], out[1]


def inv_project(cam: OCamera, px: int, py: int):
    out = (ct.c_double * 3)()
    lib.svo_cam_inv_project(ct.byref(cam), px, py, out)
    return out[0], out[1], out[2]


def bresenham(p1, p2):
    cap = 4 * (abs(p1[0] - p2[0]) + abs(p1[1] - p2[1])) + 8
    xs = (ct.c_int * cap)()
    ys = (ct.c_int * cap)()
    n = lib.svo_bresenham(p1[0], p1[1], p2[0], p2[1], xs, ys, cap)
    return [(xs[i], ys[i]) for i in range(n)]


def ref_endpoints(cref, coth, W, H, k, t_near, t_far, x, y):
    a = (ct.c_int * 2)()
    b = (ct.c_int * 2)()
    ok = lib.svo_ref_endpoints(ct.byref(cref), ct.byref(coth), W, H, k, t_near, t_far, x, y, a, b)
    return bool(ok), (a[0], a[1]), (b[0], b[1])


def ref_pair(ref, other, cref, coth, k=20, t_near=0.5, t_far=1.0, mask=None,
             disp_u8=None, disp_u16=None, valid=None):
    ref = _c(ref, np.uint8)
    other = _c(other, np.uint8)
    H, W = ref.shape
    disp_u8 = np.zeros((H, W), np.uint8) if disp_u8 is None else disp_u8
    disp_u16 = np.zeros((H, W), np.uint16) if disp_u16 is None else disp_u16
    valid = np.zeros((H, W), np.uint8) if valid is None else valid
    m = None if mask is None else _c(mask, np.uint8)
    n = lib.svo_ref_pair(_p(ref), _p(other), W, H, W, _p(m), ct.byref(cref), ct.byref(coth), k,
                         t_near, t_far, _p(disp_u8), _p(disp_u16), _p(valid))
    return disp_u8, disp_u16, valid, n


def disp_to_depth(disp, cam_distance, f, pixel_size):
    d = _c(disp, np.uint8)
    out = np.zeros(d.shape, np.float64)
    lib.svo_disp_to_depth(_p(d), d.size, cam_distance, f, pixel_size, _p(out))
    return out


# ------------------------------------------------------------------ Mode S --
def census(img):
    img = _c(img, np.uint8)
    H, W = img.shape
    out = np.zeros((H, W), np.uint64)
    lib.svo_census(_p(img), W, H, W, _p(out))
    return out


def cost(cl, cr, D, dmin, dir):
    cl = _c(cl, np.uint64)
    cr = _c(cr, np.uint64)
    H, W = cl.shape
    C = np.zeros((H, W, D), np.uint8)
    lib.svo_cost(_p(cl), _p(cr), W, H, D, dmin, dir, _p(C))
    return C


def direction(r):
    rx, ry = ct.c_int(), ct.c_int()
    lib.svo_direction(r, ct.byref(rx), ct.byref(ry))
    return rx.value, ry.value


def path(C, r, P1=10, P2=120):
    C = _c(C, np.uint8)
    H, W, D = C.shape
    rx, ry = direction(r)
    L = np.zeros_like(C)
    lib.svo_path(_p(C), W, H, D, rx, ry, P1, P2, _p(L))
    return L


def aggregate(C, P1=10, P2=120, threads=1):
    C = _c(C, np.uint8)
    H, W, D = C.shape
    S = np.zeros((H, W, D), np.uint16)
    lib.svo_aggregate(_p(C), W, H, D, P1, P2, _p(S), threads)
    return S


def wta(S, dmin=0, subpixel=True):
    S = _c(S, np.uint16)
    H, W, D = S.shape
    disp = np.zeros((H, W), np.uint16)
    sub = np.zeros((H, W), np.float32) if subpixel else None
    lib.svo_wta(_p(S), W, H, D, dmin, _p(disp), _p(sub))
    return disp, sub


def sgm(left, right, D, dmin=0, dir=-1, P1=10, P2=120, subpixel=True, threads=1):
    left = _c(left, np.uint8)
    right = _c(right, np.uint8)
    H, W = left.shape
    disp = np.zeros((H, W), np.uint16)
    sub = np.zeros((H, W), np.float32) if subpixel else None
    lib.svo_sgm(_p(left), _p(right), W, H, W, D, dmin, dir, P1, P2, _p(disp), _p(sub), threads)
    return disp, sub


def lr_check(disp_l, disp_r, dir, max_diff=1, invalid=0xFFFF):
    dl = _c(disp_l, np.uint16).copy()
    dr = _c(disp_r, np.uint16)
    H, W = dl.shape
    lib.svo_lr_check(_p(dl), _p(dr), W, H, dir, max_diff, invalid)
    return dl


def lr_sub(disp, sub, invalid=0xFFFF):
    """the f32 map is NaN wherever the checked disparity is
    `invalid`."""
    d = _c(disp, np.uint16)
    out = _c(sub, np.float32).copy()
    lib.svo_lr_sub(_p(d), _p(out), d.size, invalid)
    return out


def step_offset(s, bx, by):
    ox, oy = ct.c_int(0), ct.c_int(0)
    lib.svo_step_offset(s, bx, by, ct.byref(ox), ct.byref(oy))
    return ox.value, oy.value


def cost2(cl, cr, D, dmin, sx, sy):
    cl = _c(cl, np.uint64)
    cr = _c(cr, np.uint64)
    H, W = cl.shape
    C = np.zeros((H, W, D), np.uint8)
    lib.svo_cost2(_p(cl), _p(cr), W, H, D, dmin, sx, sy, _p(C))
    return C


def sgm2(left, right, D, dmin=0, sx=-1, sy=0, P1=10, P2=120, subpixel=True, threads=8):
    """Mode S with a 2-D matching step (census -> cost2 -> 8 paths -> WTA)."""
    left = _c(left, np.uint8)
    right = _c(right, np.uint8)
    H, W = left.shape
    disp = np.zeros((H, W), np.uint16)
    sub = np.zeros((H, W), np.float32) if subpixel else None
    lib.svo_sgm2(_p(left), _p(right), W, H, W, D, dmin, sx, sy, P1, P2, _p(disp), _p(sub),
                 threads)
    return disp, sub


def lr_check2(disp_l, disp_r, sx, sy, max_diff=1, invalid=0xFFFF):
    dl = _c(disp_l, np.uint16).copy()
    dr = _c(disp_r, np.uint16)
    H, W = dl.shape
    lib.svo_lr_check2(_p(dl), _p(dr), W, H, sx, sy, max_diff, invalid)
    return dl


def fuse_depth(disps, baselines, f, pixel_size, invalid=0xFFFF):
    d = _c(disps, np.uint16)
    N, H, W = d.shape
    b = np.ascontiguousarray(baselines, dtype=np.float64)
    out = np.zeros((H, W), np.float64)
    nv = np.zeros((H, W), np.uint8)
    lib.svo_fuse_depth(_p(d), N, W, H, _p(b), f, pixel_size, invalid, _p(out), _p(nv))
    return out, nv


# ---- refinement / 3-D ---------------------------------

def shift_perspective(cin, cout, disp, img, init=None):
    disp = _c(disp, np.uint8)
    img = _c(img, np.uint8)
    H, W = disp.shape
    out = np.zeros((H, W), np.uint8) if init is None else _c(init, np.uint8).copy()
    lib.svo_shift_perspective(ct.byref(cin), ct.byref(cout), _p(disp), _p(img), W, H, W, _p(out))
    return out


def improve_with_disparity(disp, center, images, cam_pairs, window=21, mask=None, strict=False,
                           init=None):
    """cam_pairs: list of (OCamera, OCamera); returns (status, out)."""
    disp = _c(disp, np.uint8)
    center = _c(center, np.uint8)
    H, W = disp.shape
    imgs = [_c(i, np.uint8) for i in images]
    ptrs = (ct.c_void_p * len(imgs))(*[i.ctypes.data for i in imgs])
    cams = (OCamera * (2 * len(cam_pairs)))()
    for i, (a, b) in enumerate(cam_pairs):
        cams[2 * i], cams[2 * i + 1] = a, b
    out = np.zeros((H, W), np.uint8) if init is None else _c(init, np.uint8).copy()
    m = None if mask is None else _c(mask, np.uint8)
    st = lib.svo_improve_with_disparity(_p(disp), _p(center), ptrs, cams, len(imgs), W, H, W,
                                        _p(m), window, int(strict), _p(out))
    return st, out


def shift_perspective2(cin, cout, depth, init=None):
    depth = _c(depth, np.float64)
    H, W = depth.shape
    out = np.zeros((H, W), np.float64) if init is None else _c(init, np.float64).copy()
    lib.svo_shift_perspective2(ct.byref(cin), ct.byref(cout), _p(depth), W, H, _p(out))
    return out


def points_to_depth(points, cam, W, H, init=None):
    pts = _c(points, np.float64).reshape(-1, 3)
    out = np.zeros((H, W), np.float64) if init is None else _c(init, np.float64).copy()
    lib.svo_points_to_depth(_p(pts), pts.shape[0], ct.byref(cam), W, H, _p(out))
    return out


def depth_to_points(depth, cam):
    depth = _c(depth, np.float64)
    H, W = depth.shape
    pts = np.zeros((W * H, 3), np.float64)
    n = lib.svo_depth_to_points(_p(depth), W, H, ct.byref(cam), _p(pts))
    return pts[:n].copy()


def resize_half(img):
    img = _c(img, np.uint8)
    H, W = img.shape
    dw, dh = ct.c_int(0), ct.c_int(0)
    lib.svo_resize_half_size(W, H, ct.byref(dw), ct.byref(dh))
    out = np.zeros((dh.value, dw.value), np.uint8)
    lib.svo_resize_half(_p(img), W, H, W, _p(out), max(1, dw.value))
    return out


def resize_linear_f64(src, dw, dh):
    src = _c(src, np.float64)
    sh, sw = src.shape
    out = np.zeros((dh, dw), np.float64)
    lib.svo_resize_linear_f64(_p(src), sw, sh, _p(out), dw, dh)
    return out


def ref_error(depth, ref, scale=50.0):
    depth = _c(depth, np.float64)
    ref = _c(ref, np.float64)
    h, w = depth.shape
    rh, rw = ref.shape
    out = np.zeros((rh, rw), np.float64)
    lib.svo_ref_error(_p(depth), w, h, _p(ref), rw, rh, scale, _p(out))
    return out


def masked_mean(image, mask=None):
    image = _c(image, np.float64)
    h, w = image.shape
    m = None if mask is None else _c(mask, np.uint8)
    return lib.svo_masked_mean(_p(image), _p(m), w, h)
