"""stereovisionarray_amd -- MI355X-native stereo disparity engine.

The product is the C-ABI shared library ``libsva.so`` (hand-written HIP
kernels for gfx950 + a C++ host layer, declared in ``include/sva.h``).  This
module is a thin ctypes binding used by the tests and ``bench.py``; it adds no
compute of its own and has no CPU fallback: if ``libsva.so`` is missing, import
fails loudly, and if no GPU is present every compute call raises.

Host-pointer calls take numpy arrays; ``*_d`` calls take device pointers
(ints), e.g. ``torch_tensor.data_ptr()``.
"""
from __future__ import annotations

import ctypes as ct
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SVA_LIB_PATH: load an alternative build of the same library (kernel-variant
# experiments under tools/); the default is the in-tree libsva.so.
LIB_PATH = os.environ.get("SVA_LIB_PATH") or os.path.join(_HERE, "libsva.so")

SVA_OK = 0
SVA_ERR_INVALID_ARG = 1
SVA_ERR_UNSUPPORTED = 2
SVA_ERR_DEVICE = 3
SVA_ERR_OUT_OF_MEMORY = 4
SVA_ERR_NO_DEVICE = 5
SVA_PATH_KERNEL_COST_VOLUME = 0
SVA_PATH_KERNEL_FUSED = 1
SVA_PATH_KERNEL_AUTO = 2
SVA_TIMING_OFF = 0
SVA_TIMING_ALL = 1
SVA_TIMING_PATHS = 2
SVA_TIMING_AGG = 3
SVA_DEBUG_PLANE_SPLIT = 1
SVA_DEBUG_FAIL_COST_AT = 2
SVA_DEBUG_SIDE_IDLE = 3
SVA_DEBUG_PLACEMENT_TRIALS = 4
SVA_DEBUG_PLACEMENT_NS = 5
SVA_DEBUG_PLACEMENT_WORST_NS = 6
# The ABI this binding is written against (include/sva.h SVA_ABI_VERSION).
ABI_VERSION = 6

# Symbols declared in include/sva.h (checked by tests/test_abi.py).
EXPORTED = [
    "sva_sgm_params_default", "sva_abi_version", "sva_device_count", "sva_create",
    "sva_destroy", "sva_set_stream", "sva_synchronize", "sva_last_error",
    "sva_status_string", "sva_reserve", "sva_set_path_kernel", "sva_set_timing", "sva_reset_timing",
    "sva_kernel_time", "sva_disparity_sgm", "sva_disparity_sgm_d", "sva_census_d",
    "sva_cost_d", "sva_census_cost_d", "sva_paths_d", "sva_aggregate_d", "sva_wta_d", "sva_disparity_ref",
    "sva_disparity_ref_d", "sva_ref_endpoints_d", "sva_disparity_to_depth_d",
    "sva_disparity_to_depth", "sva_fuse_depth_d", "sva_fuse_depth",
    "sva_shift_perspective_d", "sva_shift_perspective", "sva_improve_with_disparity_d",
    "sva_improve_with_disparity", "sva_shift_perspective2_d", "sva_shift_perspective2",
    "sva_points_to_depth_d", "sva_points_to_depth", "sva_depth_to_points_d",
    "sva_depth_to_points", "sva_resize_half_size", "sva_resize_half_d", "sva_resize_half",
    "sva_batch_sgm", "sva_resize_linear_f64_d", "sva_resize_linear_f64", "sva_ref_error_d",
    "sva_ref_error", "sva_masked_mean_d", "sva_masked_mean", "sva_tile_layout_of",
    "sva_tile_check", "sva_paths_tile_d", "sva_wta_hv_d", "sva_multi_create", "sva_multi_destroy",
    "sva_multi_synchronize", "sva_multi_last_error", "sva_multi_plan", "sva_multi_context",
    "sva_batch_sgm_d", "sva_array_depth", "sva_disparity_sgm_batch_d", "sva_set_debug",
    "sva_get_debug",
]
SVA_MULTI_GATHER_RCCL = 0
SVA_MULTI_GATHER_PEER = 1
SVA_MULTI_GATHER_ALL = 2


class SgmParams(ct.Structure):
    """Mirror of ``sva_sgm_params`` (include/sva.h)."""
    _fields_ = [
        ("D", ct.c_int32), ("dmin", ct.c_int32), ("dir", ct.c_int32),
        ("P1", ct.c_int32), ("P2", ct.c_int32), ("subpixel", ct.c_int32),
        ("lr_check", ct.c_int32), ("lr_max_diff", ct.c_int32),
        ("invalid", ct.c_uint16), ("_pad", ct.c_uint16), ("dir_y", ct.c_int32),
    ]


class Camera(ct.Structure):
    """Mirror of ``sva_camera`` = class Camera (include/Camera.h:6-21)."""
    _fields_ = [("f", ct.c_double), ("pos", ct.c_double * 3), ("pixel_size", ct.c_double)]

    @classmethod
    def make(cls, f, pos, pixel_size):
        c = cls()
        c.f = f
        c.pos[0], c.pos[1], c.pos[2] = pos
        c.pixel_size = pixel_size
        return c


class TileLayout(ct.Structure):
    """Mirror of ``sva_tile_layout`` (include/sva.h): the tile stages' buffers."""
    _fields_ = [("seg", ct.c_int32), ("nsx", ct.c_int32), ("nsy", ct.c_int32),
                ("diag_volumes", ct.c_int32),
                ("cost_bytes", ct.c_size_t), ("diag_bytes", ct.c_size_t),
                ("hckpt_bytes", ct.c_size_t), ("vckpt_bytes", ct.c_size_t)]


class PairJob(ct.Structure):
    _fields_ = [
        ("left", ct.c_void_p), ("right", ct.c_void_p), ("width", ct.c_int32),
        ("height", ct.c_int32), ("pitch", ct.c_size_t), ("disp", ct.c_void_p),
        ("subpix", ct.c_void_p),
    ]


class PairD(ct.Structure):
    """sva_pair_d: one device-resident pair for sva_batch_sgm_d."""
    _fields_ = [("left", ct.c_void_p), ("right", ct.c_void_p), ("params", SgmParams)]


class ArrayPair(ct.Structure):
    """sva_array_pair: one camera-array pair for sva_array_depth."""
    _fields_ = [("ref", ct.c_int32), ("other", ct.c_int32), ("params", SgmParams),
                ("baseline", ct.c_double)]


class SvaError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"sva status {status}: {msg}")
        self.status = status


def _preload_single_hip_runtime() -> None:
    """Keep ONE HIP runtime per process.  PyTorch-ROCm wheels bundle their own
    libamdhip64 (same SONAME as /opt/rocm's).  If libsva.so were loaded first it
    would bind /opt/rocm's copy and a later `import torch` would map a second
    runtime whose device init then fails.  Preloading torch's copy by path makes
    libsva.so (and torch, whenever imported) bind that single runtime."""
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return
    cand = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(cand):
        ct.CDLL(cand, mode=ct.RTLD_GLOBAL)


def _load() -> ct.CDLL:
    _preload_single_hip_runtime()
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback)")
    lib = ct.CDLL(LIB_PATH)
    vp, i32, sz, dbl = ct.c_void_p, ct.c_int, ct.c_size_t, ct.c_double
    P = ct.POINTER
    sig = {
        "sva_sgm_params_default": (None, [P(SgmParams)]),
        "sva_abi_version": (i32, []),
        "sva_device_count": (i32, [P(i32)]),
        "sva_create": (i32, [i32, P(vp)]),
        "sva_destroy": (i32, [vp]),
        "sva_set_stream": (i32, [vp, vp]),
        "sva_synchronize": (i32, [vp]),
        "sva_last_error": (ct.c_char_p, [vp]),
        "sva_status_string": (ct.c_char_p, [i32]),
        "sva_reserve": (i32, [vp, i32, i32, i32]),
        "sva_set_path_kernel": (i32, [vp, i32]),
        "sva_set_timing": (i32, [vp, i32]),
        "sva_reset_timing": (i32, [vp]),
        "sva_kernel_time": (i32, [vp, ct.c_char_p, P(dbl), P(ct.c_int64)]),
        "sva_set_debug": (i32, [vp, i32, ct.c_int64]),
        "sva_get_debug": (i32, [vp, i32, P(ct.c_int64)]),
        "sva_disparity_sgm": (i32, [vp, vp, vp, i32, i32, sz, P(SgmParams), vp, vp]),
        "sva_disparity_sgm_d": (i32, [vp, vp, vp, i32, i32, sz, P(SgmParams), vp, vp]),
        "sva_census_d": (i32, [vp, vp, i32, i32, sz, vp]),
        "sva_cost_d": (i32, [vp, vp, vp, i32, i32, P(SgmParams), vp]),
        "sva_paths_d": (i32, [vp, vp, i32, i32, P(SgmParams), vp]),
        "sva_census_cost_d": (i32, [vp, vp, vp, i32, i32, sz, P(SgmParams), vp]),
        "sva_aggregate_d": (i32, [vp, vp, i32, i32, P(SgmParams), vp]),
        "sva_wta_d": (i32, [vp, vp, i32, i32, P(SgmParams), vp, vp]),
        "sva_tile_layout_of": (i32, [i32, i32, i32, P(TileLayout)]),
        "sva_tile_check": (i32, [i32, i32, i32, sz, sz, sz, sz]),
        "sva_paths_tile_d": (i32, [vp, vp, sz, i32, i32, P(SgmParams), vp, sz, vp, sz, vp, sz]),
        "sva_wta_hv_d": (i32, [vp, vp, sz, vp, sz, vp, sz, vp, sz, i32, i32, P(SgmParams), vp,
                               vp]),
        "sva_disparity_ref": (i32, [vp, vp, vp, i32, i32, sz, vp, P(Camera), P(Camera), i32,
                                    dbl, dbl, vp, vp, vp]),
        "sva_disparity_ref_d": (i32, [vp, vp, vp, i32, i32, sz, vp, P(Camera), P(Camera), i32,
                                      dbl, dbl, vp, vp, vp]),
        "sva_ref_endpoints_d": (i32, [vp, i32, i32, P(Camera), P(Camera), i32, dbl, dbl, vp, vp]),
        "sva_disparity_to_depth_d": (i32, [vp, vp, i32, dbl, dbl, dbl, vp]),
        "sva_disparity_to_depth": (i32, [vp, vp, i32, dbl, dbl, dbl, vp]),
        "sva_fuse_depth_d": (i32, [vp, vp, i32, i32, i32, P(dbl), dbl, dbl, ct.c_uint16, vp, vp]),
        "sva_fuse_depth": (i32, [vp, vp, i32, i32, i32, P(dbl), dbl, dbl, ct.c_uint16, vp, vp]),
        "sva_shift_perspective_d": (i32, [vp, P(Camera), P(Camera), vp, vp, i32, i32, sz, vp]),
        "sva_shift_perspective": (i32, [vp, P(Camera), P(Camera), vp, vp, i32, i32, sz, vp]),
        "sva_improve_with_disparity_d": (i32, [vp, vp, vp, P(vp), P(Camera), i32, i32, i32, sz,
                                               vp, i32, i32, vp]),
        "sva_improve_with_disparity": (i32, [vp, vp, vp, P(vp), P(Camera), i32, i32, i32, sz,
                                             vp, i32, i32, vp]),
        "sva_shift_perspective2_d": (i32, [vp, P(Camera), P(Camera), vp, i32, i32, vp]),
        "sva_shift_perspective2": (i32, [vp, P(Camera), P(Camera), vp, i32, i32, vp]),
        "sva_points_to_depth_d": (i32, [vp, vp, ct.c_int64, P(Camera), i32, i32, vp]),
        "sva_points_to_depth": (i32, [vp, vp, ct.c_int64, P(Camera), i32, i32, vp]),
        "sva_depth_to_points_d": (i32, [vp, vp, i32, i32, P(Camera), vp, P(ct.c_int64)]),
        "sva_depth_to_points": (i32, [vp, vp, i32, i32, P(Camera), vp, P(ct.c_int64)]),
        "sva_resize_half_size": (i32, [i32, i32, P(i32), P(i32)]),
        "sva_resize_half_d": (i32, [vp, vp, i32, i32, sz, vp, sz]),
        "sva_resize_half": (i32, [vp, vp, i32, i32, sz, vp, sz]),
        "sva_batch_sgm": (i32, [P(vp), i32, P(PairJob), i32, P(SgmParams), P(i32)]),
        "sva_multi_create": (i32, [P(i32), i32, i32, i32, P(vp)]),
        "sva_multi_destroy": (i32, [vp]),
        "sva_multi_synchronize": (i32, [vp]),
        "sva_multi_last_error": (ct.c_char_p, [vp]),
        "sva_multi_plan": (i32, [i32, i32, i32, P(i32), P(i32), P(i32)]),
        "sva_multi_context": (i32, [vp, i32, i32, P(vp)]),
        "sva_batch_sgm_d": (i32, [vp, P(PairD), i32, i32, i32, sz, vp, vp]),
        "sva_disparity_sgm_batch_d": (i32, [vp, P(PairD), i32, i32, i32, sz, vp, vp]),
        "sva_array_depth": (i32, [vp, P(vp), i32, i32, i32, sz, P(ArrayPair), i32, P(i32), i32,
                                  dbl, dbl, vp, vp, vp]),
        "sva_resize_linear_f64_d": (i32, [vp, vp, i32, i32, vp, i32, i32]),
        "sva_resize_linear_f64": (i32, [vp, vp, i32, i32, vp, i32, i32]),
        "sva_ref_error_d": (i32, [vp, vp, i32, i32, vp, i32, i32, ct.c_double, vp]),
        "sva_ref_error": (i32, [vp, vp, i32, i32, vp, i32, i32, ct.c_double, vp]),
        "sva_masked_mean_d": (i32, [vp, vp, vp, i32, i32, P(ct.c_double)]),
        "sva_masked_mean": (i32, [vp, vp, vp, i32, i32, P(ct.c_double)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    # a stale build exports the same symbols with other semantics: refuse it
    have = lib.sva_abi_version()
    if have != ABI_VERSION:
        raise ImportError(f"{LIB_PATH} implements ABI v{have}, this binding needs v{ABI_VERSION}: "
                          "rebuild it (python -c 'import __graft_entry__ as g; g.build()')")
    return lib


lib = _load()


def default_params(**kw) -> SgmParams:
    p = SgmParams()
    lib.sva_sgm_params_default(ct.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def resize_half_size(W: int, H: int):
    """Output size of the ingestion resize: (cvRound(W/2), cvRound(H/2))."""
    dw, dh = ct.c_int(0), ct.c_int(0)
    if lib.sva_resize_half_size(W, H, ct.byref(dw), ct.byref(dh)) != 0:
        raise ValueError("bad size")
    return dw.value, dh.value


def tile_layout(W: int, H: int, D: int) -> TileLayout:
    """Plane sizes of the tile stages (sva_tile_layout_of; no device needed)."""
    out = TileLayout()
    st = lib.sva_tile_layout_of(W, H, D, ct.byref(out))
    if st != SVA_OK:
        raise SvaError(st, "sva_tile_layout_of")
    return out


def device_count() -> int:
    n = ct.c_int(0)
    lib.sva_device_count(ct.byref(n))
    return n.value


def _ptr(a) -> int | None:
    if a is None:
        return None
    if isinstance(a, int):
        return a
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()  # torch tensor


class Context:
    """One device + one stream (``sva_create``)."""

    def __init__(self, device: int = 0):
        h = ct.c_void_p()
        st = lib.sva_create(device, ct.byref(h))
        if st != SVA_OK:
            raise SvaError(st, lib.sva_status_string(st).decode())
        self.h = h
        self.device = device
        self._owned = True

    @classmethod
    def borrowed(cls, handle: int, device: int):
        """A non-owning view of a context another owner destroys (e.g. one of
        a Multi engine's, sva_multi_context)."""
        c = cls.__new__(cls)
        c.h = ct.c_void_p(handle)
        c.device = device
        c._owned = False
        return c

    def close(self):
        if self.h and self._owned:
            lib.sva_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _chk(self, st: int):
        if st != SVA_OK:
            raise SvaError(st, lib.sva_last_error(self.h).decode())

    # -- plumbing
    def set_stream(self, stream_ptr: int | None):
        self._chk(lib.sva_set_stream(self.h, stream_ptr))

    def synchronize(self):
        self._chk(lib.sva_synchronize(self.h))

    def reserve(self, W, H, D):
        self._chk(lib.sva_reserve(self.h, W, H, D))

    def set_path_kernel(self, kernel: int):
        self._chk(lib.sva_set_path_kernel(self.h, kernel))

    def set_timing(self, on):
        """on: False/True, SVA_TIMING_PATHS (the path kernel only) or SVA_TIMING_AGG
        (the path kernel and wta_hv, the two aggregation kernels)."""
        self._chk(lib.sva_set_timing(self.h, int(on)))

    def reset_timing(self):
        self._chk(lib.sva_reset_timing(self.h))

    def set_debug(self, key: int, value: int):
        """sva_set_debug: SVA_DEBUG_PLANE_SPLIT / SVA_DEBUG_FAIL_COST_AT (tests),
        SVA_DEBUG_PLACEMENT_TRIALS (sva_reserve's placement check)."""
        self._chk(lib.sva_set_debug(self.h, key, int(value)))

    def get_debug(self, key: int) -> int:
        v = ct.c_int64(0)
        self._chk(lib.sva_get_debug(self.h, key, ct.byref(v)))
        return v.value

    def kernel_time(self, name: str) -> tuple[float, int]:
        ms = ct.c_double(0)
        n = ct.c_int64(0)
        self._chk(lib.sva_kernel_time(self.h, name.encode(), ct.byref(ms), ct.byref(n)))
        return ms.value, n.value

    # -- Mode S, host arrays
    def disparity_sgm(self, left: np.ndarray, right: np.ndarray, params: SgmParams):
        assert left.dtype == np.uint8 and right.dtype == np.uint8 and left.shape == right.shape
        left = np.ascontiguousarray(left)
        right = np.ascontiguousarray(right)
        H, W = left.shape
        disp = np.zeros((H, W), np.uint16)
        sub = np.zeros((H, W), np.float32) if params.subpixel else None
        self._chk(lib.sva_disparity_sgm(self.h, _ptr(left), _ptr(right), W, H, W,
                                        ct.byref(params), _ptr(disp), _ptr(sub)))
        return disp, sub

    # -- Mode S, device pointers (async on the context stream)
    def disparity_sgm_d(self, left, right, W, H, pitch, params, disp, sub=None):
        self._chk(lib.sva_disparity_sgm_d(self.h, _ptr(left), _ptr(right), W, H, pitch,
                                          ct.byref(params), _ptr(disp), _ptr(sub)))

    def disparity_sgm_batch_d(self, pairs, W, H, pitch, maps, sub=None):
        """pairs: list of (left_ptr, right_ptr, SgmParams) on this context's device;
        maps: [n][H][W] u16 device, sub: [n][H][W] f32 device or None."""
        jobs = (PairD * len(pairs))()
        for i, (l, r, p) in enumerate(pairs):
            jobs[i] = PairD(_ptr(l), _ptr(r), p)
        self._chk(lib.sva_disparity_sgm_batch_d(self.h, jobs, len(pairs), W, H, pitch,
                                                _ptr(maps), _ptr(sub)))

    def census_d(self, img, W, H, pitch, out):
        self._chk(lib.sva_census_d(self.h, _ptr(img), W, H, pitch, _ptr(out)))

    def cost_d(self, cl, cr, W, H, params, C):
        self._chk(lib.sva_cost_d(self.h, _ptr(cl), _ptr(cr), W, H, ct.byref(params), _ptr(C)))

    def paths_d(self, C, W, H, params, L8):
        self._chk(lib.sva_paths_d(self.h, _ptr(C), W, H, ct.byref(params), _ptr(L8)))

    def census_cost_d(self, left, right, W, H, pitch, params, C):
        self._chk(lib.sva_census_cost_d(self.h, _ptr(left), _ptr(right), W, H, pitch,
                                        ct.byref(params), _ptr(C)))

    def aggregate_d(self, C, W, H, params, S):
        self._chk(lib.sva_aggregate_d(self.h, _ptr(C), W, H, ct.byref(params), _ptr(S)))

    def paths_tile_d(self, C, C_bytes, W, H, params, diag, diag_bytes, hck, hck_bytes, vck,
                     vck_bytes):
        self._chk(lib.sva_paths_tile_d(self.h, _ptr(C), C_bytes, W, H, ct.byref(params),
                                       _ptr(diag), diag_bytes, _ptr(hck), hck_bytes, _ptr(vck),
                                       vck_bytes))

    def wta_hv_d(self, C, C_bytes, diag, diag_bytes, hck, hck_bytes, vck, vck_bytes, W, H, params,
                 disp, sub=None):
        self._chk(lib.sva_wta_hv_d(self.h, _ptr(C), C_bytes, _ptr(diag), diag_bytes, _ptr(hck),
                                   hck_bytes, _ptr(vck), vck_bytes, W, H, ct.byref(params),
                                   _ptr(disp), _ptr(sub)))

    def wta_d(self, S, W, H, params, disp, sub=None):
        self._chk(lib.sva_wta_d(self.h, _ptr(S), W, H, ct.byref(params), _ptr(disp), _ptr(sub)))

    # -- Mode R
    def disparity_ref(self, ref: np.ndarray, other: np.ndarray, cref: Camera, coth: Camera,
                      k: int = 20, t_near: float = 0.5, t_far: float = 1.0, mask=None,
                      disp_u8=None, disp_u16=None, valid=None):
        ref = np.ascontiguousarray(ref)
        other = np.ascontiguousarray(other)
        H, W = ref.shape
        if disp_u8 is None:
            disp_u8 = np.zeros((H, W), np.uint8)
        if disp_u16 is None:
            disp_u16 = np.zeros((H, W), np.uint16)
        if valid is None:
            valid = np.zeros((H, W), np.uint8)
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        self._chk(lib.sva_disparity_ref(self.h, _ptr(ref), _ptr(other), W, H, W, _ptr(m),
                                        ct.byref(cref), ct.byref(coth), k, t_near, t_far,
                                        _ptr(disp_u8), _ptr(disp_u16), _ptr(valid)))
        return disp_u8, disp_u16, valid

    def disparity_ref_d(self, ref, other, W, H, pitch, mask, cref, coth, k, t_near, t_far,
                        disp_u8, disp_u16=None, valid=None):
        self._chk(lib.sva_disparity_ref_d(self.h, _ptr(ref), _ptr(other), W, H, pitch, _ptr(mask),
                                          ct.byref(cref), ct.byref(coth), k, t_near, t_far,
                                          _ptr(disp_u8), _ptr(disp_u16), _ptr(valid)))

    def ref_endpoints_d(self, W, H, cref, coth, k, t_near, t_far, ends, valid):
        self._chk(lib.sva_ref_endpoints_d(self.h, W, H, ct.byref(cref), ct.byref(coth), k,
                                          t_near, t_far, _ptr(ends), _ptr(valid)))

    # -- refinement / 3-D, host arrays
    def shift_perspective(self, cin: Camera, cout: Camera, disp, image, init=None):
        disp = np.ascontiguousarray(disp, dtype=np.uint8)
        image = np.ascontiguousarray(image, dtype=np.uint8)
        H, W = disp.shape
        out = np.zeros((H, W), np.uint8) if init is None else np.array(init, np.uint8)
        self._chk(lib.sva_shift_perspective(self.h, ct.byref(cin), ct.byref(cout), _ptr(disp),
                                            _ptr(image), W, H, W, _ptr(out)))
        return out

    def improve_with_disparity(self, disp, center, images, cam_pairs, window=21, mask=None,
                               strict=False, init=None):
        disp = np.ascontiguousarray(disp, dtype=np.uint8)
        center = np.ascontiguousarray(center, dtype=np.uint8)
        H, W = disp.shape
        imgs = [np.ascontiguousarray(i, dtype=np.uint8) for i in images]
        ptrs = (ct.c_void_p * max(1, len(imgs)))(*[i.ctypes.data for i in imgs])
        cams = (Camera * max(1, 2 * len(cam_pairs)))()
        for i, (a, b) in enumerate(cam_pairs):
            cams[2 * i], cams[2 * i + 1] = a, b
        out = np.zeros((H, W), np.uint8) if init is None else np.array(init, np.uint8)
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        self._chk(lib.sva_improve_with_disparity(self.h, _ptr(disp), _ptr(center), ptrs, cams,
                                                 len(imgs), W, H, W, _ptr(m), window,
                                                 int(strict), _ptr(out)))
        return out

    def improve_with_disparity_d(self, disp, center, images, cam_pairs, W, H, pitch, mask,
                                 window, strict, out):
        ptrs = (ct.c_void_p * max(1, len(images)))(*images)
        cams = (Camera * max(1, 2 * len(cam_pairs)))()
        for i, (a, b) in enumerate(cam_pairs):
            cams[2 * i], cams[2 * i + 1] = a, b
        self._chk(lib.sva_improve_with_disparity_d(self.h, _ptr(disp), _ptr(center), ptrs, cams,
                                                   len(images), W, H, pitch, _ptr(mask), window,
                                                   int(strict), _ptr(out)))

    def shift_perspective2(self, cin: Camera, cout: Camera, depth, init=None):
        depth = np.ascontiguousarray(depth, dtype=np.float64)
        H, W = depth.shape
        out = np.zeros((H, W), np.float64) if init is None else np.array(init, np.float64)
        self._chk(lib.sva_shift_perspective2(self.h, ct.byref(cin), ct.byref(cout), _ptr(depth),
                                             W, H, _ptr(out)))
        return out

    def points_to_depth(self, points, cam: Camera, W, H, init=None):
        pts = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 3)
        out = np.zeros((H, W), np.float64) if init is None else np.array(init, np.float64)
        self._chk(lib.sva_points_to_depth(self.h, _ptr(pts), pts.shape[0], ct.byref(cam), W, H,
                                          _ptr(out)))
        return out

    def depth_to_points(self, depth, cam: Camera):
        depth = np.ascontiguousarray(depth, dtype=np.float64)
        H, W = depth.shape
        pts = np.zeros((W * H, 3), np.float64)
        n = ct.c_int64(0)
        self._chk(lib.sva_depth_to_points(self.h, _ptr(depth), W, H, ct.byref(cam), _ptr(pts),
                                          ct.byref(n)))
        return pts[:n.value].copy()

    def depth_to_points_d(self, depth, W, H, cam: Camera, points) -> int:
        n = ct.c_int64(0)
        self._chk(lib.sva_depth_to_points_d(self.h, _ptr(depth), W, H, ct.byref(cam),
                                            _ptr(points), ct.byref(n)))
        return n.value

    # -- ingestion
    def resize_half(self, img):
        img = np.ascontiguousarray(img, dtype=np.uint8)
        H, W = img.shape
        dw, dh = resize_half_size(W, H)
        out = np.zeros((dh, dw), np.uint8)
        self._chk(lib.sva_resize_half(self.h, _ptr(img), W, H, W, _ptr(out), max(1, dw)))
        return out

    def resize_half_d(self, src, W, H, pitch, dst, dst_pitch):
        self._chk(lib.sva_resize_half_d(self.h, _ptr(src), W, H, pitch, _ptr(dst), dst_pitch))

    # ---- evaluation (CameraStereoVision.cpp:107-119) ----
    def resize_linear(self, src, dw: int, dh: int):
        """resize(src, dst, Size(dw, dh)) INTER_LINEAR on a f64 matrix."""
        src = np.ascontiguousarray(src, dtype=np.float64)
        sh, sw = src.shape
        out = np.zeros((dh, dw), np.float64)
        self._chk(lib.sva_resize_linear_f64(self.h, _ptr(src), sw, sh, _ptr(out), dw, dh))
        return out

    def resize_linear_d(self, src, sw, sh, dst, dw, dh):
        self._chk(lib.sva_resize_linear_f64_d(self.h, _ptr(src), sw, sh, _ptr(dst), dw, dh))

    def ref_error(self, depth, ref, scale: float = 50.0):
        """(resize(depth, ref.size()) - ref) * scale, as the reference's
        ``Mat error = (depth2 - ref) * 50``."""
        depth = np.ascontiguousarray(depth, dtype=np.float64)
        ref = np.ascontiguousarray(ref, dtype=np.float64)
        h, w = depth.shape
        rh, rw = ref.shape
        out = np.zeros((rh, rw), np.float64)
        self._chk(lib.sva_ref_error(self.h, _ptr(depth), w, h, _ptr(ref), rw, rh, scale,
                                    _ptr(out)))
        return out

    def ref_error_d(self, depth, w, h, ref, rw, rh, scale, error):
        self._chk(lib.sva_ref_error_d(self.h, _ptr(depth), w, h, _ptr(ref), rw, rh, scale,
                                      _ptr(error)))

    def masked_mean(self, image, mask=None) -> float:
        """cv::mean(image, mask)[0] (calculateAverageError, functions.cpp:348-354)."""
        image = np.ascontiguousarray(image, dtype=np.float64)
        h, w = image.shape
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        out = ct.c_double(0)
        self._chk(lib.sva_masked_mean(self.h, _ptr(image), _ptr(m), w, h, ct.byref(out)))
        return out.value

    def masked_mean_d(self, image, mask, w, h) -> float:
        out = ct.c_double(0)
        self._chk(lib.sva_masked_mean_d(self.h, _ptr(image), _ptr(mask), w, h, ct.byref(out)))
        return out.value

    def fuse_depth(self, disps: np.ndarray, baselines, f, pixel_size, invalid=0xFFFF):
        d = np.ascontiguousarray(disps, dtype=np.uint16)
        N, H, W = d.shape
        b = (ct.c_double * N)(*[float(v) for v in baselines])
        out = np.zeros((H, W), np.float64)
        nv = np.zeros((H, W), np.uint8)
        self._chk(lib.sva_fuse_depth(self.h, _ptr(d), N, W, H, b, f, pixel_size, invalid,
                                     _ptr(out), _ptr(nv)))
        return out, nv

    def fuse_depth_d(self, disps, n_maps, W, H, baselines, f, pixel_size, invalid, depth,
                     n_valid=None):
        b = (ct.c_double * n_maps)(*[float(v) for v in baselines])
        self._chk(lib.sva_fuse_depth_d(self.h, _ptr(disps), n_maps, W, H, b, f, pixel_size,
                                       invalid, _ptr(depth), _ptr(n_valid)))

    def disparity_to_depth(self, disp: np.ndarray, cam_distance, f, pixel_size):
        d = np.ascontiguousarray(disp, dtype=np.uint8)
        out = np.zeros(d.shape, np.float64)
        self._chk(lib.sva_disparity_to_depth(self.h, _ptr(d), d.size, cam_distance, f, pixel_size,
                                             _ptr(out)))
        return out

    def disparity_to_depth_d(self, disp, n, cam_distance, f, pixel_size, depth):
        self._chk(lib.sva_disparity_to_depth_d(self.h, _ptr(disp), n, cam_distance, f,
                                               pixel_size, _ptr(depth)))


def batch_sgm(contexts: list[Context], pairs: list[tuple[np.ndarray, np.ndarray]],
              params: SgmParams, statuses: list | None = None):
    """Match independent pairs round-robin over ``contexts`` (``sva_batch_sgm``).
    With ``statuses`` (a list), per-pair status codes are appended to it and a
    failing pair does not raise; otherwise the first failure raises."""
    jobs = (PairJob * len(pairs))()
    outs = []
    keep = []
    for i, (l, r) in enumerate(pairs):
        l = np.ascontiguousarray(l)
        r = np.ascontiguousarray(r)
        H, W = l.shape
        d = np.zeros((H, W), np.uint16)
        s = np.zeros((H, W), np.float32) if params.subpixel else None
        keep += [l, r]
        outs.append((d, s))
        jobs[i] = PairJob(_ptr(l), _ptr(r), W, H, W, _ptr(d), _ptr(s))
    hs = (ct.c_void_p * len(contexts))(*[c.h.value for c in contexts])
    js = (ct.c_int * max(1, len(pairs)))()
    st = lib.sva_batch_sgm(hs, len(contexts), jobs, len(pairs), ct.byref(params), js)
    if statuses is not None:
        statuses.extend(js[:len(pairs)])
    elif st != SVA_OK:
        raise SvaError(st, lib.sva_status_string(st).decode())
    return outs


def multi_plan(n_devices: int, streams: int, n_jobs: int):
    """(device_index, context_index, slot_index) arrays of sva_multi_plan."""
    d = np.zeros(max(n_jobs, 1), np.int32)
    c = np.zeros(max(n_jobs, 1), np.int32)
    s = np.zeros(max(n_jobs, 1), np.int32)
    st = lib.sva_multi_plan(n_devices, streams, n_jobs,
                            d.ctypes.data_as(ct.POINTER(ct.c_int32)),
                            c.ctypes.data_as(ct.POINTER(ct.c_int32)),
                            s.ctypes.data_as(ct.POINTER(ct.c_int32)))
    if st != SVA_OK:
        raise SvaError(st, "sva_multi_plan")
    return d[:n_jobs], c[:n_jobs], s[:n_jobs]


class Multi:
    """The multi-GPU engine (sva_multi_*): pairs shard over ``devices`` (pair j
    -> device j mod N, round-robin over ``streams`` contexts per device) and
    the maps are gathered to devices[0] (RCCL or peer copies)."""

    def __init__(self, devices, streams: int = 2, flags: int = SVA_MULTI_GATHER_RCCL):
        self.devices = list(devices)
        arr = (ct.c_int * len(self.devices))(*self.devices)
        self.h = ct.c_void_p()
        st = lib.sva_multi_create(arr, len(self.devices), streams, flags, ct.byref(self.h))
        if st != SVA_OK:
            raise SvaError(st, f"sva_multi_create ({lib.sva_status_string(st).decode()})")

    def close(self):
        if self.h:
            lib.sva_multi_destroy(self.h)
            self.h = ct.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, st: int):
        if st != SVA_OK:
            raise SvaError(st, lib.sva_multi_last_error(self.h).decode(errors="replace"))

    def synchronize(self):
        self._chk(lib.sva_multi_synchronize(self.h))

    def context_handle(self, device_index: int, stream_index: int) -> int:
        out = ct.c_void_p()
        self._chk(lib.sva_multi_context(self.h, device_index, stream_index, ct.byref(out)))
        return out.value

    def context(self, device_index: int, stream_index: int) -> "Context":
        """The engine's context (device_index, stream_index), borrowed (the
        engine destroys it): kernel timing, or direct per-device calls."""
        return Context.borrowed(self.context_handle(device_index, stream_index),
                                self.devices[device_index])

    def batch_sgm_d(self, pairs, W, H, pitch, maps, sub=None):
        """pairs: list of (left_ptr, right_ptr, SgmParams) on their owner devices."""
        jobs = (PairD * len(pairs))()
        for i, (l, r, p) in enumerate(pairs):
            jobs[i] = PairD(_ptr(l), _ptr(r), p)
        self._chk(lib.sva_batch_sgm_d(self.h, jobs, len(pairs), W, H, pitch, _ptr(maps),
                                      _ptr(sub)))

    def array_depth(self, images, pairs, group_start, f, pixel_size, want_maps=False):
        """images: list of HxW u8 numpy views; pairs: list of (ref, other,
        SgmParams, baseline); group_start: n_groups + 1 offsets.  Returns
        (depth [G,H,W] f64, n_valid [G,H,W] u8, maps [P,H,W] u16 or None)."""
        imgs = [np.ascontiguousarray(a, dtype=np.uint8) for a in images]
        H, W = imgs[0].shape
        ptrs = (ct.c_void_p * len(imgs))(*[_ptr(a) for a in imgs])
        jp = (ArrayPair * len(pairs))()
        for i, (a, b, p, base) in enumerate(pairs):
            jp[i] = ArrayPair(a, b, p, base)
        gs = (ct.c_int32 * len(group_start))(*group_start)
        G = len(group_start) - 1
        depth = np.zeros((G, H, W), np.float64)
        nv = np.zeros((G, H, W), np.uint8)
        maps = np.zeros((len(pairs), H, W), np.uint16) if want_maps else None
        self._chk(lib.sva_array_depth(self.h, ptrs, len(imgs), W, H, W, jp, len(pairs), gs, G,
                                      f, pixel_size, _ptr(depth), _ptr(nv), _ptr(maps)))
        return depth, nv, maps
