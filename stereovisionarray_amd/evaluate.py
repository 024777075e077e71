"""Evaluation helpers, SURVEY.md §8f row 4: the reference's ground-truth
comparison and its OpenCV-YAML matrix files.

* ``get_ideal_ref`` -- getIdealRef (functions.cpp:323-329): ``idealRef.yml``, key ``R``.
* ``save_image`` / ``load_image`` -- saveImage / loadImage (functions.cpp:331-346):
  one matrix under key ``image``.
* ``Context.ref_error`` -- ``(resize(depth, ref.size()) - ref) * 50``
  (CameraStereoVision.cpp:107-110,118-119), on the GPU.
* ``calculate_average_error`` -- calculateAverageError (functions.cpp:348-354):
  ``cv::mean(image, mask)[0]``, on the GPU.  The reference derives the mask
  from dlib's face detector (``getFaceMask``, absent here), so the caller passes it.

The files are OpenCV ``FileStorage`` YAML, i.e. a ``%YAML:1.0`` header and
``!!opencv-matrix`` nodes with ``rows``, ``cols``, ``dt`` and a flat ``data``
list.  Standard YAML loaders reject that header, so the node is parsed here
directly.  Only host I/O lives here; no compute.
"""
from __future__ import annotations

import math
import re

import numpy as np

# FileStorage element codes <-> numpy
_DT = {"u": np.uint8, "c": np.int8, "w": np.uint16, "s": np.int16, "i": np.int32,
       "f": np.float32, "d": np.float64}
_CODE = {np.dtype(v): k for k, v in _DT.items()}


def _num(tok: str) -> float:
    t = tok.strip()
    low = t.lower()
    if low in (".inf", "+.inf"):
        return math.inf
    if low == "-.inf":
        return -math.inf
    if low == ".nan":
        return math.nan
    return float(t)


def read_matrix(path: str, key: str) -> np.ndarray:
    """``FileStorage(path, READ)[key] >> Mat`` for an ``!!opencv-matrix`` node.
    Multi-channel ``dt`` ("3u") gives shape (rows, cols, channels)."""
    with open(path, "r", encoding="utf-8") as f:
        text = f.read()
    m = re.search(r"^" + re.escape(key) + r"\s*:\s*!!opencv-matrix\s*$", text, re.M)
    if not m:
        raise KeyError(f"{key!r}: no !!opencv-matrix node in {path}")
    body = text[m.end():]
    fields = {}
    for name in ("rows", "cols", "dt"):
        fm = re.search(r"^\s+" + name + r"\s*:\s*(\S+)\s*$", body, re.M)
        if not fm:
            raise ValueError(f"{key!r}: missing {name}")
        fields[name] = fm.group(1)
    dm = re.search(r"^\s+data\s*:\s*\[(.*?)\]", body, re.M | re.S)
    if not dm:
        raise ValueError(f"{key!r}: missing data")
    rows, cols = int(fields["rows"]), int(fields["cols"])
    dt = fields["dt"]
    cn = int(dt[:-1]) if len(dt) > 1 else 1
    if dt[-1] not in _DT:
        raise ValueError(f"{key!r}: unsupported dt {dt!r}")
    toks = [t for t in re.split(r"[,\s]+", dm.group(1)) if t]
    if len(toks) != rows * cols * cn:
        raise ValueError(f"{key!r}: {len(toks)} values for {rows}x{cols}x{cn}")
    vals = np.array([_num(t) for t in toks], dtype=np.float64)
    out = vals.astype(_DT[dt[-1]])
    return out.reshape((rows, cols, cn) if cn > 1 else (rows, cols))


def _fmt(v, is_float: bool) -> str:
    if not is_float:
        return str(int(v))
    v = float(v)
    if math.isnan(v):
        return ".Nan"
    if math.isinf(v):
        return ".Inf" if v > 0 else "-.Inf"
    return repr(v)          # shortest round-trip form


def write_matrix(path: str, key: str, mat: np.ndarray) -> None:
    """``FileStorage(path, WRITE) << key << mat`` (a new file with one node)."""
    a = np.ascontiguousarray(mat)
    if a.dtype not in _CODE:
        raise ValueError(f"unsupported dtype {a.dtype}")
    if a.ndim not in (2, 3):
        raise ValueError("matrix must be 2-D (or 3-D for channels)")
    rows, cols = a.shape[:2]
    cn = a.shape[2] if a.ndim == 3 else 1
    dt = (str(cn) if cn > 1 else "") + _CODE[a.dtype]
    is_float = a.dtype.kind == "f"
    flat = [_fmt(v, is_float) for v in a.reshape(-1)]
    lines = []
    for i in range(0, len(flat), 8):
        lines.append(", ".join(flat[i:i + 8]))
    data = (",\n       ").join(lines)
    with open(path, "w", encoding="utf-8") as f:
        f.write("%YAML:1.0\n---\n")
        f.write(f"{key}: !!opencv-matrix\n   rows: {rows}\n   cols: {cols}\n   dt: {dt}\n")
        f.write(f"   data: [ {data} ]\n")


def get_ideal_ref(path: str = "idealRef.yml") -> np.ndarray:
    """getIdealRef (functions.cpp:323-329)."""
    return read_matrix(path, "R")


def save_image(filename: str, image: np.ndarray) -> None:
    """saveImage (functions.cpp:331-337)."""
    write_matrix(filename, "image", image)


def load_image(filename: str) -> np.ndarray:
    """loadImage (functions.cpp:339-346)."""
    return read_matrix(filename, "image")


def calculate_average_error(ctx, image: np.ndarray, mask=None) -> float:
    """calculateAverageError (functions.cpp:348-354): cv::mean(image, mask)[0]
    on the GPU; ``mask`` replaces dlib's getFaceMask (nullable = all pixels)."""
    return ctx.masked_mean(np.asarray(image, dtype=np.float64), mask)
