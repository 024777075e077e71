"""The index math of census_cost2_mma_kernel (csrc/census_cost2.hip,
DESIGN.md §4.2b) restated in numpy and checked against the oracle's 2-D cost
(oracle.cost2 over oracle.census): no GPU needed.

The kernel walks lattice lines q0 + r*v of a 2-D array step, stages the image
around 8 adjacent lines into two sheared LDS patches, reads every census
window from them at a per-row byte offset, and maps MFMA tile rows to path
positions so that each lane's four products are one aligned u8x4 word of the
cost volume.  This test mirrors the kernel's integer expressions one for one
-- the patch staging, the window addresses (a0 + r * rowstep), the slot <->
pixel map, the tile-row <-> path map and the word index -- and rebuilds the
whole cost volume from them, with every write counted.  Hamming distances are
taken from the census bits the emulated windows yield (the dot-product
identity itself is pinned in test_mfma_hamming_cpu.py).

Mirrored constants: LINE 64, XB = tune::kCensusCost2Lines (8), CC2Geom.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as oracle  # noqa: E402

LINE, XB, BLOCK = 64, 8, 256


def reduce_step(sx, sy):
    a, b = abs(sx), abs(sy)
    while b:
        a, b = b, a % b
    return sx // a, sy // a


def supported(D, sx, sy):
    if D not in (64, 128, 192, 256) or sy == 0:
        return False
    bx, by = reduce_step(sx, sy)
    return abs(by) == 1 and abs(bx) <= 3


def geom(NC, M):
    D = NC * 16
    K = 1 if M % 4 == 0 else (2 if M % 2 == 0 else 4)
    KM, S = K * M, 4 // K
    T = (15 * KM + D + 15) // 16
    NT = (LINE - 1) * M + D
    NA = M * (K - 1) + 16 * KM * (S - 1) + 16 * T
    NAP = (NA + 15) // 16 * 16
    HALF = (M + 1) // 2
    E = 3 * M + HALF + 4
    PW0 = (XB + 11 + 6 * M + 2 * HALF + 3) // 4 * 4
    PW = PW0 if (PW0 // 4) % 2 else PW0 + 4
    LR, RR = LINE + 6, (NT + M - 1) // M + 8
    return dict(D=D, K=K, KM=KM, S=S, T=T, NT=NT, NAP=NAP, E=E, PW=PW, LR=LR, RR=RR)


def cdiv(a, b):          # C integer division (truncation toward zero)
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def census_from_patch(pat, a0, rowstep, cx_ok):
    """The 62-bit census word of each window read at byte offsets
    a0 + r * rowstep (r = 0..6) + 0..8 of the flat patch, as the kernel's
    census_bytes_at reads it: bit order dy-major, dx-minor, centre skipped
    (the Hamming distance does not depend on the order, only on both sides
    sharing it).  Windows with cx_ok False get word 0."""
    rows = a0[:, None] + np.arange(7)[None, :] * rowstep          # [n][7]
    addr = rows[:, :, None] + np.arange(9)[None, None, :]         # [n][7][9]
    if cx_ok.any():
        a = addr[cx_ok]
        assert a.min() >= 0 and a.max() < pat.size - 16, "window read outside the patch"
    win = pat[np.where(cx_ok[:, None, None], addr, 0)].astype(np.int32)
    c = win[:, 3, 4][:, None, None]
    bits = (win < c).reshape(len(a0), 63)
    bits = np.delete(bits, 31, axis=1)                            # the centre
    words = (bits.astype(np.uint64) << np.arange(61, -1, -1, dtype=np.uint64)).sum(axis=1)
    return np.where(cx_ok, words, np.uint64(0)).astype(np.uint64)


def popcount64(v):
    v = v.copy()
    c = np.zeros(v.shape, np.int64)
    while np.any(v):
        c += (v & np.uint64(1)).astype(np.int64)
        v >>= np.uint64(1)
    return c


def emulate(left, right, D, dmin, sx, sy):
    """The cost volume census_cost2_mma_kernel writes, and per-pixel write counts."""
    H, W = left.shape
    NC = D // 16
    bx, by = reduce_step(sx, sy)
    abx = abs(bx)
    M = max(abx, 1)
    g = geom(NC, M)
    K, KM, S, T, NT, NAP, E, PW, LR, RR = (g[k] for k in
                                           ("K", "KM", "S", "T", "NT", "NAP", "E", "PW", "LR", "RR"))
    ngroups = (W + (LINE - 1) * abx + XB - 1) // XB
    nchunks = (H + LINE - 1) // LINE
    sgx = (bx > 0) - (bx < 0)
    bt = (lambda u: u) if M == 1 else (lambda u: cdiv(2 * u + M, 2 * M))
    rowstep = by * PW - bx * by
    C = np.full((H, W, D), 0, np.int64)
    writes = np.zeros((H, W, D), np.int64)

    # tile mapping of one line: (wave w, tile tt, quarter lq, lane ln, e)
    w_, tt_, lq_, ln_, e_ = np.meshgrid(np.arange(4), np.arange(T), np.arange(4), np.arange(16),
                                        np.arange(4), indexing="ij")
    c_, sp_ = w_ // S, w_ % S
    idx_ = M * c_ + 16 * KM * sp_ + 16 * tt_ + 4 * lq_ + e_        # operand row of tile row
    assert idx_.max() < NAP
    jw_ = 4 * tt_ + lq_ - (KM // 4) * ln_
    slot_ = 16 * w_ + ln_
    keep = (jw_ >= 0) & (jw_ < NC * 4)
    idx_k, jw_k, slot_k, e_k = idx_[keep], jw_[keep], slot_[keep], e_[keep]

    def slot_r(b):
        w, n = b >> 4, b & 15
        return w // S + K * n + 16 * K * (w % S)

    slots = np.arange(LINE)
    r_of = slot_r(slots)
    assert sorted(r_of) == list(range(LINE))
    for blk in range(ngroups * nchunks):
        gi, h = blk % ngroups, blk // ngroups
        Y0 = LINE * h if by > 0 else H - 1 - LINE * h
        X0 = gi * XB - (LINE - 1) * max(bx, 0)
        rhoR0 = bt(dmin) - 3
        # ---- staging: flat patch [left LR | right RR][PW]
        pat = np.zeros((LR + RR) * PW + 16, np.uint8)
        i = np.arange((LR + RR) * PW)
        isR = i >= LR * PW
        q = np.where(isR, i - LR * PW, i)
        pr, cb = q // PW, q % PW
        rho = np.where(isR, rhoR0 + pr, pr - 3)
        yy, xx = Y0 + by * rho, X0 + bx * rho - E + cb
        ok = (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)
        src = np.where(isR, right[np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1)],
                       left[np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1)])
        pat[i] = np.where(ok, src, 0)
        patL, patR = pat, pat[LR * PW:]
        for j in range(XB):
            # left pixels of line j (slot order)
            x = X0 + j + bx * r_of
            y = Y0 + by * r_of
            inner = (y >= 3) & (y < H - 3) & (x >= 4) & (x < W - 4)
            a0 = (r_of - 3 * by + 3) * PW + j - 4 + E + 3 * bx * by
            a0 = np.where(inner, a0, 0)
            cl = census_from_patch(patL, a0, rowstep, inner)
            # path pixels t = dmin + i
            ii = np.arange(NT)
            u = dmin + ii
            b = np.array([bt(int(v)) for v in u])
            px, py = X0 + j + sgx * u, Y0 + by * b
            outside = (px < 0) | (px >= W) | (py < 0) | (py >= H)
            innerR = ~outside & (py >= 3) & (py < H - 3) & (px >= 4) & (px < W - 4)
            a0R = (b - 3 * by - rhoR0) * PW + j + sgx * u - bx * b - 4 + E + 3 * bx * by
            a0R = np.where(innerR, a0R, 0)
            cr = census_from_patch(patR, a0R, rowstep, innerR)
            crp = np.zeros(NAP, np.uint64)
            crp[:NT] = cr
            outp = np.zeros(NAP, bool)
            outp[:NT] = outside
            # rows >= NT are uninitialised LDS in the kernel: they must only feed dumps
            assert idx_k.max() < NT
            ham = popcount64(cl[slot_k] ^ crp[idx_k])
            val = np.where(outp[idx_k], 62, ham)
            pxl, pyl = x[slot_k], y[slot_k]
            st = (pxl >= 0) & (pxl < W) & (pyl >= 0) & (pyl < H)
            d = 4 * jw_k + e_k
            np.add.at(writes, (pyl[st], pxl[st], d[st]), 1)
            C[pyl[st], pxl[st], d[st]] = val[st]
    return C, writes


CASES = [
    # (H, W, D, dmin, sx, sy)
    (37, 29, 64, 0, 0, 1),
    (37, 29, 64, 3, 0, -1),
    (70, 41, 64, 0, 1, 1),
    (70, 41, 64, 2, -1, 1),
    (45, 52, 64, 0, 1, -1),
    (45, 52, 64, 1, -1, -1),
    (33, 60, 64, 0, 2, 1),
    (33, 60, 64, 5, -2, -1),
    (33, 60, 64, 0, 4, -2),         # non-primitive (2, -1)
    (29, 75, 64, 0, 3, 1),
    (29, 75, 64, 4, -3, 1),
    (29, 75, 64, 0, 3, -1),
    (20, 26, 128, 0, 1, -1),
    (20, 26, 128, 7, -2, 1),
    (66, 17, 64, 90, 0, 1),         # dmin past the image
]


@pytest.mark.parametrize("H,W,D,dmin,sx,sy", CASES)
def test_emulated_kernel_matches_oracle_cost2(H, W, D, dmin, sx, sy):
    rng = np.random.default_rng(H * 1000 + W + sx * 7 + sy)
    L = rng.integers(0, 256, (H, W), dtype=np.uint8)
    R = rng.integers(0, 256, (H, W), dtype=np.uint8)
    R[::3] = L[::3]                        # some equal bytes (ties in the compare)
    assert supported(D, sx, sy)
    C, writes = emulate(L, R, D, dmin, sx, sy)
    assert writes.min() == 1 and writes.max() == 1, "every (pixel, d) written exactly once"
    want = oracle.cost2(oracle.census(L), oracle.census(R), D, dmin, sx, sy)
    assert np.array_equal(C.astype(np.uint8), want)


def test_supported_steps():
    """The rig steps of getCameraPairs (5x5: unit steps) and of the 2x4 grid
    of config 4 ((k, 1) for k <= 3, vertical) take the matrix-core kernel;
    steps with |by| > 1 after reduction keep the census-word route."""
    for s in [(0, 1), (0, -1), (1, 1), (-1, -1), (1, -1), (-1, 1), (2, 1), (-2, -1), (3, 1),
              (-3, 1), (3, -1), (4, 2), (0, 3), (6, -2)]:
        assert supported(128, *s), s
    for s in [(1, 2), (2, 3), (1, 0), (-1, 0), (4, 1), (1, -2), (0, 0) if False else (5, 1)]:
        assert not supported(128, *s), s
    assert not supported(100, 0, 1)
