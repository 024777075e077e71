"""The arithmetic of census_cost_mma_kernel, on the
CPU against the oracle: no GPU needed.

The kernel forms every census window's 64 operand bytes straight from the
image bytes with a SWAR byte compare, computes Hamming distances as int8 dot
products on v_mfma_i32_16x16x64_i8, and maps tile rows to disparities so that
each lane's four products are one aligned u8x4 word of the cost volume.
These tests restate those three steps in numpy and check them:
  * the SWAR compare against n < c for all 65,536 byte pairs;
  * the encoding (left b_k = 1 - 2 l_k, b_63 = popcount; right a_k = r_k,
    a_63 = 1; outside a_k = 1 off the centre, a_63 = 2) against
    popcount(CL ^ CR) and the border cost 62 of oracle.cost;
  * the residue-class tile mapping (R = 16 t + 4 q + i, d = R - 4 n, both
    step directions, dmin, 128- and 64-pixel rows) against a full oracle.cost
    row, every disparity written exactly once.
The GPU tests (test_census_cost_gpu.py) prove the kernel's bytes; these pin
the index math it was derived from.
"""
import numpy as np
import pytest

HX, HY = 4, 3


def swar_lt(x, c4):
    """census_bytes' per-byte x < c on packed u32 words: the 0/1 bytes."""
    x = x.astype(np.uint32)
    c4 = c4.astype(np.uint32)
    cH1 = ((c4 | np.uint32(0x80808080)) - np.uint32(0x01010101)).astype(np.uint32)
    t3 = (cH1 - (x & np.uint32(0x7F7F7F7F))).astype(np.uint32)
    m = x ^ c4
    lt = (m & c4) | (~m & t3)
    return (lt >> np.uint32(7)) & np.uint32(0x01010101)


def test_swar_compare_all_byte_pairs():
    n = np.arange(256, dtype=np.uint32)
    c = np.arange(256, dtype=np.uint32)
    N, Cc = np.meshgrid(n, c, indexing="ij")
    N, Cc = N.ravel(), Cc.ravel()
    # four lanes of the word hold (n, n+1, n+2, n+3) mod 256 against one centre
    x = N | ((N + 1) & 255) << 8 | ((N + 2) & 255) << 16 | ((N + 3) & 255) << 24
    c4 = Cc * np.uint32(0x01010101)
    got = swar_lt(x.astype(np.uint32), c4.astype(np.uint32))
    for b in range(4):
        want = (((N + b) & 255) < Cc).astype(np.uint32)
        assert np.array_equal((got >> np.uint32(8 * b)) & np.uint32(1), want), b


def window_bytes(img, x, y):
    """The 63 compare bytes of the kernel's K layout: window row r's columns
    0-7 at 8r .. 8r+7, column 8 at 56 + r (the centre, row 3 column 4, is
    byte 28 and always 0)."""
    c = img[y, x]
    k = np.zeros(64, np.int64)
    for r in range(7):
        for col in range(9):
            n = img[y + r - HY, x + col - HX]
            k[8 * r + col if col < 8 else 56 + r] = 1 if n < c else 0
    return k


def operands(img, W, H, y):
    """A rows (right columns) and B rows (left pixels) as the kernel encodes
    them, for every column of the image row y; outside columns come from
    outside_a()."""
    yin = HY <= y < H - HY
    A = np.zeros((W, 64), np.int64)
    B = np.zeros((W, 64), np.int64)
    for x in range(W):
        if yin and HX <= x < W - HX:
            k = window_bytes(img, x, y)
        else:
            k = np.zeros(64, np.int64)        # census word 0
        A[x, :63] = k[:63]
        A[x, 63] = 1
        B[x, :63] = 1 - 2 * k[:63]
        B[x, 63] = int(k[:63].sum())
    return A, B


def outside_a():
    a = np.ones(64, np.int64)
    a[28] = 0                                 # the centre position
    a[63] = 2
    return a


@pytest.fixture(scope="module")
def frame(oracle):
    rng = np.random.default_rng(7)
    H, W = 12, 200
    L = rng.integers(0, 256, (H, W), dtype=np.uint8)
    L[:, 50:70] = 128                          # flat patch: many equal bytes
    R = np.roll(L, -9, axis=1)
    R[:, ::13] ^= rng.integers(0, 256, (H, (W + 12) // 13), dtype=np.uint8)
    return L, R, oracle.census(L), oracle.census(R)


def popcount64(v):
    v = np.asarray(v, np.uint64)
    return np.array([bin(int(u)).count("1") for u in v.ravel()]).reshape(v.shape)


def test_dot_product_is_hamming(oracle, frame):
    L, R, cl, cr = frame
    H, W = L.shape
    for y in (3, 6, H - 4):
        A, _ = operands(R, W, H, y)
        _, B = operands(L, W, H, y)
        dots = A @ B.T                         # [right column][left pixel]
        ham = popcount64(cr[y][:, None] ^ cl[y][None, :])
        assert np.array_equal(dots, ham)
        # an outside column costs 62 against every pixel
        assert np.array_equal(outside_a() @ B.T, np.full(W, 62))


def mma_row(L, R, y, D, dmin, DIR, PXB):
    """One image row of the cost volume assembled exactly as the kernel's
    MFMA phase does (tile rows, lanes, residue classes, dump of d >= D)."""
    H, W = L.shape
    NC, T = D // 16, (D + 60 + 15) // 16
    A_img, _ = operands(R, W, H, y)
    _, B_img = operands(L, W, H, y)
    out = np.full((W, D), -1, np.int64)
    writes = np.zeros((W, D), np.int64)
    for x0 in range(0, W, PXB):
        xlo = x0 + dmin if DIR > 0 else x0 + 1 - dmin - D
        for c in range(4):                      # wave = residue class
            for s in range(PXB // 64):
                for ln in range(16):
                    m = ln if DIR > 0 else 15 - ln
                    lp = 64 * s + c + 4 * m
                    x = x0 + lp
                    b = B_img[x] if x < W else B_img[0] * 0
                    for tt in range(T):
                        for lq in range(4):
                            j = 4 * tt + lq - ln
                            for i in range(4):
                                Rr = 16 * tt + 4 * lq + i
                                idx = 64 * s + c + Rr if DIR > 0 else 64 * s + c + D + 59 - Rr
                                col = xlo + idx
                                if not 0 <= j < NC * 4 or x >= W:
                                    continue    # dump word / pixel off the image
                                a = A_img[col] if 0 <= col < W else outside_a()
                                out[x, 4 * j + i] = int(a @ b)
                                writes[x, 4 * j + i] += 1
    return out, writes


@pytest.mark.parametrize("D,dmin,DIR,PXB", [(64, 0, -1, 64), (64, 5, 1, 64),
                                            (128, 0, -1, 128), (128, 3, 1, 128)])
def test_tile_mapping_matches_oracle_row(oracle, frame, D, dmin, DIR, PXB):
    L, R, cl, cr = frame
    y = 5
    C = oracle.cost(cl, cr, D, dmin, DIR)
    got, writes = mma_row(L, R, y, D, dmin, DIR, PXB)
    assert (writes == 1).all()                 # every disparity exactly once
    assert np.array_equal(got, C[y].astype(np.int64))
