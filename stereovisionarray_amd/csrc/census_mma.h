// census_mma.h -- the census windows as i8 MFMA operand bytes, shared by the
// 1-D census + cost kernel (census_cost.hip) and the 2-D array-step one
// (census_cost2.hip).  DESIGN.md §4.2; SURVEY.md §8a rows A10 + A11.
#pragma once

#include "sva_device.h"

namespace sva {

// ---- the Hamming costs on the matrix cores --------------------------------
// popcount(l ^ r) over the 62 census bits is one integer dot product of
// K = 64 bytes: with the left word as b_k = 1 - 2 l_k (plus b_63 = popcount(l))
// and the right word as a_k = r_k (plus a_63 = 1),
//   sum_k a_k b_k = sum r - 2 sum l r + sum l = popcount(l ^ r).
// A right column outside the image takes a_k = 1 on its 62 census positions
// (0 at the window centre's, which is 0 in every left word too) and a_63 = 2:
// 62 - 2 popcount(l) + 2 popcount(l) = 62, the reference's border cost.  The
// bit order inside K is free (a sum), as long as both operands share it
// (tests/test_mfma_hamming_cpu.py restates all of this against the oracle).
typedef int v4i __attribute__((ext_vector_type(4)));

// K layout: dwords 2r, 2r+1 = window row r's bytes 0-3, 4-7; dword 14 = byte 8
// of rows 0-3, dword 15 = byte 8 of rows 4-6 and the bias.  d[0..13] hold the
// window bytes on entry and a8[r] has window row r's byte 8 in its byte 0.
// The centre compares with itself (0 in every word), so K holds the 62 census
// bits plus one position that is 0 on both sides.
//   PM false (right pixel, A): byte k = (n_k < c), bias 1;
//   PM true  (left pixel, B):  byte k = 1 - 2 (n_k < c), bias = popcount.
template <bool PM>
__device__ __forceinline__ void census_swar(unsigned (&d)[16], const unsigned (&a8)[7]) {
    const unsigned c4 = __builtin_amdgcn_perm(0u, d[7], 0u);  // the centre in all 4 bytes
    d[14] = __builtin_amdgcn_perm(a8[1], a8[0], 0x0c0c0400u) | __builtin_amdgcn_perm(a8[3], a8[2], 0x04000c0cu);
    d[15] = __builtin_amdgcn_perm(a8[5], a8[4], 0x0c0c0400u) | ((a8[6] & 0xffu) << 16);
    // per byte x < c: where the top bits differ, c's top bit; else the low 7
    // bits' borrow, (c7 | 0x80) - 1 - x7 (no byte borrows into the next)
    const unsigned cH1 = (c4 | 0x80808080u) - 0x01010101u;
    unsigned sum = 0;
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const unsigned x = d[q];
        const unsigned t3 = cH1 - (x & 0x7f7f7f7fu);
        const unsigned m = x ^ c4;
        const unsigned lt = (m & c4) | (~m & t3);            // v_bfi_b32: top bit = x < c
        const unsigned b01 = (lt >> 7) & 0x01010101u;
        if constexpr (PM) {
            sum += q < 15 ? b01 : (b01 & 0x00ffffffu);     // bytes <= 16: no carry
            d[q] = __builtin_amdgcn_perm(0x0000ff01u, 0u, b01 | 0x04040404u);
        } else {
            d[q] = b01;
        }
    }
    if constexpr (PM) {
        const unsigned pc = __builtin_amdgcn_sad_u8(sum, 0u, 0u);   // byte sum
        d[15] = (d[15] & 0x00ffffffu) | (pc << 24);
    } else {
        d[15] = (d[15] & 0x00ffffffu) | 0x01000000u;
    }
}

// The 64 operand bytes of one census window straight from the image bytes
// (no census word in between), 4 comparisons per SWAR step.  rows[0..6] are
// dword views of ring rows y-3 .. y+3 and the 9-byte window row starts at
// byte s of each.
template <bool PM>
__device__ __forceinline__ void census_bytes(const unsigned* const* rows, int s, unsigned (&d)[16]) {
    const int base = s >> 2;
    const unsigned sh = (unsigned)(s & 3);
    unsigned a8[7];
#pragma unroll
    for (int r = 0; r < 7; r++) {
        const unsigned* row = rows[r];
        const unsigned w0 = row[base], w1 = row[base + 1], w2 = row[base + 2];
        d[2 * r] = __builtin_amdgcn_alignbyte(w1, w0, sh);
        d[2 * r + 1] = __builtin_amdgcn_alignbyte(w2, w1, sh);
        a8[r] = __builtin_amdgcn_alignbyte(w2, w2, sh);     // byte 0 = window byte 8
    }
    census_swar<PM>(d, a8);
}

// The same from a sheared LDS patch: window row r (image row y - 3 + r) starts
// at byte a0 + r * rowstep of `patch` (4-byte aligned), so every row may start
// at its own byte offset (census_cost2.hip stages the image along the step).
template <bool PM>
__device__ __forceinline__ void census_bytes_at(const uint8_t* patch, int a0, int rowstep,
                                                unsigned (&d)[16]) {
    unsigned a8[7];
#pragma unroll
    for (int r = 0; r < 7; r++) {
        const int a = a0 + r * rowstep;
        const unsigned* row = reinterpret_cast<const unsigned*>(patch) + (a >> 2);
        const unsigned sh = (unsigned)(a & 3);
        const unsigned w0 = row[0], w1 = row[1], w2 = row[2];
        d[2 * r] = __builtin_amdgcn_alignbyte(w1, w0, sh);
        d[2 * r + 1] = __builtin_amdgcn_alignbyte(w2, w1, sh);
        a8[r] = __builtin_amdgcn_alignbyte(w2, w2, sh);
    }
    census_swar<PM>(d, a8);
}

// Operand of a census word 0 (a window that leaves the image), as the left
// pixel (B: b_k = 1, b_63 = popcount 0) or the right pixel (A: a_k = 0, a_63 = 1).
template <bool PM>
__device__ __forceinline__ void census_zero(unsigned (&d)[16]) {
#pragma unroll
    for (int q = 0; q < 15; q++) d[q] = PM ? 0x01010101u : 0u;
    d[15] = PM ? 0x00010101u : 0x01000000u;
}

// Operand of a right pixel outside the image: a_k = 1 on the 62 census
// positions (not the centre, dword 7 byte 0), a_63 = 2 -> cost 62.
__device__ __forceinline__ void census_outside(unsigned (&d)[16]) {
#pragma unroll
    for (int q = 0; q < 15; q++) d[q] = 0x01010101u;
    d[7] = 0x01010100u;
    d[15] = 0x02010101u;
}

// Store one operand row as four 16-byte K-quarter planes: op[(q4 * nrow + row) * 16].
__device__ __forceinline__ void put_operand_row(uint8_t* op, int nrow, int row, const unsigned (&d)[16]) {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int q4 = 0; q4 < 4; q4++)
        *reinterpret_cast<v4u*>(&op[(q4 * nrow + row) * 16]) =
            (v4u){d[4 * q4], d[4 * q4 + 1], d[4 * q4 + 2], d[4 * q4 + 3]};
}

}  // namespace sva
