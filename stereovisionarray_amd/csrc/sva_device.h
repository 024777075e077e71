// sva_device.h -- CDNA4 (gfx950) device helpers shared by the kernels:
// packed-u16 SIMD types and wave64 DPP cross-lane primitives.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace sva {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned as_u32(u16x2 v) { return __builtin_bit_cast(unsigned, v); }
__device__ __forceinline__ u16x2 as_v2(unsigned v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ u16x2 splat2(unsigned v) {
    return (u16x2){(unsigned short)v, (unsigned short)v};
}
__device__ __forceinline__ u16x2 vmin2(u16x2 a, u16x2 b) { return __builtin_elementwise_min(a, b); }

// DPP control words (GFX9 encoding).
enum : int {
    DPP_QUAD_1032 = 0xb1,       // quad_perm [1,0,3,2]
    DPP_QUAD_2301 = 0x4e,       // quad_perm [2,3,0,1]
    DPP_ROW_SHL1 = 0x101,       // lane i <- lane i+1 within a 16-lane row
    DPP_ROW_SHR1 = 0x111,       // lane i <- lane i-1 within a 16-lane row
    DPP_ROW_MIRROR = 0x140,     // lane i <- lane 15-i
    DPP_ROW_HALF_MIRROR = 0x141 // lane i <- lane 7-i within each half row
};

// Lane i of each 16-lane row receives lane i-1's value; lane 0 receives `edge`.
__device__ __forceinline__ unsigned row_shr1(unsigned v, unsigned edge) {
    return (unsigned)__builtin_amdgcn_update_dpp((int)edge, (int)v, DPP_ROW_SHR1, 0xf, 0xf, false);
}
// Lane i of each 16-lane row receives lane i+1's value; lane 15 receives `edge`.
__device__ __forceinline__ unsigned row_shl1(unsigned v, unsigned edge) {
    return (unsigned)__builtin_amdgcn_update_dpp((int)edge, (int)v, DPP_ROW_SHL1, 0xf, 0xf, false);
}

// Minimum over the 16 lanes of a DPP row, result broadcast to all 16 lanes.
// PIN: keep the last min next to its DPP move (an empty asm on the result), so
// that it folds into one v_min_u32_dpp; unpinned, the compiler may sink it past
// a caller's branch and emit v_mov 0 + v_mov_dpp + v_min.
template <bool PIN = false>
__device__ __forceinline__ unsigned row_min_u32(unsigned v) {
    unsigned x;
    x = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, DPP_QUAD_1032, 0xf, 0xf, false);
    v = v < x ? v : x;
    x = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, DPP_QUAD_2301, 0xf, 0xf, false);
    v = v < x ? v : x;
    x = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_HALF_MIRROR, 0xf, 0xf, false);
    v = v < x ? v : x;
    x = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_MIRROR, 0xf, 0xf, false);
    v = v < x ? v : x;
    if constexpr (PIN) asm("" : "+v"(v));
    return v;
}

// Unpack 4 u8 (one dword) into two u16x2 pairs: (b0,b1) and (b2,b3).
__device__ __forceinline__ void unpack4(unsigned w, unsigned& p01, unsigned& p23) {
    // v_perm_b32 selector: byte k of result = sel byte; 0x0c = zero.
    p01 = __builtin_amdgcn_perm(0u, w, 0x0c010c00u);
    p23 = __builtin_amdgcn_perm(0u, w, 0x0c030c02u);
}
// Pack two u16x2 pairs (values < 256) into one dword of 4 u8.
__device__ __forceinline__ unsigned pack4(unsigned p01, unsigned p23) {
    // result bytes: [p01.b0, p01.b2, p23.b0, p23.b2]; src0 = p23 (bytes 4..7), src1 = p01 (0..3)
    return __builtin_amdgcn_perm(p23, p01, 0x06040200u);
}

// Disparity padding: a frame with D not in {64,128,192,256}
// runs at the next native width Dp with cost 255 at d >= D.  pad_bytes gives
// the byte mask of the dword holding disparities d0 .. d0+3: 0xff in byte b
// when d0 + b >= dreal (OR it into the packed costs).
__device__ __forceinline__ unsigned pad_bytes(int d0, int dreal) {
    const int n = dreal - d0;   // real disparities in this dword
    return n <= 0 ? 0xffffffffu : (n >= 4 ? 0u : 0xffffffffu << (8 * n));
}

// Matched-pixel offset for match distance s >= 0 along the integer baseline
// direction (bx, by): s pixels along the major axis,
// round_half_up(s*m/M) along the minor one, each with its component's sign.
// Same integer expression as oracle svo_step_offset.
__device__ __forceinline__ int2 step_offset(int s, int bx, int by) {
    const int ax = bx < 0 ? -bx : bx, ay = by < 0 ? -by : by;
    const int M = ax > ay ? ax : ay, m = ax > ay ? ay : ax;
    const int minor = (m == 0) ? 0 : (m == M ? s : (2 * s * m + M) / (2 * M));
    const int mx = ax >= ay ? s : minor, my = ax >= ay ? minor : s;
    return make_int2(bx < 0 ? -mx : (bx > 0 ? mx : 0), by < 0 ? -my : (by > 0 ? my : 0));
}

// Sum |a-b| over one 2k-byte row pair.  ND = ceil(2k/4) dwords; `lastmask`
// keeps the valid bytes of the final dword (0xffff when 2k % 4 == 2).
template <int ND>
__device__ __forceinline__ unsigned sad_row(const uint8_t* a, const uint8_t* b, unsigned lastmask,
                                            int nbytes, unsigned acc) {
    const uintptr_t ua = (uintptr_t)a, ub = (uintptr_t)b;
    const unsigned* wa = (const unsigned*)(ua & ~(uintptr_t)3);
    const unsigned* wb = (const unsigned*)(ub & ~(uintptr_t)3);
    const unsigned sa = (unsigned)(ua & 3), sb = (unsigned)(ub & 3);
    // Never touch a dword past the one holding the last valid byte.
    const int la = (int)(((ua + nbytes - 1) & ~(uintptr_t)3) - (ua & ~(uintptr_t)3)) >> 2;
    const int lb = (int)(((ub + nbytes - 1) & ~(uintptr_t)3) - (ub & ~(uintptr_t)3)) >> 2;
    unsigned ra[ND + 1], rb[ND + 1];
#pragma unroll
    for (int j = 0; j <= ND; j++) {
        ra[j] = wa[j < la ? j : la];
        rb[j] = wb[j < lb ? j : lb];
    }
#pragma unroll
    for (int j = 0; j < ND; j++) {
        unsigned oa = __builtin_amdgcn_alignbyte(ra[j + 1], ra[j], sa);
        unsigned ob = __builtin_amdgcn_alignbyte(rb[j + 1], rb[j], sb);
        if (j == ND - 1) { oa &= lastmask; ob &= lastmask; }
        acc = __builtin_amdgcn_sad_u8(oa, ob, acc);
    }
    return acc;
}

// 9x7 Census word in the oracle's bit
// order: element e (row-major over the window, centre skipped) at bit 61 - e,
// bit = neighbour < centre.  rows[0..6] are dword views of image rows y-3..y+3
// whose 9-byte window row starts at byte 4*base + sh.  Each window row is its
// own chain of 8-9 dependent (acc << 1) | sign(n - c) steps (one
// v_sub_u32_sdwa + v_alignbit each); the seven chains are independent and
// are merged with shifts at the end (one 62-long chain stalled on issue).
__device__ __forceinline__ uint64_t census9x7(const unsigned* const* rows, int base, unsigned sh) {
    const unsigned* crow = rows[3];
    const int c = (int)(__builtin_amdgcn_alignbyte(crow[base + 2], crow[base + 1], sh) & 0xff);
    unsigned P[7];
#pragma unroll
    for (int r = 0; r < 7; r++) {
        const unsigned* row = rows[r];
        const unsigned w0 = row[base], w1 = row[base + 1], w2 = row[base + 2];
        const unsigned a[3] = {__builtin_amdgcn_alignbyte(w1, w0, sh),
                               __builtin_amdgcn_alignbyte(w2, w1, sh),
                               __builtin_amdgcn_alignbyte(w2, w2, sh)};
        unsigned acc = 0;
#pragma unroll
        for (int i = 0; i < 9; i++) {
            if (r == 3 && i == 4) continue;
            const int n = (int)((a[i >> 2] >> (8 * (i & 3))) & 0xff);
            acc = __builtin_amdgcn_alignbit(acc, (unsigned)(n - c), 31);
        }
        P[r] = acc;
    }
    // rows start at elements 0, 9, 18, 27 (centre row: 8), 35, 44, 53
    const unsigned lo = (P[6] | (P[5] << 9)) | ((P[4] << 18) | (P[3] << 27));
    const unsigned hi = ((P[3] >> 5) | (P[2] << 3)) | ((P[1] << 12) | (P[0] << 21));
    return ((uint64_t)hi << 32) | lo;
}

}  // namespace sva
