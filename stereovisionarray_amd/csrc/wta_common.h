// wta_common.h -- first-minimum WTA + parabola sub-pixel on one 16-lane DPP
// row, shared by wta.hip and wta_hv.hip.
//
// Lane k holds S(d) for d in [k*DPL, k*DPL + DPL) as DPL/2 packed u16 pairs:
// pair j = (d0 + 2j, d0 + 2j + 1), or with SPLIT (the recurrence state's
// layout under tune::kSplitPairs, sgm_common.h) (d0 + j, d0 + j + DPL/2).  The first minimum is a u32 min over keys (S << 16 | d):
// the smaller d wins ties, mirroring std::min_element at
// CameraStereoVision.cpp:85.  S(d*-1), S(d*+1) come from a DPP OR-reduce.
#pragma once

#include "sva_device.h"

namespace sva {

__device__ __forceinline__ unsigned row_or_u32(unsigned v) {
    v |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, DPP_QUAD_1032, 0xf, 0xf, false);
    v |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, DPP_QUAD_2301, 0xf, 0xf, false);
    v |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_HALF_MIRROR, 0xf, 0xf, false);
    v |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_MIRROR, 0xf, 0xf, false);
    return v;
}

// The parabola through S(d*-1), S(d*), S(d*+1), in f32:
// dmin + d* (+ (a - c) / (2 (a - 2b + c)) when 0 < d* < D-1 and the
// denominator is positive).
__device__ __forceinline__ float subpixel(int dmin, int ds, int D, unsigned a, unsigned b,
                                          unsigned c) {
    float r = (float)(dmin + ds);
    if (ds > 0 && ds < D - 1) {
        const int den = (int)a - 2 * (int)b + (int)c;
        if (den > 0) r = r + (float)((int)a - (int)c) / (float)(2 * den);
    }
    return r;
}

// First-minimum WTA on the row: returns d* (0-based, the same in all 16
// lanes) and, when want_sub, S(d*-1) | S(d*+1) << 16 in *spm and S(d*) in
// *s0 (all lanes; a neighbour outside [0, D) reads 0, unused by subpixel()).
// d*-1 and d*+1 have the same parity, so they sit in the same half of two
// adjacent pairs: each lane selects pair q = (d*-1-d0) >> 1 and q + 1 of
// its own (zero outside the lane) and one v_perm packs the two halves; a
// single DPP OR-reduction then gathers both values.
template <int DPL, bool PIN = false, bool SPLIT = false>
__device__ __forceinline__ int wta_pick_raw(const unsigned (&S)[DPL / 2], int k, bool want_sub,
                                            unsigned* spm, unsigned* s0) {
    constexpr int NP = DPL / 2;
    const int d0 = k * DPL;
    unsigned best = 0xffffffffu;
#pragma unroll
    for (int j = 0; j < NP; j++) {
        const unsigned dl = (unsigned)(d0 + (SPLIT ? j : 2 * j)), dh = (unsigned)(d0 + (SPLIT ? j + NP : 2 * j + 1));
        const unsigned lo = ((S[j] & 0xffffu) << 16) | dl;
        const unsigned hi = (S[j] & 0xffff0000u) | dh;
        best = best < lo ? best : lo;
        best = best < hi ? best : hi;
    }
    best = row_min_u32<PIN>(best);
    const int ds = (int)(best & 0xffffu);
    if (want_sub) {
        const int im = ds - 1 - d0;             // local index of d*-1 (may leave the lane)
        if constexpr (SPLIT) {
            // split pairs (j, j + NP): select each neighbour's half on its own
            unsigned vm = 0, vp = 0;
#pragma unroll
            for (int j = 0; j < NP; j++) {
                vm = im == j ? S[j] & 0xffffu : (im == j + NP ? S[j] >> 16 : vm);
                vp = im + 2 == j ? S[j] & 0xffffu : (im + 2 == j + NP ? S[j] >> 16 : vp);
            }
            *spm = row_or_u32(vm | (vp << 16));
        } else {
            const int q = im >> 1;              // arithmetic shift: -1 for im in {-2, -1}
            unsigned pm = 0, pp = 0;
#pragma unroll
            for (int j = 0; j < NP; j++) {
                pm = (q == j) ? S[j] : pm;
                pp = (q == j - 1) ? S[j] : pp;
            }
            const unsigned sel = (im & 1) ? 0x07060302u : 0x05040100u;
            *spm = row_or_u32(__builtin_amdgcn_perm(pp, pm, sel));
        }
        *s0 = best >> 16;
    }
    return ds;
}

// The first-minimum key of the row, (S(d*) << 16) | d*, in all 16 lanes.
template <int DPL, bool PIN = false, bool SPLIT = false>
__device__ __forceinline__ unsigned wta_pick_key(const unsigned (&S)[DPL / 2], int k) {
    constexpr int NP = DPL / 2;
    const int d0 = k * DPL;
    unsigned best = 0xffffffffu;
#pragma unroll
    for (int j = 0; j < NP; j++) {
        const unsigned dl = (unsigned)(d0 + (SPLIT ? j : 2 * j)), dh = (unsigned)(d0 + (SPLIT ? j + NP : 2 * j + 1));
        const unsigned lo = ((S[j] & 0xffffu) << 16) | dl;
        const unsigned hi = (S[j] & 0xffff0000u) | dh;
        best = best < lo ? best : lo;
        best = best < hi ? best : hi;
    }
    return row_min_u32<PIN>(best);
}

// The same key with each pair's two keys formed by one v_perm each: dpair[j]
// holds the pair's disparities (its low | high half's d << 16), so the key of
// the low half is [dpair.lo16 | S.lo16 << 16] and of the high half
// [dpair.hi16 | S.hi16 << 16]: 2 VALU per pair where the shift/mask + or
// forms took 4.
template <int DPL, bool PIN = false>
__device__ __forceinline__ unsigned wta_pick_key_perm(const unsigned (&S)[DPL / 2],
                                                      const unsigned (&dpair)[DPL / 2]) {
    constexpr int NP = DPL / 2;
    unsigned key[2 * NP];
#pragma unroll
    for (int j = 0; j < NP; j++) {
        key[2 * j] = __builtin_amdgcn_perm(S[j], dpair[j], 0x05040100u);
        key[2 * j + 1] = __builtin_amdgcn_perm(S[j], dpair[j], 0x07060302u);
    }
    unsigned best = key[0];
#pragma unroll
    for (int i = 1; i < 2 * NP; i++) best = best < key[i] ? best : key[i];
    return row_min_u32<PIN>(best);
}

// Returns d* (0-based, the same in all 16 lanes of the row) and, when
// want_sub, the f32 sub-pixel disparity dmin + d* (+ parabola offset) in *v.
template <int DPL>
__device__ __forceinline__ int wta_pick(const unsigned (&S)[DPL / 2], int k, int D, int dmin,
                                        bool want_sub, float* v) {
    unsigned spm = 0, b = 0;
    const int ds = wta_pick_raw<DPL>(S, k, want_sub, &spm, &b);
    *v = want_sub ? subpixel(dmin, ds, D, spm & 0xffffu, b, spm >> 16) : (float)(dmin + ds);
    return ds;
}

}  // namespace sva
