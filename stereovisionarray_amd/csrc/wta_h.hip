// wta_h.hip -- horizontal-path recompute + path sum + WTA (+ sub-pixel) in one
// launch: the second half of the cost-volume frame pipeline (DESIGN.md §4.6,
// SURVEY.md §8a rows A12-A13).
//
// sgm_paths in checkpoint mode leaves six u8 volumes (the vertical and
// diagonal directions) and, for the two horizontal directions, only the
// L state at every seg-th column.  Here one 16-lane DPP row (the same lane
// layout as the path kernel: lane k owns disparities [k*DPL, k*DPL + DPL))
// owns one row segment of seg pixels (32, or 16 above D = 128) and
//   1. runs the left-to-right recurrence over the segment from the
//      checkpoint at its left edge, keeping L_0 of every pixel in registers
//      (u8-packed, seg x DPL/4 dwords), then
//   2. runs the right-to-left recurrence backwards from the checkpoint at its
//      right edge; at each pixel S = L_1 + L_0 + the six volumes is complete,
//      and the first-minimum WTA (+ parabola) picks d*.
// The recurrences are the path kernel's (sgm_step), started from the exact
// state the path kernel had at the checkpoint column, so every L value and
// therefore S, d* and the sub-pixel value are bit-identical to the 8-volume
// route (tests/test_wta_h_gpu.py).
//
// HBM bytes per disparity: 1 C read (the second pass takes the segment's cost
// words from LDS) + 6 volume reads, against 8 volume reads for wta.hip -- and
// the path kernel writes 6 volumes instead of 8.
#include "sgm_common.h"
#include "wta_common.h"
#include "sva_tuning.h"

namespace sva {
namespace {

using namespace sgm;

constexpr int HB = 256;             // 16 lines: 16 rows of one segment
constexpr int HROWS = HB / 16;

struct WtaHGeom {
    int W, H, D, P1, P2, dmin, ns;
    int dreal;        // disparities of the caller (< D: padded frame)
    unsigned vol;     // bytes of one [H][W][D] volume (< 2^32)
    unsigned ckvol;   // bytes of one checkpoint plane [H][ns][D]
};

// Prefetch depths of the two passes (tune::kWtahPf*).
template <int DPL> constexpr int pf_fwd() { return DPL <= 8 ? tune::kWtahPfFwd : tune::kWtahPfFwdWide; }
template <int DPL> constexpr int pf_bwd() { return DPL <= 8 ? tune::kWtahPfBwd : tune::kWtahPfBwdWide; }
// Cache policy of the six volume loads (their last use): nt above D = 64, so
// the stream does not evict the cost bytes other workgroups are still reading
// (default loads: +9 % at 1080p D=128, +12 % at 4K D=256); at D = 64 the
// default policy is 9 % faster (profiles/r02_v9/ab_wtah_pf.log).
template <int DPL> constexpr int vol_aux() { return DPL <= 4 ? 0 : 2; }

template <int DPL, bool PAD>
__global__ __launch_bounds__(HB) void wta_h_kernel(const uint8_t* __restrict__ C,
                                                   const uint8_t* __restrict__ L6,
                                                   const uint8_t* __restrict__ CK, WtaHGeom g,
                                                   uint16_t* __restrict__ disp,
                                                   float* __restrict__ sub) {
    constexpr int NW = DPL / 4, NP = DPL / 2;
    constexpr int K = 1 << seg_log2<DPL>(), R = K / 16;   // segment, results per lane
    constexpr int PF1 = pf_fwd<DPL>(), PF2 = pf_bwd<DPL>();
    const int s = (int)(blockIdx.x % (unsigned)g.ns);
    const int y = (int)(blockIdx.x / (unsigned)g.ns) * HROWS + (int)(threadIdx.x >> 4);
    const int k = threadIdx.x & 15;
    if (y >= g.H) return;                      // whole 16-lane row leaves together
    const int W = g.W, D = g.D;
    const unsigned P1 = (unsigned)g.P1, P2 = (unsigned)g.P2;
    const int x0 = s * K;
    const int n = W - x0 < K ? W - x0 : K;     // pixels in this segment (uniform)
    const unsigned uD = (unsigned)D;
    const unsigned base = (unsigned)y * (unsigned)W * uD + (unsigned)(k * DPL);   // (0, y)
    const rsrc_t rC = make_rsrc(C, g.vol);
    const rsrc_t rCK0 = make_rsrc(CK, g.ckvol);
    const rsrc_t rCK1 = make_rsrc(CK + g.ckvol, g.ckvol);
    rsrc_t rV[6];
#pragma unroll
    for (int r = 0; r < 6; r++) rV[r] = make_rsrc(L6 + (size_t)r * g.vol, g.vol);
    const unsigned ckrow = (unsigned)y * (unsigned)g.ns;
    // PAD: per pair, 0xffff in the halves of padded disparities (d >= dreal),
    // OR-ed into S so they never win the first-minimum WTA
    unsigned padm[NP];
#pragma unroll
    for (int j = 0; j < NP; j++) {
        const int d = k * DPL + 2 * j;
        padm[j] = PAD ? ((d >= g.dreal ? 0x0000ffffu : 0u) | (d + 1 >= g.dreal ? 0xffff0000u : 0u))
                      : 0u;
    }

    unsigned A[NP], m;
    Edges edges;
    // ---- pass 1: left-to-right (direction 0) over the segment ------------
    if (s > 0) {
        load_state<DPL, PAD>(rCK0, (ckrow + (unsigned)(s - 1)) * uD + (unsigned)(k * DPL), A, m,
                             padm);
    } else {
#pragma unroll
        for (int j = 0; j < NP; j++) A[j] = 0u;   // L(q) = 0, m = 0  =>  L = C
        m = 0u;
    }
    // The forward pass keeps the segment's cost words for the backward pass in
    // LDS, lane-major per (pixel, word) so that accesses are conflict-free:
    // re-reading C instead cost 2-5 % (it came from HBM a second time at D > 128).
    // pixels [0, KL) of the segment keep their cost words in LDS; the rest
    // (read late by the forward pass, early by the backward one) are re-read
    // from global memory, where they are still cached (tune::kWtahLdsPix)
    constexpr int KL = tune::kWtahLdsPix > 0 && tune::kWtahLdsPix < K ? tune::kWtahLdsPix : K;
    __shared__ unsigned cseg[KL * NW * HB];
    const int tid = (int)threadIdx.x;
    unsigned LR[K][NW];
    Words<NW> r1[PF1];
#pragma unroll
    for (int p = 0; p < PF1; p++) r1[p] = bload<NW>(rC, base + (unsigned)(x0 + p) * uD);
    for_seq<K>([&](auto J) {
        constexpr int j = decltype(J)::value;
        constexpr int slot = j % PF1;
        unsigned cw[NW];
#pragma unroll
        for (int w = 0; w < NW; w++) cw[w] = r1[slot].w[w];
#pragma unroll
        for (int w = 0; w < NW; w++)
            if constexpr (j < KL) cseg[(j * NW + w) * HB + tid] = cw[w];
        if (j < n) sgm_step<DPL>(cw, A, m, LR[j], P1, P2, edges);
        if constexpr (j + PF1 < K) {
            __builtin_amdgcn_sched_barrier(0);
            r1[slot] = bload<NW>(rC, base + (unsigned)(x0 + j + PF1) * uD);
            __builtin_amdgcn_sched_barrier(0);
        }
    });

    // ---- pass 2: right-to-left (direction 1), sum, WTA --------------------
    if (x0 + K < W) {
        load_state<DPL, PAD>(rCK1, (ckrow + (unsigned)(s + 1)) * uD + (unsigned)(k * DPL), A, m,
                             padm);
    } else {
#pragma unroll
        for (int j = 0; j < NP; j++) A[j] = 0u;
        m = 0u;
    }
    Words<NW> rv[PF2][6];
    Words<NW> rc[KL < K ? PF2 : 1];
    auto issue = [&](int slot, int j) {
        const unsigned off = base + (unsigned)(x0 + j) * uD;
#pragma unroll
        for (int r = 0; r < 6; r++) rv[slot][r] = bload<NW, vol_aux<DPL>()>(rV[r], off);
        if constexpr (KL < K) {
            if (j >= KL) rc[slot] = bload<NW>(rC, off);
        }
    };
#pragma unroll
    for (int q = 0; q < PF2; q++) issue(q, K - 1 - q);
    // per owned pixel: d* and S(d*-1), S(d*), S(d*+1); the owning lane forms
    // the sub-pixel value after the loop (one division per pixel, not 16)
    unsigned dres[R], sres[R][2];
#pragma unroll
    for (int e = 0; e < R; e++) dres[e] = sres[e][0] = sres[e][1] = 0u;
    const bool want_sub = sub != nullptr;
    for_seq<K>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        constexpr int j = K - 1 - q;
        constexpr int slot = q % PF2;
        if (j < n) {
            unsigned cw[NW], ow[NW];
#pragma unroll
            for (int w = 0; w < NW; w++) {
                if constexpr (j < KL) cw[w] = cseg[(j * NW + w) * HB + tid];
                else cw[w] = rc[KL < K ? slot : 0].w[w];
            }
            sgm_step<DPL>(cw, A, m, ow, P1, P2, edges);
            unsigned S[NP];
#pragma unroll
            for (int p = 0; p < NP; p++) S[p] = A[p];      // L_1 (u16 pairs, < 256)
            unpack_add<NW>(LR[j], S);                        // L_0
#pragma unroll
            for (int r = 0; r < 6; r++) unpack_add<NW>(rv[slot][r].w, S);
            if constexpr (PAD) {
#pragma unroll
                for (int p = 0; p < NP; p++) S[p] |= padm[p];
            }
            unsigned spm, s0;
            const int ds = wta_pick_raw<DPL>(S, k, want_sub, &spm, &s0);
            if (k == j / R) {
                dres[j % R] = (unsigned)ds;
                sres[j % R][0] = spm;
                sres[j % R][1] = s0;
            }
        }
        if constexpr (j - PF2 >= 0) {
            __builtin_amdgcn_sched_barrier(0);
            issue(slot, j - PF2);
            __builtin_amdgcn_sched_barrier(0);
        }
    });
    const size_t row = (size_t)y * (size_t)W;
#pragma unroll
    for (int e = 0; e < R; e++) {
        const int x = x0 + k * R + e;
        if (x < W) {
            disp[row + x] = (uint16_t)(g.dmin + (int)dres[e]);
            if (want_sub)
                sub[row + x] = subpixel(g.dmin, (int)dres[e], g.dreal, sres[e][0] & 0xffffu, sres[e][1],
                                        sres[e][0] >> 16);
        }
    }
}

}  // namespace

bool wta_h_supported(int D) { return D == 64 || D == 128 || D == 192 || D == 256; }

hipError_t launch_wta_h(Ctx& c, const uint8_t* C, const uint8_t* L6, const uint8_t* CK, int W,
                        int H, int D, int P1, int P2, int dmin, uint16_t* disp, float* sub,
                        int dreal) {
    ScopedKernelTimer t(c, "wta_h");
    WtaHGeom g;
    g.W = W; g.H = H; g.D = D; g.P1 = P1; g.P2 = P2; g.dmin = dmin;
    g.dreal = dreal > 0 && dreal < D ? dreal : D;
    const bool pad = g.dreal < D;
    g.ns = ckpt_segments(W, D);
    const size_t vol = (size_t)W * H * D;
    if (vol >= (size_t)1 << 32) return hipErrorInvalidValue;
    g.vol = (unsigned)vol;
    g.ckvol = (unsigned)((size_t)H * g.ns * D);
    const dim3 grid((unsigned)(g.ns * ((H + HROWS - 1) / HROWS)));
#define SVA_WTAH(DPL_)                                                                          \
    if (pad)                                                                                    \
        hipLaunchKernelGGL((wta_h_kernel<DPL_, true>), grid, dim3(HB), 0, c.stream, C, L6, CK,  \
                           g, disp, sub);                                                       \
    else                                                                                        \
        hipLaunchKernelGGL((wta_h_kernel<DPL_, false>), grid, dim3(HB), 0, c.stream, C, L6, CK, \
                           g, disp, sub)
    switch (D) {
        case 64: SVA_WTAH(4); break;
        case 128: SVA_WTAH(8); break;
        case 192: SVA_WTAH(12); break;
        case 256: SVA_WTAH(16); break;
        default: return hipErrorInvalidValue;
    }
#undef SVA_WTAH
    return hipGetLastError();
}

}  // namespace sva
