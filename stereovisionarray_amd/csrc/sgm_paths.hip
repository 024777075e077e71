// sgm_paths.hip -- 8-direction SGM path aggregation (DESIGN.md §2.3 / §4.3,
// SURVEY.md §8a row A12).  All eight directions run in ONE launch.
//
//   L_r(p,d) = C(p,d) + min(L_r(q,d), L_r(q,d-1)+P1, L_r(q,d+1)+P1, m+P2) - m
//   m = min_k L_r(q,k),  q = p - r;  L_r(p,d) = C(p,d) where q leaves the image.
//
// Mapping (CDNA4, wave64):
//   * A path LINE is owned by one 16-lane DPP row; lane k holds disparities
//     [k*DPL, k*DPL + DPL) as DPL/2 packed u16 pairs, so every per-disparity
//     op is one v_pk_* for two disparities.
//   * The d-1 / d+1 neighbours are v_alignbit within the lane plus one DPP
//     row_shr:1 / row_shl:1 across lanes (INF fed in at the row edges).
//   * min_k L is a lane-local v_pk_min tree + a 4-step DPP row reduction
//     (quad_perm, half-mirror, mirror) that leaves the minimum in all 16
//     lanes -- no LDS, no barrier.  The state carried to the next pixel is
//     normalised, B = L - min_k L, so m + P2 becomes the constant P2.
//   * A wave carries 4 lines, a 256-thread workgroup 16 lines of one
//     direction.  Vertical lines: consecutive x; diagonal lines: consecutive
//     (x - y) mod W, so the 4 pixels a wave touches per step are adjacent in
//     memory (one 4*D-byte span); horizontal lines: 4 rows, one D-byte span
//     each.  Diagonals use the wrap-around trick: line i visits
//     ((i + rx*t) mod W, t) and restarts (L = C) where x wraps, so every line
//     has exactly H steps and no lane idles on ragged diagonal lengths.
//   * Cost bytes are prefetched PF steps ahead into a register ring (the
//     loads do not depend on the recurrence), hiding HBM latency behind the
//     dependent DPP chain of the current step.
// HBM bytes per disparity: 8 C reads (1 B each, one per direction) + 8 L
// writes (u8 per direction volume, [8][H][W][D]).
#include "sgm_common.h"

#include <cstdlib>

namespace sva {
namespace {

using namespace sgm;

constexpr int PATH_BLOCK = 256;
constexpr int LINES_PER_BLOCK = PATH_BLOCK / 16;
// Prefetch depth in steps, per line kind.  Horizontal lines are the longest
// (W steps) and few (2H lines): once the vertical/diagonal lines drain they
// run alone and latency-bound, so they get a deeper ring (their next steps
// are contiguous bytes, and VGPRs are not what limits occupancy here: the
// grid has ~3.3 waves per SIMD at 1080p).
// Measured in-process A/B (tools/ab_paths.py, 1080p D=128, same buffers,
// alternating builds): PF_H/PF_V 8/8 0.755-0.788 ms; 32/8 0.665; 32/12 0.661;
// 28/8 0.664; 40/8 0.689 (181 VGPRs -> 2 waves/SIMD); 32/4 0.770.  Part of the
// gain is the occupancy cap itself: 149 VGPRs -> 3 waves/SIMD, and 8/8 with
// LDS forcing 3 workgroups/CU is 0.730 vs 0.788 -- fewer concurrent line
// streams, better DRAM locality.
// Per disparities-per-lane (D = 16*DPL) overrides: SVA_PF_H<DPL>/SVA_PF_V<DPL>.
// Chosen by the same in-process A/B: D=64 (1080p) 40/12 0.372 ms vs 8/8 0.416;
// D=192 24/8 0.996 vs 12/8 1.154; D=256 (4K) 12/8 stays best (16/8 equal,
// 20/8 and 12/12 +3 %).
#ifndef SVA_PF_H4
#define SVA_PF_H4 40
#endif
#ifndef SVA_PF_V4
#define SVA_PF_V4 12
#endif
#ifndef SVA_PF_H8
#define SVA_PF_H8 32
#endif
#ifndef SVA_PF_V8
#define SVA_PF_V8 12
#endif
#ifndef SVA_PF_H12
#define SVA_PF_H12 24
#endif
#ifndef SVA_PF_V12
#define SVA_PF_V12 8
#endif
#ifndef SVA_PF_H16
#define SVA_PF_H16 12
#endif
#ifndef SVA_PF_V16
#define SVA_PF_V16 8
#endif
template <int DPL> constexpr int pf_h() {
    return DPL == 4 ? SVA_PF_H4 : DPL == 8 ? SVA_PF_H8 : DPL == 12 ? SVA_PF_H12 : SVA_PF_H16;
}
template <int DPL> constexpr int pf_v() {
    return DPL == 4 ? SVA_PF_V4 : DPL == 8 ? SVA_PF_V8 : DPL == 12 ? SVA_PF_V12 : SVA_PF_V16;
}
template <int DPL, bool DIAG, int VAR, int PF>
__device__ __forceinline__ void path_line(rsrc_t rC, rsrc_t rL, const PathGeom& g, int rx, int ry,
                                          int line, int k) {
    constexpr int NW = DPL / 4, NP = DPL / 2;
    const int W = g.W, H = g.H, D = g.D;
    const unsigned P1 = (unsigned)g.P1, P2 = (unsigned)g.P2;
    const int steps = ry == 0 ? W : H;
    const unsigned WD = (unsigned)W * (unsigned)D;
    const unsigned stride = (unsigned)((ry * W + rx) * D);
    int x0, y0;
    if (ry == 0) { y0 = line; x0 = rx > 0 ? 0 : W - 1; }
    else { y0 = ry > 0 ? 0 : H - 1; x0 = line; }
    Cursor<DIAG> cc;
    cc.x = x0;
    cc.off = ((unsigned)y0 * (unsigned)W + (unsigned)x0) * (unsigned)D + (unsigned)(k * DPL);
    // Prefetch cursor: runs PF steps ahead and may run past the line's end;
    // those loads land in-range garbage or, past the volume, the buffer range
    // check returns 0 -- never consumed either way.
    Cursor<DIAG> pc = cc;

    unsigned A[NP];
#pragma unroll
    for (int j = 0; j < NP; j++) A[j] = 0u;   // L(q) = 0, m = 0  =>  L = C
    unsigned m = 0u;

    Words<NW> ring[PF];
#pragma unroll
    for (int p = 0; p < PF; p++) {
        if constexpr (VAR == 3 || VAR == 4) {
#pragma unroll
            for (int w = 0; w < NW; w++) ring[p].w[w] = (0x05030201u * (unsigned)(p + 1) + (unsigned)k) & 0x1f1f1f1fu;
        } else {
            ring[p] = bload<NW>(rC, pc.off);
        }
        pc.advance(rx, stride, W, WD);
    }

    // One step consumes ring slot p in place (loaded PF steps ago) and only
    // then refills that slot with the load for step t+PF, so the old and new
    // values never overlap and the slot keeps its registers: no copies, and
    // every wait is for a load issued ~PF steps earlier.  (Refilling first
    // made hipcc copy the whole ring at the loop head behind vmcnt(1..3).)
    auto step = [&](int p, bool refill) {
        unsigned cw[NW];
#pragma unroll
        for (int w = 0; w < NW; w++) cw[w] = ring[p].w[w];
        unsigned ow[NW];
        sgm_step<DPL>(cw, A, m, ow, P1, P2);
        bstore<NW, VAR>(rL, cc.off, ow, g.store_aux);
        const bool wrapped = cc.advance(rx, stride, W, WD);
        if constexpr (DIAG) {
            if (wrapped) {
#pragma unroll
                for (int j = 0; j < NP; j++) A[j] = 0u;
                m = 0u;
            }
        }
        if (refill) {
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (VAR == 3 || VAR == 4) {
#pragma unroll
                for (int w = 0; w < NW; w++) ring[p].w[w] = (cw[w] * 3u + (unsigned)p) & 0x1f1f1f1fu;
            } else {
                ring[p] = bload<NW>(rC, pc.off);
            }
            pc.advance(rx, stride, W, WD);
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    int t = 0;
    for (; t + PF <= steps; t += PF) {
#pragma unroll
        for (int p = 0; p < PF; p++) step(p, true);
    }
    // tail: fewer than PF steps left, all already in the ring
#pragma unroll
    for (int p = 0; p < PF; p++)
        if (t + p < steps) step(p, false);
}


template <int DPL, int VAR = 0>
__global__ __launch_bounds__(PATH_BLOCK) void sgm_paths_kernel(const uint8_t* __restrict__ C,
                                                               uint8_t* __restrict__ L8,
                                                               PathGeom g) {
    // Horizontal directions (W steps per line, the longest) get the lowest
    // block ids and issue priority so they are never the tail.
    int b = blockIdx.x, r, lb;
    if (b < 2 * g.blk_h) {
        r = b / g.blk_h;
        lb = b - r * g.blk_h;
        __builtin_amdgcn_s_setprio(1);
    } else {
        b -= 2 * g.blk_h;
        r = 2 + b / g.blk_w;
        lb = b - (r - 2) * g.blk_w;
    }
    const int line = lb * LINES_PER_BLOCK + (threadIdx.x >> 4);
    const int k = threadIdx.x & 15;
    const int nlines = r < 2 ? g.H : g.W;
    if (line >= nlines) return;  // whole 16-lane row leaves together
    int rx, ry;
    dir_of(r, rx, ry);
    const rsrc_t rC = make_rsrc(C, g.vol);
    const rsrc_t rL = make_rsrc(L8 + (size_t)r * g.vol, g.vol);
    if (r >= 4) path_line<DPL, true, VAR, pf_v<DPL>()>(rC, rL, g, rx, ry, line, k);
    else if (r >= 2) path_line<DPL, false, VAR, pf_v<DPL>()>(rC, rL, g, rx, ry, line, k);
    else path_line<DPL, false, VAR, pf_h<DPL>()>(rC, rL, g, rx, ry, line, k);
}

}  // namespace

bool paths_supported(int D) { return D == 64 || D == 128 || D == 192 || D == 256; }

hipError_t launch_paths(Ctx& c, const uint8_t* C, int W, int H, int D, int P1, int P2,
                        uint8_t* L8) {
    ScopedKernelTimer t(c, "sgm_paths");
    PathGeom g;
    g.W = W; g.H = H; g.D = D; g.P1 = P1; g.P2 = P2;
    g.blk_h = (H + LINES_PER_BLOCK - 1) / LINES_PER_BLOCK;
    g.blk_w = (W + LINES_PER_BLOCK - 1) / LINES_PER_BLOCK;
    g.vol = (size_t)W * H * D;
    g.store_aux = 0;
    if (g.vol >= (size_t)1 << 32) return hipErrorInvalidValue;  // 32-bit buffer offsets
    dim3 grid(2 * g.blk_h + 6 * g.blk_w);
#ifdef SVA_PATHS_LDS_KB
    // occupancy experiment: reserve dynamic LDS to cap workgroups per CU
    {
        const size_t lds = (size_t)SVA_PATHS_LDS_KB * 1024;
        switch (D) {
            case 64: hipLaunchKernelGGL(sgm_paths_kernel<4>, grid, dim3(PATH_BLOCK), lds, c.stream, C, L8, g); break;
            case 128: hipLaunchKernelGGL(sgm_paths_kernel<8>, grid, dim3(PATH_BLOCK), lds, c.stream, C, L8, g); break;
            case 192: hipLaunchKernelGGL(sgm_paths_kernel<12>, grid, dim3(PATH_BLOCK), lds, c.stream, C, L8, g); break;
            case 256: hipLaunchKernelGGL(sgm_paths_kernel<16>, grid, dim3(PATH_BLOCK), lds, c.stream, C, L8, g); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
#endif
#ifdef SVA_PATHS_ABLATION
    static int var = getenv("SVA_PATHS_VARIANT") ? atoi(getenv("SVA_PATHS_VARIANT")) : 0;
    if (D == 128 && var > 0) {
        switch (var) {
            case 2: hipLaunchKernelGGL((sgm_paths_kernel<8, 2>), grid, dim3(PATH_BLOCK), 0, c.stream, C, L8, g); break;
            case 3: hipLaunchKernelGGL((sgm_paths_kernel<8, 3>), grid, dim3(PATH_BLOCK), 0, c.stream, C, L8, g); break;
            case 4: hipLaunchKernelGGL((sgm_paths_kernel<8, 4>), grid, dim3(PATH_BLOCK), 0, c.stream, C, L8, g); break;
            case 9: case 10: case 11: case 12: case 13: {
                static const int auxv[5] = {2, 16, 18, 17, 0};   // 13 = default write-back
                g.store_aux = auxv[var - 9];
                hipLaunchKernelGGL((sgm_paths_kernel<8, 9>), grid, dim3(PATH_BLOCK), 0, c.stream, C, L8, g); break; }
            case 5: hipLaunchKernelGGL((sgm_paths_kernel<8, 4>), dim3(2 * g.blk_h), dim3(PATH_BLOCK), 0, c.stream, C, L8, g); break;
            case 6: { PathGeom g2 = g; g2.blk_h = 0;   // vertical + diagonal only (r = 2..7)
                      hipLaunchKernelGGL((sgm_paths_kernel<8, 4>), dim3(6 * g.blk_w), dim3(PATH_BLOCK), 0, c.stream, C, L8, g2); break; }
            case 7: hipLaunchKernelGGL((sgm_paths_kernel<8, 0>), dim3(2 * g.blk_h), dim3(PATH_BLOCK), 0, c.stream, C, L8, g); break;
            case 8: { PathGeom g2 = g; g2.blk_h = 0;
                      hipLaunchKernelGGL((sgm_paths_kernel<8, 0>), dim3(6 * g.blk_w), dim3(PATH_BLOCK), 0, c.stream, C, L8, g2); break; }
            default: break;
        }
        return hipGetLastError();
    }
#endif
    switch (D) {
        case 64: hipLaunchKernelGGL(sgm_paths_kernel<4>, grid, dim3(PATH_BLOCK), 0, c.stream, C, L8, g); break;
        case 128: hipLaunchKernelGGL(sgm_paths_kernel<8>, grid, dim3(PATH_BLOCK), 0, c.stream, C, L8, g); break;
        case 192: hipLaunchKernelGGL(sgm_paths_kernel<12>, grid, dim3(PATH_BLOCK), 0, c.stream, C, L8, g); break;
        case 256: hipLaunchKernelGGL(sgm_paths_kernel<16>, grid, dim3(PATH_BLOCK), 0, c.stream, C, L8, g); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace sva
