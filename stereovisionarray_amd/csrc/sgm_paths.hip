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
template <int DPL, int VAR = 0>
__global__ __launch_bounds__(PATH_BLOCK) void sgm_paths_kernel(const uint8_t* __restrict__ C,
                                                               uint8_t* __restrict__ L8,
                                                               PathGeom g) {
    // Horizontal directions (W steps per line, the longest) get the lowest
    // block ids and issue priority so they are never the tail.
#ifndef SVA_PATHS_ORDER
#define SVA_PATHS_ORDER 0
#endif
    int b = blockIdx.x, r, lb;
#if SVA_PATHS_ORDER == 0
    if (b < 2 * g.blk_h) {
        r = b / g.blk_h;
        lb = b - r * g.blk_h;
        __builtin_amdgcn_s_setprio(1);
    } else {
        b -= 2 * g.blk_h;
        r = 2 + b / g.blk_w;
        lb = b - (r - 2) * g.blk_w;
    }
#else
    // experiment: diagonals first, then horizontal, up, down (the fastest last)
    {
        constexpr int ORD[8] = {4, 5, 6, 7, 0, 1, 3, 2};
        r = ORD[7];
        lb = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int nb = ORD[i] < 2 ? g.blk_h : g.blk_w;
            if (b < nb) { r = ORD[i]; lb = b; break; }
            b -= nb;
        }
#if SVA_PATHS_ORDER == 1
        if (r < 2) __builtin_amdgcn_s_setprio(1);
#elif SVA_PATHS_ORDER == 2
        if (r >= 4) __builtin_amdgcn_s_setprio(1);
#endif
    }
#endif
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

#ifdef SVA_PATHS_TRACE
unsigned long long*& trace_buffer() {
    static unsigned long long* p = nullptr;
    return p;
}
extern "C" int sva_debug_paths_trace_copy(void* host, size_t bytes) {
    if (!trace_buffer()) return 1;
    return hipMemcpy(host, trace_buffer(), bytes, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 2;
}
#endif

bool paths_supported(int D) { return D == 64 || D == 128 || D == 192 || D == 256; }

hipError_t launch_paths(Ctx& c, const uint8_t* C, int W, int H, int D, int P1, int P2,
                        uint8_t* L8) {
    DispatchTimer t(c, "sgm_paths");
#ifdef SVA_PATHS_TRACE
    {
        static unsigned long long* buf = nullptr;
        const size_t n = (size_t)4 * 65536 * kTraceSlots;
        if (!buf) {
            if (hipMalloc(&buf, n * 8) != hipSuccess) return hipErrorOutOfMemory;
            if (hipMemcpyToSymbol(HIP_SYMBOL(g_paths_trace), &buf, sizeof(buf)) != hipSuccess)
                return hipErrorInvalidValue;
        }
        (void)hipMemsetAsync(buf, 0, n * 8, c.stream);
        trace_buffer() = buf;
    }
#endif
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
#define SVA_PATHS_LAUNCH(DPL_)                                                               \
    hipExtLaunchKernelGGL(sgm_paths_kernel<DPL_>, grid, dim3(PATH_BLOCK), 0, c.stream, t.start, \
                          t.stop, 0, C, L8, g);                                        \
    t.used = true
    switch (D) {
        case 64: SVA_PATHS_LAUNCH(4); break;
        case 128: SVA_PATHS_LAUNCH(8); break;
        case 192: SVA_PATHS_LAUNCH(12); break;
        case 256: SVA_PATHS_LAUNCH(16); break;
        default: return hipErrorInvalidValue;
    }
#undef SVA_PATHS_LAUNCH
    return hipGetLastError();
}

}  // namespace sva
