// sgm_paths_wide.hip -- the 8-path aggregation with ONE path line per wave
// (SURVEY.md §8a row A12): the layout for frames too small
// to fill the chip with the 16-lane layout of sgm_paths.hip.
//
// Same recurrence, same bytes out (volumes and tile-pipeline checkpoints are
// byte-identical to sgm_paths_kernel's), different lane map:
//   * lane k of the wave holds disparities [k*DPL, k*DPL + DPL), DPL = D/64
//     (1, 2 or 4 at D = 64, 128, 256);
//   * the d-1 / d+1 neighbours cross lanes with one DPP wave_shr:1 /
//     wave_shl:1 each (INF kept in lane 0 / lane 63 for the whole line);
//   * min_k L is the 16-lane row minimum (4 DPP steps), row_bcast:15 and
//     row_bcast:31 into lane 63, and one v_readlane: m, m + P2 and -m are
//     scalars, and so are the line's cursors (one line per wave).
// Why: a small frame has few lines (640x480: 4,800), which the 16-lane layout
// packs into 1,200 waves -- about one per SIMD -- so each wave issues its
// step alone and the step's ~26 VALU set the pace (the horizontal lines'
// 640 steps took 0.075 ms).  Here a step is ~13-17 VALU and every line is
// its own wave: 4,800 waves, about 5 per SIMD.  Large frames keep the
// 16-lane layout, which carries 4 lines per instruction.
#include "sgm_common.h"
#include "sva_tuning.h"

namespace sva {
namespace {

using namespace sgm;

constexpr int WIDE_BLOCK = 256;                 // 4 waves = 4 lines
constexpr int WIDE_LINES = WIDE_BLOCK / 64;

enum : int {
    DPP_WAVE_SHL1 = 0x130,      // lane i <- lane i+1 across the wave
    DPP_WAVE_SHR1 = 0x138       // lane i <- lane i-1 across the wave
};

// lane i <- lane i-1 (lane 0 keeps `edge`) / lane i+1 (lane 63 keeps `edge`)
__device__ __forceinline__ unsigned wave_shr1(unsigned v, unsigned edge) {
    return (unsigned)__builtin_amdgcn_update_dpp((int)edge, (int)v, DPP_WAVE_SHR1, 0xf, 0xf, false);
}
__device__ __forceinline__ unsigned wave_shl1(unsigned v, unsigned edge) {
    return (unsigned)__builtin_amdgcn_update_dpp((int)edge, (int)v, DPP_WAVE_SHL1, 0xf, 0xf, false);
}

// Minimum over the 64 lanes, as a wave-uniform (scalar) value: the row
// minimum in every lane (4 DPP steps), then lane 15 of rows 0 / 2 into rows
// 1 / 3 and lane 31 into rows 2 / 3 as v_min_u32_dpp with a row mask (rows
// outside the mask keep their value, so no copy is needed), lane 63 read out.
// The s_nop cover the DPP read-after-VALU-write wait states.
__device__ __forceinline__ unsigned wave_min_u32(unsigned v) {
    v = row_min_u32<false>(v);
    asm("s_nop 1\n\t"
        "v_min_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_u32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
        "s_nop 1"
        : "+v"(v));
    return (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}

// v_add3_u32 with a scalar third operand (the step's -m)
__device__ __forceinline__ unsigned add3_s(unsigned a, unsigned b, unsigned s) {
    unsigned r;
    asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(s));
    return r;
}

// The lane's DPL cost bytes: C[off + lane*DPL ..], scalar off.
template <int DPL>
__device__ __forceinline__ unsigned wload(rsrc_t r, unsigned voff, unsigned soff) {
    if constexpr (DPL == 1)
        return __builtin_amdgcn_raw_buffer_load_b8(r, voff, soff, tune::kCLoadAux);
    else if constexpr (DPL == 2)
        return __builtin_amdgcn_raw_buffer_load_b16(r, voff, soff, tune::kCLoadAux);
    else
        return __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, tune::kCLoadAux);
}
template <int DPL, int AUX>
__device__ __forceinline__ void wstore(rsrc_t r, unsigned v, unsigned voff, unsigned soff) {
    if constexpr (DPL == 1)
        __builtin_amdgcn_raw_buffer_store_b8((unsigned char)v, r, voff, soff, AUX);
    else if constexpr (DPL == 2)
        __builtin_amdgcn_raw_buffer_store_b16((unsigned short)v, r, voff, soff, AUX);
    else
        __builtin_amdgcn_raw_buffer_store_b32(v, r, voff, soff, AUX);
}

// Path state of one line: NP = max(DPL/2, 1) registers of the lane's
// disparities (DPL = 1: one u32; otherwise packed u16 pairs), the scalar
// minimum m of the previous pixel, and the edge registers of the shifts.
template <int DPL>
struct WideState {
    static constexpr int NP = DPL == 1 ? 1 : DPL / 2;
    unsigned A[NP];
    unsigned m;
    unsigned X, Y;
};

// One recurrence step (the same arithmetic as sgm_step_c):
//   u = min(min(A(d-1), A(d+1)) + P1, A(d), m + P2);  L = u + C - m.
// cw: the lane's DPL cost bytes; returns the DPL result bytes.
template <int DPL>
__device__ __forceinline__ unsigned wide_step(unsigned cw, WideState<DPL>& s, unsigned P1,
                                              unsigned P2) {
    constexpr int NP = WideState<DPL>::NP;
    if constexpr (DPL == 1) {
        s.X = wave_shr1(s.A[0], s.X);
        s.Y = wave_shl1(s.A[0], s.Y);
        const unsigned K = 0u - s.m, mP2 = s.m + P2;        // scalars
        unsigned t = (s.X < s.Y ? s.X : s.Y) + P1;
        t = t < s.A[0] ? t : s.A[0];
        t = t < mP2 ? t : mP2;
        s.A[0] = add3_s(t, cw, K);
        s.m = wave_min_u32(s.A[0]);
        return s.A[0];
    } else {
        // X = lane k-1's last pair, Y = lane k+1's first pair
        s.X = wave_shr1(s.A[NP - 1], s.X);
        s.Y = wave_shl1(s.A[0], s.Y);
        unsigned M[NP];
        M[0] = __builtin_amdgcn_alignbit(s.A[0], s.X, 16);
#pragma unroll
        for (int j = 1; j < NP; j++) M[j] = __builtin_amdgcn_alignbit(s.A[j], s.A[j - 1], 16);
        const unsigned Qlast = __builtin_amdgcn_alignbit(s.Y, s.A[NP - 1], 16);
        const unsigned K = 0u - s.m * 0x10001u;              // scalars
        const unsigned mP2 = P2 * 0x10001u - K;
        unsigned c[NP];
        if constexpr (DPL == 2) c[0] = __builtin_amdgcn_perm(0u, cw, 0x0c010c00u);
        else unpack4(cw, c[0], c[1]);
        u16x2 t[NP];
#pragma unroll
        for (int j = 0; j < NP; j++) t[j] = vmin2(as_v2(M[j]), as_v2(j < NP - 1 ? M[j + 1] : Qlast));
#pragma unroll
        for (int j = 0; j < NP; j++) t[j] = t[j] + splat2(P1);
#pragma unroll
        for (int j = 0; j < NP; j++)
            s.A[j] = add3_s(as_u32(vmin2(vmin2(t[j], as_v2(s.A[j])), as_v2(mP2))), c[j], K);
        unsigned lm;
        if constexpr (NP == 1) {
            const u16x2 a = as_v2(s.A[0]);
            lm = a.x < a.y ? a.x : a.y;
        } else {
            lm = lane_min_u16<NP>(s.A);
        }
        s.m = wave_min_u32(lm);
        if constexpr (DPL == 2) return __builtin_amdgcn_perm(0u, s.A[0], 0x0c0c0200u);
        else return pack4(s.A[0], s.A[1]);
    }
}

// One path line per wave over the materialised cost volume.  CKPT as in
// path_line (sgm_common.h): 0 writes the direction's volume, 1 / 2 the tile
// pipeline's horizontal / vertical checkpoints every 2^SL pixels.  Every
// cursor is a scalar; the lane's byte offset (lane * DPL) is the VGPR part.
template <int DPL, bool DIAG, int PF, int CKPT = 0, int SL = 0>
__device__ __forceinline__ void wide_line(rsrc_t rC, rsrc_t rOut, const PathGeom& g, int rx,
                                          int ry, int line) {
    const int W = g.W, H = g.H, D = g.D;
    const unsigned P1 = (unsigned)g.P1, P2 = (unsigned)g.P2;
    const int steps = ry == 0 ? W : H;
    const unsigned WD = (unsigned)W * (unsigned)D;
    const unsigned stride = (unsigned)((ry * W + rx) * D);
    const unsigned lane_off = (unsigned)((threadIdx.x & 63) * DPL);
    // the last pixel whose DPL bytes of every lane are inside the volume
    const unsigned last = (unsigned)(g.vol - (size_t)D);
    int x0, y0;
    if (ry == 0) { y0 = line; x0 = rx > 0 ? 0 : W - 1; }
    else { y0 = ry > 0 ? 0 : H - 1; x0 = line; }
    unsigned off = ((unsigned)y0 * (unsigned)W + (unsigned)x0) * (unsigned)D;
    unsigned poff = off;
    int x = x0, px = x0;        // DIAG: the compute / prefetch cursors' columns

    WideState<DPL> s;
#pragma unroll
    for (int j = 0; j < WideState<DPL>::NP; j++) s.A[j] = 0u;   // L(q) = 0, m = 0 => L = C
    s.m = 0u;
    s.X = s.Y = DPL == 1 ? 0x7fffu : INF2;

    // Prefetch cursor: PF pixels ahead, wrapping with the line; past the
    // line's end it would leave the volume, so it is clamped to offset 0
    // (loaded, never consumed).
    auto padvance = [&]() {
        poff += stride;
        if constexpr (DIAG) {
            px += rx;
            if (px >= W) { px -= W; poff -= WD; }
            else if (px < 0) { px += W; poff += WD; }
        }
        poff = poff <= last ? poff : 0u;
    };
    unsigned ring[PF];
#pragma unroll
    for (int p = 0; p < PF; p++) {
        ring[p] = wload<DPL>(rC, lane_off, poff);
        padvance();
    }

    auto step = [&](int p, bool refill, int ts) {
        const unsigned ow = wide_step<DPL>(ring[p], s, P1, P2);
        if constexpr (CKPT == 1) {
            const int xx = rx > 0 ? ts : W - 1 - ts;
            constexpr int SEG = 1 << SL;
            const bool hit = rx > 0 ? (((xx + 1) & (SEG - 1)) == 0 && xx + 1 < W)
                                    : ((xx & (SEG - 1)) == 0 && xx > 0);
            if (hit)
                wstore<DPL, tune::kCkptStoreAux>(
                    rOut, ow, lane_off, (unsigned)(y0 * g.ns + (xx >> SL)) * (unsigned)D);
        } else if constexpr (CKPT == 2) {
            const int y = ry > 0 ? ts : H - 1 - ts;
            constexpr int SEG = 1 << SL;
            const bool hit = ry > 0 ? (((y + 1) & (SEG - 1)) == 0 && y + 1 < H)
                                    : ((y & (SEG - 1)) == 0 && y > 0);
            if (hit)
                wstore<DPL, tune::kCkptStoreAux>(
                    rOut, ow, lane_off, (unsigned)((y >> SL) * W + x0) * (unsigned)D);
        } else {
            wstore<DPL, kStoreNT>(rOut, ow, lane_off, off);
        }
        off += stride;
        if constexpr (DIAG) {
            // the line wraps in x and restarts there (L = C), as in path_line
            x += rx;
            if ((unsigned)x >= (unsigned)W) {
                x = rx > 0 ? x - W : x + W;
                off = rx > 0 ? off - WD : off + WD;
#pragma unroll
                for (int j = 0; j < WideState<DPL>::NP; j++) s.A[j] = 0u;
                s.m = 0u;
            }
        }
        if (refill) {
            if constexpr (tune::kWideSchedBarrier) __builtin_amdgcn_sched_barrier(0);
            ring[p] = wload<DPL>(rC, lane_off, poff);
            padvance();
            if constexpr (tune::kWideSchedBarrier) __builtin_amdgcn_sched_barrier(0);
        }
    };

    int t = 0;
    for (; t + PF <= steps; t += PF) {
#pragma unroll
        for (int p = 0; p < PF; p++) step(p, true, t + p);
    }
#pragma unroll
    for (int p = 0; p < PF; p++)
        if (t + p < steps) step(p, false, t + p);
}

template <int DPL>
__global__ __launch_bounds__(WIDE_BLOCK) void sgm_paths_wide_kernel(const uint8_t* __restrict__ C,
                                                                    uint8_t* __restrict__ L8,
                                                                    uint8_t* __restrict__ CK,
                                                                    uint8_t* __restrict__ CKV,
                                                                    PathGeom g) {
    // Block order as in sgm_paths_kernel: the horizontal lines (the longest
    // chains when W > H) first with issue priority, then the six vertical /
    // diagonal directions of a 4-line band next to each other.
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int bh = (g.H + WIDE_LINES - 1) / WIDE_LINES;
    int b = blockIdx.x, r, lb;
    if (b < 2 * bh) {
        r = b / bh;
        lb = b - r * bh;
        __builtin_amdgcn_s_setprio(1);
    } else {
        b -= 2 * bh;
        r = 2 + b % 6;
        lb = b / 6;
    }
    const int line = lb * WIDE_LINES + wv;
    if (line >= (r < 2 ? g.H : g.W)) return;   // whole wave
    int rx, ry;
    dir_of(r, rx, ry);
    const rsrc_t rC = make_rsrc(C, g.vol);
    constexpr int PF = tune::kPfWide;
    constexpr int SL = DPL <= 2 ? tune::kWtahvTileLog2 : tune::kWtahvTileLog2Wide;
    if (r >= 4) {
        const int slot = g.ckpt ? r - 4 : r;
        wide_line<DPL, true, PF>(rC, make_rsrc(L8 + (size_t)slot * g.vol, g.vol), g, rx, ry, line);
    } else if (r >= 2 && g.ckpt) {
        wide_line<DPL, false, PF, 2, SL>(rC, make_rsrc(CKV + (size_t)(r - 2) * g.ckvvol, g.ckvvol), g,
                                         rx, ry, line);
    } else if (g.ckpt) {
        wide_line<DPL, false, PF, 1, SL>(rC, make_rsrc(CK + (size_t)r * g.ckvol, g.ckvol), g, rx, ry,
                                         line);
    } else {
        wide_line<DPL, false, PF>(rC, make_rsrc(L8 + (size_t)r * g.vol, g.vol), g, rx, ry, line);
    }
}

}  // namespace

bool paths_wide_supported(int D) {
    return (D == 64 || D == 128 || D == 256) && !tune::kTileDiagDown && !tune::kTileDiagUp;
}

hipError_t launch_paths_wide(Ctx& c, const PathGeom& g, const uint8_t* C, uint8_t* L8, uint8_t* CK,
                             uint8_t* CKV) {
    DispatchTimer t(c, "sgm_paths");
    const int bh = (g.H + WIDE_LINES - 1) / WIDE_LINES, bw = (g.W + WIDE_LINES - 1) / WIDE_LINES;
    const dim3 grid((unsigned)(2 * bh + 6 * bw));
#define SVA_WIDE_LAUNCH(DPL_)                                                                      \
    hipExtLaunchKernelGGL(sgm_paths_wide_kernel<DPL_>, grid, dim3(WIDE_BLOCK), 0, c.stream, t.start, \
                          t.stop, 0, C, L8, CK, CKV, g);                                          \
    t.used = true
    switch (g.D) {
        case 64: SVA_WIDE_LAUNCH(1); break;
        case 128: SVA_WIDE_LAUNCH(2); break;
        case 256: SVA_WIDE_LAUNCH(4); break;
        default: return hipErrorInvalidValue;
    }
#undef SVA_WIDE_LAUNCH
    return hipGetLastError();
}

}  // namespace sva
