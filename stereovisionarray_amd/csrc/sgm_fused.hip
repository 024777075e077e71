// sgm_fused.hip -- census-fused 8-direction SGM aggregation (DESIGN.md §4.5,
// SURVEY.md §8a rows A11 + A12).  All eight directions run in ONE launch.
//
// Same recurrence, lane layout and output as sgm_paths.hip ([8][H][W][D] u8
// path volumes, then wta.hip), but the matching cost
//     C(p,d) = popcount(CL(p) ^ CR(p + dir*(dmin+d), y)),  62 outside the image
// is formed in registers from the two census maps instead of being read back
// from a materialised W*H*D cost volume.  That removes the cost kernel's
// 1 B/disp write and the 8 B/disp of cost re-reads (one per direction): the
// path kernel's HBM traffic drops from 16 to 8 B/disp plus the census windows
// (about half of them L2 hits).  The price is ~36 more VALU per lane-step at
// D=128: on one stream this kernel wins at D=256 and loses at D<=192; with
// frames overlapping on two streams it wins at every D (DESIGN.md §4.5,
// sva_set_path_kernel).
//
// Census layout (census.hip, padded form): each map has row stride
// Wp = W + pr words, and columns W .. W+pr-1 repeat the row cyclically.  The
// pad is what lets a diagonal wave's lines share one window when some of
// them have wrapped around x (see fused_vd).  Columns outside [0, W) are read
// as whatever lies there (or 0 past the buffer: raw buffer loads are range
// checked) and masked to 62 by mask_outside from the column arithmetic alone.
//
// Line kinds:
//   * horizontal (W steps): lane k keeps its DPL census words of the matched
//     row in registers.  One step moves the window by one column, so one word
//     enters per line per step: DPP row_shl/shr by one lane plus a
//     row_newbcast of the entering word, which lane j of the line loaded for
//     step 16q + j (one u64 load per lane per 16 steps, likewise for CL).
//     The register slots rotate with the step (compile-time, no moves).
//   * vertical / diagonal (H steps): the 4 lines of a wave sit DPL columns
//     apart, so their D-word windows overlap in D + 3*DPL words.  The wave
//     loads that window once per step (D/64 words per lane, plus 3*DPL tail
//     words and the 4 CL words), stages it DPL-way transposed in a
//     wave-private LDS slot (conflict-free reads) and each lane reads its DPL
//     words back.  Loads run PF steps ahead in a register ring, the LDS read
//     of step t+1 overlaps step t's compute.
//   * every step is branch-free apart from wave-uniform branches: the DPP
//     neighbour exchange needs a full exec mask (a divergent store guard
//     around it miscompiled under a guarded unroll).
#include <cstdlib>

#include "sgm_common.h"

namespace sva {
namespace {

using namespace sgm;

constexpr int FBLOCK = 256;
constexpr int FLINES = FBLOCK / 16;

// Prefetch depth (steps) of the vertical/diagonal ring, per DPL: the ring holds
// D/64 + 1 u64 per step.
#ifndef SVA_FPF4
#define SVA_FPF4 12
#endif
#ifndef SVA_FPF8
#define SVA_FPF8 8
#endif
#ifndef SVA_FPF12
#define SVA_FPF12 6
#endif
#ifndef SVA_FPF16
#define SVA_FPF16 4
#endif
template <int DPL> constexpr int fpf() {
    return DPL == 4 ? SVA_FPF4 : DPL == 8 ? SVA_FPF8 : DPL == 12 ? SVA_FPF12 : SVA_FPF16;
}

struct FusedGeom {
    int W, H, dmin, P1, P2;
    int Wp;               // padded census row stride (words)
    unsigned offL, offR;  // byte offsets of the reference / matched census maps
    unsigned cen_bytes;   // bytes covered by the census buffer resource
    int blk_h, blk_w;
    unsigned vol;         // bytes of one path volume
};

__device__ __forceinline__ uint2 bload_u64(rsrc_t r, unsigned off) {
    auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
    return make_uint2(v[0], v[1]);
}

// Hamming distance of two census words: 2 v_xor + a v_bcnt chain.
__device__ __forceinline__ unsigned hd(uint2 a, uint2 b) {
    return (unsigned)__builtin_popcount(a.x ^ b.x) + (unsigned)__builtin_popcount(a.y ^ b.y);
}

// Lane J of each 16-lane row, broadcast over the row (DPP row_newbcast).
template <int J>
__device__ __forceinline__ uint2 bcast_row(uint2 v) {
    return make_uint2(
        (unsigned)__builtin_amdgcn_update_dpp(0, (int)v.x, 0x150 + J, 0xf, 0xf, false),
        (unsigned)__builtin_amdgcn_update_dpp(0, (int)v.y, 0x150 + J, 0xf, 0xf, false));
}

// The lane's first `nvalid` disparities (of DPL) are inside the image, the rest
// cost 62: per u16 pair, s = sat(i + 1 - nvalid) > 0 exactly for i >= nvalid,
// then c = min(c + 62 s, 62) (c <= 62 already).
template <int NP>
__device__ __forceinline__ void mask_outside(unsigned (&c)[NP], int nvalid) {
    const u16x2 nv = splat2((unsigned)nvalid);
    u16x2 s[NP];
#pragma unroll
    for (int j = 0; j < NP; j++) {
        const u16x2 dd = {(unsigned short)(2 * j + 1), (unsigned short)(2 * j + 2)};
        s[j] = __builtin_elementwise_sub_sat(dd, nv);
    }
#pragma unroll
    for (int j = 0; j < NP; j++) s[j] = s[j] * splat2(62) + as_v2(c[j]);
#pragma unroll
    for (int j = 0; j < NP; j++) c[j] = as_u32(vmin2(s[j], splat2(62)));
}

// Number of disparities d in [0, D) whose matched column x + SD*(dmin + d)
// lies inside [0, W), i.e. the first d outside.
template <int SD>
__device__ __forceinline__ int inside_count(int x, int W, int dmin) {
    return SD < 0 ? x - dmin + 1 : W - x - dmin;
}

// ------------------------------------------------------------- horizontal --
template <int DPL, int SD, int RX>
__device__ __forceinline__ void fused_h(rsrc_t rC, rsrc_t rL, const FusedGeom& g, int line,
                                        int k) {
    constexpr int NP = DPL / 2, NW = DPL / 4, D = 16 * DPL;
    constexpr int U = DPL == 12 ? 48 : 16;   // unroll: multiple of 16 and of DPL
    constexpr int SG = RX * SD;              // +1: a word moves to d-1 per step
    const int W = g.W, dmin = g.dmin;
    const unsigned P1 = (unsigned)g.P1, P2 = (unsigned)g.P2;
    const int y = line;
    const int x0 = RX > 0 ? 0 : W - 1;
    const unsigned rowL = g.offL + (unsigned)y * (unsigned)g.Wp * 8u;
    const unsigned rowR = g.offR + (unsigned)y * (unsigned)g.Wp * 8u;
    // column of the word entering at step t: cn0 + RX*t (d = D-1 or d = 0)
    const int cn0 = SG > 0 ? x0 + SD * (dmin + D - 1) : x0 + SD * dmin;

    // Window at the virtual position x0 - RX: logical word i (d = k*DPL + i)
    // in physical slot i.  At step t logical i lives in slot (i + SG*(t+1)) mod DPL.
    uint2 w[DPL];
#pragma unroll
    for (int i = 0; i < DPL; i++)
        w[i] = bload_u64(rC, rowR + (unsigned)(x0 - RX + SD * (dmin + k * DPL + i)) * 8u);
    // chunk q: lane j holds the entering word and CL of step 16q + j
    auto ld_chunk = [&](int q, uint2& r, uint2& l) {
        const int t = 16 * q + k;
        r = bload_u64(rC, rowR + (unsigned)(cn0 + RX * t) * 8u);
        l = bload_u64(rC, rowL + (unsigned)(x0 + RX * t) * 8u);
    };
    uint2 curR, curL, nxtR, nxtL;
    ld_chunk(0, nxtR, nxtL);

    unsigned A[NP];
#pragma unroll
    for (int j = 0; j < NP; j++) A[j] = 0u;   // L(q) = 0, m = 0  =>  L = C
    unsigned m = 0u;
    unsigned soff = ((unsigned)y * (unsigned)W + (unsigned)x0) * (unsigned)D + (unsigned)(k * DPL);
    const unsigned sstride = (unsigned)(RX * D);

    auto step = [&](auto S, int t) {
        constexpr int s = decltype(S)::value;
        constexpr int j = s % 16;
        if constexpr (j == 0) {
            __builtin_amdgcn_sched_barrier(0);
            curR = nxtR;
            curL = nxtL;
            ld_chunk(t / 16 + 1, nxtR, nxtL);
            __builtin_amdgcn_sched_barrier(0);
        }
        const uint2 nw = bcast_row<j>(curR);
        const uint2 cl = bcast_row<j>(curL);
        if constexpr (SG > 0) {
            constexpr int u = s % DPL;
            w[u] = make_uint2(row_shl1(w[u].x, nw.x), row_shl1(w[u].y, nw.y));
        } else {
            constexpr int u = ((-s - 1) % DPL + DPL) % DPL;
            w[u] = make_uint2(row_shr1(w[u].x, nw.x), row_shr1(w[u].y, nw.y));
        }
        unsigned c[NP];
#pragma unroll
        for (int q = 0; q < NP; q++) {
            constexpr int rot = ((SG * (s + 1)) % DPL + DPL) % DPL;
            const int p0 = (2 * q + rot) % DPL, p1 = (2 * q + 1 + rot) % DPL;
            c[q] = hd(cl, w[p0]) | (hd(cl, w[p1]) << 16);
        }
        const int nin = inside_count<SD>(x0 + RX * t, W, dmin);   // wave-uniform
        if (nin < D) {
            const int nv = nin - k * DPL;
            mask_outside<NP>(c, nv < 0 ? 0 : (nv > DPL ? DPL : nv));
        }
        unsigned ow[NW];
        sgm_step_c<DPL>(c, A, m, ow, P1, P2);
        bstore<NW, 0>(rL, soff, ow);
        soff += sstride;
    };

    // one unrolled copy with a scalar guard per step (no separate tail copy:
    // the hot code of all line kinds has to share the instruction cache)
    const int steps = W;
    for (int t0 = 0; t0 < steps; t0 += U) {
        for_seq<U>([&](auto S) {
            if (t0 + S < steps) step(S, t0 + S);
        });
    }
}

// ------------------------------------------------------ vertical/diagonal --
// A wave's 4 lines sit DPL columns apart (x_0 + DPL*l), so lane k of line l
// needs window words DPL*(l + k) + i: for one i, every lane of the wave reads
// one of 19 consecutive words of a DPL-way transposed window -- no LDS bank
// conflicts (lines one column apart made every ds_read 4-way conflicted:
// 83 % of the LDS cycles in SQ_LDS_BANK_CONFLICT).
// LDS slot (per wave): window word w (w < D + 3*DPL) at (w % DPL)*SROW + w/DPL,
// then the 4 CL words.
constexpr int SROW = 20;   // >= 19 columns; 2*SROW*NWL spreads the write groups over the banks
template <int DPL> constexpr int slot_words() { return DPL * SROW + 4 + 64; }

template <int NWL>
struct VLoad {
    uint2 a[NWL];   // window words lane*NWL .. +NWL-1
    uint2 b;        // lanes < 3*DPL: window word D + lane; next 4 lanes: CL of line lane-3*DPL
};

template <int NWL>
__device__ __forceinline__ VLoad<NWL> vload(rsrc_t r, unsigned o1, unsigned o2) {
    VLoad<NWL> v;
    if constexpr (NWL == 1) {
        v.a[0] = bload_u64(r, o1);
    } else {
#pragma unroll
        for (int h = 0; h < NWL / 2; h++) {
            auto q = __builtin_amdgcn_raw_buffer_load_b128(r, o1 + 16u * h, 0, 0);
            v.a[2 * h] = make_uint2(q[0], q[1]);
            v.a[2 * h + 1] = make_uint2(q[2], q[3]);
        }
        if constexpr (NWL & 1) v.a[NWL - 1] = bload_u64(r, o1 + 16u * (NWL / 2));
    }
    v.b = bload_u64(r, o2);
    return v;
}

template <int DPL, int SD, bool DIAG, int PF>
__device__ __forceinline__ void fused_vd(rsrc_t rC, rsrc_t rL, const FusedGeom& g,
                                         uint2* __restrict__ stg, int rx, int ry, int b, int l,
                                         int k, int lane) {
    constexpr int NP = DPL / 2, NW = DPL / 4, D = 16 * DPL, NWL = D / 64;
    static_assert(PF % 2 == 0, "word buffers alternate by step parity");
    static_assert(DPL == 4 * NWL, "ld1 rows: lane%4 * NWL + j");
    const int W = g.W, H = g.H, dmin = g.dmin;
    const unsigned P1 = (unsigned)g.P1, P2 = (unsigned)g.P2;
    const int steps = H;
    const int line = b + DPL * l;
    const bool live = line < W;
    const int y0 = ry > 0 ? 0 : H - 1;
    const unsigned WD = (unsigned)W * (unsigned)D;
    // per-line store cursor (true x; wraps for diagonals)
    Cursor<DIAG> cc;
    cc.x = live ? line : 0;
    cc.off = ((unsigned)y0 * (unsigned)W + (unsigned)cc.x) * (unsigned)D + (unsigned)(k * DPL);
    const unsigned sstride = (unsigned)((ry * W + rx) * D);
    // group window cursor: the window starts at column x_0 + cofs (x_0 = line
    // 0's column); line l sits at x_0 + DPL*l, unwrapped (the census pad repeats
    // the row, so a diagonal group straddling the wrap still reads one window)
    const int cofs = SD > 0 ? dmin : -(dmin + D - 1);
    const unsigned WB = (unsigned)W * 8u;
    const unsigned gstride = (unsigned)(ry * g.Wp + rx) * 8u;
    int px = b;
    unsigned pofs = g.offR + ((unsigned)y0 * (unsigned)g.Wp + (unsigned)(b + cofs)) * 8u;
    auto gadv = [&]() {
        pofs += gstride;
        if constexpr (DIAG) {
            px += rx;
            if (px >= W) { px -= W; pofs -= WB; }
            else if (px < 0) { px += W; pofs += WB; }
        }
    };
    // load offsets relative to pofs, and LDS positions, per lane (constants)
    const unsigned k1 = (unsigned)(lane * NWL) * 8u;
    const int cl_lane = lane - 3 * DPL;
    const bool w2 = lane < 3 * DPL + 4;
    const unsigned k2 = lane < 3 * DPL ? (unsigned)(D + lane) * 8u
                      : w2 ? (g.offL - g.offR) + (unsigned)(DPL * cl_lane - cofs) * 8u
                           : (unsigned)D * 8u;
    const int p1 = (lane & 3) * NWL * SROW + (lane >> 2);
    // lanes past the 3*DPL + 4 useful ones write a private dummy word (no
    // divergent branch in the step: DPP results need a full exec mask)
    const int p2 = lane < 3 * DPL ? (lane % DPL) * SROW + 16 + lane / DPL
                 : w2 ? DPL * SROW + cl_lane : DPL * SROW + 4 + lane;
    const int rb = SD > 0 ? l + k : (DPL - 1) * SROW + l + 15 - k;
    auto stage = [&](const VLoad<NWL>& v, uint2 (&wv)[DPL], uint2& cl) {
#pragma unroll
        for (int j = 0; j < NWL; j++) stg[p1 + j * SROW] = v.a[j];
        stg[p2] = v.b;
#pragma unroll
        for (int i = 0; i < DPL; i++) wv[i] = stg[SD > 0 ? rb + i * SROW : rb - i * SROW];
        cl = stg[DPL * SROW + l];
    };

    VLoad<NWL> ring[PF];
#pragma unroll
    for (int p = 0; p < PF; p++) {
        ring[p] = vload<NWL>(rC, pofs + k1, pofs + k2);
        gadv();
    }
    uint2 wbuf[2][DPL], clb[2];
    stage(ring[0], wbuf[0], clb[0]);
    ring[0] = vload<NWL>(rC, pofs + k1, pofs + k2);
    gadv();

    unsigned A[NP];
#pragma unroll
    for (int j = 0; j < NP; j++) A[j] = 0u;
    unsigned m = 0u;

    // step t = t0 + p: stage step t+1 (ring slot (p+1)%PF) into the other
    // word buffer, refill that ring slot with step t+1+PF, compute step t.
    auto step = [&](auto P, bool next, bool refill) {
        constexpr int p = decltype(P)::value;
        constexpr int cur = p & 1, nb = cur ^ 1, pn = (p + 1) % PF;
        if (next) stage(ring[pn], wbuf[nb], clb[nb]);
        if (refill) {
            __builtin_amdgcn_sched_barrier(0);
            ring[pn] = vload<NWL>(rC, pofs + k1, pofs + k2);
            gadv();
            __builtin_amdgcn_sched_barrier(0);
        }
        const uint2 cl = clb[cur];
        unsigned c[NP];
#pragma unroll
        for (int q = 0; q < NP; q++)
            c[q] = hd(cl, wbuf[cur][2 * q]) | (hd(cl, wbuf[cur][2 * q + 1]) << 16);
        const int nin = inside_count<SD>(cc.x, W, dmin);
        if (__builtin_amdgcn_ballot_w64(nin < D)) {
            const int nv = nin - k * DPL;
            mask_outside<NP>(c, nv < 0 ? 0 : (nv > DPL ? DPL : nv));
        }
        unsigned ow[NW];
        sgm_step_c<DPL>(c, A, m, ow, P1, P2);
        bstore<NW, 0>(rL, live ? cc.off : g.vol, ow);   // phantom line: past the range, dropped
        const bool wrapped = cc.advance(rx, sstride, W, WD);
        if constexpr (DIAG) {
#pragma unroll
            for (int j = 0; j < NP; j++) A[j] = wrapped ? 0u : A[j];
            m = wrapped ? 0u : m;
        }
    };

    int t = 0;
    for (; t + PF <= steps; t += PF) {
        for_seq<PF>([&](auto S) { step(S, true, true); });
    }
    for_seq<PF>([&](auto S) {
        if (t + S < steps) step(S, t + S + 1 < steps, false);
    });
}

// Vertical/diagonal groups: blocks of 4*DPL consecutive lines hold DPL groups
// (waves); group j of a block owns lines base + j + DPL*l, l = 0..3.
template <int DPL> __host__ __device__ constexpr int vd_groups(int W) {
    return (W + 4 * DPL - 1) / (4 * DPL) * DPL;
}

template <int DPL, int SD>
__global__ __launch_bounds__(FBLOCK) void sgm_fused_kernel(const uint64_t* __restrict__ cen,
                                                           uint8_t* __restrict__ L8,
                                                           FusedGeom g) {
    __shared__ uint2 stage[FBLOCK / 64][slot_words<DPL>()];
    int bi = blockIdx.x, r, lb;
    if (bi < 2 * g.blk_h) {   // horizontal lines first (the longest), with priority
        r = bi / g.blk_h;
        lb = bi - r * g.blk_h;
        __builtin_amdgcn_s_setprio(1);
    } else {
        bi -= 2 * g.blk_h;
        r = 2 + bi / g.blk_w;
        lb = bi - (r - 2) * g.blk_w;
    }
    const int k = threadIdx.x & 15;
    const rsrc_t rL = make_rsrc(L8 + (size_t)r * g.vol, g.vol);
    int rx, ry;
    dir_of(r, rx, ry);
    const rsrc_t rC = make_rsrc(cen, g.cen_bytes);
    if (r < 2) {
        const int line = lb * FLINES + (threadIdx.x >> 4);
        if (line >= g.H) return;   // horizontal lines are independent: the row leaves
        if (r == 0) fused_h<DPL, SD, 1>(rC, rL, g, line, k);
        else fused_h<DPL, SD, -1>(rC, rL, g, line, k);
        return;
    }
    // vertical / diagonal: a wave's 4 lines share one staged window, so a
    // partially filled wave keeps its phantom lines (they load, never store)
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int grp = lb * (FBLOCK / 64) + wave;
    if (grp >= vd_groups<DPL>(g.W)) return;
    const int base = grp / DPL * (4 * DPL) + grp % DPL;
    if (base >= g.W) return;
    constexpr int PF = fpf<DPL>();
    if (r >= 4) fused_vd<DPL, SD, true, PF>(rC, rL, g, stage[wave], rx, ry, base, lane >> 4, k, lane);
    else fused_vd<DPL, SD, false, PF>(rC, rL, g, stage[wave], rx, ry, base, lane >> 4, k, lane);
}

}  // namespace

int fused_pad(int W, int D, int dmin) {
    // lines of a vertical/diagonal wave reach 3*DPL columns past x_0 (unwrapped);
    // matched columns of wrapped lines reach min(W, dmin + D) further
    const long long md = (long long)dmin + D;
    return (int)(3 * (D / 16) + (md < W ? md : W));
}

bool fused_fits(int W, int H, int D, int dmin) {
    const unsigned long long Wp = (unsigned long long)W + (unsigned long long)fused_pad(W, D, dmin);
    const unsigned long long cen = 2ull * H * Wp * 8ull;
    const unsigned long long vol = (unsigned long long)W * H * D;
    // negative window offsets must wrap past the census buffer: keep it < 2 GiB
    return cen < (1ull << 31) && vol < (1ull << 32);
}

hipError_t launch_paths_fused(Ctx& c, const uint64_t* cen, size_t cen_words, size_t map_l,
                              size_t map_r, int W, int H, int D, int dmin, int dir, int P1,
                              int P2, uint8_t* L8) {
    DispatchTimer t(c, "sgm_fused");
    if (!paths_supported(D) || !fused_fits(W, H, D, dmin) || cen_words * 8 >= (1ull << 31))
        return hipErrorInvalidValue;
    FusedGeom g;
    g.W = W; g.H = H; g.dmin = dmin; g.P1 = P1; g.P2 = P2;
    g.Wp = W + fused_pad(W, D, dmin);
    g.offL = (unsigned)(map_l * 8);
    g.offR = (unsigned)(map_r * 8);
    g.cen_bytes = (unsigned)(cen_words * 8);
    g.blk_h = (H + FLINES - 1) / FLINES;
    const int groups = D == 64 ? vd_groups<4>(W) : D == 128 ? vd_groups<8>(W)
                     : D == 192 ? vd_groups<12>(W) : vd_groups<16>(W);
    g.blk_w = (groups + FBLOCK / 64 - 1) / (FBLOCK / 64);
    g.vol = (unsigned)((size_t)W * H * D);
    dim3 grid(2 * g.blk_h + 6 * g.blk_w);
#ifdef SVA_PATHS_ABLATION   // A/B builds only: SVA_FUSED_KIND 1 = horizontal lines only,
                            // 2 = vertical + diagonal only
    {
        static const int kind = getenv("SVA_FUSED_KIND") ? atoi(getenv("SVA_FUSED_KIND")) : 0;
        if (kind == 1) grid = dim3(2 * g.blk_h);
        if (kind == 2) { g.blk_h = 0; grid = dim3(6 * g.blk_w); }
    }
#endif
#define SVA_FUSED_LAUNCH(DPL)                                                                   \
    do {                                                                                        \
        if (dir > 0)                                                                            \
            hipExtLaunchKernelGGL((sgm_fused_kernel<DPL, 1>), grid, dim3(FBLOCK), 0, c.stream,  \
                                  t.start, t.stop, 0, cen, L8, g);                              \
        else                                                                                    \
            hipExtLaunchKernelGGL((sgm_fused_kernel<DPL, -1>), grid, dim3(FBLOCK), 0, c.stream, \
                                  t.start, t.stop, 0, cen, L8, g);                              \
        t.used = true;                                                                          \
    } while (0)
    switch (D) {
        case 64: SVA_FUSED_LAUNCH(4); break;
        case 128: SVA_FUSED_LAUNCH(8); break;
        case 192: SVA_FUSED_LAUNCH(12); break;
        default: SVA_FUSED_LAUNCH(16); break;
    }
#undef SVA_FUSED_LAUNCH
    return hipGetLastError();
}

}  // namespace sva
