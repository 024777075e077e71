// wta_strip.hip -- the tile pipeline's final kernel with all eight
// directions recomputed per tile (SURVEY.md §8a rows
// A12-A13).  Built for D <= 128 when tune::kStripRoute.
//
// sgm_paths (checkpoint mode 2 + 3) leaves no path volume at all: only the
// states of every line at the checkpoint columns / rows (every 8 pixels):
// horizontal [2][H][nsx][D], vertical [2][nty][W][D] and, for the four
// diagonals, [4][nty][W][D] (direction 4 and 6 at the last row of every
// 8-row band, 5 and 7 at the first; vckpt planes 2..5).  This kernel re-runs
// all eight recurrences from those states, sums S and picks d* -- so the
// 2 B/disp x 4 of diagonal-volume traffic of the wta_hv route (a u8 write in
// sgm_paths and a read here, 2.12 GB per 1080p D=128 frame) never happens.
//
// The round-4 per-tile diagonal recompute (§4.11) lost because a 16 x 8 tile
// is crossed by 23 lines per diagonal direction: 44 % of its diagonal steps
// were halo.  Here a workgroup walks a STRIP of g.nt tiles (TW columns x 8
// rows each) of one 8-row band from left to right, and assigns the lines of
// each diagonal direction to tiles so that every line is run exactly once:
//   * group t holds TW lines per direction, line li starting at checkpoint
//     column  c = x0 - 1 + li  (directions 4, 7: +x)  or
//             c = x0 + 8 + li  (directions 6, 5: -x),  x0 = t * TW;
//     its 8 pixels lie in tile t, except a triangle of at most 7 columns that
//     spills into tile t + 1 (never into t - 1);
//   * the accumulators live in an LDS ring of TW + 8 columns x 8 rows, so
//     tile t + 1's spill columns are ready when its turn comes;
//   * a strip's first tile also needs the 7 spilling lines per direction of
//     the group before it (the prologue): 28 runs, the only halo left.
// Per tile: phase V (directions 2, 3: one column per slot) and phase D (the
// group's 4 x TW lines, one line of each direction per slot) add into the
// ring with LDS atomics (ds_add_u32 on packed u16 pairs: S <= 8 x 448 per
// half, no carry); barrier; phase H (directions 0, 1 over one 8-pixel row
// segment per slot, from the horizontal checkpoints) adds L_0 + L_1, picks
// d* (+ parabola) and zeroes the tile's blocks for reuse; barrier.
// Every recurrence restarts from the exact state the path kernel had, so S,
// d* and the sub-pixel value are bit-identical to the 8-volume route.
//
// LDS block of pixel (ring column rc, row r): [pair p][lane k] dwords, so 16
// lanes touch 16 consecutive dwords per pair (conflict-free single-dword
// atomics).  At D = 128, TW = 16: 24 x 8 x 64 x 4 B = 48 KB, three workgroups
// per CU (168 VGPRs, 3 waves per SIMD).
//
// MEASURED SLOWER than the wta_hv route and OFF (tune::kStripRoute = 0):
// 1080p D=128 frame 0.962 vs 0.883 ms, this kernel VALU-issue-bound at 0.83
// of the measured mix ceiling (profiles/r06_v2/).
#include "sgm_common.h"
#include "wta_common.h"
#include "sva_tuning.h"

namespace sva {
namespace {

using namespace sgm;

struct StripGeom {
    int W, H, D, P1, P2, dmin;
    int dreal;        // disparities of the caller (< D: padded frame)
    int nty, nsx;     // 8-row bands; horizontal checkpoint segments per row
    int ntx;          // tiles per band (TW columns each)
    int nt;           // tiles per strip
    int nstrip;       // strips per band
    int blocks;       // workgroups per frame (nty * nstrip; a batch: frame = block / blocks)
    unsigned vol;     // bytes of one [H][W][D] volume (< 2^32)
    unsigned hck;     // bytes of one horizontal checkpoint plane [H][nsx][D]
    unsigned vck;     // bytes of one row checkpoint plane [nty][W][D]
};

template <int DPL, int TW, bool PAD>
__global__ __launch_bounds__(TW * 16, tune::kStripMinWaves) void wta_strip_kernel(const uint8_t* __restrict__ C,
                                                          const uint8_t* __restrict__ CK,
                                                          const uint8_t* __restrict__ CKV,
                                                          StripGeom g, uint16_t* __restrict__ disp,
                                                          float* __restrict__ sub) {
    constexpr int NW = DPL / 4, NP = DPL / 2;
    constexpr int TY = 8;                 // band rows = checkpoint segment
    constexpr int TB = TW * 16;           // TW slots of 16 lanes
    constexpr int RC = TW + 8;            // ring columns
    constexpr int PIX = 16 * NP;          // dwords per pixel block
    constexpr int SPR = TW / TY;          // phase H: row segments per tile row
    constexpr bool PIN = tune::kWtahvPinRowMin != 0;
    static_assert(TW % TY == 0 && TW >= 16, "tile width");
    __shared__ unsigned acc[RC * TY * PIX];

    const unsigned f = blockIdx.x / (unsigned)g.blocks;
    const unsigned bb = blockIdx.x - f * (unsigned)g.blocks;
    const int ty = (int)(bb / (unsigned)g.nstrip);
    const int st = (int)(bb - (unsigned)ty * (unsigned)g.nstrip);
    C += (size_t)f * g.vol;
    CK += (size_t)f * 2 * g.hck;
    CKV += (size_t)f * 6 * g.vck;
    disp += (size_t)f * (size_t)g.W * (size_t)g.H;
    if (sub) sub += (size_t)f * (size_t)g.W * (size_t)g.H;
    const int slot = (int)(threadIdx.x >> 4);
    const int k = (int)(threadIdx.x & 15);
    const int W = g.W, H = g.H;
    const unsigned uD = (unsigned)g.D, uW = (unsigned)W;
    const unsigned P1 = (unsigned)g.P1, P2 = (unsigned)g.P2;
    const int y0 = ty * TY;
    const int ny = H - y0 < TY ? H - y0 : TY;         // band rows inside the image (uniform)
    const int t0 = st * g.nt;
    const int t1 = t0 + g.nt < g.ntx ? t0 + g.nt : g.ntx;
    const int xs = t0 * TW;                           // the strip's first column
    const unsigned lane_d = (unsigned)(k * DPL);
    const rsrc_t rC = make_rsrc(C, g.vol);
    const rsrc_t rCKV = make_rsrc(CKV, 6u * g.vck);
    unsigned padm[NP];
#pragma unroll
    for (int j = 0; j < NP; j++) {
        const int dl = k * DPL + pair_d<DPL>(j, 0), dh = k * DPL + pair_d<DPL>(j, 1);
        padm[j] = PAD ? ((dl >= g.dreal ? 0x0000ffffu : 0u) | (dh >= g.dreal ? 0xffff0000u : 0u))
                      : 0u;
    }
    // has an up checkpoint row (the band is not the image's last)
    const bool has_up = y0 + TY < H;

    auto zero_state = [](unsigned (&A)[NP], unsigned& m) {
#pragma unroll
        for (int j = 0; j < NP; j++) A[j] = 0u;     // L(q) = 0, m = 0  =>  L = C
        m = 0u;
    };
    // pixel block of ring column rc, row r; lane k's pair p at + p * 16
    auto blk = [&](int rc, int r) -> unsigned* { return &acc[(rc * TY + r) * PIX + k]; };
    auto add_blk = [&](unsigned* b, const unsigned (&A)[NP]) {
#pragma unroll
        for (int p = 0; p < NP; p++) atomicAdd(b + p * 16, A[p]);
    };

    for (int i = (int)threadIdx.x; i < RC * TY * PIX; i += TB) acc[i] = 0u;
    __syncthreads();

    // ---- one diagonal line: direction dd (vckpt plane 2 + dd: 0 -> 4 (+x,
    // down), 1 -> 6 (-x, down), 2 -> 5 (-x, up), 3 -> 7 (+x, up)), starting at
    // checkpoint column c; its pixels add into the ring (base column rb at
    // window column wx0) where x >= xmin.
    // Diagonal line li of the group whose tiles start at x0g, direction DD
    // (vckpt plane 2 + DD: 0 -> 4 (+x, down), 1 -> 6 (-x, down), 2 -> 5 (-x,
    // up), 3 -> 7 (+x, up)): its checkpoint column c and the 8 pixels
    // (c + rx (s + 1), row r(s)).  Step s is always computed; off the image
    // the state is zeroed (the path kernel restarts there) and the add is 0,
    // so the run has no per-lane branch.  PRO (the prologue): only pixels at
    // x >= xmin add.
    auto col_of = [&](int dd, int li, int x0g) -> int {
        return (dd == 0 || dd == 3) ? x0g - 1 + li : x0g + 8 + li;
    };
    auto issue_run = [&](auto DDc, int c, Words<NW>& ck, Words<NW> (&cd)[TY])
        __attribute__((always_inline)) {
        constexpr int DD = decltype(DDc)::value;
        constexpr bool up = DD >= 2;
        constexpr int rx = (DD == 0 || DD == 3) ? 1 : -1;
        const bool ckin = (up ? has_up : ty > 0) && (unsigned)c < uW;
        const int yck = up ? ty + 1 : ty - 1;
        ck = bload<NW>(rCKV, ckin ? ((unsigned)(2 + DD) * (unsigned)g.nty + (unsigned)yck) * uW * uD +
                                        (unsigned)c * uD + lane_d
                                  : 0u);
        for_seq<TY>([&](auto S) {
            constexpr int s = decltype(S)::value;
            constexpr int r = up ? TY - 1 - s : s;
            const int x = c + rx * (s + 1);
            cd[s] = bload<NW>(rC, (unsigned)x < uW && r < ny
                                      ? ((unsigned)(y0 + r) * uW + (unsigned)x) * uD + lane_d
                                      : 0u);
        });
    };
    auto run_line = [&](auto DDc, auto PROc, int c, const Words<NW>& ck, const Words<NW> (&cd)[TY],
                        int wx0, int rb, int xmin) __attribute__((always_inline)) {
        constexpr int DD = decltype(DDc)::value;
        constexpr bool PRO = decltype(PROc)::value;
        constexpr bool up = DD >= 2;
        constexpr int rx = (DD == 0 || DD == 3) ? 1 : -1;
        unsigned A[NP], m;
        if ((up ? has_up : ty > 0) && (unsigned)c < uW) state_from_words<DPL, PAD, PIN>(ck, A, m, padm);
        else zero_state(A, m);
        Edges e;
        // ring column of the line's first pixel (window column c + rx - wx0)
        int rc = rb + c + rx - wx0;                   // in (-RC, 2 RC)
        rc = rc >= RC ? rc - RC : (rc < 0 ? rc + RC : rc);
        for_seq<TY>([&](auto S) {
            constexpr int s = decltype(S)::value;
            constexpr int r = up ? TY - 1 - s : s;
            const int x = c + rx * (s + 1);
            unsigned ow[NW];
            sgm_step<DPL, PIN>(cd[s].w, A, m, ow, P1, P2, e);
            const bool in = (unsigned)x < uW && r < ny;
#pragma unroll
            for (int j = 0; j < NP; j++) A[j] = in ? A[j] : 0u;   // off the image: restart
            m = in ? m : 0u;
            if constexpr (PRO) {
                unsigned Ad[NP];
#pragma unroll
                for (int j = 0; j < NP; j++) Ad[j] = x >= xmin ? A[j] : 0u;
                add_blk(blk(rc, r), Ad);
            } else {
                add_blk(blk(rc, r), A);
            }
            if constexpr (s + 1 < TY) {
                rc += rx;
                if constexpr (rx > 0) rc = rc >= RC ? rc - RC : rc;
                else rc = rc < 0 ? rc + RC : rc;
            }
        });
    };

    // ---- prologue: the 7 spilling lines per direction of the group before
    // the strip (group t0 - 1), their pixels at x >= xs only
    {
        constexpr int NPRO = 4 * 7;
        const int x0g = xs - TW;
        for (int q = slot; q < NPRO; q += TW) {
            const int dd = q / 7, li = TW - 7 + q % 7;
            const int c = col_of(dd, li, x0g);
            Words<NW> ck, cd[TY];
            auto go = [&](auto DDc) {
                issue_run(DDc, c, ck, cd);
                run_line(DDc, std::true_type{}, c, ck, cd, xs, 0, xs);
            };
            switch (dd) {                              // uniform per 16-lane row
                case 0: go(std::integral_constant<int, 0>{}); break;
                case 1: go(std::integral_constant<int, 1>{}); break;
                case 2: go(std::integral_constant<int, 2>{}); break;
                default: go(std::integral_constant<int, 3>{}); break;
            }
        }
    }
    __builtin_amdgcn_sched_barrier(0);

    const int hr = slot / SPR, hseg = slot % SPR;     // phase H: row hr, segment hseg
    const unsigned yh = (unsigned)(y0 + hr);
    unsigned dpair[NP];                               // each pair's two d (kWtahvKeyPerm)
#pragma unroll
    for (int j = 0; j < NP; j++)
        dpair[j] = (lane_d + (unsigned)pair_d<DPL>(j, 0)) | ((lane_d + (unsigned)pair_d<DPL>(j, 1)) << 16);
    const bool want_sub = sub != nullptr;
    const rsrc_t rCK0 = make_rsrc(CK, g.hck), rCK1 = make_rsrc(CK + g.hck, g.hck);

    int rb = 0;                                       // ring column of the tile's first column
    for (int t = t0; t < t1; t++) {
        const int x0 = t * TW;
        const int nx = W - x0 < TW ? W - x0 : TW;     // tile columns inside the image (uniform)
        // ---- phase V: column x0 + slot, down (2) then up (3); V = L_2 + L_3
        const bool vcol = slot < nx;
        const unsigned xv = (unsigned)(x0 + slot);
        if (vcol) {
            Words<NW> cv[TY];
#pragma unroll
            for (int r = 0; r < TY; r++)
                cv[r] = bload<NW>(rC, r < ny ? ((unsigned)(y0 + r) * uW + xv) * uD + lane_d : 0u);
            unsigned Aa[NP], ma, Ab[NP], mb;
            if (ty > 0)
                load_state<DPL, PAD, PIN>(make_rsrc(CKV, g.vck), ((unsigned)(ty - 1) * uW + xv) * uD + lane_d,
                                          Aa, ma, padm);
            else
                zero_state(Aa, ma);
            if (has_up)
                load_state<DPL, PAD, PIN>(make_rsrc(CKV + g.vck, g.vck),
                                          ((unsigned)(ty + 1) * uW + xv) * uD + lane_d, Ab, mb, padm);
            else
                zero_state(Ab, mb);
            Edges ea, eb;
            // L_2 of each row kept u8-packed (the step's own ow words; <= 255
            // except at padded disparities, whose S is masked anyway)
            unsigned LD[TY][NW];
            for_seq<TY>([&](auto I) {
                constexpr int i = decltype(I)::value;
                unsigned ow[NW];
                if (i < ny) {
                    sgm_step<DPL, PIN>(cv[i].w, Aa, ma, ow, P1, P2, ea);
#pragma unroll
                    for (int q = 0; q < NW; q++) LD[i][q] = ow[q];
                }
            });
            int rc = rb + slot;
            rc = rc >= RC ? rc - RC : rc;
            for_seq<TY>([&](auto Q) {
                constexpr int r = TY - 1 - decltype(Q)::value;
                if (r < ny) {
                    unsigned lu[NW];
                    sgm_step<DPL, PIN>(cv[r].w, Ab, mb, lu, P1, P2, eb);
                    unsigned V[NP];
#pragma unroll
                    for (int p = 0; p < NP; p++) V[p] = Ab[p];
                    unpack_add<NW>(LD[r], V);                 // + L_2
                    add_blk(blk(rc, r), V);
                }
            });
        }
        // (phase fences: the scheduler would otherwise hoist the next phase's
        // loads into this one and hold both phases' registers at once)
        __builtin_amdgcn_sched_barrier(0);
        // ---- phase D: line `slot` of each diagonal direction of group t
        {
            for_seq<4>([&](auto DDc) {
                constexpr int dd = decltype(DDc)::value;
                const int c = col_of(dd, slot, x0);
                Words<NW> ck, cd[TY];
                issue_run(DDc, c, ck, cd);
                run_line(DDc, std::false_type{}, c, ck, cd, x0, rb, x0);
                __builtin_amdgcn_sched_barrier(0);
            });
        }
        __builtin_amdgcn_sched_barrier(0);
        // phase H's first loads go out before the barrier
        const int hx = x0 + hseg * TY;                // first column of the row segment
        const int nh = W - hx < TY ? W - hx : TY;     // its pixels inside the image
        const bool hrow = hr < ny && nh > 0;
        const int hs = hx >> 3;
        const unsigned ckrow = yh * (unsigned)g.nsx;
        Words<NW> ch[TY], ckw[2];
        if (hrow) {
#pragma unroll
            for (int j = 0; j < TY; j++)
                ch[j] = bload<NW>(rC, j < nh ? (yh * uW + (unsigned)(hx + j)) * uD + lane_d : 0u);
            // (words outside the image are never used: the first / last
            // segment starts from zero state)
            ckw[0] = bload<NW>(rCK0, (ckrow + (unsigned)(hs - 1)) * uD + lane_d);
            ckw[1] = bload<NW>(rCK1, (ckrow + (unsigned)(hs + 1)) * uD + lane_d);
        }
        __syncthreads();

        // ---- phase H: left-to-right (0), then right-to-left (1) with the
        // sum and the WTA per pixel
        if (hrow) {
            unsigned A[NP], m;
            if (hs > 0) state_from_words<DPL, PAD, PIN>(ckw[0], A, m, padm);
            else zero_state(A, m);
            Edges e0, e1;
            unsigned LF[TY][NW];                      // L_0, u8-packed like phase V's L_2
            for_seq<TY>([&](auto I) {
                constexpr int i = decltype(I)::value;
                unsigned ow[NW];
                if (i < nh) {
                    sgm_step<DPL, PIN>(ch[i].w, A, m, ow, P1, P2, e0);
#pragma unroll
                    for (int q = 0; q < NW; q++) LF[i][q] = ow[q];
                }
            });
            if (hx + TY < W) state_from_words<DPL, PAD, PIN>(ckw[1], A, m, padm);
            else zero_state(A, m);
            int rc0 = rb + hseg * TY;
            rc0 = rc0 >= RC ? rc0 - RC : rc0;
            unsigned dres = 0u, s0 = 0u, sm = 0u;
            for_seq<TY>([&](auto Q) {
                constexpr int j = TY - 1 - decltype(Q)::value;
                if (j < nh) {
                    unsigned ow[NW];
                    sgm_step<DPL, PIN>(ch[j].w, A, m, ow, P1, P2, e1);
                    int rc = rc0 + j;
                    rc = rc >= RC ? rc - RC : rc;
                    unsigned* const b = blk(rc, hr);
                    unsigned Sv[NP];
#pragma unroll
                    for (int p = 0; p < NP; p++) Sv[p] = b[p * 16] + A[p];
                    unpack_add<NW>(LF[j], Sv);              // + L_0
                    if constexpr (PAD) {
#pragma unroll
                        for (int p = 0; p < NP; p++) Sv[p] |= padm[p];
                    }
                    const unsigned best = wta_pick_key_perm<DPL, PIN && tune::kWtahvPinWta>(Sv, dpair);
                    // S over the pixel's block (read back below by the lane
                    // that owns the pixel, same wave), or zero for reuse
#pragma unroll
                    for (int p = 0; p < NP; p++) b[p * 16] = want_sub ? Sv[p] : 0u;
                    dres = k == j ? (best & 0xffffu) : dres;
                    s0 = k == j ? best >> 16 : s0;
                }
            });
            if (want_sub) {
                // S(d*-1), S(d*+1) of lane k's pixel (j = k) from the S its row
                // wrote over the pixel's block (same wave: issue order)
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (k < nh) {
                    int rc = rc0 + k;
                    rc = rc >= RC ? rc - RC : rc;
                    const unsigned* bk = &acc[(rc * TY + hr) * PIX];
                    const uint16_t* s16 = reinterpret_cast<const uint16_t*>(bk);
                    const int ds = (int)dres;
                    const int dm = ds > 0 ? ds - 1 : 0, dp = ds + 1 < 16 * DPL ? ds + 1 : ds;
                    // u16 of disparity d: pair (d / 2) % NP of lane d / DPL
                    auto at = [&](int d) {
                        const int kk = d / DPL, pp = pair_of<DPL>(d % DPL), hh = half_of<DPL>(d % DPL);
                        return (unsigned)s16[2 * (pp * 16 + kk) + hh];
                    };
                    sm = at(dm) | (at(dp) << 16);
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                // the segment's blocks back to zero for the ring's next use
                for_seq<TY>([&](auto J) {
                    constexpr int j = decltype(J)::value;
                    if (j < nh) {
                        int rc = rc0 + j;
                        rc = rc >= RC ? rc - RC : rc;
                        unsigned* const b = blk(rc, hr);
#pragma unroll
                        for (int p = 0; p < NP; p++) b[p * 16] = 0u;
                    }
                });
            }
            if (k < nh) {
                const size_t at = (size_t)yh * (size_t)W + (size_t)(hx + k);
                disp[at] = (uint16_t)(g.dmin + (int)dres);
                if (want_sub) sub[at] = subpixel(g.dmin, (int)dres, g.dreal, sm & 0xffffu, s0, sm >> 16);
            }
        }
        __syncthreads();                              // the tile's blocks are free again
        __builtin_amdgcn_sched_barrier(0);
        rb += TW;
        rb = rb >= RC ? rb - RC : rb;
    }
}

}  // namespace

bool wta_strip_supported(int D) { return D == 64 || D == 128; }

hipError_t launch_wta_strip(Ctx& c, const uint8_t* C, const uint8_t* CK, const uint8_t* CKV, int W,
                            int H, int D, int P1, int P2, int dmin, uint16_t* disp, float* sub,
                            int dreal, int npair) {
    DispatchTimer t(c, "wta_hv");
    if (!wta_strip_supported(D) || npair < 1) return hipErrorInvalidValue;
    const TileGeom tg = tile_geom(W, H, D);
    if (tg.seg_log2 != 3 || tg.nvol != 0) return hipErrorInvalidValue;
    constexpr int TW = tune::kStripTileW;
    StripGeom g;
    g.W = W; g.H = H; g.D = D; g.P1 = P1; g.P2 = P2; g.dmin = dmin;
    g.dreal = dreal > 0 && dreal < D ? dreal : D;
    g.nty = tg.nty;
    g.nsx = tg.nsx;
    g.ntx = (W + TW - 1) / TW;
    // strips of about kStripCols columns, evened out over the band
    const int want = (W + tune::kStripCols - 1) / tune::kStripCols;
    g.nt = (g.ntx + want - 1) / want;
    g.nstrip = (g.ntx + g.nt - 1) / g.nt;
    g.blocks = g.nty * g.nstrip;
    const size_t vol = (size_t)W * H * D;
    if (vol >= (size_t)1 << 32) return hipErrorInvalidValue;
    g.vol = (unsigned)vol;
    g.hck = (unsigned)(tg.hck_bytes / 2);
    g.vck = (unsigned)(tg.vck_bytes / 2);
    const bool pad = g.dreal < D;
    const dim3 grid((unsigned)(g.blocks * npair));
#define SVA_STRIP(DPL_)                                                                          \
    if (pad)                                                                                     \
        hipExtLaunchKernelGGL((wta_strip_kernel<DPL_, TW, true>), grid, dim3(TW * 16), 0,        \
                              c.stream, t.start, t.stop, 0, C, CK, CKV, g, disp, sub);           \
    else                                                                                         \
        hipExtLaunchKernelGGL((wta_strip_kernel<DPL_, TW, false>), grid, dim3(TW * 16), 0,       \
                              c.stream, t.start, t.stop, 0, C, CK, CKV, g, disp, sub);           \
    t.used = true
    switch (D) {
        case 64: SVA_STRIP(4); break;
        case 128: SVA_STRIP(8); break;
        default: return hipErrorInvalidValue;
    }
#undef SVA_STRIP
    return hipGetLastError();
}

}  // namespace sva
