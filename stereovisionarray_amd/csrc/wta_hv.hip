// wta_hv.hip -- the tile pipeline's final kernel (SURVEY.md
// §8a rows A12-A13): horizontal AND vertical path recompute + path sum + WTA
// (+ sub-pixel) per 16 x TY pixel tile.
//
// sgm_paths in tile mode (ckpt 2) leaves four u8 volumes (the diagonal
// directions) and checkpoints every TY pixels: the horizontal lines' L state
// at the last / first column of every TY-column segment, the vertical lines'
// at the last / first row of every TY-row segment.  One 256-thread workgroup
// owns one tile of 16 columns x TY rows, with the path kernel's lane layout
// (lane k of a 16-lane DPP row owns disparities [k*DPL, k*DPL + DPL)):
//   phase V  row-slot s runs column x0 + s: the downward recurrence over the
//            tile's rows from the checkpoint above the tile, and the upward
//            one from the checkpoint below it; V = L_2 + L_3 of every pixel
//            goes to LDS (u16 pairs).
//   phase H  row-slot s runs one TY-pixel row segment (16 / TY per tile row):
//            left-to-right from the checkpoint left of it (L_0 kept in
//            registers, u8-packed), then right-to-left from the one right of
//            it; at each pixel S = L_1 + L_0 + V + the four diagonal volumes,
//            and the first-minimum WTA (+ parabola) picks d*.
// Every recurrence restarts from the exact state the path kernel had, so L,
// S, d* and the sub-pixel value are bit-identical to the 8-volume route.
//
// Bytes per disparity: 1 C read (phase H re-reads the tile's cost words from
// L2, where phase V just brought them) + 4 volume reads, and the path kernel
// writes 4 volumes instead of 6: -4 B/disp against the wta_h route (§4.6).
#include "sgm_common.h"
#include "wta_common.h"
#include "sva_tuning.h"

namespace sva {
namespace {

using namespace sgm;

constexpr int TB = 256;             // 16 slots of 16 lanes
constexpr int TW = 16;              // tile columns

struct WtaHvGeom {
    int W, H, D, P1, P2, dmin;
    int ntx, nty;     // tiles per row / per column
    int nsx;          // horizontal checkpoint segments per row, ceil(W / TY)
    int dreal;        // disparities of the caller (< D: padded frame)
    unsigned vol;     // bytes of one [H][W][D] volume (< 2^32)
    unsigned hck;     // bytes of one horizontal checkpoint plane [H][nsx][D]
    unsigned vck;     // bytes of one vertical checkpoint plane [nty][W][D]
    int tiles;        // tiles per frame, ntx * nty (a batch: frame = block / tiles)
};

// Prefetch depth (pixels) of the diagonal volumes in the last pass.
template <int DPL> constexpr int pf_vol() {
    return DPL >= 16 ? tune::kWtahvPfVol16 : DPL <= 4 ? tune::kWtahvPfVol4 : tune::kWtahvPfVol;
}

template <int DPL, int TYL, bool PAD>
__global__ __launch_bounds__(TB, tune::kWtahvMinWaves) void wta_hv_kernel(const uint8_t* __restrict__ C,
                                                    const uint8_t* __restrict__ L4,
                                                    const uint8_t* __restrict__ CK,
                                                    const uint8_t* __restrict__ CKV, WtaHvGeom g,
                                                    uint16_t* __restrict__ disp,
                                                    float* __restrict__ sub) {
    constexpr int NW = DPL / 4, NP = DPL / 2;
    constexpr int TY = 1 << TYL;        // tile rows = checkpoint segment (rows and columns)
    constexpr int kPfVol = pf_vol<DPL>();
    // bit 0: phase V keeps L_2 as u16, bit 1: phase H keeps L_0 as u16
    constexpr int KEEPM = DPL <= 8 ? tune::kWtahvKeepU16 : tune::kWtahvKeepU16Wide;
    constexpr bool KEEP16 = (KEEPM & 1) != 0, KEEP16H = (KEEPM & 2) != 0;
    constexpr bool PIN = tune::kWtahvPinRowMin != 0;     // row_min_u32<PIN>
    // cost words expanded once per phase (tune::kWtahvUnpackOnce)
    constexpr bool UNPACK1 = ((tune::kWtahvUnpackOnce >> (DPL / 4 - 1)) & 1) != 0;

    constexpr int SPR = TW / TY;        // phase H: row segments per tile row
    static_assert(TY <= TW && TW % TY == 0, "tile rows must divide 16");
    // a batch of frames: frame f's planes follow frame f-1's
    const unsigned f = blockIdx.x / (unsigned)g.tiles;
    const unsigned tb = blockIdx.x - f * (unsigned)g.tiles;
    const int tx = (int)(tb % (unsigned)g.ntx);
    const int ty = (int)(tb / (unsigned)g.ntx);
    // diagonals recomputed per tile (§4.11): the down pair (4, 6), the up pair (5, 7)
    constexpr bool DOWN = diag_ckpt_down(DPL), UP = diag_ckpt_up(DPL);
    constexpr int ND = (DOWN ? 2 : 0) + (UP ? 2 : 0);   // recomputed diagonals
    constexpr int NV = 4 - ND;                          // diagonal volumes read
    C += (size_t)f * g.vol;
    L4 += (size_t)f * NV * g.vol;
    CK += (size_t)f * 2 * g.hck;
    CKV += (size_t)f * (2 + ND) * g.vck;
    disp += (size_t)f * (size_t)g.W * (size_t)g.H;
    if (sub) sub += (size_t)f * (size_t)g.W * (size_t)g.H;
    const int slot = (int)(threadIdx.x >> 4);
    const int k = (int)(threadIdx.x & 15);
    const int W = g.W, H = g.H;
    const unsigned uD = (unsigned)g.D, uW = (unsigned)W;
    const unsigned P1 = (unsigned)g.P1, P2 = (unsigned)g.P2;
    const int x0 = tx * TW, y0 = ty * TY;
    const int nx = W - x0 < TW ? W - x0 : TW;       // tile columns inside the image (uniform)
    const int ny = H - y0 < TY ? H - y0 : TY;       // tile rows inside the image (uniform)
    const unsigned lane_d = (unsigned)(k * DPL);
    const rsrc_t rC = make_rsrc(C, g.vol);
    unsigned padm[NP];
#pragma unroll
    for (int j = 0; j < NP; j++) {
        const int dl = k * DPL + pair_d<DPL>(j, 0), dh = k * DPL + pair_d<DPL>(j, 1);
        padm[j] = PAD ? ((dl >= g.dreal ? 0x0000ffffu : 0u) | (dh >= g.dreal ? 0xffff0000u : 0u))
                      : 0u;
    }

    // V = L_2 + L_3 per tile pixel, [pixel = r * TW + c][lane k][NP pairs]:
    // each 16-lane row reads / writes 16 consecutive NP-dword chunks.  At
    // NP = 8 a lane's two 16-byte chunks trade places when ((k >> 2) ^
    // (k >> 3)) & 1 (tune::kWtahvVSwizzle): bank-conflict-free b128 reads and
    // writes.  vw(p) = the word of pair p inside a pixel block.
    __shared__ unsigned vsum[TY * TW * 16 * NP];
    constexpr bool VSW = NP == 8 && tune::kWtahvVSwizzle != 0;
    auto vsw_of = [](int kk) -> int { return VSW ? (((kk >> 2) ^ (kk >> 3)) & 1) * 4 : 0; };
    const int vb0 = k * NP + vsw_of(k), vb1 = k * NP + (4 ^ vsw_of(k));
    auto vw = [&](int p) -> int { return (p < 4 ? vb0 : vb1) + (p & 3); };

    // phase V: column x0 + slot; phase H: row hr, columns [hx, hx + TY)
    const bool vcol = slot < nx;
    const int hr = slot / SPR, hseg = slot % SPR;
    const int hx = x0 + hseg * TY;                    // first column of the row segment
    const int nh = W - hx < TY ? W - hx : TY;         // its pixels inside the image
    const bool hrow = hr < ny && nh > 0;
    const unsigned xv = (unsigned)(x0 + slot), yh = (unsigned)(y0 + hr);

    // Both phases' cost words are loaded up front (tune::kWtahvRowCFirst): the
    // tile's column slice for phase V and its row slice for phase H (the same
    // bytes, L2-hot the second time).
    Words<NW> cv[TY], ch[TY];
#pragma unroll
    for (int r = 0; r < TY; r++)
        cv[r] = bload<NW>(rC, ((unsigned)(y0 + r) * uW + xv) * uD + lane_d);
    auto load_row = [&]() {
#pragma unroll
        for (int j = 0; j < TY; j++)
            ch[j] = bload<NW>(rC, (yh * uW + (unsigned)(hx + j)) * uD + lane_d);
    };
    if constexpr (tune::kWtahvRowCFirst != 0) load_row();

    auto zero_state = [](unsigned (&A)[NP], unsigned& m) {
#pragma unroll
        for (int j = 0; j < NP; j++) A[j] = 0u;   // L(q) = 0, m = 0  =>  L = C
        m = 0u;
    };
    unsigned Aa[NP], Ab[NP], ma, mb;
    Edges ea, eb;
    // ---- phase V: down (direction 2) and up (direction 3) ------------------
    // tune::kWtahvInterleaveV: one after the other (0), or interleaved, step i
    // of one next to step TY-1-i of the other (1: two independent dependency
    // chains per wave).
    if (vcol) {
        if (ty > 0)
            load_state<DPL, PAD, PIN>(make_rsrc(CKV, g.vck), ((unsigned)(ty - 1) * uW + xv) * uD + lane_d,
                                 Aa, ma, padm);
        else
            zero_state(Aa, ma);
        if (y0 + TY < H)
            load_state<DPL, PAD, PIN>(make_rsrc(CKV + g.vck, g.vck),
                                 ((unsigned)(ty + 1) * uW + xv) * uD + lane_d, Ab, mb, padm);
        else
            zero_state(Ab, mb);
        // The down pass keeps each pixel's L_2 (KEEP16, tune::kWtahvKeepU16: as the
        // step's u16 pairs, so V = L_2 + L_3 is NP packed adds; else u8-packed,
        // re-expanded here with two v_perm per word).
        constexpr int NK = KEEP16 ? NP : NW;
        auto keep = [&](unsigned (&dst)[NK], const unsigned (&A)[NP], const unsigned (&ow)[NW]) {
#pragma unroll
            for (int q = 0; q < NK; q++) dst[q] = KEEP16 ? A[q] : ow[q];
        };
        auto put_v = [&](int r, const unsigned (&ld)[NK], const unsigned (&Au)[NP],
                         const unsigned (&lu)[NW]) {
            unsigned V[NP];
            if constexpr (KEEP16) {
#pragma unroll
                for (int p = 0; p < NP; p++) V[p] = ld[p] + Au[p];   // L_2 + L_3 (<= 510 per half)
            } else {
                words_to_pairs<DPL>(ld, V);
                unpack_add<NW>(lu, V);
            }
            unsigned* dst = &vsum[(r * TW + slot) * 16 * NP];
#pragma unroll
            for (int p = 0; p < NP; p++) dst[vw(p)] = V[p];
        };
        unsigned LD[TY][NK];
        if constexpr (tune::kWtahvInterleaveV != 0) {
            unsigned LU[TY][NK];
            for_seq<TY>([&](auto I) {
                constexpr int i = decltype(I)::value, ru = TY - 1 - i;
                unsigned ow[NW];
                if (i < ny) { sgm_step<DPL, PIN>(cv[i].w, Aa, ma, ow, P1, P2, ea); keep(LD[i], Aa, ow); }
                if (ru < ny) { sgm_step<DPL, PIN>(cv[ru].w, Ab, mb, ow, P1, P2, eb); keep(LU[ru], Ab, ow); }
            });
            for_seq<TY>([&](auto R) {
                constexpr int r = decltype(R)::value;
                if (r < ny) {
                    if constexpr (KEEP16) {
                        const unsigned none[NW] = {};
                        put_v(r, LD[r], LU[r], none);
                    } else {
                        unsigned V[NP] = {};
                        put_v(r, LD[r], V, LU[r]);
                    }
                }
            });
        } else {
            unsigned cvp[UNPACK1 ? TY : 1][NP];           // row r's cost pairs (UNPACK1)
            for_seq<TY>([&](auto I) {
                constexpr int i = decltype(I)::value;
                unsigned ow[NW];
                if (i < ny) {
                    if constexpr (UNPACK1) {
                        words_to_pairs<DPL>(cv[i].w, cvp[i]);
                        sgm_step_c<DPL, PIN>(cvp[i], Aa, ma, ow, P1, P2, ea);
                    } else {
                        sgm_step<DPL, PIN>(cv[i].w, Aa, ma, ow, P1, P2, ea);
                    }
                    keep(LD[i], Aa, ow);
                }
            });
            for_seq<TY>([&](auto Q) {
                constexpr int r = TY - 1 - decltype(Q)::value;
                if (r < ny) {
                    unsigned lu[NW];
                    if constexpr (UNPACK1) sgm_step_c<DPL, PIN>(cvp[UNPACK1 ? r : 0], Ab, mb, lu, P1, P2, eb);
                    else sgm_step<DPL, PIN>(cv[r].w, Ab, mb, lu, P1, P2, eb);
                    put_v(r, LD[r], Ab, lu);
                }
            });
        }
    }
    if constexpr (ND > 0) {
        // ---- phase D: diagonals recomputed per tile ------
        // Direction 4 (+x) and 6 (-x) come down from the row checkpoint at
        // y0 - 1, 5 (-x) and 7 (+x) up from the one at y0 + TY (zero state at
        // the image's top / bottom edge).  Each has NL = 16 + TY - 1 lines
        // crossing the tile; a line's first TY - 1 pixels can lie in the halo
        // beside it.  In-tile pixels add L into V with LDS atomics (packed u16
        // pairs: V + four diagonals <= 1530 per half, no carry), so every
        // direction's runs share the slots in any order.  A line off the
        // image restarts (zero state) like the path kernel's wrapped lines.
        __syncthreads();                              // V stored before the adds
        constexpr int NL = TW + TY - 1;
        constexpr int NRUN = (ND * NL + 15) / 16;     // runs per slot
        const rsrc_t rCKD = make_rsrc(CKV + 2 * (size_t)g.vck, (unsigned)ND * g.vck);
        // run i of this slot: line q = slot + 16 i of the ND * NL
        struct Run {
            int c, rx, yck;   // column at the checkpoint row, x step, checkpoint segment
            unsigned plane;   // its plane in rCKD
            bool up, ok;
        };
        auto run_of = [&](int i) __attribute__((always_inline)) -> Run {
            Run u;
            const int q = slot + 16 * i;
            const int dd = q / NL, li = q - dd * NL;
            u.ok = q < ND * NL;
            u.up = !DOWN || dd >= 2;
            const int e = u.up && DOWN ? dd - 2 : dd;     // 0 or 1 within its pair
            // down: 4 (+x), 6 (-x); up: 5 (-x), 7 (+x)
            u.rx = u.up ? (e ? 1 : -1) : (e ? -1 : 1);
            u.c = u.rx > 0 ? x0 - TY + li : x0 + 1 + li;
            u.plane = (unsigned)dd;
            u.yck = u.up ? (y0 + TY < H ? ty + 1 : -1) : ty - 1;   // -1: no checkpoint
            return u;
        };
        auto issue_d = [&](int i, Words<NW>& ck, Words<NW> (&cd)[TY]) __attribute__((always_inline)) {
            const Run u = run_of(i);
            const bool ckin = u.yck >= 0 && (unsigned)u.c < (unsigned)W;
            ck = bload<NW>(rCKD, ckin ? u.plane * g.vck + ((unsigned)u.yck * uW + (unsigned)u.c) * uD +
                                            lane_d
                                      : 0u);
#pragma unroll
            for (int s = 0; s < TY; s++) {
                const int x = u.c + u.rx * (s + 1);
                const int y = u.up ? y0 + TY - 1 - s : y0 + s;
                cd[s] = bload<NW>(rC, (unsigned)x < (unsigned)W && y < H
                                          ? ((unsigned)y * uW + (unsigned)x) * uD + lane_d
                                          : 0u);
            }
        };
        auto run_d = [&](int i, const Words<NW>& ck, const Words<NW> (&cd)[TY]) __attribute__((always_inline)) {
            const Run u = run_of(i);
            if (!u.ok) return;                        // uniform per 16-lane row
            unsigned A[NP], m;
            if (u.yck >= 0 && (unsigned)u.c < (unsigned)W) state_from_words<DPL, PAD, PIN>(ck, A, m, padm);
            else zero_state(A, m);
            for_seq<TY>([&](auto R) {
                constexpr int s = decltype(R)::value;
                const int x = u.c + u.rx * (s + 1);
                const int r = u.up ? TY - 1 - s : s;      // tile row
                if ((unsigned)x < (unsigned)W && r < ny) {
                    unsigned ow[NW];
                    sgm_step<DPL, PIN>(cd[s].w, A, m, ow, P1, P2, eb);
                    if (x >= x0 && x < x0 + nx) {
                        unsigned* dst = &vsum[(r * TW + (x - x0)) * 16 * NP];
#pragma unroll
                        for (int p = 0; p < NP; p++) atomicAdd(&dst[vw(p)], A[p]);
                    }
                } else {
                    zero_state(A, m);                   // off the image: restart
                }
            });
        };
        if constexpr (DPL <= 8) {
            // the next run's loads go out before this run's recurrence
            Words<NW> ck[2], cd[2][TY];
            issue_d(0, ck[0], cd[0]);
            for_seq<NRUN>([&](auto I) {
                constexpr int i = decltype(I)::value;
                if constexpr (i + 1 < NRUN) issue_d(i + 1, ck[(i + 1) & 1], cd[(i + 1) & 1]);
                run_d(i, ck[i & 1], cd[i & 1]);
            });
        } else {
            Words<NW> ck, cd[TY];
            for_seq<NRUN>([&](auto I) {
                constexpr int i = decltype(I)::value;
                issue_d(i, ck, cd);
                run_d(i, ck, cd);
            });
        }
    }
    if constexpr (tune::kWtahvRowCFirst == 0) load_row();
    // phase H's first global loads (checkpoints, diagonal volumes) go out
    // before the barrier (tune::kWtahvEarlyLoads)
    const int hs = hx >> TYL;                          // the row segment's index
    const unsigned ckrow = yh * (unsigned)g.nsx;
    Words<NW> ckw[2];
    constexpr int NVA = NV > 0 ? NV : 1;               // (array extent; NV may be 0)
    rsrc_t rV[NVA];
#pragma unroll
    for (int r = 0; r < NV; r++) rV[r] = make_rsrc(L4 + (size_t)r * g.vol, g.vol);
    Words<NW> rv[kPfVol][NVA];
    auto issue = [&](int s, int j) {
        const unsigned off = (yh * uW + (unsigned)(hx + j)) * uD + lane_d;
#pragma unroll
        for (int r = 0; r < NV; r++) rv[s][r] = bload<NW, 2>(rV[r], off);   // last use: nt
    };
    auto issue_first = [&]() {
        // (words outside the image are never used: the first / last segment
        // starts from zero state)
        ckw[0] = bload<NW>(make_rsrc(CK, g.hck), (ckrow + (unsigned)(hs - 1)) * uD + lane_d);
        ckw[1] = bload<NW>(make_rsrc(CK + g.hck, g.hck), (ckrow + (unsigned)(hs + 1)) * uD + lane_d);
#pragma unroll
        for (int q = 0; q < kPfVol && q < TY; q++) issue(q, TY - 1 - q);
    };
    if constexpr (tune::kWtahvEarlyLoads != 0) {
        if (hrow) issue_first();
    }
    __syncthreads();

    // ---- phase H: left-to-right (direction 0), then right-to-left (1) with
    // the sum and the WTA per pixel
    if (!hrow) return;                                 // whole 16-lane row leaves together
    if constexpr (tune::kWtahvEarlyLoads == 0) issue_first();
    if (hs > 0) state_from_words<DPL, PAD, PIN>(ckw[0], Aa, ma, padm);
    else zero_state(Aa, ma);
    // L_0 of the segment's pixels, kept like phase V's L_2 (KEEP16H)
    constexpr int NKH = KEEP16H ? NP : NW;
    unsigned LF[TY][NKH];
    unsigned chp[UNPACK1 ? TY : 1][NP];                // pixel i's cost pairs (UNPACK1)
    for_seq<TY>([&](auto I) {
        constexpr int i = decltype(I)::value;
        unsigned ow[NW];
        if (i < nh) {
            if constexpr (UNPACK1) {
                words_to_pairs<DPL>(ch[i].w, chp[i]);
                sgm_step_c<DPL, PIN>(chp[i], Aa, ma, ow, P1, P2, ea);
            } else {
                sgm_step<DPL, PIN>(ch[i].w, Aa, ma, ow, P1, P2, ea);
            }
#pragma unroll
            for (int q = 0; q < NKH; q++) LF[i][q] = KEEP16H ? Aa[q] : ow[q];
        }
    });
    if (hx + TY < W) state_from_words<DPL, PAD, PIN>(ckw[1], Aa, ma, padm);
    else zero_state(Aa, ma);
    unsigned dres = 0u, sm = 0u, s0 = 0u;
    const bool want_sub = sub != nullptr;
    unsigned dpair[NP];                                // each pair's two d (kWtahvKeyPerm)
#pragma unroll
    for (int j = 0; j < NP; j++)
        dpair[j] = (lane_d + (unsigned)pair_d<DPL>(j, 0)) | ((lane_d + (unsigned)pair_d<DPL>(j, 1)) << 16);
    constexpr bool DEFER = tune::kWtahvSubLds != 0 && tune::kWtahvSubDeferred != 0;
    unsigned* const vrow = &vsum[(hr * TW + hseg * TY) * 16 * NP];   // the segment's V blocks
    for_seq<TY>([&](auto Q) {
        constexpr int q = decltype(Q)::value, j = TY - 1 - q, s = q % kPfVol;
        if (j < nh) {
            unsigned ow[NW];
            if constexpr (UNPACK1) sgm_step_c<DPL, PIN>(chp[UNPACK1 ? j : 0], Aa, ma, ow, P1, P2, ea);
            else sgm_step<DPL, PIN>(ch[j].w, Aa, ma, ow, P1, P2, ea);
            unsigned* const vpix = vrow + j * 16 * NP;                     // this pixel's V
            unsigned S[NP];
#pragma unroll
            for (int p = 0; p < NP; p++) S[p] = vpix[vw(p)] + Aa[p];   // V + L_1
            if constexpr (KEEP16H) {
#pragma unroll
                for (int p = 0; p < NP; p++) S[p] += LF[j][p];     // + L_0
            } else {
                unpack_add<NW>(LF[j], S);
            }
#pragma unroll
            for (int r = 0; r < NV; r++) unpack_add<NW>(rv[s][r].w, S);
            if constexpr (PAD) {
#pragma unroll
                for (int p = 0; p < NP; p++) S[p] |= padm[p];
            }
            unsigned spm, sb;
            if constexpr (tune::kWtahvSubLds != 0) {
                // S(d*-1) and S(d*+1) through LDS: every lane writes its S
                // pairs over the pixel's V block, which nothing reads again;
                // as u16 the block is S indexed by d (up to the swizzle).  The owning lane reads
                // the two neighbours (same wave, behind a wave barrier).
                const unsigned best = tune::kWtahvKeyPerm
                                          ? wta_pick_key_perm<DPL, PIN && tune::kWtahvPinWta>(S, dpair)
                                          : wta_pick_key<DPL, PIN && tune::kWtahvPinWta, tune::kSplitPairs != 0>(S, k);
                const int ds = (int)(best & 0xffffu);
                if (want_sub) {
#pragma unroll
                    for (int p = 0; p < NP; p++) vpix[vw(p)] = S[p];
                    if constexpr (!DEFER) {
                        // the owning lane reads what other lanes of this wave just
                        // wrote: state the ordering (a wave's LDS operations
                        // execute in issue order, so this costs no instruction)
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    }
                }
                if constexpr (DEFER) {
                    dres = k == j ? (unsigned)ds : dres;
                    s0 = k == j ? best >> 16 : s0;
                } else if (k == j) {
                    dres = (unsigned)ds;
                    s0 = best >> 16;
                    if (want_sub) {
                        const uint16_t* s16 = reinterpret_cast<const uint16_t*>(vpix);
                        const int dm = ds > 0 ? ds - 1 : 0, dp = ds + 1 < 16 * DPL ? ds + 1 : ds;
                        // u16 of disparity d: pair (d / 2) % NP of lane d / DPL
                        auto at = [&](int d) {
                            const int kk = d / DPL, pp = pair_of<DPL>(d % DPL), hh = half_of<DPL>(d % DPL);
                            return (unsigned)s16[2 * (kk * NP + (pp ^ vsw_of(kk))) + hh];
                        };
                        sm = at(dm) | (at(dp) << 16);
                    }
                }
            } else {
                const int ds = wta_pick_raw<DPL, PIN && tune::kWtahvPinWta, tune::kSplitPairs != 0>(S, k, want_sub, &spm, &sb);
                if (k == j) {
                    dres = (unsigned)ds;
                    sm = spm;
                    s0 = sb;
                }
            }
        }
        if constexpr (q + kPfVol < TY) {
            __builtin_amdgcn_sched_barrier(0);
            issue(s, TY - 1 - (q + kPfVol));
            __builtin_amdgcn_sched_barrier(0);
        }
    });
    if constexpr (DEFER) {
        // S(d*-1), S(d*+1) of lane k's pixel (j = k) from the S its row wrote
        // over the pixel's V block (same wave: order, no barrier instruction)
        if (want_sub) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (k < nh) {
                const uint16_t* s16 = reinterpret_cast<const uint16_t*>(vrow + k * 16 * NP);
                const int ds = (int)dres;
                const int dm = ds > 0 ? ds - 1 : 0, dp = ds + 1 < 16 * DPL ? ds + 1 : ds;
                auto at = [&](int d) {
                    const int kk = d / DPL, pp = pair_of<DPL>(d % DPL), hh = half_of<DPL>(d % DPL);
                    return (unsigned)s16[2 * (kk * NP + (pp ^ vsw_of(kk))) + hh];
                };
                sm = at(dm) | (at(dp) << 16);
            }
        }
    }
    if (k < nh) {
        const size_t at = (size_t)yh * (size_t)W + (size_t)(hx + k);
        disp[at] = (uint16_t)(g.dmin + (int)dres);
        if (want_sub) sub[at] = subpixel(g.dmin, (int)dres, g.dreal, sm & 0xffffu, s0, sm >> 16);
    }
}

}  // namespace

bool wta_hv_supported(int D) { return D == 64 || D == 128 || D == 192 || D == 256; }

hipError_t launch_wta_hv(Ctx& c, const uint8_t* C, const uint8_t* L4, const uint8_t* CK,
                         const uint8_t* CKV, int W, int H, int D, int P1, int P2, int dmin,
                         uint16_t* disp, float* sub, int dreal, int npair) {
    // D <= 128 on the strip route: all eight directions recomputed per tile
    // from checkpoints, no diagonal volume (wta_strip.hip)
    if (tune::kStripRoute != 0 && wta_strip_supported(D))
        return launch_wta_strip(c, C, CK, CKV, W, H, D, P1, P2, dmin, disp, sub, dreal, npair);
    DispatchTimer t(c, "wta_hv");
    if (!wta_hv_supported(D)) return hipErrorInvalidValue;
    const TileGeom tg = tile_geom(W, H, D);
    WtaHvGeom g;
    g.W = W; g.H = H; g.D = D; g.P1 = P1; g.P2 = P2; g.dmin = dmin;
    g.dreal = dreal > 0 && dreal < D ? dreal : D;
    g.ntx = tg.ntx;
    g.nty = tg.nty;
    g.nsx = tg.nsx;
    const size_t vol = (size_t)W * H * D;
    if (vol >= (size_t)1 << 32) return hipErrorInvalidValue;
    g.vol = (unsigned)vol;
    g.hck = (unsigned)(tg.hck_bytes / 2);
    g.vck = (unsigned)(tg.vck_bytes / 2);
    const bool pad = g.dreal < D;
    if (npair < 1) return hipErrorInvalidValue;
    g.tiles = g.ntx * g.nty;
    const dim3 grid((unsigned)(g.tiles * npair));
#define SVA_WTAHV(DPL_, TYL_)                                                                 \
    if (pad)                                                                                  \
        hipExtLaunchKernelGGL((wta_hv_kernel<DPL_, TYL_, true>), grid, dim3(TB), 0, c.stream, \
                              t.start, t.stop, 0, C, L4, CK, CKV, g, disp, sub);              \
    else                                                                                      \
        hipExtLaunchKernelGGL((wta_hv_kernel<DPL_, TYL_, false>), grid, dim3(TB), 0,          \
                              c.stream, t.start, t.stop, 0, C, L4, CK, CKV, g, disp, sub);    \
    t.used = true
    constexpr int TYL = tune::kWtahvTileLog2, TYLW = tune::kWtahvTileLog2Wide;
    if (tg.seg_log2 != (D <= 128 ? TYL : TYLW)) return hipErrorInvalidValue;
    switch (D) {
        case 64: SVA_WTAHV(4, TYL); break;
        case 128: SVA_WTAHV(8, TYL); break;
        case 192: SVA_WTAHV(12, TYLW); break;
        case 256: SVA_WTAHV(16, TYLW); break;
        default: return hipErrorInvalidValue;
    }
#undef SVA_WTAHV
    return hipGetLastError();
}

}  // namespace sva
