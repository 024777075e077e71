// census_cost.hip -- 9x7 Census + Hamming cost volume in one kernel, for 1-D
// matching steps (SURVEY.md §8a rows A10 + A11).
//
// Produces exactly the bytes of census9x7_rows_kernel followed by
// hamming_cost_rows_kernel -- C[(y*W + x)*D + d] = popcount(CL(x,y) ^
// CR(x + dir*(dmin+d), y)), 62 where the matched column leaves the image --
// without the census maps ever reaching HBM, and with the Hamming distances
// on the matrix cores (round 4; the round-1 kernel computed them with two
// v_xor + two v_bcnt + a pack per disparity on the VALU).
//
// A 256-thread workgroup owns PXB = 64 or 128 consecutive pixels (per D,
// tune::kCensusCostPx*) of a band of 8 rows (4 for frames too small to fill
// the chip that way), from an 8-row LDS ring of image bytes (the 7-row window
// plus the row being staged).  Per row, between two barriers:
//   A  every census window of the row -- its PXB left pixels and the
//      PXB + D - 1 right columns they match -- becomes one 64-byte operand
//      row in LDS, straight from the image bytes (census_bytes: four
//      comparisons per SWAR step, no census word in between); the staged
//      costs of the previous row leave as whole 128-byte lines (nt stores);
//   B  each wave takes one residue class of pixels mod 4 and multiplies its
//      16-pixel tiles by the right columns' tiles on v_mfma_i32_16x16x64_i8;
//      each lane packs its four results -- four consecutive disparities of
//      one pixel -- into a u8x4 word of the staged row; the next image row
//      is staged into the ring slot nobody reads now.
// HBM bytes: 1 B/disparity written + ~1.4 B/pixel of image read.
// dreal < D (a padded frame): disparities d >= dreal get 255.
#include "census_mma.h"
#include "sva_device.h"
#include "sva_internal.h"
#include "sva_tuning.h"

namespace sva {
namespace {

constexpr int CC_BLOCK = 256;
constexpr int RING = 8;              // image rows in LDS (power of two)
constexpr int HX = 4, HY = 3;        // half window (9 wide, 7 high)

__device__ __forceinline__ void store16_nt(uint8_t* p, const unsigned (&o)[4]) {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    if constexpr (tune::kCostStoreNT)
        __builtin_nontemporal_store((v4u){o[0], o[1], o[2], o[3]}, (v4u*)p);
    else
        *(v4u*)p = (v4u){o[0], o[1], o[2], o[3]};
}

// The operand bytes of a census window and the dot-product identity behind
// them: census_mma.h.

// pixels per workgroup row (a multiple of 64: 4 residue classes x 16)
template <int NC> constexpr int mma_px() {
    return NC == 4 ? tune::kCensusCostPx4 : NC == 8 ? tune::kCensusCostPx8
                   : NC == 12 ? tune::kCensusCostPx12 : tune::kCensusCostPx16;
}

template <int NC, int DIR>
__global__ __launch_bounds__(CC_BLOCK) void census_cost_mma_kernel(
    const uint8_t* __restrict__ left, const uint8_t* __restrict__ right, int W, int H,
    size_t pitch, int dmin, int rows, int dreal, uint8_t* __restrict__ C) {
    constexpr int D = NC * 16;
    constexpr int PXB = mma_px<NC>();                    // pixels per workgroup row
    constexpr int NSPAN = PXB / 64;                      // N-tiles per residue class
    constexpr int T = (D + 60 + 15) / 16;                // M-tiles per N-tile (16 T = D + 64)
    constexpr int NWM = PXB + D - 1;                     // right columns some pixel matches
    // operand rows: 16 front rows + NWM, rounded to 16 (planes 256-B aligned); the
    // tiles' last 4 rows (d >= D for every pixel) read the padding rows
    constexpr int NWMP = (16 + NWM + 4 + 15) / 16 * 16;
    constexpr int RW = (NWM + 8 + 4 + 3) / 4 * 4;        // right ring row bytes (+ dword overrun)
    constexpr int LW = (PXB + 8 + 4 + 3) / 4 * 4;        // left ring row bytes
    constexpr int SPAN = NWM + 8 + PXB + 8;              // image bytes staged per row
    constexpr int LOADS = (SPAN + CC_BLOCK - 1) / CC_BLOCK;
    constexpr int NWORDS = PXB + NWM;                    // census words formed per row (left first)
    constexpr int WPT = (NWORDS + CC_BLOCK - 1) / CC_BLOCK;
    // staging dwords per pixel slot: the D / 4 words, then 4 dump words (lane
    // quarter q's word when it holds no disparity of this pixel) and 3 spare;
    // S4 = 3 mod 4 keeps a wave's 32-lane write groups on distinct banks
    constexpr int S4 = NC * 4 + 7;
    static_assert(CC_BLOCK == 256 && PXB % 64 == 0, "four waves, one residue class each");
    __shared__ __attribute__((aligned(16))) uint8_t ringR[RING][RW];
    __shared__ __attribute__((aligned(16))) uint8_t ringL[RING][LW];
    __shared__ __attribute__((aligned(16))) uint8_t opA[4 * NWMP * 16];   // [K quarter][column][16]
    __shared__ __attribute__((aligned(16))) uint8_t opB[4 * PXB * 16];    // [K quarter][pixel][16]
    __shared__ unsigned stg[PXB * S4];                                     // [pixel slot][S4]

    const int bpr = (W + PXB - 1) / PXB;
    const int bx = blockIdx.x % bpr, by = blockIdx.x / bpr;
    const int x0 = bx * PXB, y0 = by * rows;
    const int nrows = min(H, y0 + rows) - y0;
    const int t = threadIdx.x;
    // operand row 16 + i of opA <-> right column xlo + i; ring byte i <-> column cbR + i
    const int xlo = DIR > 0 ? x0 + dmin : x0 + 1 - dmin - D;
    const int cbR = xlo - HX, cbL = x0 - HX;

    auto fetch = [&](int gy, uint8_t (&v)[LOADS]) {
#pragma unroll
        for (int k = 0; k < LOADS; k++) {
            const int i = t + k * CC_BLOCK;
            int col;
            const uint8_t* img;
            if (i < NWM + 8) { col = cbR + i; img = right; }
            else { col = cbL + (i - (NWM + 8)); img = left; }
            v[k] = (i < SPAN && (unsigned)col < (unsigned)W && (unsigned)gy < (unsigned)H)
                       ? img[(size_t)gy * pitch + col] : 0;
        }
    };
    auto stage = [&](int gy, const uint8_t (&v)[LOADS]) {
        const int slot = gy & (RING - 1);
#pragma unroll
        for (int k = 0; k < LOADS; k++) {
            const int i = t + k * CC_BLOCK;
            if (i < NWM + 8) ringR[slot][i] = v[k];
            else if (i < SPAN) ringL[slot][i - (NWM + 8)] = v[k];
        }
    };
    uint8_t pro[2 * HY + 1][LOADS];
#pragma unroll
    for (int r = -HY; r <= HY; r++) fetch(y0 + r, pro[r + HY]);
    uint8_t pre[LOADS];
    fetch(y0 + HY + 1, pre);
#pragma unroll
    for (int r = -HY; r <= HY; r++) stage(y0 + r, pro[r + HY]);
    __syncthreads();

    const int wv = t >> 6, l = t & 63, ln = l & 15, lq = l >> 4;
    for (int p = 0; p <= nrows; p++) {
        // ---- census of row y0+p into the operand rows; store of row y0+p-1
        if (p < nrows) {
            const int y = y0 + p;
            const bool yin = y >= HY && y < H - HY;
            const unsigned* rR[7];
            const unsigned* rL[7];
#pragma unroll
            for (int dy = -HY; dy <= HY; dy++) {
                rR[dy + HY] = reinterpret_cast<const unsigned*>(ringR[(y + dy) & (RING - 1)]);
                rL[dy + HY] = reinterpret_cast<const unsigned*>(ringL[(y + dy) & (RING - 1)]);
            }
#pragma unroll
            for (int k = 0; k < WPT; k++) {
                const int w = t + k * CC_BLOCK;
                unsigned d[16];
                if (w < PXB) {
                    // operand row b <-> pixel 4 (b % (PXB/4)) + b / (PXB/4): the
                    // rows of one residue class are consecutive
                    const int b = w;
                    const int lp = 4 * (b % (PXB / 4)) + b / (PXB / 4), x = x0 + lp;
                    if (yin && x >= HX && x < W - HX) {
                        census_bytes<true>(rL, lp, d);
                    } else {                                       // census word 0
#pragma unroll
                        for (int q = 0; q < 15; q++) d[q] = 0x01010101u;
                        d[15] = 0x00010101u;                       // b_63 = popcount 0
                    }
                    put_operand_row(opB, PXB, b, d);
                } else if (w < NWORDS) {
                    const int i = w - PXB, col = xlo + i;
                    if ((unsigned)col >= (unsigned)W) {
                        // outside: a_k = 1 on the 62 census positions (not the
                        // centre, dword 7 byte 0), a_63 = 2 -> cost 62
#pragma unroll
                        for (int q = 0; q < 15; q++) d[q] = 0x01010101u;
                        d[7] = 0x01010100u;
                        d[15] = 0x02010101u;
                    } else if (yin && col >= HX && col < W - HX) {
                        census_bytes<false>(rR, i, d);
                    } else {                                       // census word 0
#pragma unroll
                        for (int q = 0; q < 15; q++) d[q] = 0u;
                        d[15] = 0x01000000u;                       // a_63 = 1
                    }
                    put_operand_row(opA, NWMP, 16 + i, d);
                }
            }
        }
        if (p > 0) {
            // pixel lp's slot: class c = lp & 3, span s = lp >> 6, lane n
            const int y = y0 + p - 1;
#pragma unroll
            for (int k = 0; k < PXB * NC / CC_BLOCK; k++) {
                const int ch = t + k * CC_BLOCK;
                int lp, sl;
                const int ci = ch % NC;
                if constexpr (tune::kCensusCostSlotOrder) {
                    // chunks in staging-slot order: the 32 lanes of a read
                    // group take consecutive slots, whose rows start on
                    // distinct banks (S4 odd); in pixel order they took
                    // slots 16 apart, all on one bank set (4-way conflicts)
                    sl = ch / NC;
                    const int c = sl / (PXB / 4), r = sl % (PXB / 4), n = r & 15;
                    lp = 64 * (r >> 4) + 4 * (DIR > 0 ? n : 15 - n) + c;
                } else {
                    lp = ch / NC;
                    const int m = (lp >> 2) & 15, n = DIR > 0 ? m : 15 - m;
                    sl = (lp & 3) * (PXB / 4) + 16 * (lp >> 6) + n;
                }
                const int x = x0 + lp;
                if (x >= W) continue;
                const unsigned* src = &stg[sl * S4 + 4 * ci];
                unsigned out[4] = {src[0], src[1], src[2], src[3]};
                if (dreal < D) {                 // padded disparities: cost 255
#pragma unroll
                    for (int q = 0; q < 4; q++) out[q] |= pad_bytes(16 * ci + 4 * q, dreal);
                }
                store16_nt(C + ((size_t)y * W + x) * D + 16 * ci, out);
            }
        }
        __syncthreads();
        // ---- the costs of row y0+p on the matrix cores, into the staging rows
        if (p < nrows) {
            const int c = wv;                                   // this wave's residue class
            const v4i zero = {0, 0, 0, 0};
#pragma unroll
            for (int s = 0; s < NSPAN; s++) {
                const int m = DIR > 0 ? ln : 15 - ln;
                const v4i bf = *reinterpret_cast<const v4i*>(
                    &opB[(lq * PXB + c * (PXB / 4) + 16 * s + m) * 16]);
                // lane (n = ln, q = lq) holds rows 16 tt + 4q + i = disparities 4j + i;
                // tiles go in groups of G (G fragments + G accumulators live)
                unsigned* dst = &stg[(c * (PXB / 4) + 16 * s + ln) * S4];
                constexpr int G = 4;
#pragma unroll
                for (int g = 0; g < T; g += G) {
                    v4i acc[G];
#pragma unroll
                    for (int i = 0; i < G && g + i < T; i++) {
                        // row R = 4 n + d of pixel lane n (DIR < 0: that class's pixel 15 - n)
                        const int R = 16 * (g + i) + ln;
                        const int idx = DIR > 0 ? 64 * s + c + R : 64 * s + c + D + 59 - R;
                        const v4i af = *reinterpret_cast<const v4i*>(&opA[(lq * NWMP + 16 + idx) * 16]);
                        acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af, bf, zero, 0, 0, 0);
                    }
#pragma unroll
                    for (int i = 0; i < G && g + i < T; i++) {
                        const int j = 4 * (g + i) + lq - ln;
                        unsigned wd = (unsigned)acc[i][0] | ((unsigned)acc[i][1] << 8);
                        wd |= ((unsigned)acc[i][2] << 16) | ((unsigned)acc[i][3] << 24);
                        dst[(unsigned)j < (unsigned)(NC * 4) ? j : NC * 4 + lq] = wd;   // else: dump
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            stage(y0 + p + HY + 1, pre);
            if (p + 1 < nrows) fetch(y0 + p + HY + 2, pre);
        }
        __syncthreads();
    }
}

// The same census + cost with the two phases on different waves (round 6,
// tune::kCensusCostWS): a 512-thread workgroup whose waves 0-3 form the census
// operand rows of row p + 1 while waves 4-7 multiply row p's (two operand
// buffers) and store their own residue class's pixels, one barrier per row
// instead of two.  PXB = 64: each MFMA wave's 16 pixels are its own class, so
// it stores them behind a wave barrier.  Bit-identical to the kernel above.
template <int NC, int DIR>
__global__ __launch_bounds__(2 * CC_BLOCK) void census_cost_ws_kernel(
    const uint8_t* __restrict__ left, const uint8_t* __restrict__ right, int W, int H,
    size_t pitch, int dmin, int rows, int dreal, uint8_t* __restrict__ C) {
    constexpr int D = NC * 16;
    constexpr int PXB = 64;
    constexpr int T = (D + 60 + 15) / 16;
    constexpr int NWM = PXB + D - 1;
    constexpr int NWMP = (16 + NWM + 4 + 15) / 16 * 16;
    constexpr int RW = (NWM + 8 + 4 + 3) / 4 * 4;
    constexpr int LW = (PXB + 8 + 4 + 3) / 4 * 4;
    constexpr int SPAN = NWM + 8 + PXB + 8;
    constexpr int LOADS = (SPAN + CC_BLOCK - 1) / CC_BLOCK;
    constexpr int NWORDS = PXB + NWM;
    constexpr int WPT = (NWORDS + CC_BLOCK - 1) / CC_BLOCK;
    constexpr int S4 = NC * 4 + 7;
    __shared__ __attribute__((aligned(16))) uint8_t ringR[RING][RW];
    __shared__ __attribute__((aligned(16))) uint8_t ringL[RING][LW];
    __shared__ __attribute__((aligned(16))) uint8_t opA[2][4 * NWMP * 16];
    __shared__ __attribute__((aligned(16))) uint8_t opB[2][4 * PXB * 16];
    __shared__ unsigned stg[PXB * S4];

    const int bpr = (W + PXB - 1) / PXB;
    const int bx = blockIdx.x % bpr, by = blockIdx.x / bpr;
    const int x0 = bx * PXB, y0 = by * rows;
    const int nrows = min(H, y0 + rows) - y0;
    const int t = threadIdx.x, grp = t >> 8, tl = t & (CC_BLOCK - 1);   // grp: wave-uniform
    const int xlo = DIR > 0 ? x0 + dmin : x0 + 1 - dmin - D;
    const int cbR = xlo - HX, cbL = x0 - HX;

    auto fetch = [&](int gy, uint8_t (&v)[LOADS]) {
#pragma unroll
        for (int k = 0; k < LOADS; k++) {
            const int i = tl + k * CC_BLOCK;
            int col;
            const uint8_t* img;
            if (i < NWM + 8) { col = cbR + i; img = right; }
            else { col = cbL + (i - (NWM + 8)); img = left; }
            v[k] = (i < SPAN && (unsigned)col < (unsigned)W && (unsigned)gy < (unsigned)H)
                       ? img[(size_t)gy * pitch + col] : 0;
        }
    };
    auto stage = [&](int gy, const uint8_t (&v)[LOADS]) {
        const int slot = gy & (RING - 1);
#pragma unroll
        for (int k = 0; k < LOADS; k++) {
            const int i = tl + k * CC_BLOCK;
            if (i < NWM + 8) ringR[slot][i] = v[k];
            else if (i < SPAN) ringL[slot][i - (NWM + 8)] = v[k];
        }
    };
    // census operand rows of image row y into buffer b (group 0)
    auto census_row = [&](int y, int b) {
        const bool yin = y >= HY && y < H - HY;
        const unsigned* rR[7];
        const unsigned* rL[7];
#pragma unroll
        for (int dy = -HY; dy <= HY; dy++) {
            rR[dy + HY] = reinterpret_cast<const unsigned*>(ringR[(y + dy) & (RING - 1)]);
            rL[dy + HY] = reinterpret_cast<const unsigned*>(ringL[(y + dy) & (RING - 1)]);
        }
#pragma unroll
        for (int k = 0; k < WPT; k++) {
            const int w = tl + k * CC_BLOCK;
            unsigned d[16];
            if (w < PXB) {
                const int lp = 4 * (w % (PXB / 4)) + w / (PXB / 4), x = x0 + lp;
                if (yin && x >= HX && x < W - HX) census_bytes<true>(rL, lp, d);
                else census_zero<true>(d);
                put_operand_row(opB[b], PXB, w, d);
            } else if (w < NWORDS) {
                const int i = w - PXB, col = xlo + i;
                if ((unsigned)col >= (unsigned)W) census_outside(d);
                else if (yin && col >= HX && col < W - HX) census_bytes<false>(rR, i, d);
                else census_zero<false>(d);
                put_operand_row(opA[b], NWMP, 16 + i, d);
            }
        }
    };

    // prologue: image rows y0 - 3 .. y0 + 4 (the whole ring: the census of
    // rows 0 and 1), then row 0's operands
    {
        uint8_t v[4][LOADS];
#pragma unroll
        for (int r = 0; r < 4; r++) fetch(y0 - HY + 4 * grp + r, v[r]);
#pragma unroll
        for (int r = 0; r < 4; r++) stage(y0 - HY + 4 * grp + r, v[r]);
    }
    __syncthreads();
    if (grp == 0) census_row(y0, 0);
    uint8_t pre[LOADS];
    if (grp == 1) fetch(y0 + HY + 2, pre);
    __syncthreads();

    const int wv = (t >> 6) & 3, l = t & 63, ln = l & 15, lq = l >> 4;
    for (int p = 0; p < nrows; p++) {
        if (grp == 0) {
            if (p + 1 < nrows) census_row(y0 + p + 1, (p + 1) & 1);
        } else {
            const int b = p & 1, c = wv;                 // this wave's residue class
            const v4i zero = {0, 0, 0, 0};
            const int m = DIR > 0 ? ln : 15 - ln;
            const v4i bf = *reinterpret_cast<const v4i*>(&opB[b][(lq * PXB + c * (PXB / 4) + m) * 16]);
            unsigned* dst = &stg[(c * (PXB / 4) + ln) * S4];
            constexpr int G = 4;
#pragma unroll
            for (int g = 0; g < T; g += G) {
                v4i acc[G];
#pragma unroll
                for (int i = 0; i < G && g + i < T; i++) {
                    const int R = 16 * (g + i) + ln;
                    const int idx = DIR > 0 ? c + R : c + D + 59 - R;
                    const v4i af = *reinterpret_cast<const v4i*>(&opA[b][(lq * NWMP + 16 + idx) * 16]);
                    acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af, bf, zero, 0, 0, 0);
                }
#pragma unroll
                for (int i = 0; i < G && g + i < T; i++) {
                    const int j = 4 * (g + i) + lq - ln;
                    unsigned wd = (unsigned)acc[i][0] | ((unsigned)acc[i][1] << 8);
                    wd |= ((unsigned)acc[i][2] << 16) | ((unsigned)acc[i][3] << 24);
                    dst[(unsigned)j < (unsigned)(NC * 4) ? j : NC * 4 + lq] = wd;   // else: dump
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            // this wave's 16 pixels (class c) leave as whole lines: the lanes
            // read other lanes' staging words (same wave: LDS order, no barrier
            // instruction)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const int y = y0 + p;
#pragma unroll
            for (int k = 0; k < 16 * NC / 64; k++) {
                const int ch = l + 64 * k;
                const int sl = ch / NC, ci = ch % NC;      // slot sl of the class: pixel lane n = sl
                const int lp = 4 * (DIR > 0 ? sl : 15 - sl) + c, x = x0 + lp;
                if (x >= W) continue;
                const unsigned* src = &stg[(c * (PXB / 4) + sl) * S4 + 4 * ci];
                unsigned out[4] = {src[0], src[1], src[2], src[3]};
                if (dreal < D) {                 // padded disparities: cost 255
#pragma unroll
                    for (int q = 0; q < 4; q++) out[q] |= pad_bytes(16 * ci + 4 * q, dreal);
                }
                store16_nt(C + ((size_t)y * W + x) * D + 16 * ci, out);
            }
            stage(y0 + p + HY + 2, pre);
            if (p + 1 < nrows) fetch(y0 + p + HY + 3, pre);
        }
        __syncthreads();
    }
}

}  // namespace

bool census_cost_supported(int D) { return D == 64 || D == 128 || D == 192 || D == 256; }

hipError_t launch_census_cost(Ctx& c, const uint8_t* left, const uint8_t* right, int W, int H,
                              size_t pitch, int D, int dmin, int dir, uint8_t* C, int dreal) {
    if (dreal <= 0) dreal = D;
    ScopedKernelTimer t(c, "cost");
    // the wave-specialised kernel for D < 256 (PXB 64), tune::kCensusCostWS
    const bool ws = tune::kCensusCostWS != 0 && D <= 192;
    const int px = ws ? 64 : D == 64 ? mma_px<4>() : D == 128 ? mma_px<8>() : D == 192 ? mma_px<12>() : mma_px<16>();
    const long long bpr = (W + px - 1) / px;
    const int rows = bpr * ((H + tune::kCensusCostRows - 1) / tune::kCensusCostRows) >=
                             tune::kCensusCostMinGroups
                         ? tune::kCensusCostRows
                         : tune::kCensusCostRowsSmall;
    const dim3 grid((unsigned)(bpr * ((H + rows - 1) / rows)));
#define SVA_CC_MMA(NC_)                                                                            \
    if (ws && NC_ <= 12) {                                                                         \
        if (dir > 0)                                                                               \
            hipLaunchKernelGGL((census_cost_ws_kernel<(NC_ <= 12 ? NC_ : 12), 1>), grid,            \
                               dim3(2 * CC_BLOCK), 0, c.stream, left, right, W, H, pitch, dmin,    \
                               rows, dreal, C);                                                    \
        else                                                                                       \
            hipLaunchKernelGGL((census_cost_ws_kernel<(NC_ <= 12 ? NC_ : 12), -1>), grid,           \
                               dim3(2 * CC_BLOCK), 0, c.stream, left, right, W, H, pitch, dmin,    \
                               rows, dreal, C);                                                    \
    } else if (dir > 0)                                                                            \
        hipLaunchKernelGGL((census_cost_mma_kernel<NC_, 1>), grid, dim3(CC_BLOCK), 0, c.stream, left, \
                           right, W, H, pitch, dmin, rows, dreal, C);                             \
    else                                                                                           \
        hipLaunchKernelGGL((census_cost_mma_kernel<NC_, -1>), grid, dim3(CC_BLOCK), 0, c.stream,     \
                           left, right, W, H, pitch, dmin, rows, dreal, C);
    switch (D) {
        case 64: SVA_CC_MMA(4) break;
        case 128: SVA_CC_MMA(8) break;
        case 192: SVA_CC_MMA(12) break;
        case 256: SVA_CC_MMA(16) break;
        default: return hipErrorInvalidValue;
    }
#undef SVA_CC_MMA
    return hipGetLastError();
}

}  // namespace sva
