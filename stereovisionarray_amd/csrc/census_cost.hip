// census_cost.hip -- 9x7 Census + Hamming cost volume in one kernel, for 1-D
// matching steps (SURVEY.md §8a rows A10 + A11).
//
// Produces exactly the bytes of census9x7_rows_kernel followed by
// hamming_cost_rows_kernel -- C[(y*W + x)*D + d] = popcount(CL(x,y) ^
// CR(x + dir*(dmin+d), y)), 62 where the matched column leaves the image --
// without the census maps ever reaching HBM, and without the census launch.
//
// A 256-thread workgroup owns PXB = 128 consecutive pixels of a band of 4
// rows.  Per row it needs the census words of its own 128 left pixels and of
// the NW = PXB + D - 1 right-image columns they match against; it forms them
// from an 8-row LDS ring of image bytes (the 7-row window plus the row being
// staged), exactly as the census kernel does (aligned dwords realigned with
// v_alignbyte, one v_sub_sdwa + v_alignbit per bit).  The right census is
// formed (PXB + D - 1) / PXB ~ 2x over at D = 128 -- VALU the bandwidth-bound
// cost kernel has spare.  One barrier per row, phase p:
//   census of row y0+p         -> words[p & 1]          (ring rows y0+p-3..+3)
//   cost of row y0+p-1         <- words[(p-1) & 1]      (16-byte nt stores)
//   stage image row y0+p+4     -> ring slot of row y0+p-4 (read by no one now)
// HBM bytes: 1 B/disparity written + ~1.4 B/pixel of image read.
// dreal < D (a padded frame): disparities d >= dreal get 255.
#include "sva_device.h"
#include "sva_internal.h"
#include "sva_tuning.h"

namespace sva {
namespace {

constexpr int CC_BLOCK = 256;
// pixels per workgroup row, per disparity width (tune::kCensusCostPx*)
template <int NC> constexpr int pxb_of() { return NC > 8 ? tune::kCensusCostPxWide : tune::kCensusCostPx; }
constexpr int RING = 8;              // image rows in LDS (power of two)
constexpr int HX = 4, HY = 3;        // half window (9 wide, 7 high)
constexpr uint64_t kOutsideCC = 1ull << 63;   // never set in a census word (bits 0..61)

__device__ __forceinline__ void store16_nt(uint8_t* p, const unsigned (&o)[4]) {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    if constexpr (tune::kCostStoreNT)
        __builtin_nontemporal_store((v4u){o[0], o[1], o[2], o[3]}, (v4u*)p);
    else
        *(v4u*)p = (v4u){o[0], o[1], o[2], o[3]};
}

// Census word of the pixel whose 9-byte window row starts at byte s of each
// ring row; `rows[dy+3]` are the dword views of ring rows y-3 .. y+3.
__device__ __forceinline__ uint64_t census_at(const unsigned* const* rows, int s) {
    return census9x7(rows, s >> 2, (unsigned)(s & 3));
}

template <int NC>
__global__ __launch_bounds__(CC_BLOCK) void census_cost_kernel(
    const uint8_t* __restrict__ left, const uint8_t* __restrict__ right, int W, int H,
    size_t pitch, int dmin, int dir, int rows, int dreal, uint8_t* __restrict__ C) {
    constexpr int D = NC * 16;
    constexpr int PXB = pxb_of<NC>();
    constexpr int NW = PXB + D - 1;                      // right census words per row
    constexpr int RW = (NW + 8 + 4 + 3) / 4 * 4;         // right ring row bytes (+ dword overrun)
    constexpr int LW = (PXB + 8 + 4 + 3) / 4 * 4;        // left ring row bytes
    constexpr int SPAN = NW + 8 + PXB + 8;               // image bytes staged per row
    constexpr int LOADS = (SPAN + CC_BLOCK - 1) / CC_BLOCK;
    constexpr int NWORDS = NW + PXB;                     // census words formed per row
    constexpr int WPT = (NWORDS + CC_BLOCK - 1) / CC_BLOCK;
    static_assert(PXB % 64 == 0 && NC % 4 == 0, "cost tasks must tile the workgroup");
    __shared__ __attribute__((aligned(16))) uint8_t ringR[RING][RW];
    __shared__ __attribute__((aligned(16))) uint8_t ringL[RING][LW];
    __shared__ uint64_t rw[2][NW];
    __shared__ uint64_t lw[2][PXB];

    const int bpr = (W + PXB - 1) / PXB;
    const int bx = blockIdx.x % bpr, by = blockIdx.x / bpr;
    const int x0 = bx * PXB, y0 = by * rows;
    const int nrows = min(H, y0 + rows) - y0;
    const int t = threadIdx.x;
    // right word j <-> column colR(j); ring byte i <-> image column cbR + i
    const int colR0 = dir > 0 ? x0 + dmin : x0 + PXB - 1 - dmin;        // column of word 0
    const int cminR = dir > 0 ? colR0 : colR0 - (NW - 1);
    const int cbR = cminR - HX, cbL = x0 - HX;
    const bool border = cminR < 0 || cminR + NW > W;

    auto fetch = [&](int gy, uint8_t (&v)[LOADS]) {
#pragma unroll
        for (int k = 0; k < LOADS; k++) {
            const int i = t + k * CC_BLOCK;
            int col;
            const uint8_t* img;
            if (i < NW + 8) { col = cbR + i; img = right; }
            else { col = cbL + (i - (NW + 8)); img = left; }
            v[k] = (i < SPAN && (unsigned)col < (unsigned)W && (unsigned)gy < (unsigned)H)
                       ? img[(size_t)gy * pitch + col] : 0;
        }
    };
    auto stage = [&](int gy, const uint8_t (&v)[LOADS]) {
        const int slot = gy & (RING - 1);
#pragma unroll
        for (int k = 0; k < LOADS; k++) {
            const int i = t + k * CC_BLOCK;
            if (i < NW + 8) ringR[slot][i] = v[k];
            else if (i < SPAN) ringL[slot][i - (NW + 8)] = v[k];
        }
    };

    // prologue: rows y0-3 .. y0+3 in the ring, row y0+4 in registers
    // (all 8 rows' loads are issued before any is waited on)
    uint8_t pro[2 * HY + 1][LOADS];
#pragma unroll
    for (int r = -HY; r <= HY; r++) fetch(y0 + r, pro[r + HY]);
    uint8_t pre[LOADS];
    fetch(y0 + HY + 1, pre);
#pragma unroll
    for (int r = -HY; r <= HY; r++) stage(y0 + r, pro[r + HY]);
    __syncthreads();

    for (int p = 0; p <= nrows; p++) {
        if (p < nrows) {                                  // census of row y
            const int y = y0 + p;
            const bool yin = y >= HY && y < H - HY;
            const unsigned* rR[7];
            const unsigned* rL[7];
#pragma unroll
            for (int dy = -HY; dy <= HY; dy++) {
                rR[dy + HY] = reinterpret_cast<const unsigned*>(ringR[(y + dy) & (RING - 1)]);
                rL[dy + HY] = reinterpret_cast<const unsigned*>(ringL[(y + dy) & (RING - 1)]);
            }
            uint64_t* rwb = rw[p & 1];
            uint64_t* lwb = lw[p & 1];
#pragma unroll
            for (int k = 0; k < WPT; k++) {
                const int w = t + k * CC_BLOCK;
                if (w < NW) {
                    const int col = dir > 0 ? colR0 + w : colR0 - w;
                    uint64_t word;
                    if ((unsigned)col >= (unsigned)W) word = kOutsideCC;
                    else if (!yin || col < HX || col >= W - HX) word = 0;
                    else word = census_at(rR, col - cminR);
                    rwb[w] = word;
                } else if (w < NWORDS) {
                    const int lp = w - NW, x = x0 + lp;
                    uint64_t word = 0;
                    if (yin && x >= HX && x < W - HX) word = census_at(rL, lp);
                    lwb[lp] = word;
                }
            }
        }
        if (p > 0) {                                      // cost of row y - 1
            const int y = y0 + p - 1;
            const uint64_t* rwb = rw[(p - 1) & 1];
            const uint64_t* lwb = lw[(p - 1) & 1];
            // a wave owns 16 pixels x all NC chunks per pass (lane (p, c) forms
            // chunks c, c+4, ...), so each 128-byte line is written by one wave
            // in back-to-back instructions; each 32-lane LDS group reads 16
            // pixels x 2 chunks: 32 consecutive words, conflict-free
            const int wv = t >> 6, ln = t & 63;
            const int pl = ln & 15, c0 = ln >> 4;
#pragma unroll
            for (int k = 0; k < PXB / 64; k++) {
                const int lp = 16 * (wv + 4 * k) + pl;
                const int x = x0 + lp;
                if (x >= W) continue;
                const uint64_t lc = lwb[lp];
                const uint64_t* base = rwb + (dir > 0 ? lp : PXB - 1 - lp);
#pragma unroll
                for (int cc = 0; cc < NC / 4; cc++) {
                    const int c = c0 + 4 * cc;
                    const uint64_t* src = base + 16 * c;
                    unsigned out[4];
                    if (!border) {
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            unsigned ww = 0;
#pragma unroll
                            for (int b = 0; b < 4; b++)
                                ww |= (unsigned)__popcll(lc ^ src[q * 4 + b]) << (8 * b);
                            out[q] = ww;
                        }
                    } else {
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            unsigned ww = 0;
#pragma unroll
                            for (int b = 0; b < 4; b++) {
                                const uint64_t v = lc ^ src[q * 4 + b];
                                const unsigned cst = (v >> 63) ? 62u : (unsigned)__popcll(v);
                                ww |= cst << (8 * b);
                            }
                            out[q] = ww;
                        }
                    }
                    if (dreal < D) {                 // padded disparities: cost 255
#pragma unroll
                        for (int q = 0; q < 4; q++) out[q] |= pad_bytes(16 * c + 4 * q, dreal);
                    }
                    store16_nt(C + ((size_t)y * W + x) * D + 16 * c, out);
                }
            }
        }
        if (p < nrows) {                                  // stage row y0+p+4, fetch the next
            stage(y0 + p + HY + 1, pre);
            if (p + 1 < nrows) fetch(y0 + p + HY + 2, pre);
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
    const int rows = tune::kCensusCostRows;
    const int PXB = D > 128 ? pxb_of<16>() : pxb_of<8>();
    const int bpr = (W + PXB - 1) / PXB;
    const dim3 grid((unsigned)(bpr * ((H + rows - 1) / rows)));
    const int sd = dir > 0 ? 1 : -1;
    switch (D) {
        case 64: hipLaunchKernelGGL(census_cost_kernel<4>, grid, dim3(CC_BLOCK), 0, c.stream, left, right, W, H, pitch, dmin, sd, rows, dreal, C); break;
        case 128: hipLaunchKernelGGL(census_cost_kernel<8>, grid, dim3(CC_BLOCK), 0, c.stream, left, right, W, H, pitch, dmin, sd, rows, dreal, C); break;
        case 192: hipLaunchKernelGGL(census_cost_kernel<12>, grid, dim3(CC_BLOCK), 0, c.stream, left, right, W, H, pitch, dmin, sd, rows, dreal, C); break;
        case 256: hipLaunchKernelGGL(census_cost_kernel<16>, grid, dim3(CC_BLOCK), 0, c.stream, left, right, W, H, pitch, dmin, sd, rows, dreal, C); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace sva
