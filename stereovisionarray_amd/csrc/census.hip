// census.hip -- 9x7 Census transform.
//
// One thread per pixel.  A 64x4 workgroup tile stages its (64+8)x(4+6) halo
// through LDS so every image byte is read from HBM once (coalesced row
// segments), then each thread forms its 62-bit word from LDS.
// HBM bytes: 1 B/pixel read + 8 B/pixel write.
#include <cstdlib>

#include "sva_device.h"
#include "sva_internal.h"

namespace sva {
namespace {

constexpr int TX = 64, TY = 4;           // pixels per tile
constexpr int HX = 4, HY = 3;            // half window (9 wide, 7 high)
constexpr int LW = TX + 2 * HX;          // 72 LDS columns
constexpr int LH = TY + 2 * HY;          // 10 LDS rows

// blockIdx.z selects the image: the left and right census of a pair are one
// launch (img1/out1 may repeat img0/out0 for a single image).
__global__ __launch_bounds__(TX* TY) void census9x7_kernel(const uint8_t* __restrict__ img0,
                                                            const uint8_t* __restrict__ img1,
                                                            int W, int H, size_t pitch,
                                                            uint64_t* __restrict__ out0,
                                                            uint64_t* __restrict__ out1) {
    const uint8_t* __restrict__ img = blockIdx.z ? img1 : img0;
    uint64_t* __restrict__ out = blockIdx.z ? out1 : out0;
    __shared__ uint8_t tile[LH][LW];
    const int x0 = blockIdx.x * TX, y0 = blockIdx.y * TY;
    const int tid = threadIdx.y * TX + threadIdx.x;
    for (int i = tid; i < LW * LH; i += TX * TY) {
        int ly = i / LW, lx = i - ly * LW;
        int gx = x0 + lx - HX, gy = y0 + ly - HY;
        uint8_t v = 0;
        if (gx >= 0 && gx < W && gy >= 0 && gy < H) v = img[(size_t)gy * pitch + gx];
        tile[ly][lx] = v;
    }
    __syncthreads();
    const int x = x0 + threadIdx.x, y = y0 + threadIdx.y;
    if (x >= W || y >= H) return;
    uint64_t word = 0;
    if (x >= HX && x < W - HX && y >= HY && y < H - HY) {
        const int cx = threadIdx.x + HX, cy = threadIdx.y + HY;
        const unsigned c = tile[cy][cx];
        // Row-major window order, centre skipped: the first element lands in
        // bit 61.  Build the word in two 32-bit halves to keep VALU work short.
        unsigned hi = 0, lo = 0;
        int e = 0;
#pragma unroll
        for (int dy = -HY; dy <= HY; dy++) {
#pragma unroll
            for (int dx = -HX; dx <= HX; dx++) {
                if (dx == 0 && dy == 0) continue;
                unsigned bit = (unsigned)tile[cy + dy][cx + dx] < c ? 1u : 0u;
                if (e < 30) hi = (hi << 1) | bit;
                else lo = (lo << 1) | bit;
                e++;
            }
        }
        word = ((uint64_t)hi << 32) | lo;
    }
    out[(size_t)y * W + x] = word;
}

// Multi-row form: a 64x4 workgroup walks a 64-column strip of kCensusRows
// rows in steps of TY rows.  The 7-row window lives in a 16-row LDS ring, so
// each step loads only its TY new rows (prefetched into registers during the
// previous step's compute); rows outside the image stage as 0.  One barrier
// per step: ring slots are rewritten 4 steps after their rows were loaded and
// 2 steps after their last reads (a step reads rows y-3 .. y+TY+2).
constexpr int RING = 16;
#ifndef SVA_CENSUS_ROWS
#define SVA_CENSUS_ROWS 16
#endif
constexpr int kCensusRows = SVA_CENSUS_ROWS;
constexpr int LOADS = (TY * LW + TX * TY - 1) / (TX * TY);   // bytes per thread per step

__global__ __launch_bounds__(TX* TY) void census9x7_rows_kernel(
    const uint8_t* __restrict__ img0, const uint8_t* __restrict__ img1, int W, int H,
    size_t pitch, uint64_t* __restrict__ out0, uint64_t* __restrict__ out1, int rows,
    size_t ostride, int pr) {
    const uint8_t* __restrict__ img = blockIdx.z ? img1 : img0;
    uint64_t* __restrict__ out = blockIdx.z ? out1 : out0;
    __shared__ __attribute__((aligned(16))) uint8_t ring[RING][LW];   // LW = 72: rows dword-aligned
    const int x0 = blockIdx.x * TX, yb = blockIdx.y * rows;
    const int ye = min(H, yb + rows);
    const int tid = threadIdx.y * TX + threadIdx.x;
    auto load = [&](int gy, int lx) -> uint8_t {
        const int gx = x0 + lx - HX;
        return (gx >= 0 && gx < W && gy >= 0 && gy < H) ? img[(size_t)gy * pitch + gx] : 0;
    };
    // halo rows yb-3 .. yb+TY-2 (directly), then the TY rows of step 0 via registers
    for (int i = tid; i < (HY + TY - 1) * LW; i += TX * TY) {
        const int r = i / LW, lx = i - r * LW;
        const int gy = yb - HY + r;
        ring[(gy + RING) & (RING - 1)][lx] = load(gy, lx);
    }
    uint8_t pre[LOADS];
    auto prefetch = [&](int ybase) {   // rows ybase + HY .. ybase + HY + TY - 1
#pragma unroll
        for (int k = 0; k < LOADS; k++) {
            const int i = tid + k * TX * TY;
            const int r = i / LW, lx = i - r * LW;
            pre[k] = i < TY * LW ? load(ybase + HY + r, lx) : 0;
        }
    };
    prefetch(yb);
    const int x = x0 + threadIdx.x;
    for (int ys = yb; ys < ye; ys += TY) {
#pragma unroll
        for (int k = 0; k < LOADS; k++) {
            const int i = tid + k * TX * TY;
            const int r = i / LW, lx = i - r * LW;
            if (i < TY * LW) ring[(ys + HY + r) & (RING - 1)][lx] = pre[k];
        }
        __syncthreads();
        if (ys + TY < ye) prefetch(ys + TY);
        const int y = ys + threadIdx.y;
        if (x < W && y < ye) {
            uint64_t word = 0;
            if (x >= HX && x < W - HX && y >= HY && y < H - HY) {
                // the window of lane tx is ring bytes [tx, tx+8]: three aligned
                // dwords per row, realigned with v_alignbyte (no unaligned LDS)
                const unsigned* rows[7];
#pragma unroll
                for (int dy = -HY; dy <= HY; dy++)
                    rows[dy + HY] = reinterpret_cast<const unsigned*>(ring[(y + dy) & (RING - 1)]);
                word = census9x7(rows, threadIdx.x >> 2, threadIdx.x & 3);
            }
            uint64_t* orow = out + (size_t)y * ostride;
            orow[x] = word;
            // padded layout (fused path): columns W .. W+pr-1
            // repeat the row cyclically, orow[W + j] = orow[j mod W]
            for (int cpad = x + W; cpad < W + pr; cpad += W) orow[cpad] = word;
        }
    }
}

}  // namespace

static hipError_t census_launch(Ctx& c, const uint8_t* a, const uint8_t* b, int W, int H,
                                size_t pitch, uint64_t* oa, uint64_t* ob, int n,
                                size_t ostride = 0, int pr = 0) {
#ifdef SVA_PATHS_ABLATION   // A/B builds only: SVA_CENSUS_VARIANT=1 selects the single-tile kernel
    static const int variant = getenv("SVA_CENSUS_VARIANT") ? atoi(getenv("SVA_CENSUS_VARIANT")) : 0;
#else
    constexpr int variant = 0;
#endif
    if (ostride == 0) ostride = (size_t)W;
    if (variant == 1 && ostride == (size_t)W) {   // single-tile kernel
        dim3 grid((W + TX - 1) / TX, (H + TY - 1) / TY, n);
        hipLaunchKernelGGL(census9x7_kernel, grid, dim3(TX, TY), 0, c.stream, a, b, W, H, pitch,
                           oa, ob);
        return hipGetLastError();
    }
    dim3 grid((W + TX - 1) / TX, (H + kCensusRows - 1) / kCensusRows, n);
    hipLaunchKernelGGL(census9x7_rows_kernel, grid, dim3(TX, TY), 0, c.stream, a, b, W, H, pitch,
                       oa, ob, kCensusRows, ostride, pr);
    return hipGetLastError();
}

hipError_t launch_census(Ctx& c, const uint8_t* img, int W, int H, size_t pitch,
                         uint64_t* out) {
    ScopedKernelTimer t(c, "census");
    return census_launch(c, img, img, W, H, pitch, out, out, 1);
}

hipError_t launch_census_pair(Ctx& c, const uint8_t* left, const uint8_t* right, int W, int H,
                              size_t pitch, uint64_t* out_l, uint64_t* out_r) {
    ScopedKernelTimer t(c, "census");
    return census_launch(c, left, right, W, H, pitch, out_l, out_r, 2);
}

hipError_t launch_census_pair_padded(Ctx& c, const uint8_t* left, const uint8_t* right, int W,
                                     int H, size_t pitch, int pr, uint64_t* out_l,
                                     uint64_t* out_r) {
    ScopedKernelTimer t(c, "census");
    return census_launch(c, left, right, W, H, pitch, out_l, out_r, 2, (size_t)W + pr, pr);
}

}  // namespace sva
