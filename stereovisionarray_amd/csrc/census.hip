// census.hip -- 9x7 Census transform.
//
// One thread per pixel; a 64x4 workgroup walks a 64-column strip (below), so
// every image byte is read from HBM once (coalesced row segments) and each
// thread forms its 62-bit word from an LDS ring.  blockIdx.z selects the
// image: the left and right census of a pair are one launch.
// HBM bytes: 1 B/pixel read + 8 B/pixel write.
#include "sva_device.h"
#include "sva_internal.h"
#include "sva_tuning.h"

namespace sva {
namespace {

constexpr int TX = 64, TY = 4;           // pixels per tile
constexpr int HX = 4, HY = 3;            // half window (9 wide, 7 high)
constexpr int LW = TX + 2 * HX;          // 72 LDS columns

// Multi-row form: a 64x4 workgroup walks a 64-column strip of kCensusRows
// rows in steps of TY rows.  The 7-row window lives in a 16-row LDS ring, so
// each step loads only its TY new rows (prefetched into registers during the
// previous step's compute); rows outside the image stage as 0.  One barrier
// per step: ring slots are rewritten 4 steps after their rows were loaded and
// 2 steps after their last reads (a step reads rows y-3 .. y+TY+2).
constexpr int RING = 16;
constexpr int kCensusRows = tune::kCensusRows;
constexpr int LOADS = (TY * LW + TX * TY - 1) / (TX * TY);   // bytes per thread per step

__global__ __launch_bounds__(TX* TY) void census9x7_rows_kernel(
    const uint8_t* __restrict__ img0, const uint8_t* __restrict__ img1, int W, int H,
    size_t pitch, uint64_t* __restrict__ out0, uint64_t* __restrict__ out1, int rows) {
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
            out[(size_t)y * W + x] = word;
        }
    }
}

}  // namespace

static hipError_t census_launch(Ctx& c, const uint8_t* a, const uint8_t* b, int W, int H,
                                size_t pitch, uint64_t* oa, uint64_t* ob, int n) {
    dim3 grid((W + TX - 1) / TX, (H + kCensusRows - 1) / kCensusRows, n);
    hipLaunchKernelGGL(census9x7_rows_kernel, grid, dim3(TX, TY), 0, c.stream, a, b, W, H, pitch,
                       oa, ob, kCensusRows);
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

}  // namespace sva
