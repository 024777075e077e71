// census.hip -- 9x7 Census transform.
//
// One thread per pixel.  A 64x4 workgroup tile stages its (64+8)x(4+6) halo
// through LDS so every image byte is read from HBM once (coalesced row
// segments), then each thread forms its 62-bit word from LDS.
// HBM bytes: 1 B/pixel read + 8 B/pixel write.
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

}  // namespace

hipError_t launch_census(Ctx& c, const uint8_t* img, int W, int H, size_t pitch,
                         uint64_t* out) {
    ScopedKernelTimer t(c, "census");
    dim3 grid((W + TX - 1) / TX, (H + TY - 1) / TY, 1);
    hipLaunchKernelGGL(census9x7_kernel, grid, dim3(TX, TY), 0, c.stream, img, img, W, H, pitch,
                       out, out);
    return hipGetLastError();
}

hipError_t launch_census_pair(Ctx& c, const uint8_t* left, const uint8_t* right, int W, int H,
                              size_t pitch, uint64_t* out_l, uint64_t* out_r) {
    ScopedKernelTimer t(c, "census");
    dim3 grid((W + TX - 1) / TX, (H + TY - 1) / TY, 2);
    hipLaunchKernelGGL(census9x7_kernel, grid, dim3(TX, TY), 0, c.stream, left, right, W, H,
                       pitch, out_l, out_r);
    return hipGetLastError();
}

}  // namespace sva
