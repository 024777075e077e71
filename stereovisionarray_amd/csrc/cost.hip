// cost.hip -- Hamming matching-cost volume.
//
// C[(y*W + x)*D + d] = popcount(CL(x,y) ^ CR(x + dir*(dmin+d), y)), 62 outside.
// A 256-thread workgroup owns PX = 4096/D consecutive pixels of one row; the
// right-census words they touch (PX + D - 1 of them) are staged once in LDS.
// Each thread produces 16 disparities = one 16-byte store, so a wave writes
// 1 KiB contiguous.  HBM bytes: 1 B/disparity written + 16 B/pixel read.
#include "sva_device.h"
#include "sva_internal.h"

namespace sva {
namespace {

constexpr int BLOCK = 256;
constexpr int MAXW = 4096 / 64 + 256;  // LDS words for the smallest D (64): PX=64, +D

// LDS word swizzle.  The D/16 lanes of one pixel read words 16 apart (one per
// 16-disparity chunk): unswizzled that is a 4-way ds_read_b64 bank conflict at
// D=128.  XOR-ing bits 0-2 of the word index with bits 4-6 (the chunk) spreads
// the chunks of a pixel over 8 different bank pairs.  Bijective within each
// aligned 128-word block, so MAXW rounded up to 128 words is enough.
__device__ __forceinline__ int swz(int j) { return j ^ ((j >> 4) & 7); }

__global__ __launch_bounds__(BLOCK) void hamming_cost_kernel(const uint64_t* __restrict__ cl,
                                                              const uint64_t* __restrict__ cr,
                                                              int W, int H, int D, int dmin,
                                                              int dir, uint8_t* __restrict__ C) {
    __shared__ uint64_t rw[(MAXW + 127) / 128 * 128];
    __shared__ uint8_t rvalid[MAXW];
    const int tpp = D / 16;                  // threads per pixel
    const int px_per_block = BLOCK / tpp;    // pixels per block
    const int blocks_per_row = (W + px_per_block - 1) / px_per_block;
    const int y = blockIdx.x / blocks_per_row;
    const int x0 = (blockIdx.x - y * blocks_per_row) * px_per_block;
    // Right-census range touched by pixels [x0, x0+px) and d in [0, D):
    // column = x + dir*(dmin + d).  Index LDS by j = (x - x0) + d, column =
    // x0 + dir*dmin + (dir>0 ? j : ...) -- handled below for both signs.
    const int nwords = px_per_block + D - 1;
    for (int j = threadIdx.x; j < nwords; j += BLOCK) {
        // dir = +1: word j <-> column x0 + dmin + j          (x - x0) + d = j
        // dir = -1: word j <-> column x0 + px - 1 - dmin - j  (px-1-(x-x0)) + d = j
        int col = dir > 0 ? x0 + dmin + j : x0 + px_per_block - 1 - dmin - j;
        bool ok = col >= 0 && col < W;
        rw[swz(j)] = ok ? cr[(size_t)y * W + col] : 0ull;
        rvalid[j] = ok;
    }
    __syncthreads();
    const int lp = threadIdx.x / tpp;        // pixel within block
    const int x = x0 + lp;
    if (lp >= px_per_block || x >= W) return;  // D=192: 256 % 12 != 0 leaves idle lanes
    const int d0 = (threadIdx.x - lp * tpp) * 16;
    const uint64_t l = cl[(size_t)y * W + x];
    unsigned out[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        unsigned w = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int d = d0 + q * 4 + b;
            const int j = dir > 0 ? lp + d : (px_per_block - 1 - lp) + d;
            unsigned cst = rvalid[j] ? (unsigned)__popcll(l ^ rw[swz(j)]) : 62u;
            w |= cst << (8 * b);
        }
        out[q] = w;
    }
    *(uint4*)(C + ((size_t)y * W + x) * D + d0) = make_uint4(out[0], out[1], out[2], out[3]);
}

}  // namespace

hipError_t launch_cost(Ctx& c, const uint64_t* cl, const uint64_t* cr, int W, int H, int D,
                       int dmin, int dir, uint8_t* C) {
    ScopedKernelTimer t(c, "cost");
    const int px_per_block = BLOCK / (D / 16);
    const int blocks_per_row = (W + px_per_block - 1) / px_per_block;
    hipLaunchKernelGGL(hamming_cost_kernel, dim3(blocks_per_row * H), dim3(BLOCK), 0, c.stream,
                       cl, cr, W, H, D, dmin, dir, C);
    return hipGetLastError();
}

}  // namespace sva
