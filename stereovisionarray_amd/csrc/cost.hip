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

// 2-D matching step: the word for (x, y, d) sits at
// (x, y) + step_offset(s, bx, by), s = dmin + d, by != 0 (vertical, diagonal
// and any other integer baseline direction of an array pair).  The per-block
// offset table (one division per disparity) lives in LDS.  Consecutive disparities now walk down rows, so no word is shared
// between the D disparities of one pixel; what a row of pixels shares is the
// word at the same s: the PX pixels of a block read, per s, PX consecutive
// words of one census row.  The block stages that D x PX tile in LDS once
// (coalesced row segments) and every thread then reads its 16 words from LDS.
// LDS slot of (s-index e, pixel p): e*PX + (p + G*(e>>4)) % PX.  The 32 lanes of
// a half-wave are 32/NC pixels x NC chunks; rotating each chunk's row by G =
// 32/NC words puts the 32 lanes' reads in 32 distinct bank pairs (D=64, 128;
// D=192/256 keep a 2-way conflict, the rows are narrower than a bank sweep).
// Out-of-image words are staged as a word with bit 63 set, which no census
// word has (bits 0..61), and read back as cost 62.
constexpr uint64_t kOutside = 1ull << 63;

template <int NC>
__global__ __launch_bounds__(BLOCK) void hamming_cost2_kernel(const uint64_t* __restrict__ cl,
                                                               const uint64_t* __restrict__ cr,
                                                               int W, int H, int dmin, int bx,
                                                               int by, uint8_t* __restrict__ C) {
    constexpr int D = NC * 16, PX = BLOCK / NC, G = 32 / NC > 0 ? 32 / NC : 1;
    __shared__ uint64_t rw[D * PX];
    __shared__ int2 off[D];
    const int blocks_per_row = (W + PX - 1) / PX;
    const int y = blockIdx.x / blocks_per_row;
    const int x0 = (blockIdx.x - y * blocks_per_row) * PX;
    for (int e = threadIdx.x; e < D; e += BLOCK) off[e] = step_offset(dmin + e, bx, by);
    __syncthreads();
    for (int i = threadIdx.x; i < D * PX; i += BLOCK) {
        const int e = i / PX, p = i - e * PX;
        const int2 o = off[e];
        const int xr = x0 + p + o.x, yr = y + o.y;
        uint64_t w = kOutside;
        if ((unsigned)xr < (unsigned)W && (unsigned)yr < (unsigned)H) w = cr[(size_t)yr * W + xr];
        rw[e * PX + (p + G * (e >> 4)) % PX] = w;
    }
    __syncthreads();
    const int lp = threadIdx.x / NC;
    const int x = x0 + lp;
    if (lp >= PX || x >= W) return;  // D=192: 256 % 12 != 0 leaves idle lanes
    const int c = threadIdx.x - lp * NC;
    const uint64_t l = cl[(size_t)y * W + x];
    const uint64_t* col = rw + (c * 16) * PX + (lp + G * c) % PX;
    unsigned out[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        unsigned w = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const uint64_t v = l ^ col[(q * 4 + b) * PX];
            const unsigned cst = (v >> 63) ? 62u : (unsigned)__popcll(v);
            w |= cst << (8 * b);
        }
        out[q] = w;
    }
    *(uint4*)(C + ((size_t)y * W + x) * D + c * 16) = make_uint4(out[0], out[1], out[2], out[3]);
}

}  // namespace

hipError_t launch_cost2(Ctx& c, const uint64_t* cl, const uint64_t* cr, int W, int H, int D,
                        int dmin, int sx, int sy, uint8_t* C) {
    if (sy == 0) return launch_cost(c, cl, cr, W, H, D, dmin, sx > 0 ? 1 : -1, C);
    ScopedKernelTimer t(c, "cost");
    const int nc = D / 16, px = BLOCK / nc;
    const dim3 grid(((W + px - 1) / px) * H);
    switch (nc) {
        case 4: hipLaunchKernelGGL(hamming_cost2_kernel<4>, grid, dim3(BLOCK), 0, c.stream, cl, cr, W, H, dmin, sx, sy, C); break;
        case 8: hipLaunchKernelGGL(hamming_cost2_kernel<8>, grid, dim3(BLOCK), 0, c.stream, cl, cr, W, H, dmin, sx, sy, C); break;
        case 12: hipLaunchKernelGGL(hamming_cost2_kernel<12>, grid, dim3(BLOCK), 0, c.stream, cl, cr, W, H, dmin, sx, sy, C); break;
        case 16: hipLaunchKernelGGL(hamming_cost2_kernel<16>, grid, dim3(BLOCK), 0, c.stream, cl, cr, W, H, dmin, sx, sy, C); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

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
