// cost.hip -- Hamming matching-cost volume.
//
// C[(y*W + x)*D + d] = popcount(CL(x,y) ^ CR(x + dir*(dmin+d), y)), 62 outside,
// from two census maps: the 1-D kernel (hamming_cost_rows_kernel, below) and
// the 2-D array-step kernel (hamming_cost2_kernel).  Each thread produces 16
// disparities = one 16-byte store.  HBM bytes: 1 B/disparity written +
// 16 B/pixel read.
#include "sva_device.h"
#include "sva_internal.h"

namespace sva {
namespace {

constexpr int BLOCK = 256;

// Cost bytes are stored non-temporally: the 8 path directions re-read C long
// after it is written and it does not fit the caches anyway (265 MB at 1080p
// D=128).  Measured effect: none beyond noise -- an in-process A/B with each
// build listed twice gave temporal 1.155/1.172 ms vs nt 1.169/1.142 ms per
// full frame (a first, single-listing A/B had suggested -3.8 %).
__device__ __forceinline__ void store_cost_nt(uint8_t* p, const unsigned (&o)[4]) {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store((v4u){o[0], o[1], o[2], o[3]}, (v4u*)p);
}

// Out-of-image marker: bit 63 is never set in a census word (bits 0..61).
constexpr uint64_t kOutside = 1ull << 63;

// 2-D matching step: the word for (x, y, d) sits at
// q + off(s), off = step_offset(., bx, by), s = dmin + d, by != 0 (vertical,
// diagonal and any other integer baseline direction of an array pair).
//
// Reuse along the lattice step v = (bx, by): rounding commutes with adding an
// integer, so off(s + r*M) = off(s) + r*v (M = max(|bx|, |by|)) and pixel
// q + r*v at distance s reads the word that q reads at distance s + r*M.  A
// workgroup therefore owns PX base pixels b of one row y0 and the R pixels
// b + r*v (r < R) above each: a sheared PX x R tile.  It needs, per base pixel,
// only the words q_b + off(dmin + t) for t < T = D + M*(R-1) -- staged once in
// LDS as coalesced row segments (about T/R ~ 5 words per pixel at D=128 instead
// of D) -- then writes R rows of PX*D contiguous cost bytes.
// Tiling: rows y0 + r*by of band/phase (|by| interleaved phases per band of
// R*|by| rows; by < 0 bands run up from the bottom); base columns over
// [bmin, bmin + ncolb*PX) so the sheared rows cover [0, W); pixels outside the
// image are skipped.
// LDS slot of (t, b): t*PX + (b + G*(t>>4)) % PX.  A half-wave is 32/NC pixels
// x NC chunks reading t = 16c + j (same j): t>>4 = c + (j>>4), so rotating by
// G = 32/NC words per 16 t puts the 32 lanes on 32 distinct bank pairs (D=64,
// 128; D=192/256 keep a 2-way conflict).  Out-of-image words are staged with
// bit 63 set, which no census word has (bits 0..61), and read back as 62.
constexpr int kCost2LdsBytes = 64 * 1024;

template <int NC>
__global__ __launch_bounds__(BLOCK) void hamming_cost2_kernel(
    const uint64_t* __restrict__ cl, const uint64_t* __restrict__ cr, int W, int H, int dmin,
    int bx, int by, int R, int T, int ncolb, int bmin, int dreal, uint8_t* __restrict__ C) {
    constexpr int D = NC * 16, PX = BLOCK / NC, G = 32 / NC > 0 ? 32 / NC : 1;
    extern __shared__ uint64_t smem[];
    uint64_t* rw = smem;                       // [T][PX] census words
    int2* off = reinterpret_cast<int2*>(smem + (size_t)T * PX);
    const int aby = by < 0 ? -by : by, abx = bx < 0 ? -bx : bx;
    const int M = abx > aby ? abx : aby;
    const int colb = blockIdx.x % ncolb, rb = blockIdx.x / ncolb;
    const int band = rb / aby, phase = rb - band * aby;
    const int y0 = by > 0 ? band * R * aby + phase : (H - 1) - (band * R * aby + phase);
    const int X0 = bmin + colb * PX;
    for (int t = threadIdx.x; t < T; t += BLOCK) off[t] = step_offset(dmin + t, bx, by);
    __syncthreads();
    for (int i = threadIdx.x; i < T * PX; i += BLOCK) {
        const int t = i / PX, b = i - t * PX;
        const int2 o = off[t];
        const int xr = X0 + b + o.x, yr = y0 + o.y;
        uint64_t w = kOutside;
        if ((unsigned)xr < (unsigned)W && (unsigned)yr < (unsigned)H) w = cr[(size_t)yr * W + xr];
        rw[t * PX + (b + G * (t >> 4)) % PX] = w;
    }
    __syncthreads();
    const int lp = threadIdx.x / NC;
    if (lp >= PX) return;  // D=192: 256 % 12 != 0 leaves idle lanes
    const int c = threadIdx.x - lp * NC;
    for (int r = 0; r < R; r++) {
        const int x = X0 + lp + r * bx, y = y0 + r * by;
        if ((unsigned)x >= (unsigned)W || (unsigned)y >= (unsigned)H) continue;
        const uint64_t l = cl[(size_t)y * W + x];
        const int j0 = r * M;                 // t = 16c + j0 + k
        unsigned out[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            unsigned w = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const int j = j0 + q * 4 + b, t = c * 16 + j;
                const uint64_t v = l ^ rw[t * PX + (lp + G * c + G * (j >> 4)) % PX];
                const unsigned cst = (v >> 63) ? 62u : (unsigned)__popcll(v);
                w |= cst << (8 * b);
            }
            out[q] = w;
        }
        if (dreal < D) {                             // padded disparities: cost 255
#pragma unroll
            for (int q = 0; q < 4; q++) out[q] |= pad_bytes(16 * c + 4 * q, dreal);
        }
        store_cost_nt(C + ((size_t)y * W + x) * D + c * 16, out);
    }
}

// Multi-row cost kernel (production).  A workgroup owns PX pixels x ROWS
// consecutive rows; the next row's right-census words and left word are
// prefetched into registers while the current row computes, into a second LDS
// buffer, so HBM latency overlaps compute instead of being paid once per
// 4 KiB-output workgroup.  One barrier per row: a buffer is rewritten two rows
// after its last reads and the barrier of the row in between separates them.
//
// Lane mapping: 16 consecutive pixels x NC chunks per 16*NC threads (lane
// l of a 16*NC group: pixel 16g + (l & 15), chunk l >> 4), so a half-wave is
// 16 pixels x 2 chunks and, for each k, reads words j = lp + 16c + k that are
// 32 distinct consecutive-or-16-apart words: 32 distinct ds_read_b64 bank
// pairs with NO swizzle, and each thread's 16 words are consecutive (one base
// address, immediate offsets).  Out-of-image words carry the bit-63 marker;
// only workgroups whose word range touches the image border test it.
// (Measured at 1080p D=128, PMC: the single-row XOR-swizzled kernel spent
// 7.3M of 16.3M LDS cycles in bank conflicts and ~19 VALU per disparity.)
// Tried and rejected: 64-pixel workgroups (2-4 passes over the 16-pixel
// groups, less staging traffic per cost byte) -- cost-only A/B: D=128 -2.5 %,
// D=64 equal, D=192 +22 %, D=256 (4K) +13 %.
// Rows per workgroup.  Fewer rows = more workgroups in flight; measured
// in-process (1080p, rows 1/2/4/16): D=64 0.038/0.033/0.032/0.033 ms, D=128
// 0.072/0.067/0.072/0.079, D=192 0.115/0.099/0.104/0.113, D=256
// 0.145/0.124/0.128/0.138; 4K D=256 0.61/0.52/0.50/0.49.
__host__ __device__ constexpr int cost_rows(int W, int H, int D) {
    return (D >= 128 && (long long)W * H <= 4000000ll) ? 2 : 4;
}

template <int NC>
__global__ __launch_bounds__(256) void hamming_cost_rows_kernel(
    const uint64_t* __restrict__ cl, const uint64_t* __restrict__ cr, int W, int H, int dmin,
    int dir, int rows, int dreal, uint8_t* __restrict__ C) {
    constexpr int D = NC * 16, NT = (256 / (16 * NC) > 0 ? 256 / (16 * NC) : 1) * 16 * NC;
    constexpr int PX = NT / NC, NW = PX + D - 1;
    constexpr int WPT = (NW + NT - 1) / NT;  // staged words per thread
    __shared__ uint64_t rw[2][NW];
    const int blocks_per_row = (W + PX - 1) / PX;
    const int bx = blockIdx.x % blocks_per_row, by = blockIdx.x / blocks_per_row;
    const int x0 = bx * PX, y0 = by * rows;
    const int y1 = min(H, y0 + rows);
    const int t = threadIdx.x;
    const int g = t / (16 * NC), r = t - g * 16 * NC;
    const int lp = 16 * g + (r & 15), c = r >> 4;
    const int x = x0 + lp;
    const bool active = x < W;
    // word j <-> column: dir > 0: x0 + dmin + j; dir < 0: x0 + PX - 1 - dmin - j
    const int first = dir > 0 ? x0 + dmin : x0 + PX - 1 - dmin - (NW - 1);
    const bool border = first < 0 || first + NW > W;
    const int j0 = (dir > 0 ? lp : PX - 1 - lp) + 16 * c;
    uint64_t w[WPT];
    uint64_t l = 0;
    auto fetch = [&](int y) {
#pragma unroll
        for (int k = 0; k < WPT; k++) {
            const int j = t + k * NT;
            const int col = dir > 0 ? x0 + dmin + j : x0 + PX - 1 - dmin - j;
            w[k] = (j < NW && (unsigned)col < (unsigned)W) ? cr[(size_t)y * W + col] : kOutside;
        }
        l = active ? cl[(size_t)y * W + x] : 0;
    };
    fetch(y0);
    for (int y = y0; y < y1; y++) {
        uint64_t* buf = rw[(y - y0) & 1];
#pragma unroll
        for (int k = 0; k < WPT; k++) {
            const int j = t + k * NT;
            if (j < NW) buf[j] = w[k];
        }
        const uint64_t lc = l;
        __syncthreads();
        if (y + 1 < y1) fetch(y + 1);
        if (active) {
            const uint64_t* src = buf + j0;
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
            if (dreal < D) {                         // padded disparities: cost 255
#pragma unroll
                for (int q = 0; q < 4; q++) out[q] |= pad_bytes(16 * c + 4 * q, dreal);
            }
            store_cost_nt(C + ((size_t)y * W + x) * D + 16 * c, out);
        }
    }
}

}  // namespace

hipError_t launch_cost2(Ctx& c, const uint64_t* cl, const uint64_t* cr, int W, int H, int D,
                        int dmin, int sx, int sy, uint8_t* C, int dreal) {
    if (dreal <= 0) dreal = D;
    if (sy == 0) return launch_cost(c, cl, cr, W, H, D, dmin, sx > 0 ? 1 : -1, C, dreal);
    ScopedKernelTimer t(c, "cost");
    // reduce the step to its primitive lattice vector (same offsets, more reuse)
    int a = sx < 0 ? -sx : sx, b = sy < 0 ? -sy : sy;
    while (b) { int r = a % b; a = b; b = r; }
    const int bx = sx / a, by = sy / a;
    const int abx = bx < 0 ? -bx : bx, aby = by < 0 ? -by : by, M = abx > aby ? abx : aby;
    const int nc = D / 16, px = BLOCK / nc;
    const int tmax = kCost2LdsBytes / (8 * (px + 1));
    int R = 1 + (tmax - D) / M;
    if (R > 32) R = 32;
    if (R < 1) return hipErrorInvalidValue;
    const int T = D + M * (R - 1);
    const int span = (R - 1) * abx;
    const int bmin = bx > 0 ? -span : 0;
    const int ncolb = (W + span + px - 1) / px;
    const int nbands = (H + R * aby - 1) / (R * aby);
    const dim3 grid((unsigned)(ncolb * nbands * aby));
    const size_t lds = (size_t)T * px * 8 + (size_t)T * 8;
#define SVA_COST2(NC)                                                                          \
    hipLaunchKernelGGL(hamming_cost2_kernel<NC>, grid, dim3(BLOCK), lds, c.stream, cl, cr, W, H, \
                       dmin, bx, by, R, T, ncolb, bmin, dreal, C)
    switch (nc) {
        case 4: SVA_COST2(4); break;
        case 8: SVA_COST2(8); break;
        case 12: SVA_COST2(12); break;
        case 16: SVA_COST2(16); break;
        default: return hipErrorInvalidValue;
    }
#undef SVA_COST2
    return hipGetLastError();
}

hipError_t launch_cost(Ctx& c, const uint64_t* cl, const uint64_t* cr, int W, int H, int D,
                       int dmin, int dir, uint8_t* C, int dreal) {
    if (dreal <= 0) dreal = D;
    ScopedKernelTimer t(c, "cost");
    const int rows = cost_rows(W, H, D);
    // threads: 16 pixels x NC chunks per group, as many groups as fit 256
    const int nc = D / 16, groups = 256 / (16 * nc) > 0 ? 256 / (16 * nc) : 1;
    const int nt = groups * 16 * nc, px = groups * 16;
    const int bpr = (W + px - 1) / px;
    const dim3 grid((unsigned)(bpr * ((H + rows - 1) / rows)));
    switch (D) {
        case 64: hipLaunchKernelGGL(hamming_cost_rows_kernel<4>, grid, dim3(nt), 0, c.stream, cl, cr, W, H, dmin, dir, rows, dreal, C); break;
        case 128: hipLaunchKernelGGL(hamming_cost_rows_kernel<8>, grid, dim3(nt), 0, c.stream, cl, cr, W, H, dmin, dir, rows, dreal, C); break;
        case 192: hipLaunchKernelGGL(hamming_cost_rows_kernel<12>, grid, dim3(nt), 0, c.stream, cl, cr, W, H, dmin, dir, rows, dreal, C); break;
        case 256: hipLaunchKernelGGL(hamming_cost_rows_kernel<16>, grid, dim3(nt), 0, c.stream, cl, cr, W, H, dmin, dir, rows, dreal, C); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace sva
