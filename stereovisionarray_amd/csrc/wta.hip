// wta.hip -- path sum, winner-take-all and sub-pixel (DESIGN.md §2.4,
// SURVEY.md §8a row A13), plus the left/right check (§2.5).
//
// Same lane layout as sgm_paths.hip: one 16-lane DPP row per pixel, lane k
// holds disparities [k*DPL, k*DPL+DPL).  S = sum of the 8 u8 path volumes is
// formed in packed u16 (no carry: S <= 8*255 < 2^16); the pick is
// wta_common.h's.  These kernels serve the stage API (sva_wta_d,
// sva_aggregate_d); the frame pipeline uses wta_hv.hip, which also recomputes
// the horizontal paths.
#include "sva_device.h"
#include "sva_internal.h"
#include "wta_common.h"

namespace sva {
namespace {

constexpr int BLOCK = 256;
constexpr int PIX_PER_BLOCK = BLOCK / 16;

template <int NW>
__device__ __forceinline__ void load_nw(const uint8_t* p, unsigned (&w)[NW]) {
    if constexpr (NW == 1) {
        w[0] = *(const unsigned*)p;
    } else if constexpr (NW == 2) {
        uint2 v = *(const uint2*)p;
        w[0] = v.x; w[1] = v.y;
    } else if constexpr (NW == 3) {
        const unsigned* q = (const unsigned*)p;
        w[0] = q[0]; w[1] = q[1]; w[2] = q[2];
    } else {
        uint4 v = *(const uint4*)p;
        w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    }
}

// Last-use reads of the path volumes: non-temporal.
template <int NW>
__device__ __forceinline__ void load_nw_nt(const uint8_t* p, unsigned (&w)[NW]) {
    const unsigned* q = (const unsigned*)p;
    if constexpr (NW == 2) {
        typedef unsigned v2u __attribute__((ext_vector_type(2)));
        v2u v = __builtin_nontemporal_load((const v2u*)q);
        w[0] = v[0]; w[1] = v[1];
    } else if constexpr (NW == 4) {
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        v4u v = __builtin_nontemporal_load((const v4u*)q);
        w[0] = v[0]; w[1] = v[1]; w[2] = v[2]; w[3] = v[3];
    } else {
#pragma unroll
        for (int i = 0; i < NW; i++) w[i] = __builtin_nontemporal_load(q + i);
    }
}

// S pairs for this lane from the 8 direction volumes.
template <int DPL>
__device__ __forceinline__ void sum_paths(const uint8_t* p, size_t vol, unsigned (&S)[DPL / 2]) {
    constexpr int NW = DPL / 4, NP = DPL / 2;
#pragma unroll
    for (int j = 0; j < NP; j++) S[j] = 0u;
    unsigned w[8][NW];
#pragma unroll
    for (int r = 0; r < 8; r++) load_nw_nt<NW>(p + (size_t)r * vol, w[r]);
#pragma unroll
    for (int r = 0; r < 8; r++)
#pragma unroll
        for (int q = 0; q < NW; q++) {
            unsigned a, b;
            unpack4(w[r][q], a, b);
            S[2 * q] += a;      // packed add, no carry across halves
            S[2 * q + 1] += b;
        }
}

template <int DPL>
__device__ __forceinline__ void wta_finish(const unsigned (&S)[DPL / 2], int k, int D, int dmin,
                                           size_t pix, uint16_t* disp, float* sub) {
    float v;
    const int ds = wta_pick<DPL>(S, k, D, dmin, sub != nullptr, &v);
    if (k == 0) {
        disp[pix] = (uint16_t)(dmin + ds);
        if (sub) sub[pix] = v;
    }
}

template <int DPL>
__global__ __launch_bounds__(BLOCK) void sum_paths_kernel(const uint8_t* __restrict__ L8,
                                                          size_t vol, int npix, int D,
                                                          uint16_t* __restrict__ Sout) {
    const size_t pix = (size_t)blockIdx.x * PIX_PER_BLOCK + (threadIdx.x >> 4);
    const int k = threadIdx.x & 15;
    if (pix >= (size_t)npix) return;
    unsigned S[DPL / 2];
    sum_paths<DPL>(L8 + pix * D + k * DPL, vol, S);
    unsigned* o = (unsigned*)(Sout + pix * D + k * DPL);
#pragma unroll
    for (int j = 0; j < DPL / 2; j++) o[j] = S[j];
}

template <int DPL>
__global__ __launch_bounds__(BLOCK) void wta_sum_kernel(const uint16_t* __restrict__ Sin,
                                                        int npix, int D, int dmin,
                                                        uint16_t* __restrict__ disp,
                                                        float* __restrict__ sub) {
    const size_t pix = (size_t)blockIdx.x * PIX_PER_BLOCK + (threadIdx.x >> 4);
    const int k = threadIdx.x & 15;
    if (pix >= (size_t)npix) return;
    unsigned S[DPL / 2];
    const unsigned* s = (const unsigned*)(Sin + pix * D + k * DPL);
#pragma unroll
    for (int j = 0; j < DPL / 2; j++) S[j] = s[j];
    wta_finish<DPL>(S, k, D, dmin, pix, disp, sub);
}

// DESIGN.md §2.5.  The sub-pixel map (nullable) follows the check: NaN
// wherever the disparity is `invalid` afterwards (oracle svo_lr_sub).
__global__ void lr_check_kernel(uint16_t* __restrict__ dl, const uint16_t* __restrict__ dr,
                                float* __restrict__ sub, int W, int H, int sx, int sy,
                                int max_diff, uint16_t invalid) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    const size_t i = (size_t)y * W + x;
    const int d = dl[i];
    bool bad = d == invalid;
    if (!bad) {
        const int2 o = step_offset(d, sx, sy);
        const int xr = x + o.x, yr = y + o.y;
        if (xr < 0 || xr >= W || yr < 0 || yr >= H) {
            bad = true;
        } else {
            const int r = dr[(size_t)yr * W + xr];
            const int diff = d > r ? d - r : r - d;
            bad = r == invalid || diff > max_diff;
        }
        if (bad) dl[i] = invalid;
    }
    if (bad && sub) sub[i] = __builtin_nanf("");
}

}  // namespace

#define SVA_DISPATCH_D(D, KERNEL, GRID, ...)                                                     \
    switch (D) {                                                                                 \
        case 64: hipLaunchKernelGGL(KERNEL<4>, GRID, dim3(BLOCK), 0, c.stream, __VA_ARGS__); break;   \
        case 128: hipLaunchKernelGGL(KERNEL<8>, GRID, dim3(BLOCK), 0, c.stream, __VA_ARGS__); break;  \
        case 192: hipLaunchKernelGGL(KERNEL<12>, GRID, dim3(BLOCK), 0, c.stream, __VA_ARGS__); break; \
        case 256: hipLaunchKernelGGL(KERNEL<16>, GRID, dim3(BLOCK), 0, c.stream, __VA_ARGS__); break; \
        default: return hipErrorInvalidValue;                                                    \
    }

hipError_t launch_sum(Ctx& c, const uint8_t* L8, int W, int H, int D, uint16_t* S) {
    ScopedKernelTimer t(c, "path_sum");
    const int npix = W * H;
    const size_t vol = (size_t)npix * D;
    dim3 grid((npix + PIX_PER_BLOCK - 1) / PIX_PER_BLOCK);
    SVA_DISPATCH_D(D, sum_paths_kernel, grid, L8, vol, npix, D, S);
    return hipGetLastError();
}

hipError_t launch_wta_from_sum(Ctx& c, const uint16_t* S, int W, int H, int D, int dmin,
                               uint16_t* disp, float* sub) {
    ScopedKernelTimer t(c, "wta_sum");
    const int npix = W * H;
    dim3 grid((npix + PIX_PER_BLOCK - 1) / PIX_PER_BLOCK);
    SVA_DISPATCH_D(D, wta_sum_kernel, grid, S, npix, D, dmin, disp, sub);
    return hipGetLastError();
}

hipError_t launch_lr_check(Ctx& c, uint16_t* disp_l, const uint16_t* disp_r, float* sub, int W,
                           int H, int sx, int sy, int max_diff, uint16_t invalid) {
    ScopedKernelTimer t(c, "lr_check");
    dim3 grid((W + 255) / 256, H);
    hipLaunchKernelGGL(lr_check_kernel, grid, dim3(256), 0, c.stream, disp_l, disp_r, sub, W, H,
                       sx, sy, max_diff, invalid);
    return hipGetLastError();
}

}  // namespace sva
