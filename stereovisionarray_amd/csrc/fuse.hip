// fuse.hip -- multi-pair depth fusion on the root.
//
// depth(p) = median over maps i with disp_i(p) != invalid and disp_i(p) > 0 of
//            (baseline_i * f) / ((double)disp_i(p) * pixel_size)
// (mean of the two middle values for an even count, 0 if no map is valid).
// One thread per pixel.  The n <= NM depths live in registers (fully unrolled);
// the median is chosen by rank counting (rank_i = #{j : z_j < z_i, or z_j == z_i
// and j < i}), O(NM^2) f64 compares, no data-dependent indexing so nothing
// spills to scratch.  Invalid entries are +inf and rank after every valid one.
// HBM bytes per pixel: 2 * n_maps read + 9 written.  f64 without contraction,
// IEEE division: the same bits as the oracle's insertion sort + mean.
#include "sva_internal.h"

#pragma clang fp contract(off)

namespace sva {
namespace {

struct FuseNum {
    double v[32];  // baseline_i * f
};

template <int NM>
__global__ __launch_bounds__(256) void fuse_depth_kernel(const uint16_t* __restrict__ disps,
                                                         int n_maps, size_t np, FuseNum num,
                                                         double pixel_size, uint16_t invalid,
                                                         double* __restrict__ depth,
                                                         uint8_t* __restrict__ n_valid) {
    const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= np) return;
    double z[NM];
    int n = 0;
#pragma unroll
    for (int i = 0; i < NM; i++) {
        const unsigned d = i < n_maps ? disps[(size_t)i * np + p] : invalid;
        const bool ok = d != invalid && d != 0;
        z[i] = ok ? num.v[i] / ((double)d * pixel_size) : __builtin_inf();
        n += ok;
    }
    const int lo = (n - 1) >> 1, hi = n >> 1;
    double a = 0.0, b = 0.0;
#pragma unroll
    for (int i = 0; i < NM; i++) {
        int r = 0;
#pragma unroll
        for (int j = 0; j < NM; j++)
            if (j != i) r += (z[j] < z[i]) || (j < i && z[j] == z[i]);
        if (r == lo) a = z[i];
        if (r == hi) b = z[i];
    }
    depth[p] = n == 0 ? 0.0 : ((n & 1) ? a : (a + b) * 0.5);
    if (n_valid) n_valid[p] = (uint8_t)n;
}

}  // namespace

hipError_t launch_fuse_depth(Ctx& c, const uint16_t* disps, int n_maps, size_t np,
                             const double* num, double pixel_size, uint16_t invalid,
                             double* depth, uint8_t* n_valid) {
    if (n_maps < 1 || n_maps > 32) return hipErrorInvalidValue;
    ScopedKernelTimer t(c, "fuse_depth");
    FuseNum k{};
    for (int i = 0; i < n_maps; i++) k.v[i] = num[i];
    const dim3 grid((unsigned)((np + 255) / 256));
#define SVA_FUSE(NM) \
    hipLaunchKernelGGL(fuse_depth_kernel<NM>, grid, dim3(256), 0, c.stream, disps, n_maps, np, k, \
                       pixel_size, invalid, depth, n_valid)
    if (n_maps <= 4) SVA_FUSE(4);
    else if (n_maps <= 8) SVA_FUSE(8);
    else if (n_maps <= 16) SVA_FUSE(16);
    else SVA_FUSE(32);
#undef SVA_FUSE
    return hipGetLastError();
}

}  // namespace sva
