// evaluate.hip -- SURVEY.md §8f row 4: the reference's evaluation step
// (CameraStereoVision.cpp:107-110,118-119; functions.cpp:348-354):
//
//   resize(depth, depth2, ref.size());   error = (depth2 - ref) * 50;
//   cv::mean(image, mask)[0]
//
// OpenCV 4.2 semantics restated in oracle/eval_oracle.c (third-party, absent
// here: parity unpinned); the kernels evaluate the same f64 expressions in
// the same order with the same float coefficients, no contraction.
//
//   resize_linear_kernel   1 thread/output pixel: float (fx, fy) and taps as
//                          resizeGeneric_ (x taps clamped with fx = 0, y rows
//                          clipped with fy kept), or the exact-2x area path
//   ref_error fused        the resize tap + a * s + b * (-s) + 0 per pixel
//   masked_sum_kernel      fixed-shape two-level f64 reduction (per-thread
//                          strided partials, LDS tree, one finishing block):
//                          deterministic run to run
#include "sva_internal.h"

#pragma clang fp contract(off)

namespace sva {
namespace {

struct ResizeGeom {
    int sw, sh, dw, dh;
    double sx, sy;   // scale = 1 / (dsize / ssize), per axis
    int mode;        // 0 copy, 1 area 2x, 2 linear
};

__device__ __forceinline__ double resize_at(const double* __restrict__ src, const ResizeGeom& g,
                                            int x, int y) {
    if (g.mode == 0) return src[(size_t)y * g.sw + x];
    if (g.mode == 1) {
        const double* s0 = src + (size_t)(2 * y) * g.sw + 2 * x;
        const double* s1 = s0 + g.sw;
        double sum = 0;
        sum += s0[0] + s0[1] + s1[0] + s1[1];
        return sum * 0.25;
    }
    float fy = (float)((y + 0.5) * g.sy - 0.5);
    const int sy = (int)floorf(fy);
    fy -= (float)sy;
    const int r0 = min(max(sy, 0), g.sh - 1), r1 = min(max(sy + 1, 0), g.sh - 1);
    float fx = (float)((x + 0.5) * g.sx - 0.5);
    int sx = (int)floorf(fx);
    fx -= (float)sx;
    if (sx < 0) { sx = 0; fx = 0.f; }
    const double* S0 = src + (size_t)r0 * g.sw;
    const double* S1 = src + (size_t)r1 * g.sw;
    double h0, h1;
    if (sx >= g.sw - 1) {
        h0 = S0[g.sw - 1];
        h1 = S1[g.sw - 1];
    } else {
        const double a0 = (double)(1.f - fx), a1 = (double)fx;
        h0 = S0[sx] * a0 + S0[sx + 1] * a1;
        h1 = S1[sx] * a0 + S1[sx + 1] * a1;
    }
    return h0 * (double)(1.f - fy) + h1 * (double)fy;
}

__global__ void resize_linear_kernel(const double* __restrict__ src, ResizeGeom g,
                                     const double* __restrict__ ref, double scale,
                                     double* __restrict__ dst) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= g.dw) return;
    const size_t o = (size_t)y * g.dw + x;
    const double v = resize_at(src, g, x, y);
    dst[o] = ref ? v * scale + ref[o] * -scale + 0.0 : v;
}

constexpr int SUM_BLOCKS = 512, SUM_THREADS = 256;

// Stage 1: block b's thread t sums elements i = b*256 + t + k*(512*256), then
// an LDS tree; partial (sum, count) per block.  Stage 2: one block folds the
// 512 partials by the same tree.  The association depends only on n.
__device__ __forceinline__ void block_tree(double* s, unsigned long long* c) {
    const int t = threadIdx.x;
    for (int w = SUM_THREADS / 2; w > 0; w >>= 1) {
        __syncthreads();
        if (t < w) {
            s[t] = s[t] + s[t + w];
            c[t] += c[t + w];
        }
    }
    __syncthreads();
}

__global__ __launch_bounds__(SUM_THREADS) void masked_sum_kernel(
    const double* __restrict__ img, const uint8_t* __restrict__ mask, size_t n,
    double* __restrict__ psum, unsigned long long* __restrict__ pcnt) {
    __shared__ double s[SUM_THREADS];
    __shared__ unsigned long long c[SUM_THREADS];
    const size_t stride = (size_t)SUM_BLOCKS * SUM_THREADS;
    double acc = 0;
    unsigned long long cnt = 0;
    for (size_t i = (size_t)blockIdx.x * SUM_THREADS + threadIdx.x; i < n; i += stride)
        if (!mask || mask[i]) {
            acc += img[i];
            cnt++;
        }
    s[threadIdx.x] = acc;
    c[threadIdx.x] = cnt;
    block_tree(s, c);
    if (threadIdx.x == 0) {
        psum[blockIdx.x] = s[0];
        pcnt[blockIdx.x] = c[0];
    }
}

__global__ __launch_bounds__(SUM_THREADS) void masked_mean_finish(
    const double* __restrict__ psum, const unsigned long long* __restrict__ pcnt,
    double* __restrict__ mean) {
    __shared__ double s[SUM_THREADS];
    __shared__ unsigned long long c[SUM_THREADS];
    const int t = threadIdx.x;
    s[t] = psum[t] + psum[t + SUM_THREADS];
    c[t] = pcnt[t] + pcnt[t + SUM_THREADS];
    block_tree(s, c);
    if (t == 0) *mean = c[0] ? s[0] / (double)c[0] : 0.0;
}

ResizeGeom resize_geom(int sw, int sh, int dw, int dh) {
    ResizeGeom g{sw, sh, dw, dh, 1.0 / ((double)dw / sw), 1.0 / ((double)dh / sh), 2};
    if (sw == dw && sh == dh) g.mode = 0;
    else if (g.sx == 2.0 && g.sy == 2.0) g.mode = 1;
    return g;
}

}  // namespace

size_t masked_mean_workspace() {
    return (size_t)SUM_BLOCKS * (sizeof(double) + sizeof(unsigned long long)) + sizeof(double);
}

hipError_t launch_resize_linear(Ctx& c, const double* src, int sw, int sh, double* dst, int dw,
                                int dh, const double* ref, double scale) {
    ScopedKernelTimer t(c, "resize_linear");
    if (dw == 0 || dh == 0) return hipSuccess;
    hipLaunchKernelGGL(resize_linear_kernel, dim3((dw + 255) / 256, dh), dim3(256), 0, c.stream,
                       src, resize_geom(sw, sh, dw, dh), ref, scale, dst);
    return hipGetLastError();
}

hipError_t launch_masked_mean(Ctx& c, const double* img, const uint8_t* mask, size_t n,
                              void* ws, double* mean) {
    ScopedKernelTimer t(c, "masked_mean");
    double* psum = (double*)ws;
    unsigned long long* pcnt = (unsigned long long*)(psum + SUM_BLOCKS);
    hipLaunchKernelGGL(masked_sum_kernel, dim3(SUM_BLOCKS), dim3(SUM_THREADS), 0, c.stream, img,
                       mask, n, psum, pcnt);
    hipLaunchKernelGGL(masked_mean_finish, dim3(1), dim3(SUM_THREADS), 0, c.stream, psum, pcnt,
                       mean);
    return hipGetLastError();
}

}  // namespace sva
