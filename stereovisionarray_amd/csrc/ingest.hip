// ingest.hip -- SURVEY.md §8f row 4: the reference's ingestion resize
// (CameraStereoVision.cpp:18, resize(img, img, Size(), 0.5, 0.5), default
// INTER_LINEAR), which OpenCV 4.2 routes to its exact-2x area path (restated
// in oracle/refine_oracle.c svo_resize_half; OpenCV is absent: parity
// unpinned).  One thread per output pixel: two 2-byte row reads, full blocks
// (s00+s01+s10+s11+2)>>2, partial edge blocks rint(sum/count).
#include "sva_internal.h"

namespace sva {
namespace {

__global__ void resize_half_kernel(const uint8_t* __restrict__ src, int W, int H, size_t pitch,
                                   uint8_t* __restrict__ dst, int dw, int dh, size_t dpitch) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= dw || y >= dh) return;
    const int sx = 2 * x, sy = 2 * y;
    const uint8_t* r0 = src + (size_t)sy * pitch + sx;
    uint8_t v;
    if (sx + 1 < W && sy + 1 < H) {
        v = (uint8_t)((r0[0] + r0[1] + r0[pitch] + r0[pitch + 1] + 2) >> 2);
    } else {
        int sum = r0[0], cnt = 1;
        if (sx + 1 < W) { sum += r0[1]; cnt++; }
        if (sy + 1 < H) {
            sum += r0[pitch]; cnt++;
            if (sx + 1 < W) { sum += r0[pitch + 1]; cnt++; }
        }
        v = (uint8_t)(int)__builtin_rint((double)sum / cnt);   // cvRound: half to even
    }
    dst[(size_t)y * dpitch + x] = v;
}

}  // namespace

void resize_half_size(int W, int H, int* dw, int* dh) {
    *dw = (int)__builtin_rint(W * 0.5);   // cvRound(W * 0.5), half to even
    *dh = (int)__builtin_rint(H * 0.5);
}

hipError_t launch_resize_half(Ctx& c, const uint8_t* src, int W, int H, size_t pitch,
                              uint8_t* dst, size_t dpitch) {
    ScopedKernelTimer t(c, "resize_half");
    int dw, dh;
    resize_half_size(W, H, &dw, &dh);
    if (dw == 0 || dh == 0) return hipSuccess;
    hipLaunchKernelGGL(resize_half_kernel, dim3((dw + 255) / 256, dh), dim3(256), 0, c.stream, src,
                       W, H, pitch, dst, dw, dh, dpitch);
    return hipGetLastError();
}

}  // namespace sva
