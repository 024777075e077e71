// refine.hip -- SURVEY.md §8f rows 1-2 on the GPU: disparity refinement
// (improveWithDisparity + shiftPerspectiveWithDisparity, functions.cpp:11-72)
// and depth <-> 3-D output (shiftPerspective2, Points3DToDepthMap,
// DepthMapToPoints3D, functions.cpp:74-146).  Semantics of the reference's
// undefined corners: DESIGN.md §2.7 (same as oracle/refine_oracle.c).
//
//   shift_perspective_kernel  1 thread/pixel gather (u8), f64 index math
//   refine_kernel<ND>          1 thread/pixel, 11 candidate 2k x 2k SADs on
//                              dword-realigned rows (v_alignbyte + v_sad_u8),
//                              first-minimum, (uchar)(int) of the f64 update
//   scatter_key_kernel /       "last write in loop order wins" scatters as two
//   scatter_write_kernel       passes: atomicMax of (loop index + 1) per target,
//                              then the owner of the winning index writes
//   d2p_count / d2p_scan /     column-major stream compaction (depth > 0.1):
//   d2p_write                  per-(column, 64-row chunk) counts, one-block
//                              exclusive scan, ordered writes
// All f64 in the reference's operand order, no contraction.
#include "sva_device.h"
#include "sva_internal.h"

#pragma clang fp contract(off)

namespace sva {
namespace {

struct CamD {
    double f, px, py, pz, ps;
};
inline CamD camd(const sva_camera& c) { return CamD{c.f, c.pos[0], c.pos[1], c.pos[2], c.pixel_size}; }

// double -> int with the skip rule: false for NaN / outside int range.
__device__ __forceinline__ bool to_int(double v, long long& out) {
    if (!(v > -2147483649.0 && v < 2147483648.0)) return false;
    out = (long long)(int)v;
    return true;
}

__global__ void shift_perspective_kernel(const uint8_t* __restrict__ disp,
                                         const uint8_t* __restrict__ img, int W, int H,
                                         size_t pitch, double preX, double preY,
                                         uint8_t* __restrict__ out) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    const double d = disp[(size_t)y * pitch + x];
    if (d == 0) return;
    long long sx, sy;
    if (!to_int(d * preX + x, sx) || !to_int(d * preY + y, sy)) return;
    if (sy >= H || sy < 0 || sx >= W || sx < 0) return;
    out[(size_t)y * pitch + x] = img[(size_t)sy * pitch + sx];
}

template <int ND>
__global__ __launch_bounds__(256) void refine_kernel(
    const uint8_t* __restrict__ disp, const uint8_t* __restrict__ center,
    const uint8_t* __restrict__ shifted, const uint8_t* __restrict__ mask, int W, int H,
    size_t pitch, int k, int ddx, int ddy, uint8_t* __restrict__ out, int* __restrict__ fault) {
    const int x = blockIdx.x * 64 + threadIdx.x, y = blockIdx.y * 4 + threadIdx.y;
    if (x >= W || y >= H) return;
    const size_t p = (size_t)y * pitch + x;
    if (mask && mask[p] == 0) return;
    const bool ok = x - k >= 0 && x + k <= W && y - k >= 0 && y + k <= H &&
                    x - 5 * ddx - k >= 0 && x + 5 * ddx + k <= W &&
                    y - 5 * ddy - k >= 0 && y + 5 * ddy + k <= H;
    if (!ok) {
        atomicOr(fault, 1);
        return;
    }
    int bi = 0;
    if constexpr (ND > 0) {
        const unsigned lastmask = (k & 1) ? 0xffffu : 0xffffffffu;  // 2k % 4 == 2 -> 2 bytes
        const uint8_t* win = center + (size_t)(y - k) * pitch + (x - k);
        unsigned best = 0;
        for (int c = 0; c <= 10; c++) {
            const int nx = x + ddx * (c - 5), ny = y + ddy * (c - 5);
            const uint8_t* sw = shifted + (size_t)(ny - k) * pitch + (nx - k);
            unsigned acc = 0;
            for (int v = 0; v < 2 * k; v++)
                acc = sad_row<ND>(sw + (size_t)v * pitch, win + (size_t)v * pitch, lastmask, 2 * k,
                                  acc);
            if (c == 0 || acc < best) { best = acc; bi = c; }
        }
    }
    const double v = (double)disp[p] + (double)(bi - 5) * (double)(ddx + ddy);
    out[p] = (uint8_t)(int)v;
}

// ---- scatters: last write in loop order wins --------------------------------
// Source s (loop index) writes target t: pass 1 keys[t] = max(idx + 1), pass 2
// the source whose idx + 1 equals keys[t] writes its value.

struct Shift2 {
    double preX, preY;
};

__device__ __forceinline__ bool shift2_target(const Shift2& g, double d, int x, int y, int W,
                                              int H, unsigned& t) {
    if (d < 0.5) return false;
    long long tx, ty;
    if (!to_int(g.preX / d, tx) || !to_int(g.preY / d, ty)) return false;
    const long long sx = tx + x, sy = ty + y;
    if (sy >= H || sy < 0 || sx >= W || sx < 0) return false;
    t = (unsigned)(sy * W + sx);
    return true;
}

__global__ void shift2_kernel(const double* __restrict__ depth, int W, int H, Shift2 g,
                              unsigned* __restrict__ keys, double* __restrict__ out, int pass) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    const double d = depth[(size_t)y * W + x];
    unsigned t;
    if (!shift2_target(g, d, x, y, W, H, t)) return;
    const unsigned key = (unsigned)x * (unsigned)H + (unsigned)y + 1u;   // x-major loop order
    if (pass == 0) atomicMax(keys + t, key);
    else if (keys[t] == key) out[t] = d;
}

__device__ __forceinline__ bool project_target(const CamD& c, const double* P, int W, int H,
                                               unsigned& t) {
    const double mult = c.f / (P[2] - c.pz) / c.ps;
    long long px, py;
    if (!to_int((P[0] - c.px) * mult, px) || !to_int((P[1] - c.py) * mult, py)) return false;
    px += W / 2;
    py += H / 2;
    if (!(px >= 0 && px < W && py >= 0 && py < H)) return false;
    t = (unsigned)(py * W + px);
    return true;
}

__global__ void points_to_depth_kernel(const double* __restrict__ pts, long long n, CamD c, int W,
                                       int H, unsigned* __restrict__ keys,
                                       double* __restrict__ out, int pass) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double P[3] = {pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]};
    unsigned t;
    if (!project_target(c, P, W, H, t)) return;
    const unsigned key = (unsigned)i + 1u;
    if (pass == 0) atomicMax(keys + t, key);
    else if (keys[t] == key) out[t] = P[2] - c.pz;
}

// ---- DepthMapToPoints3D: ordered compaction ----------------------------------
constexpr int D2P_ROWS = 64;

__global__ void d2p_count_kernel(const double* __restrict__ depth, int W, int H, int nch,
                                 unsigned* __restrict__ counts) {
    const int u = blockIdx.x * blockDim.x + threadIdx.x, ch = blockIdx.y;
    if (u >= W) return;
    const int v0 = ch * D2P_ROWS, v1 = min(H, v0 + D2P_ROWS);
    unsigned n = 0;
    for (int v = v0; v < v1; v++) n += depth[(size_t)v * W + u] > 0.1;
    counts[(size_t)u * nch + ch] = n;   // column-major unit order
}

// Inclusive wave64 scan in 6 DPP adds (row_shr 1/2/4/8, row_bcast 15/31).
__device__ __forceinline__ unsigned wave_scan_incl(unsigned v) {
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
    return v;
}

// One block: exclusive scan of counts[0..n) in place; total -> *total.
// Rounds of 1024 consecutive counts (one coalesced load per thread), a DPP
// wave scan, the 16 wave totals combined through LDS, and a running carry.
// (A per-thread walk over 32 contiguous counts serialised the loads: 58 us.)
__global__ __launch_bounds__(1024) void d2p_scan_kernel(unsigned* __restrict__ counts, int n,
                                                       long long* __restrict__ total) {
    __shared__ unsigned wsum[16];
    __shared__ unsigned long long carry_s;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    if (t == 0) carry_s = 0;
    __syncthreads();
    for (int base = 0; base < n; base += 1024) {
        const int i = base + t;
        const unsigned c = i < n ? counts[i] : 0u;
        const unsigned incl = wave_scan_incl(c);
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        unsigned before = 0, round = 0;
        for (int w = 0; w < 16; w++) {
            const unsigned ws = wsum[w];
            if (w < wave) before += ws;
            round += ws;
        }
        const unsigned long long carry = carry_s;
        if (i < n) counts[i] = (unsigned)(carry + before + incl - c);
        __syncthreads();                      // everyone has read wsum / carry_s
        if (t == 0) carry_s = carry + round;
        __syncthreads();
    }
    if (t == 0) *total = (long long)carry_s;
}

__global__ void d2p_write_kernel(const double* __restrict__ depth, int W, int H, int nch,
                                 const unsigned* __restrict__ offs, CamD c,
                                 double* __restrict__ pts) {
    const int u = blockIdx.x * blockDim.x + threadIdx.x, ch = blockIdx.y;
    if (u >= W) return;
    const int v0 = ch * D2P_ROWS, v1 = min(H, v0 + D2P_ROWS);
    size_t o = offs[(size_t)u * nch + ch];
    const double r0 = (double)(u - W / 2) * c.ps;
    for (int v = v0; v < v1; v++) {
        const double d = depth[(size_t)v * W + u];
        if (!(d > 0.1)) continue;
        // Camera::inv_project (Camera.cpp:25-33), then pos3D + r * depth
        const double r1 = (double)(v - H / 2) * c.ps, r2 = c.f;
        const double nrm = sqrt(r0 * r0 + r1 * r1 + r2 * r2);
        pts[3 * o + 0] = c.px + (r0 / nrm) * d;
        pts[3 * o + 1] = c.py + (r1 / nrm) * d;
        pts[3 * o + 2] = c.pz + (r2 / nrm) * d;
        o++;
    }
}

}  // namespace

hipError_t launch_shift_perspective(Ctx& c, const sva_camera& in, const sva_camera& out,
                                    const uint8_t* disp, const uint8_t* img, int W, int H,
                                    size_t pitch, uint8_t* shifted) {
    ScopedKernelTimer t(c, "shift_perspective");
    // preMult (functions.cpp:56-57): (in - out) / norm(in - out), host f64, no contraction
    const double dx = in.pos[0] - out.pos[0], dy = in.pos[1] - out.pos[1],
                 dz = in.pos[2] - out.pos[2];
    const double n = sqrt(dx * dx + dy * dy + dz * dz);
    hipLaunchKernelGGL(shift_perspective_kernel, dim3((W + 255) / 256, H), dim3(256), 0, c.stream,
                       disp, img, W, H, pitch, dx / n, dy / n, shifted);
    return hipGetLastError();
}

#define SVA_REFINE_CASE(ND)                                                                    \
    case ND:                                                                                   \
        hipLaunchKernelGGL(refine_kernel<ND>, grid, dim3(64, 4), 0, c.stream, disp, center,     \
                           shifted, mask, W, H, pitch, k, ddx, ddy, out, fault);               \
        break;

hipError_t launch_refine(Ctx& c, const uint8_t* disp, const uint8_t* center,
                         const uint8_t* shifted, const uint8_t* mask, int W, int H, size_t pitch,
                         int k, const sva_camera& c0, const sva_camera& c1, uint8_t* out,
                         int* fault) {
    ScopedKernelTimer t(c, "refine");
    // 0/1 direction (functions.cpp:23-25): v / norm(v) && (v > 0.001)
    const int ddx = (c0.pos[0] - c1.pos[0]) > 0.001 ? 1 : 0;
    const int ddy = (c0.pos[1] - c1.pos[1]) > 0.001 ? 1 : 0;
    const dim3 grid((W + 63) / 64, (H + 3) / 4);
    switch ((k + 1) / 2) {  // ND = ceil(2k / 4)
        SVA_REFINE_CASE(0) SVA_REFINE_CASE(1) SVA_REFINE_CASE(2) SVA_REFINE_CASE(3)
        SVA_REFINE_CASE(4) SVA_REFINE_CASE(5) SVA_REFINE_CASE(6) SVA_REFINE_CASE(7)
        SVA_REFINE_CASE(8) SVA_REFINE_CASE(9) SVA_REFINE_CASE(10) SVA_REFINE_CASE(11)
        SVA_REFINE_CASE(12) SVA_REFINE_CASE(13) SVA_REFINE_CASE(14) SVA_REFINE_CASE(15)
        SVA_REFINE_CASE(16)
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_shift_perspective2(Ctx& c, const sva_camera& in, const sva_camera& out,
                                     const double* depth, int W, int H, unsigned* keys,
                                     double* shifted) {
    ScopedKernelTimer t(c, "shift_perspective2");
    // preMult (functions.cpp:77-78): (in - out) * f / pixel_size
    Shift2 g{(in.pos[0] - out.pos[0]) * in.f / in.pixel_size,
             (in.pos[1] - out.pos[1]) * in.f / in.pixel_size};
    hipError_t e = hipMemsetAsync(keys, 0, (size_t)W * H * 4, c.stream);
    if (e != hipSuccess) return e;
    const dim3 grid((W + 255) / 256, H);
    hipLaunchKernelGGL(shift2_kernel, grid, dim3(256), 0, c.stream, depth, W, H, g, keys, shifted, 0);
    hipLaunchKernelGGL(shift2_kernel, grid, dim3(256), 0, c.stream, depth, W, H, g, keys, shifted, 1);
    return hipGetLastError();
}

hipError_t launch_points_to_depth(Ctx& c, const double* pts, long long n, const sva_camera& cam,
                                  int W, int H, unsigned* keys, double* depth) {
    ScopedKernelTimer t(c, "points_to_depth");
    hipError_t e = hipMemsetAsync(keys, 0, (size_t)W * H * 4, c.stream);
    if (e != hipSuccess) return e;
    if (n == 0) return hipSuccess;
    const dim3 grid((unsigned)((n + 255) / 256));
    hipLaunchKernelGGL(points_to_depth_kernel, grid, dim3(256), 0, c.stream, pts, n, camd(cam), W,
                       H, keys, depth, 0);
    hipLaunchKernelGGL(points_to_depth_kernel, grid, dim3(256), 0, c.stream, pts, n, camd(cam), W,
                       H, keys, depth, 1);
    return hipGetLastError();
}

size_t d2p_units(int W, int H) { return (size_t)W * ((H + D2P_ROWS - 1) / D2P_ROWS); }

hipError_t launch_depth_to_points(Ctx& c, const double* depth, int W, int H,
                                  const sva_camera& cam, unsigned* counts, long long* total,
                                  double* pts) {
    ScopedKernelTimer t(c, "depth_to_points");
    const int nch = (H + D2P_ROWS - 1) / D2P_ROWS;
    const dim3 grid((W + 255) / 256, nch);
    hipLaunchKernelGGL(d2p_count_kernel, grid, dim3(256), 0, c.stream, depth, W, H, nch, counts);
    hipLaunchKernelGGL(d2p_scan_kernel, dim3(1), dim3(1024), 0, c.stream, counts, W * nch, total);
    hipLaunchKernelGGL(d2p_write_kernel, grid, dim3(256), 0, c.stream, depth, W, H, nch, counts,
                       camd(cam), pts);
    return hipGetLastError();
}

}  // namespace sva
