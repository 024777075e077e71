// refine.hip -- SURVEY.md §8f rows 1-2 on the GPU: disparity refinement
// (improveWithDisparity + shiftPerspectiveWithDisparity, functions.cpp:11-72)
// and depth <-> 3-D output (shiftPerspective2, Points3DToDepthMap,
// DepthMapToPoints3D, functions.cpp:74-146).  Semantics of the reference's
// undefined corners: DESIGN.md §2.7 (same as oracle/refine_oracle.c).
//
//   shift_perspective_kernel  1 thread/pixel gather (u8), f64 index math
//   refine_box_kernel          1 <= k <= 16: the 11 window SADs as 2k x 2k box
//                              sums of offset AD planes (wave per column strip)
//   refine_kernel<ND>          other k: 1 thread/pixel, 11 candidate SADs on
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
                                         uint8_t* __restrict__ out, int zero_fill) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    const double d = disp[(size_t)y * pitch + x];
    long long sx, sy;
    if (d == 0 || !to_int(d * preX + x, sx) || !to_int(d * preY + y, sy) || sy >= H || sy < 0 ||
        sx >= W || sx < 0) {
        if (zero_fill) out[(size_t)y * pitch + x] = 0;   // untouched pixel of a fresh plane
        return;
    }
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

// Box-filter form of refine_kernel for 1 <= k <= REF_BOX_KMAX.  Candidate c's
// window SAD is the 2k x 2k box sum of the offset plane
// AD_c(q) = |shifted(q + (c-5)*dd) - center(q)|.  A block of 4 waves owns a
// strip of 64 columns x REF_BOX_TH output rows (lane = column x0 - k + lane,
// 65 - 2k outputs per row); wave w takes candidates 3w..3w+2 (the last wave
// repeats 10).  Per AD row and candidate: one AD, a sliding column sum (old AD
// rows packed 3 per dword in an LDS ring of 2k rows), a DPP wave prefix scan
// and one bpermute, SAD(x) = P[lane + 2k - 1] - P[lane - 1].  Each wave folds
// (SAD << 4) | c into an LDS min per output -- the minimum key is the
// first-minimum candidate -- and after one barrier the block writes the
// masked outputs.  Integer-exact.
constexpr int REF_BOX_KMAX = 16, REF_BOX_TH = 32;

typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void* base, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                             0x00020000);
}

size_t refine_box_lds(int k) { return (size_t)(REF_BOX_TH * 64 + 4 * 2 * k * 64) * 4; }

__global__ __launch_bounds__(256) void refine_box_kernel(
    const uint8_t* __restrict__ disp, const uint8_t* __restrict__ center,
    const uint8_t* __restrict__ shifted, const uint8_t* __restrict__ mask, int W, int H,
    size_t pitch, int k, int ddx, int ddy, uint8_t* __restrict__ out, int* __restrict__ fault) {
    extern __shared__ unsigned smem[];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int w2 = 2 * k, OW = 65 - w2;
    const int x0 = blockIdx.x * OW, y0 = blockIdx.y * REF_BOX_TH;
    const int q = x0 - k + lane;
    const int ylim = min(y0 + REF_BOX_TH, H);
    const int rbeg = y0 - k, rend = ylim - 1 + k;    // AD rows [rbeg, rend)
    unsigned* keys = smem;                            // [REF_BOX_TH][64]
    unsigned* ring = smem + REF_BOX_TH * 64 + wv * w2 * 64;

    if (mask) {             // nothing to do for a strip with no masked output pixel
        const int x = x0 + lane;
        // wave w checks rows y0 + w, y0 + w + 4, ... (8 independent loads per lane)
        int any = 0;
        const int xc = min(x, W - 1);
#pragma unroll
        for (int j = 0; j < REF_BOX_TH / 4; j++) {
            const int y = min(y0 + wv + 4 * j, H - 1);
            any |= mask[(size_t)y * pitch + xc];
        }
        if (!__syncthreads_or(any && lane < OW && x < W)) return;
    }
    for (int i = threadIdx.x; i < REF_BOX_TH * 64; i += 256) keys[i] = ~0u;
    __syncthreads();

    // Raw buffer loads, unconditional, used as loaded: offsets before the plane
    // wrap to huge unsigned values and offsets past it read 0 (hardware range
    // check); a column outside [0, W) may read a neighbouring row's byte, but a
    // pixel that passes the window check below only sums in-image positions, so
    // such values never reach an output.  (Guarded loads become exec branches,
    // and the compiler then waits for every load in flight, the prefetch too.)
    // Offsets in wrapping unsigned arithmetic; H * pitch < 2^31 at launch.
    const unsigned plane = (unsigned)((size_t)H * pitch);
    const rsrc_t rc = make_rsrc(center, plane), rsh = make_rsrc(shifted, plane);
    const unsigned st = (unsigned)ddy * (unsigned)pitch + (unsigned)ddx;   // candidate step
    int cand[3];
    unsigned soff[3];
#pragma unroll
    for (int j = 0; j < 3; j++) {
        cand[j] = min(3 * wv + j, 10);
        soff[j] = (unsigned)(cand[j] - 5) * st;
    }
    struct Row {
        unsigned cb, sb[3];
    };
    auto fetch = [&](int r, Row& n) {
        const unsigned ro = (unsigned)r * (unsigned)pitch + (unsigned)q;
        n.cb = __builtin_amdgcn_raw_buffer_load_b8(rc, ro, 0, 0);
#pragma unroll
        for (int j = 0; j < 3; j++) n.sb[j] = __builtin_amdgcn_raw_buffer_load_b8(rsh, ro + soff[j], 0, 0);
    };
    unsigned col[3] = {0u, 0u, 0u};
    int slot = 0;
    // One AD row: consume cur; the row after next is requested into nxt.
    auto step = [&](int r, const Row& cur, Row& nxt) {
        fetch(r + 2, nxt);
        const int i = r - rbeg;
        unsigned* rs = ring + slot * 64 + lane;
        const unsigned old = i >= w2 ? *rs : 0u;
        unsigned pk = 0;
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const unsigned ad = __builtin_amdgcn_sad_u8(cur.cb, cur.sb[j], 0u);
            col[j] = col[j] + ad - ((old >> (8 * j)) & 0xffu);
            pk |= ad << (8 * j);
        }
        *rs = pk;
        if (++slot == w2) slot = 0;
        if (i < w2 - 1) return;
        unsigned key = ~0u;
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const unsigned P = wave_scan_incl(col[j]);
            const unsigned hi =
                (unsigned)__builtin_amdgcn_ds_bpermute((lane + w2 - 1) << 2, (int)P);
            key = min(key, ((hi - (P - col[j])) << 4) | (unsigned)cand[j]);
        }
        atomicMin(keys + (r - k + 1 - y0) * 64 + lane, key);
    };
    // Two rows in flight, unrolled by three over rotating row buffers: no
    // register copies of in-flight loads (a copy at the loop end makes the
    // compiler wait for the prefetch).
    Row A, B, C;
    fetch(rbeg, A);
    fetch(rbeg + 1, B);
    for (int r = rbeg; r < rend; r += 3) {
        step(r, A, C);
        if (r + 1 >= rend) break;
        step(r + 1, B, A);
        if (r + 2 >= rend) break;
        step(r + 2, C, B);
    }
    __syncthreads();
    // write-out: all mask / disparity bytes requested before any is used
    const int xo = x0 + lane, xoc = min(xo, W - 1);
    unsigned mv[REF_BOX_TH / 4], dv[REF_BOX_TH / 4];
#pragma unroll
    for (int j = 0; j < REF_BOX_TH / 4; j++) {
        const size_t p = (size_t)min(y0 + wv + 4 * j, H - 1) * pitch + xoc;
        mv[j] = mask ? mask[p] : 1u;
        dv[j] = disp[p];
    }
    if (lane >= OW || xo >= W) return;
#pragma unroll
    for (int j = 0; j < REF_BOX_TH / 4; j++) {
        const int y = y0 + wv + 4 * j, x = xo;
        if (y >= ylim || mv[j] == 0) continue;
        const bool ok = x - k >= 0 && x + k <= W && y - k >= 0 && y + k <= H &&
                        x - 5 * ddx - k >= 0 && x + 5 * ddx + k <= W &&
                        y - 5 * ddy - k >= 0 && y + 5 * ddy + k <= H;
        if (!ok) {
            atomicOr(fault, 1);
            continue;
        }
        const int bi = (int)(keys[(y - y0) * 64 + lane] & 15u);
        const double v = (double)dv[j] + (double)(bi - 5) * (double)(ddx + ddy);
        out[(size_t)y * pitch + x] = (uint8_t)(int)v;
    }
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
                                    size_t pitch, uint8_t* shifted, bool zero_fill) {
    ScopedKernelTimer t(c, "shift_perspective");
    // preMult (functions.cpp:56-57): (in - out) / norm(in - out), host f64, no contraction
    const double dx = in.pos[0] - out.pos[0], dy = in.pos[1] - out.pos[1],
                 dz = in.pos[2] - out.pos[2];
    const double n = sqrt(dx * dx + dy * dy + dz * dz);
    hipLaunchKernelGGL(shift_perspective_kernel, dim3((W + 255) / 256, H), dim3(256), 0, c.stream,
                       disp, img, W, H, pitch, dx / n, dy / n, shifted, (int)zero_fill);
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
    if (k >= 1 && k <= REF_BOX_KMAX && (size_t)H * pitch < ((size_t)1 << 31)) {
        const int ow = 65 - 2 * k;
        hipLaunchKernelGGL(refine_box_kernel, dim3((W + ow - 1) / ow, (H + REF_BOX_TH - 1) / REF_BOX_TH),
                           dim3(256), refine_box_lds(k), c.stream, disp, center, shifted, mask, W,
                           H, pitch, k, ddx, ddy, out, fault);
        return hipGetLastError();
    }
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
