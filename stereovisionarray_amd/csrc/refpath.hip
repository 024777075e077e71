// refpath.hip -- Mode R: the reference's own disparity path, bit-exact
// (DESIGN.md §3).
//
//   ref_endpoints_kernel  one thread per pixel, IEEE f64 in the reference's
//                         operand order (Camera.cpp:15-34,
//                         CameraStereoVision.cpp:28,60-71).  FMA contraction
//                         is off for this file so every rounding matches.
//   ref_match_kernel      one wave per pixel, one lane per Bresenham
//                         candidate (functions.cpp:253-321 in closed form),
//                         2k x 2k SAD with v_sad_u8 (4 |a-b| per lane-op) on
//                         dword-realigned rows (v_alignbyte), first-minimum
//                         argmin as a wave-wide u64 min over (SAD << 32 | i),
//                         then (uchar)(int)sqrt(dx^2 + dy^2)
//                         (CameraStereoVision.cpp:85-89).
#pragma clang fp contract(off)

#include <cstdlib>

#include "sva_device.h"
#include "sva_internal.h"

namespace sva {
namespace {

struct CamD {
    double f, px, py, pz, ps;
};

__device__ __forceinline__ CamD cam_of(const sva_camera& c) {
    return CamD{c.f, c.pos[0], c.pos[1], c.pos[2], c.pixel_size};
}

// Camera::project (Camera.cpp:15-21)
__device__ __forceinline__ void project(const CamD& c, double X, double Y, double Z, int& u,
                                        int& v) {
    const double mult = c.f / (Z - c.pz) / c.ps;
    u = (int)((X - c.px) * mult);
    v = (int)((Y - c.py) * mult);
}

__global__ void ref_endpoints_kernel(int W, int H, sva_camera cref_, sva_camera coth_, int k,
                                     double t_near, double t_far, int4* __restrict__ ends,
                                     uint8_t* __restrict__ valid) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    const size_t p = (size_t)y * W + x;
    const CamD cr = cam_of(cref_), co = cam_of(coth_);
    const int hx = W / 2, hy = H / 2;  // halfRes = resolution / 2 (:28)
    // Camera::inv_project (Camera.cpp:25-33): vector / norm(vector)
    const double v0 = (double)(x - hx) * cr.ps;
    const double v1 = (double)(y - hy) * cr.ps;
    const double v2 = cr.f;
    const double n = __builtin_sqrt(v0 * v0 + v1 * v1 + v2 * v2);
    const double e0 = v0 / n, e1 = v1 / n, e2 = v2 / n;
    // p1 = pos3D + vec*t_near ; p2 = pos3D + vec*t_far (:61-62)
    int a0, a1, b0, b1;
    project(co, cr.px + e0 * t_near, cr.py + e1 * t_near, cr.pz + e2 * t_near, a0, a1);
    project(co, cr.px + e0 * t_far, cr.py + e1 * t_far, cr.pz + e2 * t_far, b0, b1);
    a0 += hx; a1 += hy; b0 += hx; b1 += hy;
    bool ok = x >= k && x < W - k && y >= k && y < H - k;   // loop bounds (:49,51)
    ok = ok && !(a0 < k || a1 < k || a0 > W - k || a1 > H - k);  // :66
    ok = ok && !(b0 < k || b1 < k || b0 > W - k || b1 > H - k);  // :69
    ends[p] = make_int4(a0, a1, b0, b1);
    valid[p] = ok ? 1 : 0;
}

// Closed form of functions.cpp:253-321.  The line is stored as its start
// point, the major-axis direction and the Bresenham slope numerator/denominator
// so candidate i is O(1):  plotLineLow emits (x0+i, y0 + yi*floor((2|dy|i + dx - 1) / (2dx))),
// plotLineHigh the transpose.  (Proof: the error term D_i = 2|dy|(i+1) - dx -
// 2dx*n_i stays in (-2dx, 2|dy|], which gives n_i = ceil((2|dy|i - dx)/(2dx)).)
struct Line {
    int x0, y0;   // first emitted point
    int high;     // 1: plotLineHigh (y major)
    int step;     // +-1 minor-axis step (yi / xi)
    int a, b;     // 2*|minor delta|, 2*major delta
    int major;    // major delta (dx for low, dy for high)
    int n;        // number of points
};

__device__ __forceinline__ Line make_line(int p1x, int p1y, int p2x, int p2y) {
    // bresenham(point2 = pixel1, point1 = pixel2), functions.cpp:299-321
    const int ax = p1x, ay = p1y, bx = p2x, by = p2y;
    int x0, y0, x1, y1;
    Line L;
    if (abs(ay - by) < abs(ax - bx)) {
        if (bx > ax) { x0 = ax; y0 = ay; x1 = bx; y1 = by; }
        else { x0 = bx; y0 = by; x1 = ax; y1 = ay; }
        int dx = x1 - x0, dy = y1 - y0;
        L.high = 0;
        L.step = dy < 0 ? -1 : 1;
        L.a = 2 * (dy < 0 ? -dy : dy);
        L.b = 2 * dx;
        L.major = dx;
        L.n = dx + 1;
    } else {
        if (by > ay) { x0 = ax; y0 = ay; x1 = bx; y1 = by; }
        else { x0 = bx; y0 = by; x1 = ax; y1 = ay; }
        int dx = x1 - x0, dy = y1 - y0;
        L.high = 1;
        L.step = dx < 0 ? -1 : 1;
        L.a = 2 * (dx < 0 ? -dx : dx);
        L.b = 2 * dy;
        L.major = dy;
        L.n = dy + 1;   // dy >= 0 here; dy == 0 only for a single point
    }
    L.x0 = x0;
    L.y0 = y0;
    return L;
}

__device__ __forceinline__ void line_point(const Line& L, int i, int& cx, int& cy) {
    const int minor = L.b > 0 ? (L.a * i + L.major - 1) / L.b : 0;
    if (L.high) { cx = L.x0 + L.step * minor; cy = L.y0 + i; }
    else { cx = L.x0 + i; cy = L.y0 + L.step * minor; }
}

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        unsigned lo = (unsigned)v, hi = (unsigned)(v >> 32);
        unsigned olo = __shfl_xor(lo, off, 64), ohi = __shfl_xor(hi, off, 64);
        unsigned long long o = ((unsigned long long)ohi << 32) | olo;
        v = o < v ? o : v;
    }
    return v;
}

// sad_row<ND>: sva_device.h

// Per-pixel wave algorithm (one wave per reference pixel, one lane per
// candidate, v_sad_u8 on v_alignbyte-realigned rows).  Used by
// ref_match_kernel and as the per-tile fallback of ref_plane_kernel.
template <int ND>
__device__ __forceinline__ void match_pixel_wave(const uint8_t* __restrict__ ref,
                                                 const uint8_t* __restrict__ other, int W,
                                                 size_t pitch, int x, int y, const int4 e, int k,
                                                 uint8_t* __restrict__ disp_u8,
                                                 uint16_t* __restrict__ disp_u16,
                                                 uint8_t* __restrict__ valid_out) {
    const int lane = threadIdx.x & 63;
    const size_t p = (size_t)y * W + x;
    const Line L = make_line(e.x, e.y, e.z, e.w);                     // :73
    const int nbytes = 2 * k;
    const unsigned lastmask = (nbytes & 3) ? 0xffffu : 0xffffffffu;
    const uint8_t* kern = ref + (size_t)(y - k) * pitch + (x - k);    // :57
    unsigned long long best = ~0ull;
    for (int base = 0; base < L.n; base += 64) {                      // :76-83
        const int i = base + lane;
        unsigned long long key = ~0ull;
        if (i < L.n) {
            int cx, cy;
            line_point(L, i, cx, cy);
            const uint8_t* sel = other + (size_t)(cy - k) * pitch + (cx - k);
            unsigned acc = 0;
            for (int v = 0; v < nbytes; v++)
                acc = sad_row<ND>(sel + (size_t)v * pitch, kern + (size_t)v * pitch, lastmask,
                                  nbytes, acc);
            key = ((unsigned long long)acc << 32) | (unsigned)i;
        }
        key = wave_min_u64(key);                                      // :85 first min
        best = key < best ? key : best;
    }
    if (lane == 0) {
        int cx, cy;
        line_point(L, (int)(best & 0xffffffffu), cx, cy);
        const double dx = (double)(cx - x), dy = (double)(cy - y);
        const int dn = (int)__builtin_sqrt(dx * dx + dy * dy);       // :89
        disp_u8[p] = (uint8_t)dn;
        if (disp_u16) disp_u16[p] = (uint16_t)dn;
        if (valid_out) valid_out[p] = 1;
    }
}

template <int ND>
__global__ __launch_bounds__(256) void ref_match_kernel(
    const uint8_t* __restrict__ ref, const uint8_t* __restrict__ other, int W, int H, size_t pitch,
    const uint8_t* __restrict__ mask, const int4* __restrict__ ends,
    const uint8_t* __restrict__ valid_in, int k, uint8_t* __restrict__ disp_u8,
    uint16_t* __restrict__ disp_u16, uint8_t* __restrict__ valid_out) {
    // one wave per pixel of the loop region [k, W-k) x [k, H-k)
    const int iw = W - 2 * k;
    const long long q = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
    if (q >= (long long)iw * (H - 2 * k)) return;
    const int y = k + (int)(q / iw), x = k + (int)(q % iw);
    const size_t p = (size_t)y * W + x;
    if (!valid_in[p]) return;
    if (mask && mask[p] == 0) return;                                 // :53
    match_pixel_wave<ND>(ref, other, W, pitch, x, y, ends[p], k, disp_u8, disp_u16, valid_out);
}

// ---- offset-plane algorithm (same results, far less work) -------------------
//
// For a fixed offset delta, AD(q) = |O(q + delta) - R(q)| is shared by every
// reference pixel, and SAD(p, delta) is the 2k x 2k box sum of AD at p.  A
// workgroup owns a tile of TW = 64 - 2k columns x PT_ROWS rows of reference
// pixels, whose window-extended region is exactly 64 columns wide.  It
//   1. collects the union of its pixels' candidate offsets c_i - p in an LDS
//      bitmap over their bounding box (neighbouring pixels' offsets nearly
//      coincide, so this is a thin band even for diagonal pairs);
//   2. per offset plane: AD bytes of the region into LDS (aligned dword loads
//      of O realigned with v_alignbyte), column sums sliding down the rows,
//      row sums sliding along x, and for each pixel a division-free test of
//      whether delta is on ITS Bresenham line -- candidate i on a low line is
//      x0 + i with minor offset m = floor((a*i + major - 1) / b), i.e.
//      t*b <= a*i + major - 1 < (t+1)*b for t = step*(c.minor - minor0) --
//      keeping min over (SAD << 32 | i): the reference's first minimum
//      (CameraStereoVision.cpp:85) whatever order the planes are visited in.
// A tile whose offset box exceeds the bitmap falls back to match_pixel_wave.
constexpr int PT_ROWS = 32;                  // tile rows
constexpr int PT_REG_W = 64;                 // region width = TW + 2k
constexpr int PT_MAXK = 28;                  // TW >= 8
constexpr int PT_REG_H = PT_ROWS + 2 * PT_MAXK;
constexpr int PT_P_W = PT_REG_W + 1;         // prefix rows: 65 u32 (odd stride spreads banks)
constexpr int PT_MAXBITS = 1 << 15;          // offset bitmap capacity
constexpr int PT_OU_BYTES = 28 * 1024;       // staged union of O over all planes (3 workgroups/CU)

// Inclusive wave64 scan in 6 DPP adds (no LDS): Hillis-Steele within each
// 16-lane row (row_shr 1, 2, 4, 8; lanes with no source read 0), then
// row_bcast:15 adds lane 15 into rows 1 and 3 and row_bcast:31 adds lane 31
// into rows 2 and 3.  (A ds_bpermute-based __shfl_up scan put 6 LDS
// round-trips on the dependency chain of every row.)
__device__ __forceinline__ unsigned scan64_dpp(unsigned v) {
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);   // row_shr:1
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);   // row_shr:2
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);   // row_shr:4
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);   // row_shr:8
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);   // row_bcast:15
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return v;
}

__device__ __forceinline__ bool on_line(const Line& L, int cx, int cy) {
    int i, t;
    if (L.high) { i = cy - L.y0; t = L.step * (cx - L.x0); }
    else { i = cx - L.x0; t = L.step * (cy - L.y0); }
    if (i < 0 || i >= L.n) return false;
    if (L.b == 0) return t == 0;
    const int num = L.a * i + L.major - 1;
    return t >= 0 && t * L.b <= num && num < (t + 1) * L.b;
}

__device__ __forceinline__ int line_index(const Line& L, int cx, int cy) {
    return L.high ? cy - L.y0 : cx - L.x0;
}

template <int ND>
__global__ __launch_bounds__(256) void ref_plane_kernel(
    const uint8_t* __restrict__ ref, const uint8_t* __restrict__ other, int W, int H, size_t pitch,
    const uint8_t* __restrict__ mask, const int4* __restrict__ ends,
    const uint8_t* __restrict__ valid_in, int k, uint8_t* __restrict__ disp_u8,
    uint16_t* __restrict__ disp_u16, uint8_t* __restrict__ valid_out) {
    __shared__ __attribute__((aligned(16))) uint8_t Rr[PT_REG_H][PT_REG_W];   // read as dwords
    __shared__ __attribute__((aligned(16))) uint8_t AD[PT_REG_H][PT_REG_W];
    __shared__ unsigned Pf[PT_ROWS][PT_P_W];   // per-row exclusive prefix of column sums
    __shared__ unsigned bits[PT_MAXBITS / 32];
    __shared__ __attribute__((aligned(16))) uint8_t OU[PT_OU_BYTES];   // O over every plane
    __shared__ int box[4];                    // dx_lo, dx_hi, dy_lo, dy_hi
    const int t = threadIdx.x;
    const int TW = PT_REG_W - 2 * k;
    const int tx0 = k + blockIdx.x * TW, ty0 = k + blockIdx.y * PT_ROWS;
    const int rx0 = tx0 - k, ry0 = ty0 - k;   // region origin (image coords)
    const int RH = PT_ROWS + 2 * k;
    // pixels of this thread: row r = t / 8, x_l in [seg*PPT, seg*PPT + PPT)
    const int PPT = (TW + 7) / 8;
    const int r = t >> 3, xs = (t & 7) * PPT;
    constexpr int MAXPPT = (PT_REG_W - 2 + 7) / 8;   // k >= 1: TW <= 62
    Line Ls[MAXPPT];
    bool ok[MAXPPT];
    unsigned long long best[MAXPPT];
    if (t < 4) box[t] = (t & 1) ? -0x7fffffff : 0x7fffffff;
    for (int i = t; i < RH * PT_REG_W; i += 256) {
        const int v = i >> 6, u = i & 63;
        const int gx = rx0 + u, gy = ry0 + v;
        Rr[v][u] = (gx < W && gy < H) ? ref[(size_t)gy * pitch + gx] : 0;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < MAXPPT; j++) {
        ok[j] = false;
        best[j] = ~0ull;
        const int xl = xs + j, x = tx0 + xl, y = ty0 + r;
        if (j >= PPT || xl >= TW || x >= W - k || y >= H - k) continue;
        const size_t p = (size_t)y * W + x;
        if (!valid_in[p] || (mask && mask[p] == 0)) continue;
        const int4 e = ends[p];
        ok[j] = true;
        Ls[j] = make_line(e.x, e.y, e.z, e.w);
        atomicMin(&box[0], min(e.x, e.z) - x);
        atomicMax(&box[1], max(e.x, e.z) - x);
        atomicMin(&box[2], min(e.y, e.w) - y);
        atomicMax(&box[3], max(e.y, e.w) - y);
    }
    __syncthreads();
    const int dxlo = box[0], dylo = box[2];
    const int bw = box[1] - box[0] + 1, bh = box[3] - box[2] + 1;
    if (box[1] < box[0]) return;             // no valid pixel in this tile
    if ((long long)bw * bh > PT_MAXBITS) {
        // offset box too large for the bitmap: per-pixel waves for this tile
        const int wave = t >> 6;
        for (int pi = wave; pi < TW * PT_ROWS; pi += 4) {
            const int x = tx0 + pi % TW, y = ty0 + pi / TW;
            if (x >= W - k || y >= H - k) continue;
            const size_t p = (size_t)y * W + x;
            if (!valid_in[p] || (mask && mask[p] == 0)) continue;
            match_pixel_wave<ND>(ref, other, W, pitch, x, y, ends[p], k, disp_u8, disp_u16,
                                 valid_out);
        }
        return;
    }
    const int nwords = (bw * bh + 31) >> 5;
    for (int i = t; i < nwords; i += 256) bits[i] = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < MAXPPT; j++) {
        if (!ok[j]) continue;
        const int x = tx0 + xs + j, y = ty0 + r;
        for (int i = 0; i < Ls[j].n; i++) {
            int cx, cy;
            line_point(Ls[j], i, cx, cy);
            const int b = (cy - y - dylo) * bw + (cx - x - dxlo);
            atomicOr(&bits[b >> 5], 1u << (b & 31));
        }
    }
    // Stage O over the union of all planes once, when it fits: rows
    // ry0 + dylo + [0, RH + bh - 1), cols rx0 + dxlo + [0, 64 + bw - 1); the
    // plane loop then reads only LDS.  Otherwise each plane loads O itself.
    const int ouw = (PT_REG_W + bw - 1 + 3) & ~3, ouh = RH + bh - 1;
    const bool staged = ouw * ouh <= PT_OU_BYTES - 8;   // slack: the realigning read may touch one dword past the region
    if (staged) {
        const int ox0 = rx0 + dxlo, oy0 = ry0 + dylo;
        for (int i = t; i < ouw * ouh; i += 256) {
            const int v = i / ouw, u = i - v * ouw;
            const int gx = ox0 + u, gy = oy0 + v;
            OU[i] = (gx >= 0 && gx < W && gy >= 0 && gy < H) ? other[(size_t)gy * pitch + gx] : 0;
        }
    }
    __syncthreads();
    const int cu = t & 63, cseg = t >> 6;    // column-sum thread: column, 8-row segment
    for (int wd = 0; wd < nwords; wd++) {
        unsigned m = bits[wd];               // uniform across the workgroup
        while (m) {
            const int bit = __builtin_ctz(m);
            m &= m - 1;
            const int b = wd * 32 + bit;
            const int ddy = dylo + b / bw, ddx = dxlo + b % bw;
            // (a) AD bytes of the region for this plane
            for (int i = t; i < RH * 16; i += 256) {
                const int v = i >> 4, u4 = (i & 15) * 4;
                const int gx = rx0 + u4 + ddx, gy = ry0 + v + ddy;
                unsigned o;
                if (staged) {
                    // bytes OU[(v + ddy - dylo) * ouw + u4 + ddx - dxlo + 0..3], realigned
                    const int bo = (v + ddy - dylo) * ouw + u4 + (ddx - dxlo);
                    const unsigned* w = reinterpret_cast<const unsigned*>(OU) + (bo >> 2);
                    const unsigned sh = (unsigned)(bo & 3);
                    o = sh ? __builtin_amdgcn_alignbyte(w[1], w[0], sh) : w[0];
                } else if (gy >= 0 && gy < H && gx >= 0 && gx + 3 < W) {
                    const uint8_t* src = other + (size_t)gy * pitch + gx;
                    const uintptr_t a = (uintptr_t)src;
                    const unsigned* w = (const unsigned*)(a & ~(uintptr_t)3);
                    const unsigned sh = (unsigned)(a & 3);
                    // never read the dword after the one holding the last byte
                    o = sh ? __builtin_amdgcn_alignbyte(w[1], w[0], sh) : w[0];
                } else {
                    o = 0;
                    for (int q = 0; q < 4; q++) {
                        const int x = gx + q;
                        if (gy >= 0 && gy < H && x >= 0 && x < W)
                            o |= (unsigned)other[(size_t)gy * pitch + x] << (8 * q);
                    }
                }
                const unsigned rr = *(const unsigned*)&Rr[v][u4];
                // |o - r| per byte on even / odd bytes as u16 pairs: max - min
                const u16x2 oe = as_v2(o & 0x00ff00ffu), oo = as_v2((o >> 8) & 0x00ff00ffu);
                const u16x2 re = as_v2(rr & 0x00ff00ffu), ro = as_v2((rr >> 8) & 0x00ff00ffu);
                const unsigned de = as_u32(__builtin_elementwise_max(oe, re) - vmin2(oe, re));
                const unsigned dd = as_u32(__builtin_elementwise_max(oo, ro) - vmin2(oo, ro));
                *(unsigned*)&AD[v][u4] = de | (dd << 8);
            }
            __syncthreads();
            // (b) column sums over 2k rows (wave = 8 output rows, lane =
            // column), each row turned into an exclusive prefix over the 64
            // columns by a cross-lane scan, so (c) needs two reads per pixel.
            // (Summing 2k consecutive u16 column sums per pixel instead let
            // the compiler merge them into unaligned wide LDS loads:
            // SQ_LDS_UNALIGNED_STALL 3.07G of 3.84G LDS cycles.)
            {
                const int r0 = cseg * 8;
                unsigned sacc = 0;
                for (int v = 0; v < 2 * k; v++) sacc += AD[r0 + v][cu];
#pragma unroll
                for (int rr2 = 0; rr2 < 8; rr2++) {
                    if (rr2 > 0) {
                        sacc += AD[r0 + rr2 - 1 + 2 * k][cu];
                        sacc -= AD[r0 + rr2 - 1][cu];
                    }
                    const unsigned sc = scan64_dpp(sacc);   // inclusive over the lanes
                    Pf[r0 + rr2][cu + 1] = sc;
                    if (cu == 0) Pf[r0 + rr2][0] = 0;
                }
            }
            __syncthreads();
            // (c) SAD from two prefix reads, membership, first-minimum key
#pragma unroll
            for (int j = 0; j < MAXPPT; j++) {
                if (!ok[j]) continue;               // ok[] implies j < PPT, xs + j < TW
                const int xl = xs + j;
                const unsigned sad = Pf[r][xl + 2 * k] - Pf[r][xl];
                const int cx = tx0 + xl + ddx, cy = ty0 + r + ddy;
                if (!on_line(Ls[j], cx, cy)) continue;
                const unsigned long long key =
                    ((unsigned long long)sad << 32) | (unsigned)line_index(Ls[j], cx, cy);
                best[j] = key < best[j] ? key : best[j];
            }
        }
    }
#pragma unroll
    for (int j = 0; j < MAXPPT; j++) {
        if (!ok[j]) continue;
        const int x = tx0 + xs + j, y = ty0 + r;
        const size_t p = (size_t)y * W + x;
        int cx, cy;
        line_point(Ls[j], (int)(best[j] & 0xffffffffu), cx, cy);
        const double dx = (double)(cx - x), dy = (double)(cy - y);
        const int dn = (int)__builtin_sqrt(dx * dx + dy * dy);       // :89
        disp_u8[p] = (uint8_t)dn;
        if (disp_u16) disp_u16[p] = (uint16_t)dn;
        if (valid_out) valid_out[p] = 1;
    }
}

typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void* base, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                             0x00020000);
}

// ---- offset-plane algorithm, v2 (the one launched) --------------------------
// Same tiles, bitmap, planes and first-minimum keys as ref_plane_kernel; what
// changes is the layout and who does what:
//   * R, the staged O union and the AD planes are held column-major in LDS
//     (byte (col, row) at col * stride + row, stride an odd number of dwords),
//     so a lane that owns a column reads 4 rows per ds_read_b32 and the 2k-row
//     column sum is k/2 v_sad_u8(dword, 0) byte sums.
//   * Wave w owns output rows 8w..8w+7 and lane = output column: it turns its
//     own column sums into SADs with a DPP scan and one ds_bpermute
//     (SAD = P[lane + 2k - 1] - P[lane] + col[lane]) and tests membership for
//     its own pixels, whose lines and best keys stay in registers.  No prefix
//     table, no second pass.
//   * Two planes per iteration: one barrier per plane instead of two.
//   * Tiles whose O union does not fit the staging buffer read O with raw
//     buffer loads (a valid pixel's windows lie inside the image, so the
//     bytes a clamped or wrapped column brings in never reach its SAD).
constexpr int P2_ROWS = 32;                           // 4 waves x 8 rows
constexpr int P2_RS = 92;                             // R / AD column stride: 23 dwords >= 88 rows
constexpr int P2_OU_BYTES = 24 * 1024;

__device__ __forceinline__ unsigned bytes4(const uint8_t* lds, int byte_off) {
    // 4 bytes at any byte offset of an LDS image: two aligned dwords, realigned
    const unsigned* w = reinterpret_cast<const unsigned*>(lds) + (byte_off >> 2);
    const unsigned sh = (unsigned)(byte_off & 3);
    return sh ? __builtin_amdgcn_alignbyte(w[1], w[0], sh) : w[0];
}

__device__ __forceinline__ unsigned absdiff4(unsigned o, unsigned r) {
    // |o - r| per byte, even and odd bytes as u16 pairs: max - min
    const u16x2 oe = as_v2(o & 0x00ff00ffu), oo = as_v2((o >> 8) & 0x00ff00ffu);
    const u16x2 re = as_v2(r & 0x00ff00ffu), ro = as_v2((r >> 8) & 0x00ff00ffu);
    const unsigned de = as_u32(__builtin_elementwise_max(oe, re) - vmin2(oe, re));
    const unsigned dd = as_u32(__builtin_elementwise_max(oo, ro) - vmin2(oo, ro));
    return de | (dd << 8);
}

template <int ND>
__global__ __launch_bounds__(256) void ref_plane2_kernel(
    const uint8_t* __restrict__ ref, const uint8_t* __restrict__ other, int W, int H, size_t pitch,
    const uint8_t* __restrict__ mask, const int4* __restrict__ ends,
    const uint8_t* __restrict__ valid_in, int k, uint8_t* __restrict__ disp_u8,
    uint16_t* __restrict__ disp_u16, uint8_t* __restrict__ valid_out) {
    __shared__ __attribute__((aligned(16))) uint8_t RT[64 * P2_RS];
    __shared__ __attribute__((aligned(16))) uint8_t ADT[2][64 * P2_RS];
    __shared__ unsigned bits[PT_MAXBITS / 32];
    __shared__ __attribute__((aligned(16))) uint8_t OUT[P2_OU_BYTES];
    __shared__ int box[4];                    // dx_lo, dx_hi, dy_lo, dy_hi
    __shared__ unsigned short uniq[P2_ROWS * 64];   // pixels with a distinct relative line
    __shared__ int nuniq;
    const int t = threadIdx.x, lane = t & 63;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
    const int TW = PT_REG_W - 2 * k, w2 = 2 * k;
    const int tx0 = k + blockIdx.x * TW, ty0 = k + blockIdx.y * P2_ROWS;
    const int rx0 = tx0 - k, ry0 = ty0 - k;   // region origin (image coords)
    const int RH = P2_ROWS + w2;
#ifdef SVA_REF_PROF
    long long tp[6];
    int nplanes = 0;
    tp[0] = clock64();
#endif
    if (t < 4) box[t] = (t & 1) ? -0x7fffffff : 0x7fffffff;
    for (int i = t; i < RH * PT_REG_W; i += 256) {
        const int v = i >> 6, u = i & 63;
        const int gx = rx0 + u, gy = ry0 + v;
        RT[u * P2_RS + v] = (gx < W && gy < H) ? ref[(size_t)gy * pitch + gx] : 0;
    }
    __syncthreads();
    // this thread's pixels: column lane, rows 8 * wv + j.  All loads are
    // issued first (clamped addresses), then used.
    // Per-pixel membership terms (on_line restated per plane with 24-bit
    // multiplies and no short-circuit): with ia = cx - x0, ib = cy - y0,
    //   i = high ? ib : ia,  tt = step * (high ? ia : ib),  num = a*i + major - 1
    //   on = i in [0, n) && (b == 0 ? tt == 0 : tt >= 0 && tt*b <= num < tt*b + b)
    // n = 0 marks a pixel that is not evaluated.
    int m_ox[8], m_oy[8], m_n[8], m_fl[8], m_a[8], m_b[8], m_mj[8];
    bool ok[8];
    int4 E[8];
    unsigned long long best[8];
    {
        unsigned vin[8], mk[8];
        const int xc = min(tx0 + lane, W - 1);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const size_t p = (size_t)min(ty0 + 8 * wv + j, H - 1) * W + xc;
            vin[j] = valid_in[p];
            mk[j] = mask ? mask[p] : 1u;
            E[j] = ends[p];
        }
        int bx0 = 0x7fffffff, bx1 = -0x7fffffff, by0 = 0x7fffffff, by1 = -0x7fffffff;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int x = tx0 + lane, y = ty0 + 8 * wv + j;
            ok[j] = lane < TW && x < W - k && y < H - k && vin[j] != 0 && mk[j] != 0;
            best[j] = ~0ull;
            const Line L = make_line(E[j].x, E[j].y, E[j].z, E[j].w);
            m_ox[j] = x - L.x0;
            m_oy[j] = y - L.y0;
            m_n[j] = ok[j] ? L.n : 0;
            m_fl[j] = (L.high ? 1 : 0) | (L.step < 0 ? 2 : 0);
            m_a[j] = L.a;
            m_b[j] = L.b;
            m_mj[j] = L.major - 1;
            if (ok[j]) {
                bx0 = min(bx0, min(E[j].x, E[j].z) - x);
                bx1 = max(bx1, max(E[j].x, E[j].z) - x);
                by0 = min(by0, min(E[j].y, E[j].w) - y);
                by1 = max(by1, max(E[j].y, E[j].w) - y);
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {   // wave min/max, then one atomic each
            bx0 = min(bx0, __shfl_xor(bx0, off, 64));
            bx1 = max(bx1, __shfl_xor(bx1, off, 64));
            by0 = min(by0, __shfl_xor(by0, off, 64));
            by1 = max(by1, __shfl_xor(by1, off, 64));
        }
        if (lane == 0) {
            atomicMin(&box[0], bx0);
            atomicMax(&box[1], bx1);
            atomicMin(&box[2], by0);
            atomicMax(&box[3], by1);
        }
    }
    __syncthreads();
    const int dxlo = box[0], dylo = box[2];
    const int bw = box[1] - box[0] + 1, bh = box[3] - box[2] + 1;
    if (box[1] < box[0]) return;             // no valid pixel in this tile
    if ((long long)bw * bh > PT_MAXBITS) {
        // offset box too large for the bitmap: per-pixel waves for this tile
        for (int pi = wv; pi < TW * P2_ROWS; pi += 4) {
            const int x = tx0 + pi % TW, y = ty0 + pi / TW;
            if (x >= W - k || y >= H - k) continue;
            const size_t p = (size_t)y * W + x;
            if (!valid_in[p] || (mask && mask[p] == 0)) continue;
            match_pixel_wave<ND>(ref, other, W, pitch, x, y, ends[p], k, disp_u8, disp_u16,
                                 valid_out);
        }
        return;
    }
    const int nwords = (bw * bh + 31) >> 5;
    for (int i = t; i < nwords; i += 256) bits[i] = 0;
    if (t == 0) nuniq = 0;
    __syncthreads();
#ifdef SVA_REF_PROF
    tp[1] = clock64();
#endif
    // Bresenham is translation-invariant: pixels whose endpoints, relative
    // to themselves, match the left neighbour's or the previous row's have the
    // same offset set.  Only the first of each such chain enters the list.
    {
        int4 prev = make_int4(0, 0, 0, 0);
        bool prev_ok = false;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int x = tx0 + lane, y = ty0 + 8 * wv + j;
            const int4 rel = make_int4(E[j].x - x, E[j].y - y, E[j].z - x, E[j].w - y);
            const int lx = __shfl_up(rel.x, 1, 64), ly = __shfl_up(rel.y, 1, 64);
            const int lz = __shfl_up(rel.z, 1, 64), lw = __shfl_up(rel.w, 1, 64);
            const int lok = __shfl_up((int)ok[j], 1, 64);
            const bool same_left = lane > 0 && lok && lx == rel.x && ly == rel.y && lz == rel.z &&
                                   lw == rel.w;
            const bool same_up = prev_ok && prev.x == rel.x && prev.y == rel.y &&
                                 prev.z == rel.z && prev.w == rel.w;
            if (ok[j] && !same_left && !same_up) uniq[atomicAdd(&nuniq, 1)] = (unsigned short)((8 * wv + j) * 64 + lane);
            prev = rel;
            prev_ok = ok[j];
        }
    }
    __syncthreads();
    // one thread per distinct line, walking it incrementally: the minor
    // coordinate of point i is floor((a*i + major - 1) / b) with a <= b, so it
    // advances by at most one per step (no division in the loop)
    for (int q = t; q < nuniq; q += 256) {
        const int pl = uniq[q], x = tx0 + (pl & 63), y = ty0 + (pl >> 6);
        const int4 e = ends[(size_t)y * W + x];
        const Line L = make_line(e.x, e.y, e.z, e.w);
        int mnr = L.b > 0 ? (L.major - 1) / L.b : 0;
        int rem = L.b > 0 ? (L.major - 1) - mnr * L.b : 0;
        // bit of point i: (cy - y - dylo) * bw + (cx - x - dxlo)
        const int bx0 = L.x0 - x - dxlo, by0 = L.y0 - y - dylo;
        for (int i = 0; i < L.n; i++) {
            const int off = L.step * mnr;
            const int b = L.high ? (by0 + i) * bw + (bx0 + off) : (by0 + off) * bw + (bx0 + i);
            atomicOr(&bits[b >> 5], 1u << (b & 31));
            rem += L.a;
            if (rem >= L.b) {
                rem -= L.b;
                mnr++;
            }
        }
    }
#ifdef SVA_REF_PROF
    __syncthreads();
    tp[2] = clock64();
#endif
    // O over the union of all planes, column-major: columns rx0 + dxlo +
    // [0, 64 + bw - 1), rows ry0 + dylo + [0, RH + bh - 1), column stride os
    // (odd dwords).  16 bytes of slack: bytes4() may touch one dword past a
    // column, and the last rows of a 4-row group may run past RH.
    const int ouw = PT_REG_W + bw - 1, ouh = RH + bh - 1 + 4;
    const int os = ((((ouh + 3) >> 2) | 1) << 2);
    const bool staged = ouw * os <= P2_OU_BYTES - 16;
    if (staged) {
        const int ox0 = rx0 + dxlo, oy0 = ry0 + dylo;
        for (int i = t; i < ouw * ouh; i += 256) {
            const int v = i / ouw, u = i - v * ouw;
            const int gx = ox0 + u, gy = oy0 + v;
            OUT[u * os + v] =
                (gx >= 0 && gx < W && gy >= 0 && gy < H) ? other[(size_t)gy * pitch + gx] : 0;
        }
    }
    const rsrc_t ro = make_rsrc(other, (unsigned)min((size_t)0xffffffffu, (size_t)H * pitch));
    __syncthreads();
#ifdef SVA_REF_PROF
    tp[3] = clock64();
#endif

    // (a) AD plane of the region, column-major.  Thread (wave w, lane u)
    // owns column u, row groups 4 * (w + 4q), q < 6 (RH <= 88 rows = 22
    // groups); every read is issued unconditionally (addresses stay inside
    // the LDS images), only the writes are guarded.
    const int nv4 = (RH + 3) >> 2;
    auto ad_plane = [&](int ddx, int ddy, uint8_t* adt) {
        const int u = lane;
        if (staged) {
            const int ob = (u + ddx - dxlo) * os + (ddy - dylo);
            unsigned o[6], r[6];
#pragma unroll
            for (int q = 0; q < 6; q++) {
                const int v = 4 * min(wv + 4 * q, nv4 - 1);
                o[q] = bytes4(OUT, ob + v);
                r[q] = *reinterpret_cast<const unsigned*>(&RT[u * P2_RS + v]);
            }
#pragma unroll
            for (int q = 0; q < 6; q++) {
                const int v4 = wv + 4 * q;
                if (v4 < nv4)
                    *reinterpret_cast<unsigned*>(&adt[u * P2_RS + 4 * v4]) = absdiff4(o[q], r[q]);
            }
        } else {
            const unsigned gx = (unsigned)(rx0 + u + ddx);
            for (int v4 = wv; v4 < nv4; v4 += 4) {
                const int v = 4 * v4;
                const unsigned base = (unsigned)(ry0 + v + ddy) * (unsigned)pitch + gx;
                unsigned o = 0;
#pragma unroll
                for (int q = 0; q < 4; q++)
                    o |= __builtin_amdgcn_raw_buffer_load_b8(ro, base + (unsigned)q * (unsigned)pitch,
                                                             0, 0) << (8 * q);
                const unsigned r = *reinterpret_cast<const unsigned*>(&RT[u * P2_RS + v]);
                *reinterpret_cast<unsigned*>(&adt[u * P2_RS + v]) = absdiff4(o, r);
            }
        }
    };
    // (b) this wave's 8 output rows of one plane: column sums, SADs, keys
    const int r0 = 8 * wv;
    const int kh = w2 >> 2;                   // whole dwords in a 2k-row column sum
    auto sad_rows = [&](int ddx, int ddy, const uint8_t* adt) {
        const uint8_t* col = adt + lane * P2_RS;
        const unsigned* cw = reinterpret_cast<const unsigned*>(col);
        unsigned s = 0;
        for (int q = 0; q < kh; q++) s = __builtin_amdgcn_sad_u8(cw[(r0 >> 2) + q], 0u, s);
        if (w2 & 2) s = __builtin_amdgcn_sad_u8(cw[(r0 >> 2) + kh] & 0xffffu, 0u, s);
        // rows leaving (r0 .. r0+6) and entering (r0+2k .. r0+2k+6)
        const unsigned out0 = cw[r0 >> 2], out1 = cw[(r0 >> 2) + 1];
        const unsigned in0 = bytes4(col, r0 + w2), in1 = bytes4(col, r0 + w2 + 4);
        unsigned sj[8], sad[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (j > 0) {
                const unsigned ow = j - 1 < 4 ? out0 : out1, iw = j - 1 < 4 ? in0 : in1;
                const unsigned sh = 8u * (unsigned)((j - 1) & 3);
                s = s + ((iw >> sh) & 0xffu) - ((ow >> sh) & 0xffu);
            }
            sj[j] = s;
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {        // 8 independent scans: interleaved
            const unsigned P = scan64_dpp(sj[j]);
            const unsigned hi = (unsigned)__builtin_amdgcn_ds_bpermute((lane + w2 - 1) << 2, (int)P);
            sad[j] = hi - P + sj[j];
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {        // membership (on_line) + first-minimum key
            const int ia = m_ox[j] + ddx, ib = m_oy[j] + ddy;
            const int high = m_fl[j] & 1, neg = -((m_fl[j] >> 1) & 1);
            const int i = high ? ib : ia;
            const int u = high ? ia : ib;
            const int tt = (u ^ neg) - neg;              // step * u, step = +-1
            const int num = __mul24(m_a[j], i) + m_mj[j];
            const int tb = __mul24(tt, m_b[j]);
            const int in_range = (unsigned)i < (unsigned)m_n[j];
            const int on_pt = (int)(tt == 0);
            const int on_ln = (int)(tt >= 0) & (int)(tb <= num) & (int)(num < tb + m_b[j]);
            const int on = in_range & (m_b[j] == 0 ? on_pt : on_ln);
            const unsigned long long key = ((unsigned long long)sad[j] << 32) | (unsigned)i;
            best[j] = (on & (int)(key < best[j])) ? key : best[j];
        }
    };
    int wd = 0;
    unsigned m = nwords > 0 ? bits[0] : 0u;  // uniform across the workgroup
    auto next_plane = [&](int& ddx, int& ddy) -> bool {
        while (m == 0) {
            if (++wd >= nwords) return false;
            m = bits[wd];
        }
        const int b = wd * 32 + __builtin_ctz(m);
        m &= m - 1;
        ddy = dylo + b / bw;
        ddx = dxlo + b % bw;
        return true;
    };
    for (;;) {
        int ax, ay, bx, by;
        const bool pa = next_plane(ax, ay);
        if (!pa) break;
        const bool pb = next_plane(bx, by);
#ifdef SVA_REF_PROF
        nplanes += 1 + (int)pb;
#endif
        ad_plane(ax, ay, ADT[0]);
        if (pb) ad_plane(bx, by, ADT[1]);
        __syncthreads();
        sad_rows(ax, ay, ADT[0]);
        if (pb) sad_rows(bx, by, ADT[1]);
        __syncthreads();
        if (!pb) break;
    }
#ifdef SVA_REF_PROF
    tp[4] = clock64();
#endif
#pragma unroll
    for (int j = 0; j < 8; j++) {
        if (!ok[j]) continue;
        const int x = tx0 + lane, y = ty0 + r0 + j;
        const size_t p = (size_t)y * W + x;
        const int4 e = ends[p];
        int cx, cy;
        line_point(make_line(e.x, e.y, e.z, e.w), (int)(best[j] & 0xffffffffu), cx, cy);
        const double dx = (double)(cx - x), dy = (double)(cy - y);
        const int dn = (int)__builtin_sqrt(dx * dx + dy * dy);       // :89
        disp_u8[p] = (uint8_t)dn;
        if (disp_u16) disp_u16[p] = (uint16_t)dn;
        if (valid_out) valid_out[p] = 1;
    }
#ifdef SVA_REF_PROF
    tp[5] = clock64();
    if (t == 0 && (blockIdx.x % 16) == 5 && (blockIdx.y % 8) == 3)
        printf("REFPROF blk %d %d planes %d staged %d box %dx%d setup %lld bitmap %lld stage %lld planes %lld out %lld\n",
               blockIdx.x, blockIdx.y, nplanes, (int)staged, bw, bh, tp[1] - tp[0], tp[2] - tp[1],
               tp[3] - tp[2], tp[4] - tp[3], tp[5] - tp[4]);
#endif
}

__global__ void disp_to_depth_kernel(const uint8_t* __restrict__ disp, int n, double num,
                                     double pixel_size, double* __restrict__ depth) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double den = (double)disp[i] * pixel_size;   // multiply(disparity, pixelSize, .., 6)
    depth[i] = den != 0.0 ? num / den : 0.0;          // camDistance * f / pixSizeDisp
}

}  // namespace

hipError_t launch_ref_endpoints(Ctx& c, int W, int H, const sva_camera& cref,
                                const sva_camera& coth, int k, double t_near, double t_far,
                                int32_t* ends, uint8_t* valid) {
    ScopedKernelTimer t(c, "ref_endpoints");
    dim3 grid((W + 255) / 256, H);
    hipLaunchKernelGGL(ref_endpoints_kernel, grid, dim3(256), 0, c.stream, W, H, cref, coth, k,
                       t_near, t_far, (int4*)ends, valid);
    return hipGetLastError();
}

#define SVA_REF_CASE(ND)                                                                       \
    case ND:                                                                                   \
        hipLaunchKernelGGL(ref_match_kernel<ND>, grid, dim3(256), 0, c.stream, ref, other, W, H, \
                           pitch, mask, (const int4*)ends, valid_in, k, disp_u8, disp_u16,      \
                           valid_out);                                                         \
        break;

hipError_t launch_ref_match(Ctx& c, const uint8_t* ref, const uint8_t* other, int W, int H,
                            size_t pitch, const uint8_t* mask, const int32_t* ends,
                            const uint8_t* valid_in, int k, uint8_t* disp_u8,
                            uint16_t* disp_u16, uint8_t* valid_out) {
    ScopedKernelTimer t(c, "ref_match");
    const long long npx = (long long)(W - 2 * k) * (H - 2 * k);
    if (npx <= 0) return hipSuccess;
    if (k <= PT_MAXK) {   // offset-plane algorithm
        const int tw = PT_REG_W - 2 * k;
        const dim3 pg((unsigned)((W - 2 * k + tw - 1) / tw), (unsigned)((H - 2 * k + PT_ROWS - 1) / PT_ROWS));
        const dim3 pg2((unsigned)((W - 2 * k + tw - 1) / tw),
                       (unsigned)((H - 2 * k + P2_ROWS - 1) / P2_ROWS));
        // A/B switch for the previous plane kernel (tools/bench_refpath.py)
        static const bool plane_v1 = getenv("SVA_REF_PLANE_V1") != nullptr;
#define SVA_PLANE_CASE(ND)                                                                     \
    case ND:                                                                                   \
        if (plane_v1)                                                                          \
            hipLaunchKernelGGL(ref_plane_kernel<ND>, pg, dim3(256), 0, c.stream, ref, other, W, \
                               H, pitch, mask, (const int4*)ends, valid_in, k, disp_u8,         \
                               disp_u16, valid_out);                                            \
        else                                                                                   \
            hipLaunchKernelGGL(ref_plane2_kernel<ND>, pg2, dim3(256), 0, c.stream, ref, other,  \
                               W, H, pitch, mask, (const int4*)ends, valid_in, k, disp_u8,      \
                               disp_u16, valid_out);                                            \
        break;
        switch ((k + 1) / 2) {
            SVA_PLANE_CASE(1) SVA_PLANE_CASE(2) SVA_PLANE_CASE(3) SVA_PLANE_CASE(4)
            SVA_PLANE_CASE(5) SVA_PLANE_CASE(6) SVA_PLANE_CASE(7) SVA_PLANE_CASE(8)
            SVA_PLANE_CASE(9) SVA_PLANE_CASE(10) SVA_PLANE_CASE(11) SVA_PLANE_CASE(12)
            SVA_PLANE_CASE(13) SVA_PLANE_CASE(14)
            default: return hipErrorInvalidValue;
        }
#undef SVA_PLANE_CASE
        return hipGetLastError();
    }
    dim3 grid((unsigned)((npx + 3) / 4));
    switch ((k + 1) / 2) {  // ND = ceil(2k / 4)
        SVA_REF_CASE(1) SVA_REF_CASE(2) SVA_REF_CASE(3) SVA_REF_CASE(4)
        SVA_REF_CASE(5) SVA_REF_CASE(6) SVA_REF_CASE(7) SVA_REF_CASE(8)
        SVA_REF_CASE(9) SVA_REF_CASE(10) SVA_REF_CASE(11) SVA_REF_CASE(12)
        SVA_REF_CASE(13) SVA_REF_CASE(14) SVA_REF_CASE(15) SVA_REF_CASE(16)
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_disp_to_depth(Ctx& c, const uint8_t* disp, int n, double cam_distance,
                                double f, double pixel_size, double* depth) {
    ScopedKernelTimer t(c, "disp_to_depth");
    const double num = cam_distance * f;
    hipLaunchKernelGGL(disp_to_depth_kernel, dim3((n + 255) / 256), dim3(256), 0, c.stream, disp,
                       n, num, pixel_size, depth);
    return hipGetLastError();
}

}  // namespace sva
