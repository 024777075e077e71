// refpath.hip -- Mode R: the reference's own disparity path, bit-exact
// (DESIGN.md §3).
//
//   ref_endpoints_kernel  one thread per pixel, IEEE f64 in the reference's
//                         operand order (Camera.cpp:15-34,
//                         CameraStereoVision.cpp:28,60-71).  FMA contraction
//                         is off for this file so every rounding matches.
//   ref_plane3_kernel     the offset-plane algorithm (below) for k = 1..32,
//                         with a per-pixel fallback (match_pixel_wave) for
//                         tiles whose offset geometry exceeds its buffers;
//                         first-minimum argmin, then
//                         (uchar)(int)sqrt(dx^2 + dy^2)
//                         (CameraStereoVision.cpp:85-89).  WIDE instances
//                         (W or H >= 4096: a line may hold 4,096 candidates
//                         or more) keep 64-bit (SAD, i) first-minimum keys.
//   ref_pixel_kernel      k > 32 (the reference bounds k only by the image,
//                         CameraStereoVision.cpp:49-51): one wave per pixel.
#pragma clang fp contract(off)

#include <cstdlib>
#include <type_traits>

#include "sva_device.h"
#include "sva_internal.h"
#include "sva_tuning.h"

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

// Per-pixel wave algorithm: one wave per reference pixel, one lane per
// Bresenham candidate (functions.cpp:253-321 in closed form), the 2k x 2k SAD
// with v_sad_u8 (4 |a-b| per lane-op) on v_alignbyte-realigned rows, and the
// first minimum as a wave-wide u64 min over (SAD << 32 | i).  The per-tile
// fallback of ref_plane3_kernel.
// sad_row over a row of any (even) length: 64-byte chunks, then the rest
// (k > 32, where the 2k-byte row outgrows one sad_row<ND> instance).
template <int N>
__device__ __forceinline__ unsigned sad_tail(const uint8_t* a, const uint8_t* b, unsigned lastmask,
                                             int nbytes, unsigned acc) {
    if constexpr (N > 16) {
        return acc;
    } else {
        if ((nbytes + 3) / 4 == N) return sad_row<N>(a, b, lastmask, nbytes, acc);
        return sad_tail<N + 1>(a, b, lastmask, nbytes, acc);
    }
}
__device__ __forceinline__ unsigned sad_span(const uint8_t* a, const uint8_t* b, int nbytes,
                                             unsigned acc) {
    int off = 0;
    for (; off + 64 <= nbytes; off += 64) acc = sad_row<16>(a + off, b + off, 0xffffffffu, 64, acc);
    const int rem = nbytes - off;
    if (rem > 0) acc = sad_tail<1>(a + off, b + off, (rem & 3) ? 0xffffu : 0xffffffffu, rem, acc);
    return acc;
}

// KEY: the type of the split plane loop's per-pixel first-minimum keys
// (u32 (SAD << 12 | i), or u64 (SAD << 32 | i) for WIDE frames).  ND = 0:
// rows of any length (sad_span, k > 32).
template <int ND, class KEY = unsigned>
__device__ __forceinline__ void match_pixel_wave(const uint8_t* __restrict__ ref,
                                                 const uint8_t* __restrict__ other, int W,
                                                 size_t pitch, int x, int y, const int4 e, int k,
                                                 uint8_t* __restrict__ disp_u8,
                                                 uint16_t* __restrict__ disp_u16,
                                                 uint8_t* __restrict__ valid_out,
                                                 KEY* __restrict__ keys = nullptr) {
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
            for (int v = 0; v < nbytes; v++) {
                if constexpr (ND == 0)
                    acc = sad_span(sel + (size_t)v * pitch, kern + (size_t)v * pitch, nbytes, acc);
                else
                    acc = sad_row<ND>(sel + (size_t)v * pitch, kern + (size_t)v * pitch, lastmask,
                                      nbytes, acc);
            }
            key = ((unsigned long long)acc << 32) | (unsigned)i;
        }
        key = wave_min_u64(key);                                      // :85 first min
        best = key < best ? key : best;
    }
    if (lane == 0 && keys) {
        // the split plane loop's first-minimum key (SAD << 12 | i, or the
        // full (SAD, i) pair for WIDE frames), finished by ref_finalize_kernel
        if constexpr (sizeof(KEY) == 8)
            atomicMin(&keys[p], (KEY)best);
        else
            atomicMin(&keys[p], ((unsigned)(best >> 32) << 12) | (unsigned)(best & 0xfffu));
    } else if (lane == 0) {
        int cx, cy;
        line_point(L, (int)(best & 0xffffffffu), cx, cy);
        const double dx = (double)(cx - x), dy = (double)(cy - y);
        const int dn = (int)__builtin_sqrt(dx * dx + dy * dy);       // :89
        disp_u8[p] = (uint8_t)dn;
        if (disp_u16) disp_u16[p] = (uint16_t)dn;
        if (valid_out) valid_out[p] = 1;
    }
}

// ---- offset-plane algorithm (same results, far less work) -------------------
//
// For a fixed offset delta, AD(q) = |O(q + delta) - R(q)| is shared by every
// reference pixel, and SAD(p, delta) is the 2k x 2k box sum of AD at p.  A
// workgroup owns a tile of reference pixels and
//   1. collects the union of its pixels' candidate offsets c_i - p in an LDS
//      bitmap over their bounding box (neighbouring pixels' offsets nearly
//      coincide, so this is a thin band even for diagonal pairs);
//   2. per offset plane forms the box sums of the tile and, for each pixel,
//      tests whether delta is on ITS Bresenham line -- candidate i has minor
//      offset floor((a*i + major - 1) / b) -- keeping the minimum key over
//      (SAD, i): the reference's first minimum (CameraStereoVision.cpp:85)
//      whatever order the planes are visited in.
// A tile whose offset geometry exceeds the kernel's buffers falls back to
// match_pixel_wave.
// largest k of the plane kernel: the ABI maximum.  Region 63 + 2k <= 127
// columns (two per lane) and SAD <= (2k)^2 * 255 < 2^20 for the u32 key.
constexpr int PT_MAXK = 32;

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

// The same scan on N pairs of values, stage by stage: each DPP add's source
// was written 2N instructions earlier, so no s_nop separates dependent adds.
template <int N>
__device__ __forceinline__ void scan64_dpp_n(unsigned (&a)[N], unsigned (&b)[N]) {
    auto stage = [&](auto ctl, int rmask) {
        (void)rmask;
#pragma unroll
        for (int j = 0; j < N; j++) {
            a[j] += (unsigned)__builtin_amdgcn_update_dpp(0, (int)a[j], decltype(ctl)::value,
                                                          decltype(ctl)::value >= 0x142
                                                              ? (decltype(ctl)::value == 0x142 ? 0xa : 0xc)
                                                              : 0xf,
                                                          0xf, false);
            b[j] += (unsigned)__builtin_amdgcn_update_dpp(0, (int)b[j], decltype(ctl)::value,
                                                          decltype(ctl)::value >= 0x142
                                                              ? (decltype(ctl)::value == 0x142 ? 0xa : 0xc)
                                                              : 0xf,
                                                          0xf, false);
        }
    };
    stage(std::integral_constant<int, 0x111>{}, 0xf);   // row_shr:1
    stage(std::integral_constant<int, 0x112>{}, 0xf);   // row_shr:2
    stage(std::integral_constant<int, 0x114>{}, 0xf);   // row_shr:4
    stage(std::integral_constant<int, 0x118>{}, 0xf);   // row_shr:8
    stage(std::integral_constant<int, 0x142>{}, 0xa);   // row_bcast:15 into rows 1, 3
    stage(std::integral_constant<int, 0x143>{}, 0xc);   // row_bcast:31 into rows 2, 3
}

// ---- offset-plane algorithm (v3) ---------------------------------------------
// The round-1 kernel (v2) spent most lanes on the window
// halo: a wave covered the 64 region columns of a (64 - 2k)-pixel tile, so at
// k = 20 only 24 of 64 lanes owned an output.  v3 gives every lane an output
// column:
//   * Tile = 64 output columns x 32 rows (wave w: rows 8w..8w+7); the region
//     is 63 + 2k columns.  Lane u owns region columns u and u + 64 (the
//     second is real for u < 2k - 1).  The 2k-column box sum reads the
//     inclusive scans of both through ONE ds_bpermute: source lanes below
//     2k - 1 hold the second scan plus the first one's total, the others the
//     first scan.
//   * No AD plane in LDS: the 2k-row column sums are v_sad_u8 of staged O
//     dwords (column-major, 4 rows per dword, one wave-uniform v_alignbyte)
//     against the lane's R dwords, which stay in registers for the whole
//     tile; rows r0+1..r0+7 follow from v_sad_u8 of the leaving and
//     entering rows (partial dwords by byte select).  Nothing is written to LDS per plane, so the four waves
//     run their plane loops with no barrier.
//   * Membership is an interval test.  Planes are visited with the tile's
//     dominant major axis innermost (row-major bitmap when most lines are
//     Low, column-major when High).  For one outer offset the inner offsets
//     on a pixel's line form one interval -- of length <= 1 when the pixel's
//     own major axis is the outer one -- recomputed only when the outer
//     offset changes.  Per plane the test is (d_in - lo) < len, and the
//     first-minimum key is the u32 (SAD << 12 | i): SAD < 2^20 for k <= 32,
//     i < 4096 when W, H < 4096.  Larger frames take the WIDE instance, whose
//     u64 key (SAD << 32 | i) holds any i (VERDICT r05 missing #3).
constexpr int P3_ROWS = 32;                          // 4 waves x 8 rows
constexpr int P3_OU_BYTES = tune::kPlaneOuKB * 1024;  // staged O chunk
constexpr int P3_WORDS = tune::kPlaneWords;            // offset bitmap per pass: 32K bits
constexpr int P3_MAX_OUT = 1024;                     // outer offsets per pass

// Interval [lo, lo + len) of inner offsets d_in on a pixel's line at outer
// offset d_out; the candidate index there is i = d_in + ib0.
//   po = o_major | o_minor << 16: the pixel minus its line start along the
//        line's major / minor axis (signed 16-bit halves);
//   pa = a | b << 16, pn = n | major << 16 (Line fields; n = 0: no pixel);
//   mi: the line's major axis is the inner axis; neg: minor step is -1.
// Candidate i of a line has minor offset floor((a*i + major - 1) / b)
// (make_line's closed form of functions.cpp:253-321).
__device__ __forceinline__ void line_interval(int po, int pa, int pn, bool mi, bool neg,
                                              int d_out, int& lo, int& len, int& ib0) {
    const int o_major = (int)(short)(po & 0xffff), o_minor = po >> 16;
    const int a = pa & 0xffff, b = (int)((unsigned)pa >> 16);
    const int n = pn & 0xffff, mj = (int)((unsigned)pn >> 16) - 1;
    if (mi) {
        // i = o_major + d_in, and floor((a*i + mj) / b) must equal the
        // candidate's minor offset tt = step * (o_minor + d_out)
        const int u = o_minor + d_out;
        const int tt = neg ? -u : u;
        int ilo = 0, ihi = 0;
        if (tt >= 0) {
            if (a == 0) {
                ihi = tt == 0 ? n : 0;
            } else {
                // i in [ceil((tt*b - mj)/a), ceil((tt*b + b - mj)/a)); the
                // lower bound at tt = 0 is <= 0, i.e. 0 after clamping
                // tune::kPlaneNoHoistDiv: an opaque copy keeps the compiler
                // from hoisting each pixel's reciprocal of a out of the outer
                // offset loop (no spill at k = 20, but the division is then
                // redone per outer offset: +9 % on diagonal pairs)
                unsigned A = (unsigned)a;
                if constexpr (tune::kPlaneNoHoistDiv != 0) asm volatile("" : "+v"(A));
                ilo = tt == 0 ? 0 : (int)(((unsigned)(tt * b - mj) + A - 1u) / A);
                ihi = (int)(((unsigned)(tt * b + b - mj) + A - 1u) / A);
            }
        }
        ihi = ihi > n ? n : ihi;
        len = ihi > ilo ? ihi - ilo : 0;
        lo = ilo - o_major;
        ib0 = o_major;
    } else {
        // i = o_major + d_out is fixed; one inner offset is on the line
        const int i = o_major + d_out;
        const bool in = (unsigned)i < (unsigned)n;
        const int t = (b > 0 && in) ? (int)((unsigned)(a * i + mj) / (unsigned)b) : 0;
        lo = (neg ? -t : t) - o_minor;
        len = in ? 1 : 0;
        ib0 = i - lo;
    }
}

template <int K, bool WIDE>
__global__ __launch_bounds__(256, tune::kPlaneMinBlocks) void ref_plane3_kernel(
    const uint8_t* __restrict__ ref, const uint8_t* __restrict__ other, int W, int H, size_t pitch,
    const uint8_t* __restrict__ mask, const int4* __restrict__ ends,
    const uint8_t* __restrict__ valid_in, uint8_t* __restrict__ disp_u8,
    uint16_t* __restrict__ disp_u16, uint8_t* __restrict__ valid_out,
    void* __restrict__ keys_) {
    // first-minimum keys: u32 (SAD << 12 | i) while every line holds < 4096
    // candidates, else u64 (SAD << 32 | i)
    using Key = typename std::conditional<WIDE, unsigned long long, unsigned>::type;
    constexpr Key KNONE = (Key)~(Key)0;
    Key* keys = (Key*)keys_;
    // Grid (shares, tiles x, tiles y): every tile is split over gridDim.x
    // workgroups (one share of its offsets each, adjacent in dispatch order)
    // whose per-pixel first-minimum keys meet in keys[] by atomicMin
    // (ref_finalize_kernel turns them into the disparity).  The key order is
    // the reference's first minimum whatever the split
    // (CameraStereoVision.cpp:85).  gridDim.x = 1: no split, no keys.
    constexpr int W2 = 2 * K;
    constexpr int ND = (W2 + 3) / 4;          // dwords holding a 2k-row column
    constexpr bool ODD = (W2 & 2) != 0;       // the 2k rows end mid-dword
    constexpr int ND2 = (W2 + 6) / 4 + 1;     // dwords holding rows r0 .. r0 + 2k + 6
    constexpr int RW = 63 + W2;
    // R column stride: rows r0 + 4*ND2 of the lowest wave, an odd dword count
    // (each lane reads its own column: conflict-free)
    constexpr int RS = (((24 + 4 * ND2) / 4) | 1) * 4;
    constexpr int RS4 = RS / 4;
    static_assert(24 + 4 * ND2 <= RS, "R column stride too small");
    static_assert(ND2 >= ND + 2, "entering rows");
    static_assert(K >= 1 && K <= PT_MAXK, "k outside the ABI range");
    static_assert(4 * K * K * 255 < (1 << 20), "SAD must fit the 20-bit key field");
    __shared__ __attribute__((aligned(16))) uint8_t RT[RW * RS];
    __shared__ unsigned bits[P3_WORDS];
    __shared__ __attribute__((aligned(16))) uint8_t OUT[P3_OU_BYTES];
    __shared__ short omn[P3_MAX_OUT], omx[P3_MAX_OUT];
    __shared__ int box[6];   // dx_lo, dx_hi, dy_lo, dy_hi, #High pixels, #pixels
    __shared__ unsigned short uniq[P3_ROWS * 64];   // pixels with a distinct relative line
    __shared__ int nuniq;
    // tune::kPlanePoLds: each thread's eight line offsets (po below) in LDS,
    // [row][thread], read back once per outer offset instead of held in
    // registers -- where that still leaves kPlaneMinBlocks workgroups per CU
    // (the arrays above plus 256 B of alignment slack)
    constexpr size_t LDS_BASE = sizeof(RT) + sizeof(bits) + sizeof(OUT) + sizeof(omn) + sizeof(omx) +
                                sizeof(box) + sizeof(uniq) + sizeof(nuniq);
    // LDS per CU: 160 KB on gfx950, the only target this file is built for
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "refpath.hip sizes its LDS for gfx950 (160 KB per CU)"
#endif
    constexpr size_t LDS_PER_CU = 160 * 1024;
    constexpr bool POLDS = tune::kPlanePoLds != 0 &&
                           LDS_BASE + 8 * 256 * sizeof(int) + 256 <= LDS_PER_CU / tune::kPlaneMinBlocks;
    __shared__ int po_lds[POLDS ? 8 * 256 : 1];
    const int t = threadIdx.x, lane = t & 63;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
    // (a share taken from a per-tile condition instead -- whole tiles plus a
    // split band -- cost 4-5 VGPRs and 20 B of scratch at k = 20)
    const int share = (int)blockIdx.x, nshare = (int)gridDim.x;
    if (nshare == 1) keys = nullptr;     // a whole tile writes its pixels directly
    const int tx0 = K + (int)blockIdx.y * 64, ty0 = K + (int)blockIdx.z * P3_ROWS;
    const int rx0 = tx0 - K, ry0 = ty0 - K;   // region origin (image coords)
    const int r0 = 8 * wv;
    if (t < 6) box[t] = t >= 4 ? 0 : ((t & 1) ? -0x7fffffff : 0x7fffffff);
    // R region, column-major; rows up to the stride are staged as well (read
    // into registers below, masked out of every sum)
    // (eight byte loads in flight per thread, from clamped in-image
    // addresses, then the eight LDS stores: a branch per byte had made every
    // load its own load-wait-store round trip)
    for (int i0 = 0; i0 < RW * RS; i0 += 8 * 256) {
        unsigned bv[8];
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const int i = i0 + q * 256 + t;
            const int v = i / RW, u = i - v * RW;
            bv[q] = ref[(size_t)min(ry0 + v, H - 1) * pitch + min(rx0 + u, W - 1)];
        }
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const int i = i0 + q * 256 + t;
            const int v = i / RW, u = i - v * RW;
            if (i < RW * RS) RT[u * RS + v] = (rx0 + u < W && ry0 + v < H) ? (uint8_t)bv[q] : 0;
        }
    }
    // this thread's pixels: column tx0 + lane, rows ty0 + r0 + j
    int ox[8], oy[8], pa[8], pn[8];
    bool high[8], neg[8];
    int4 E[8];
    {
        unsigned vin[8], mk[8];
        const int xc = min(tx0 + lane, W - 1);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const size_t p = (size_t)min(ty0 + r0 + j, H - 1) * W + xc;
            vin[j] = valid_in[p];
            mk[j] = mask ? mask[p] : 1u;
            E[j] = ends[p];
        }
        int bx0 = 0x7fffffff, bx1 = -0x7fffffff, by0 = 0x7fffffff, by1 = -0x7fffffff;
        int nh = 0, nok = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int x = tx0 + lane, y = ty0 + r0 + j;
            const bool ok = x < W - K && y < H - K && vin[j] != 0 && mk[j] != 0;
            const Line L = make_line(E[j].x, E[j].y, E[j].z, E[j].w);
            high[j] = L.high != 0;
            neg[j] = L.step < 0;
            ox[j] = x - L.x0;
            oy[j] = y - L.y0;
            pa[j] = L.a | (L.b << 16);
            pn[j] = (ok ? L.n : 0) | (L.major << 16);
            if (ok) {
                bx0 = min(bx0, min(E[j].x, E[j].z) - x);
                bx1 = max(bx1, max(E[j].x, E[j].z) - x);
                by0 = min(by0, min(E[j].y, E[j].w) - y);
                by1 = max(by1, max(E[j].y, E[j].w) - y);
                nh += L.high ? 1 : 0;
                nok++;
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {   // wave reductions, then one atomic each
            bx0 = min(bx0, __shfl_xor(bx0, off, 64));
            bx1 = max(bx1, __shfl_xor(bx1, off, 64));
            by0 = min(by0, __shfl_xor(by0, off, 64));
            by1 = max(by1, __shfl_xor(by1, off, 64));
            nh += __shfl_xor(nh, off, 64);
            nok += __shfl_xor(nok, off, 64);
        }
        if (lane == 0) {
            atomicMin(&box[0], bx0);
            atomicMax(&box[1], bx1);
            atomicMin(&box[2], by0);
            atomicMax(&box[3], by1);
            atomicAdd(&box[4], nh);
            atomicAdd(&box[5], nok);
        }
    }
    __syncthreads();
    if (box[1] < box[0]) return;             // no valid pixel in this tile
    const int dxlo = box[0], dylo = box[2];
    const int bw = box[1] - box[0] + 1, bh = box[3] - box[2] + 1;
    const bool cm = 2 * box[4] > box[5];     // inner axis y: High lines dominate
    const int n_in = cm ? bh : bw, n_out = cm ? bw : bh;
    const int wpo = (n_in + 31) >> 5;        // bitmap words per outer offset
    // outer offsets per bitmap pass: one pass at 1080p, ~3 for a 4K diagonal
    const int opp = min(P3_WORDS / wpo, P3_MAX_OUT);
    // bytes of the O rectangle staged for span_out outer x span_in inner offsets
    auto stage_bytes = [&](int span_out, int span_in) {
        const int cw = RW + (cm ? span_out : span_in) - 1;
        const int ch = 24 + (cm ? span_in : span_out) - 1 + 4 * (ND2 + 1);
        return cw * ((((ch + 3) >> 2) | 1) << 2);
    };
    if (opp < 1 || stage_bytes(1, 1) > P3_OU_BYTES) {
        // one outer offset's bitmap row or O column does not fit: per-pixel
        // waves for this tile
        if (share != 0) return;           // one share does the whole tile
        for (int pi = wv; pi < 64 * P3_ROWS; pi += 4) {
            const int x = tx0 + (pi & 63), y = ty0 + (pi >> 6);
            if (x >= W - K || y >= H - K) continue;
            const size_t p = (size_t)y * W + x;
            if (!valid_in[p] || (mask && mask[p] == 0)) continue;
            match_pixel_wave<ND, Key>(ref, other, W, pitch, x, y, ends[p], K, disp_u8, disp_u16,
                                      valid_out, keys);
        }
        return;
    }
    if (t == 0) nuniq = 0;
    __syncthreads();
    // Bresenham is translation-invariant: pixels whose endpoints, relative
    // to themselves, match the left neighbour's or the previous row's have the
    // same offset set.  Only the first of each such chain enters the list.
    {
        int4 prev = make_int4(0, 0, 0, 0);
        bool prev_ok = false;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int x = tx0 + lane, y = ty0 + r0 + j;
            const bool ok = (pn[j] & 0xffff) != 0;
            // the endpoints again from global memory (L2-hot): E[] need not
            // stay live across the tile's box reduction and barrier
            const int4 e = ends[(size_t)min(y, H - 1) * W + min(x, W - 1)];
            const int4 rel = make_int4(e.x - x, e.y - y, e.z - x, e.w - y);
            const int lx = __shfl_up(rel.x, 1, 64), ly = __shfl_up(rel.y, 1, 64);
            const int lz = __shfl_up(rel.z, 1, 64), lw = __shfl_up(rel.w, 1, 64);
            const int lok = __shfl_up((int)ok, 1, 64);
            const bool same_left = lane > 0 && lok && lx == rel.x && ly == rel.y && lz == rel.z &&
                                   lw == rel.w;
            const bool same_up = prev_ok && prev.x == rel.x && prev.y == rel.y &&
                                 prev.z == rel.z && prev.w == rel.w;
            if (ok && !same_left && !same_up)
                uniq[atomicAdd(&nuniq, 1)] = (unsigned short)((r0 + j) * 64 + lane);
            prev = rel;
            prev_ok = ok;
        }
    }
    __syncthreads();
    // widest inner window of a single outer offset (uniform)
    int iwmax = 1;
    for (int step = 1 << 12; step; step >>= 1)
        if (iwmax + step <= n_in && stage_bytes(1, iwmax + step) <= P3_OU_BYTES) iwmax += step;

    // R dwords of this lane's two region columns, rows r0 .. r0 + 4*ND2 - 1
    const int ca = lane, cb = min(lane + 64, RW - 1);
    unsigned RA[ND2], RB[ND2];
    {
        const unsigned* RT32 = reinterpret_cast<const unsigned*>(RT);
#pragma unroll
        for (int q = 0; q < ND2; q++) {
            RA[q] = RT32[ca * RS4 + (r0 >> 2) + q];
            RB[q] = RT32[cb * RS4 + (r0 >> 2) + q];
        }
    }
    // rows r0 + 2k .. r0 + 2k + 7 (the rows entering the window)
    auto entering = [](const unsigned (&X)[ND2], int e) -> unsigned {
        return ODD ? __builtin_amdgcn_alignbyte(X[ND + e], X[ND - 1 + e], 2) : X[ND + e];
    };
    const unsigned reA0 = entering(RA, 0), reA1 = entering(RA, 1);
    const unsigned reB0 = entering(RB, 0), reB1 = entering(RB, 1);
    // column sums of |O - R| over rows [r0 + j, r0 + j + 2k), j < 8, for one
    // region column whose O dwords start at byte ob of OUT
    auto colsums = [&](const unsigned (&R)[ND2], unsigned re0, unsigned re1, int ob,
                       unsigned (&cs)[8]) {
        const unsigned* w = reinterpret_cast<const unsigned*>(OUT) + (ob >> 2);
        const unsigned sh = (unsigned)(ob & 3);
        unsigned raw[ND2 + 1], O[ND2];
#pragma unroll
        for (int q = 0; q <= ND2; q++) raw[q] = w[q];
#pragma unroll
        for (int q = 0; q < ND2; q++) O[q] = __builtin_amdgcn_alignbyte(raw[q + 1], raw[q], sh);
        // |o - r| summed over the first j bytes only: the other bytes of o are
        // replaced by r's (one v_perm) so they add 0 -- cheaper than masking
        // both operands.  Selector: bytes < j from o (4..7), the rest from r.
        auto sad_first = [](unsigned o, unsigned r, int j, unsigned acc) -> unsigned {
            const unsigned sel = j == 1 ? 0x03020104u : j == 2 ? 0x03020504u : 0x03060504u;
            return __builtin_amdgcn_sad_u8(__builtin_amdgcn_perm(o, r, sel), r, acc);
        };
        unsigned s0 = 0;
#pragma unroll
        for (int q = 0; q < ND; q++) {
            if (ODD && q == ND - 1) s0 = sad_first(O[q], R[q], 2, s0);
            else s0 = __builtin_amdgcn_sad_u8(O[q], R[q], s0);
        }
        const unsigned oe0 = entering(O, 0), oe1 = entering(O, 1);
        // X_j = sum of the j rows leaving, E_j = s0 + sum of the j rows entering
        const unsigned x4 = __builtin_amdgcn_sad_u8(O[0], R[0], 0u);
        const unsigned e4 = __builtin_amdgcn_sad_u8(oe0, re0, s0);
        cs[0] = s0;
        cs[4] = e4 - x4;
#pragma unroll
        for (int j = 1; j < 4; j++) {
            cs[j] = sad_first(oe0, re0, j, s0) - sad_first(O[0], R[0], j, 0u);
            cs[4 + j] = sad_first(oe1, re1, j, e4) - sad_first(O[1], R[1], j, x4);
        }
    };

    Key best[8];
    int lo[8], len[8], ib0[8];
    unsigned lb[8];            // kPlaneStageMajor: len and lo + ib0 in one register
#pragma unroll
    for (int j = 0; j < 8; j++) {
        best[j] = KNONE;
        lo[j] = len[j] = ib0[j] = 0;
    }
    // line offsets along each line's own axes (see line_interval)
    int po[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const int omaj = high[j] ? oy[j] : ox[j], omin = high[j] ? ox[j] : oy[j];
        po[j] = (omaj & 0xffff) | (omin << 16);
        if constexpr (POLDS) po_lds[j * 256 + t] = po[j];
    }
    const int in_lo = cm ? dylo : dxlo, out_lo = cm ? dxlo : dylo;
    const int src = ((lane + W2 - 1) & 63) << 2;
    const int bstride = wpo * 32;
    // this workgroup's share of the INNER offsets (all of them unsplit): the
    // runs along the inner axis are the long ones, so every share gets a
    // piece of every outer offset's run -- an outer-offset split left the
    // thin bands of Low / High pairs with one or two uneven outer offsets
    // per share
    // (tune::kPlaneSplitInner: 1 inner, 0 outer, 2 per tile -- inner for the
    // thin offset bands of Low / High pairs, outer for the diagonal bands,
    // whose inner runs are short and shift with the outer offset)
    const bool SPLIT_IN = tune::kPlaneSplitInner == 2 ? 4 * min(bw, bh) < max(bw, bh)
                                                       : tune::kPlaneSplitInner != 0;
    const int nsplit = SPLIT_IN ? n_in : n_out;
    const int s_lo = (int)((long long)nsplit * share / nshare);
    const int s_hi = (int)((long long)nsplit * (share + 1) / nshare);
    const int i_lo = SPLIT_IN ? s_lo : 0;
    const unsigned i_len = (unsigned)(SPLIT_IN ? s_hi - s_lo : n_in);
    const int o_lo = SPLIT_IN ? 0 : s_lo, o_hi = SPLIT_IN ? n_out : s_hi;
    for (int oa = o_lo; oa < o_hi; oa += opp) {
        const int nl = min(o_hi - oa, opp);     // outer offsets of this bitmap pass
        __syncthreads();                     // the previous pass's planes are done
        for (int i = t; i < wpo * nl; i += 256) bits[i] = 0;
        __syncthreads();
        // one thread per distinct line, walking it incrementally (the minor
        // offset of point i advances by at most one per step since a <= b);
        // consecutive points mostly fall in one bitmap word (runs along the
        // major axis), so they are gathered in a mask: one atomic per word
        for (int q = t; q < nuniq; q += 256) {
            const int pl = uniq[q], x = tx0 + (pl & 63), y = ty0 + (pl >> 6);
            const int4 e = ends[(size_t)y * W + x];
            const Line L = make_line(e.x, e.y, e.z, e.w);
            const int bx0 = L.x0 - x - dxlo, by0 = L.y0 - y - dylo;
            // only the points whose major-axis coordinate (b0 + i) can lie in
            // this pass's outer range or this share's inner range, whichever
            // axis is the line's major one: a share or a later pass no longer
            // re-walks the whole line (tune::kPlaneWalkRange)
            int i0 = 0, i1 = L.n;
            if constexpr (tune::kPlaneWalkRange != 0) {
                const bool outer_major = cm != (L.high != 0);   // outer axis x (cm) is Low's major
                const int b0 = L.high ? by0 : bx0;
                const int lo = outer_major ? oa : i_lo;
                const int len = outer_major ? nl : (int)i_len;
                i0 = max(0, lo - b0);
                i1 = min(L.n, lo + len - b0);
            }
            // minor offset of point i: floor((a i + major - 1) / b), then
            // advanced incrementally (it grows by at most one per step, a <= b)
            const int num0 = L.a * i0 + L.major - 1;
            int mnr = L.b > 0 ? num0 / L.b : 0;
            int rem = L.b > 0 ? num0 - mnr * L.b : 0;
            int cur = -1;
            unsigned msk = 0;
            for (int i = i0; i < i1; i++) {
                const int off = L.step * mnr;
                const int rx = L.high ? bx0 + off : bx0 + i;
                const int ry = L.high ? by0 + i : by0 + off;
                const int ro = (cm ? rx : ry) - oa;
                if ((unsigned)ro < (unsigned)nl && (unsigned)((cm ? ry : rx) - i_lo) < i_len) {
                    const int b = ro * bstride + (cm ? ry : rx);
                    if ((b >> 5) != cur) {
                        if (msk) atomicOr(&bits[cur], msk);
                        cur = b >> 5;
                        msk = 0;
                    }
                    msk |= 1u << (b & 31);
                }
                rem += L.a;
                if (rem >= L.b) {
                    rem -= L.b;
                    mnr++;
                }
            }
            if (msk) atomicOr(&bits[cur], msk);
        }
        __syncthreads();
        // Per outer offset, the first and last inner offset with a plane.  The
        // planes are staged in chunks of consecutive outer offsets whose O
        // rectangle fits OUT (one chunk for Low/High pairs at 1080p; diagonal
        // pairs, whose offset box is a thin diagonal band, take a few); an
        // outer offset whose inner span alone does not fit is split into
        // windows.
        for (int o = t; o < nl; o += 256) {
            int mn = 0x7fff, mx = -1;
            for (int wc = 0; wc < wpo; wc++) {
                const unsigned m = bits[o * wpo + wc];
                if (m) {
                    mn = min(mn, wc * 32 + __builtin_ctz(m));
                    mx = max(mx, wc * 32 + 31 - __builtin_clz(m));
                }
            }
            omn[o] = (short)mn;
            omx[o] = (short)mx;
        }
        __syncthreads();
        for (int o0 = 0, wst = -1;;) {           // wst >= 0: outer offset o0 continues there
            if (wst < 0) {
                while (o0 < nl && __builtin_amdgcn_readfirstlane(omn[o0] > omx[o0])) o0++;
                if (o0 >= nl) break;
            }
            int o1 = o0 + 1;
            int ilo = __builtin_amdgcn_readfirstlane(omn[o0]);
            int ihi = __builtin_amdgcn_readfirstlane(omx[o0]);
            if (wst >= 0 || ihi - ilo + 1 > iwmax) {
                // one outer offset, inner window [ilo, ihi]
                const int end = ihi;
                ilo = wst >= 0 ? wst : ilo;
                ihi = min(end, ilo + iwmax - 1);
                wst = ihi < end ? ihi + 1 : -1;
            } else {
                // grow the chunk [o0, o1) while its O rectangle fits
                for (; o1 < nl; o1++) {
                    const int a = __builtin_amdgcn_readfirstlane(omn[o1]);
                    const int b = __builtin_amdgcn_readfirstlane(omx[o1]);
                    const int gl = a <= b ? min(ilo, a) : ilo, gh = a <= b ? max(ihi, b) : ihi;
                    if (stage_bytes(o1 + 1 - o0, gh - gl + 1) > P3_OU_BYTES) break;
                    ilo = gl;
                    ihi = gh;
                }
            }
            // O over the chunk: columns rx0 + dxb + [0, ouw), rows ry0 + dyb +
            // [0, ouh) (every dword a plane reads), column stride os (odd dwords)
            const int dxb = cm ? out_lo + oa + o0 : in_lo + ilo;
            const int dyb = cm ? in_lo + ilo : out_lo + oa + o0;
            const int ouw = RW + (cm ? o1 - o0 : ihi - ilo + 1) - 1;
            const int ouh = 24 + (cm ? ihi - ilo + 1 : o1 - o0) - 1 + 4 * (ND2 + 1);
            const int os = ((((ouh + 3) >> 2) | 1) << 2);
            __syncthreads();                     // the previous chunk's planes are done
            {
                const int ox0 = rx0 + dxb, oy0 = ry0 + dyb;
                for (int i = t; i < ouw * ouh; i += 256) {
                    const int v = i / ouw, u = i - v * ouw;
                    const int gx = ox0 + u, gy = oy0 + v;
                    OUT[u * os + v] = (gx >= 0 && gx < W && gy >= 0 && gy < H)
                                          ? other[(size_t)gy * pitch + gx] : 0;
                }
            }
            __syncthreads();
            for (int ot = o0; ot < o1; ot++) {
                const int d_out = out_lo + oa + ot;
                const int wlo = max(ilo, __builtin_amdgcn_readfirstlane(omn[ot]));
                const int whi = min(ihi, __builtin_amdgcn_readfirstlane(omx[ot]));
                if (wlo > whi) continue;
                if constexpr (POLDS) {
                    // reload the line offsets here (the empty asm keeps the
                    // compiler from hoisting the reads out of the loop)
                    asm volatile("" ::: "memory");
#pragma unroll
                    for (int j = 0; j < 8; j++) po[j] = po_lds[j * 256 + t];
                }
#pragma unroll
                for (int j = 0; j < 8; j++)
                    line_interval(po[j], pa[j], pn[j], high[j] == cm, neg[j], d_out, lo[j],
                                  len[j], ib0[j]);
#pragma unroll
                for (int j = 0; j < 8; j++)   // len | first candidate index << 16 (both < 65536)
                    lb[j] = (unsigned)len[j] | ((unsigned)(lo[j] + ib0[j]) << 16);
                for (int wc = wlo >> 5; wc <= (whi >> 5); wc++) {
                    unsigned m =
                        (unsigned)__builtin_amdgcn_readfirstlane((int)bits[ot * wpo + wc]);
                    if (wc == (wlo >> 5)) m &= ~0u << (wlo & 31);            // window edges
                    if (wc == (whi >> 5)) m &= ~0u >> (31 - (whi & 31));
                    while (m) {
                        const int d_in = in_lo + wc * 32 + __builtin_ctz(m);
                        m &= m - 1;
                        const int ddx = cm ? d_out : d_in, ddy = cm ? d_in : d_out;
                        const int ob = (ddx - dxb) * os + (ddy - dyb) + r0;
                        unsigned csA[8], csB[8];
                        colsums(RA, reA0, reA1, ob + ca * os, csA);
                        colsums(RB, reB0, reB1, ob + cb * os, csB);
                        if constexpr (tune::kPlaneStageMajor != 0) {
                            // the 16 scans stage by stage (independent DPP adds
                            // between dependent ones: no s_nop), all 8
                            // ds_bpermute issued before the first is consumed,
                            // and a branch-free first-minimum update
                            // rows in groups of G: 2G DPP chains in flight, and
                            // fewer live registers than all 8 rows at once
                            constexpr int G = tune::kPlaneStageMajor > 0 ? tune::kPlaneStageMajor : 1;
#pragma unroll
                            for (int j0 = 0; j0 < 8; j0 += G) {
                                unsigned Pa[G], V[G];
#pragma unroll
                                for (int j = 0; j < G; j++) { Pa[j] = csA[j0 + j]; V[j] = csB[j0 + j]; }
                                scan64_dpp_n<G>(Pa, V);
#pragma unroll
                                for (int j = 0; j < G; j++) {
                                    const unsigned ta = (unsigned)__builtin_amdgcn_readlane((int)Pa[j], 63);
                                    V[j] = lane < W2 - 1 ? V[j] + ta : Pa[j];
                                    V[j] = (unsigned)__builtin_amdgcn_ds_bpermute(src, (int)V[j]);
                                    Pa[j] -= csA[j0 + j];          // exclusive prefix
                                }
#pragma unroll
                                for (int j = 0; j < G; j++) {
                                    const unsigned sad = V[j] - Pa[j];
                                    const unsigned tt = (unsigned)(d_in - lo[j0 + j]);
                                    const unsigned x = lb[j0 + j];
                                    const Key key = WIDE ? ((Key)sad << 32) | (Key)(tt + (x >> 16))
                                                         : (Key)((sad << 12) | (tt + (x >> 16)));
                                    const bool on = tt < (x & 0xffffu);
                                    best[j0 + j] = min(best[j0 + j], on ? key : KNONE);
                                }
                            }
                        } else {
#pragma unroll
                        for (int j = 0; j < 8; j++) {
                            const unsigned Pa = scan64_dpp(csA[j]), Pb = scan64_dpp(csB[j]);
                            const unsigned ta = (unsigned)__builtin_amdgcn_readlane((int)Pa, 63);
                            const unsigned V = lane < W2 - 1 ? Pb + ta : Pa;
                            const unsigned hi =
                                (unsigned)__builtin_amdgcn_ds_bpermute(src, (int)V);
                            const unsigned sad = hi - Pa + csA[j];
                            const Key key = WIDE ? ((Key)sad << 32) | (Key)(unsigned)(d_in + ib0[j])
                                                 : (Key)((sad << 12) | (unsigned)(d_in + ib0[j]));
                            const bool on = (unsigned)(d_in - lo[j]) < (unsigned)len[j];
                            best[j] = on ? min(best[j], key) : best[j];
                        }
                        }
                    }
                }
            }
            if (wst < 0) o0 = o1;
        }
    }
    if (keys) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if ((pn[j] & 0xffff) == 0 || best[j] == KNONE) continue;
            atomicMin(&keys[(size_t)(ty0 + r0 + j) * W + tx0 + lane], best[j]);
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < 8; j++) {
        if ((pn[j] & 0xffff) == 0) continue;
        const int x = tx0 + lane, y = ty0 + r0 + j;
        const size_t p = (size_t)y * W + x;
        const int4 e = ends[p];
        int cx, cy;
        line_point(make_line(e.x, e.y, e.z, e.w), WIDE ? (int)(unsigned)best[j] : (int)(best[j] & 0xfffu),
                   cx, cy);
        const double dx = (double)(cx - x), dy = (double)(cy - y);
        const int dn = (int)__builtin_sqrt(dx * dx + dy * dy);       // :89
        disp_u8[p] = (uint8_t)dn;
        if (disp_u16) disp_u16[p] = (uint16_t)dn;
        if (valid_out) valid_out[p] = 1;
    }
}

// The split plane loop's keys -> the reference's outputs: candidate i of the
// pixel's line, (uchar)(int)sqrt(dx^2 + dy^2) (CameraStereoVision.cpp:85-89).
// Pixels without a key (not matched) keep what the maps held.  Each key read
// is put back to all-ones, so the next call needs no memset.
template <class Key>
__global__ void ref_finalize_kernel(int W, int H, const int4* __restrict__ ends,
                                    Key* __restrict__ keys,
                                    uint8_t* __restrict__ disp_u8, uint16_t* __restrict__ disp_u16,
                                    uint8_t* __restrict__ valid_out) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    const size_t p = (size_t)y * W + x;
    const Key key = keys[p];
    if (key == (Key)~(Key)0) return;
    keys[p] = (Key)~(Key)0;
    const int4 e = ends[p];
    int cx, cy;
    line_point(make_line(e.x, e.y, e.z, e.w),
               sizeof(Key) == 8 ? (int)(unsigned)key : (int)((unsigned)key & 0xfffu), cx, cy);
    const double dx = (double)(cx - x), dy = (double)(cy - y);
    const int dn = (int)__builtin_sqrt(dx * dx + dy * dy);       // :89
    disp_u8[p] = (uint8_t)dn;
    if (disp_u16) disp_u16[p] = (uint16_t)dn;
    if (valid_out) valid_out[p] = 1;
}

// k > 32: one wave per reference pixel over its Bresenham candidates (the
// 2k-byte rows through sad_span; the per-pixel first minimum is a u64
// (SAD << 32 | i) wave minimum, so neither k nor the frame size is bounded by
// a key field).  Four pixels per 256-thread workgroup.
__global__ __launch_bounds__(256) void ref_pixel_kernel(
    const uint8_t* __restrict__ ref, const uint8_t* __restrict__ other, int W, int H, size_t pitch,
    const uint8_t* __restrict__ mask, const int4* __restrict__ ends,
    const uint8_t* __restrict__ valid_in, int k, uint8_t* __restrict__ disp_u8,
    uint16_t* __restrict__ disp_u16, uint8_t* __restrict__ valid_out) {
    const int x = k + (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6), y = k + (int)blockIdx.y;
    if (x >= W - k || y >= H - k) return;                       // wave-uniform
    const size_t p = (size_t)y * W + x;
    if (!valid_in[p] || (mask && mask[p] == 0)) return;
    match_pixel_wave<0>(ref, other, W, pitch, x, y, ends[p], k, disp_u8, disp_u16, valid_out);
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

// Shares per tile: about four rounds of the chip's workgroup slots in all,
// rounded, within [kPlaneSplitMin, kPlaneSplitMax] -- 1080p (990 tiles, 768
// slots), 1440p and 4K 3, 1280x720 and smaller 6.  Measured with every tile
// split S ways (profiles/r05_v5/plane_walk/n*_*.log.txt, r6q/): the shares
// fill the last round and balance the uneven tile work (a Low pair's tiles
// near the image border carry fewer planes); more shares than that pay more
// per-share setup than they save.
static int plane_shares(long long tiles, int cu_count) {
    const long long slots = (long long)cu_count * tune::kPlaneMinBlocks;
    if (tune::kPlaneSplitMax <= 1 || slots <= 0 || tiles <= 0) return 1;
    long long s = (tune::kPlaneSplitRounds * slots + tiles / 2) / tiles;
    if (s > tune::kPlaneSplitMax) s = tune::kPlaneSplitMax;
    if (s < tune::kPlaneSplitMin) s = tune::kPlaneSplitMin;
    return (int)s;
}

hipError_t launch_ref_match(Ctx& c, const uint8_t* ref, const uint8_t* other, int W, int H,
                            size_t pitch, const uint8_t* mask, const int32_t* ends,
                            const uint8_t* valid_in, int k, uint8_t* disp_u8,
                            uint16_t* disp_u16, uint8_t* valid_out) {
    ScopedKernelTimer t(c, "ref_match");
    const long long npx = (long long)(W - 2 * k) * (H - 2 * k);
    if (npx <= 0) return hipSuccess;
    if (k > PT_MAXK) {
        // windows wider than the plane kernel's region (63 + 2k <= 127
        // columns): one wave per pixel, first minimum in a u64 wave key
        const dim3 grid((unsigned)((W - 2 * k + 3) / 4), (unsigned)(H - 2 * k));
        hipLaunchKernelGGL(ref_pixel_kernel, grid, dim3(256), 0, c.stream, ref, other, W, H, pitch,
                           mask, (const int4*)ends, valid_in, k, disp_u8, disp_u16, valid_out);
        return hipGetLastError();
    }
    // offset-plane algorithm for k = 1..32
    const int gx = (W - 2 * k + 63) / 64, gy = (H - 2 * k + P3_ROWS - 1) / P3_ROWS;
    const long long tiles = (long long)gx * gy;
    int nsh = plane_shares(tiles, c.cu_count);
    // SVA_DEBUG_PLANE_SPLIT (sva_set_debug): every tile in n shares, so the
    // parity tests cover every share count at every size
    if (c.dbg_plane_split >= 1 && c.dbg_plane_split <= 16) nsh = c.dbg_plane_split;
    const bool split = nsh > 1;
    // a line holds at most max(W, H) - 2k + 1 candidates: 4096 or more do not
    // fit the u32 key's 12-bit index field
    const bool wide = W >= 4096 || H >= 4096;
    const size_t kb = wide ? sizeof(unsigned long long) : sizeof(unsigned);
    void* keys = nullptr;
    if (split) {
        const size_t need = (size_t)W * H * kb;
        hipError_t e = c.ref_keys.ensure(need);
        if (e != hipSuccess) return e;
        keys = c.ref_keys.ptr;
        if (c.ref_keys_alloc != c.ref_keys.ptr) {   // a new allocation: nothing known clean
            c.ref_keys_alloc = c.ref_keys.ptr;
            c.ref_keys_clean = 0;
        }
        if (c.ref_keys_clean < need) {
            // the only memset: the first call, or a buffer past what earlier
            // finalize passes restored to all-ones
            e = hipMemsetAsync(keys, 0xff, need, c.stream);
            if (e != hipSuccess) return e;
            c.ref_keys_clean = need;
        }
        c.ref_keys_clean = 0;                        // until the finalize below is queued
    }
    const dim3 pg3((unsigned)nsh, (unsigned)gx, (unsigned)gy);
#define SVA_PLANE3_CASE(K_)                                                                        \
    case K_:                                                                                       \
        if (wide)                                                                                  \
            hipLaunchKernelGGL((ref_plane3_kernel<K_, true>), pg3, dim3(256), 0, c.stream, ref,    \
                               other, W, H, pitch, mask, (const int4*)ends, valid_in, disp_u8,     \
                               disp_u16, valid_out, keys);                                         \
        else                                                                                       \
            hipLaunchKernelGGL((ref_plane3_kernel<K_, false>), pg3, dim3(256), 0, c.stream, ref,   \
                               other, W, H, pitch, mask, (const int4*)ends, valid_in, disp_u8,     \
                               disp_u16, valid_out, keys);                                         \
        break;
    switch (k) {
        SVA_PLANE3_CASE(1) SVA_PLANE3_CASE(2) SVA_PLANE3_CASE(3) SVA_PLANE3_CASE(4)
        SVA_PLANE3_CASE(5) SVA_PLANE3_CASE(6) SVA_PLANE3_CASE(7) SVA_PLANE3_CASE(8)
        SVA_PLANE3_CASE(9) SVA_PLANE3_CASE(10) SVA_PLANE3_CASE(11) SVA_PLANE3_CASE(12)
        SVA_PLANE3_CASE(13) SVA_PLANE3_CASE(14) SVA_PLANE3_CASE(15) SVA_PLANE3_CASE(16)
        SVA_PLANE3_CASE(17) SVA_PLANE3_CASE(18) SVA_PLANE3_CASE(19) SVA_PLANE3_CASE(20)
        SVA_PLANE3_CASE(21) SVA_PLANE3_CASE(22) SVA_PLANE3_CASE(23) SVA_PLANE3_CASE(24)
        SVA_PLANE3_CASE(25) SVA_PLANE3_CASE(26) SVA_PLANE3_CASE(27) SVA_PLANE3_CASE(28)
        SVA_PLANE3_CASE(29) SVA_PLANE3_CASE(30) SVA_PLANE3_CASE(31) SVA_PLANE3_CASE(32)
        default: return hipErrorInvalidValue;
    }
#undef SVA_PLANE3_CASE
    if (split && wide)
        hipLaunchKernelGGL(ref_finalize_kernel<unsigned long long>,
                           dim3((unsigned)((W + 255) / 256), (unsigned)H), dim3(256), 0, c.stream, W,
                           H, (const int4*)ends, (unsigned long long*)keys, disp_u8, disp_u16,
                           valid_out);
    else if (split)
        hipLaunchKernelGGL(ref_finalize_kernel<unsigned>, dim3((unsigned)((W + 255) / 256), (unsigned)H),
                           dim3(256), 0, c.stream, W, H, (const int4*)ends, (unsigned*)keys,
                           disp_u8, disp_u16, valid_out);
    const hipError_t err = hipGetLastError();
    // the finalize pass restores every key of the W x H region to all-ones
    if (split && err == hipSuccess) c.ref_keys_clean = (size_t)W * H * (wide ? 8 : 4);
    return err;
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
