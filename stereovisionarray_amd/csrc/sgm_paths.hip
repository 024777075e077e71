// sgm_paths.hip -- 8-direction SGM path aggregation (DESIGN.md §2.3 / §4.3,
// SURVEY.md §8a row A12).  All eight directions run in ONE launch.
//
//   L_r(p,d) = C(p,d) + min(L_r(q,d), L_r(q,d-1)+P1, L_r(q,d+1)+P1, m+P2) - m
//   m = min_k L_r(q,k),  q = p - r;  L_r(p,d) = C(p,d) where q leaves the image.
//
// Mapping (CDNA4, wave64):
//   * A path LINE is owned by one 16-lane DPP row; lane k holds disparities
//     [k*DPL, k*DPL + DPL) as DPL/2 packed u16 pairs, so every per-disparity
//     op is one v_pk_* for two disparities.
//   * The d-1 / d+1 neighbours are v_alignbit within the lane plus one DPP
//     row_shr:1 / row_shl:1 across lanes (INF fed in at the row edges).
//   * min_k L is a lane-local v_pk_min tree + a 4-step DPP row reduction
//     (quad_perm, half-mirror, mirror) that leaves the minimum in all 16
//     lanes -- no LDS, no barrier.  The state carried to the next pixel is
//     normalised, B = L - min_k L, so m + P2 becomes the constant P2.
//   * A wave carries 4 lines, a 256-thread workgroup 16 lines of one
//     direction.  Vertical lines: consecutive x; diagonal lines: consecutive
//     (x - y) mod W, so the 4 pixels a wave touches per step are adjacent in
//     memory (one 4*D-byte span); horizontal lines: 4 rows, one D-byte span
//     each.  Diagonals use the wrap-around trick: line i visits
//     ((i + rx*t) mod W, t) and restarts (L = C) where x wraps, so every line
//     has exactly H steps and no lane idles on ragged diagonal lengths.
//   * Cost bytes are prefetched PF steps ahead into a register ring (the
//     loads do not depend on the recurrence), hiding HBM latency behind the
//     dependent DPP chain of the current step.
// HBM bytes per disparity: 8 C reads (1 B each, one per direction) + 8 L
// writes (u8 per direction volume, [8][H][W][D]).
#include "sva_device.h"
#include "sva_internal.h"

namespace sva {
namespace {

constexpr int PATH_BLOCK = 256;
constexpr int LINES_PER_BLOCK = PATH_BLOCK / 16;
constexpr int PF = 8;                        // prefetch depth in steps
constexpr unsigned INF2 = 0x7fff7fffu;       // neighbour beyond d range

struct PathGeom {
    int W, H, D;
    int P1, P2;
    int blk_h;    // blocks per horizontal direction (H lines)
    int blk_w;    // blocks per vertical / diagonal direction (W lines)
    size_t vol;   // bytes of one direction volume (W*H*D)
};

template <int NW>
struct Words {
    unsigned w[NW];
};

template <int NW>
__device__ __forceinline__ Words<NW> load_words(const uint8_t* p) {
    Words<NW> r;
    if constexpr (NW == 1) {
        r.w[0] = *(const unsigned*)p;
    } else if constexpr (NW == 2) {
        uint2 v = *(const uint2*)p;
        r.w[0] = v.x; r.w[1] = v.y;
    } else if constexpr (NW == 3) {
        const unsigned* q = (const unsigned*)p;
        r.w[0] = q[0]; r.w[1] = q[1]; r.w[2] = q[2];
    } else {
        uint4 v = *(const uint4*)p;
        r.w[0] = v.x; r.w[1] = v.y; r.w[2] = v.z; r.w[3] = v.w;
    }
    return r;
}

template <int NW>
__device__ __forceinline__ void store_words(uint8_t* p, const unsigned (&w)[NW]) {
    if constexpr (NW == 1) {
        *(unsigned*)p = w[0];
    } else if constexpr (NW == 2) {
        *(uint2*)p = make_uint2(w[0], w[1]);
    } else if constexpr (NW == 3) {
        unsigned* q = (unsigned*)p;
        q[0] = w[0]; q[1] = w[1]; q[2] = w[2];
    } else {
        *(uint4*)p = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

// Cursor over one path line.  DIAG lines wrap in x and report the wrap.
template <bool DIAG>
struct Cursor {
    int x, y;
    __device__ __forceinline__ bool advance(int rx, int ry, int W) {
        x += rx;
        y += ry;
        bool wrapped = false;
        if constexpr (DIAG) {
            if (x >= W) { x -= W; wrapped = true; }
            if (x < 0) { x += W; wrapped = true; }
        }
        return wrapped;
    }
    __device__ __forceinline__ size_t off(int W, int D) const {
        return ((size_t)y * (size_t)W + (size_t)x) * (size_t)D;
    }
};

// One recurrence step for the lane's DPL disparities.
template <int DPL>
__device__ __forceinline__ void sgm_step(const unsigned (&cw)[DPL / 4], unsigned (&B)[DPL / 2],
                                         unsigned (&ow)[DPL / 4], unsigned P1, unsigned P2) {
    constexpr int NW = DPL / 4, NP = DPL / 2;
    unsigned c[NP];
#pragma unroll
    for (int w = 0; w < NW; w++) unpack4(cw[w], c[2 * w], c[2 * w + 1]);
    // neighbours: X = lane k-1's last pair, Y = lane k+1's first pair
    const unsigned X = row_shr1(B[NP - 1], INF2);
    const unsigned Y = row_shl1(B[0], INF2);
    unsigned M[NP];
    M[0] = __builtin_amdgcn_alignbit(B[0], X, 16);
#pragma unroll
    for (int j = 1; j < NP; j++) M[j] = __builtin_amdgcn_alignbit(B[j], B[j - 1], 16);
    const unsigned Qlast = __builtin_amdgcn_alignbit(Y, B[NP - 1], 16);
    unsigned Ln[NP];
#pragma unroll
    for (int j = 0; j < NP; j++) {
        const u16x2 q = as_v2(j < NP - 1 ? M[j + 1] : Qlast);
        u16x2 t = vmin2(as_v2(M[j]), q) + splat2(P1);
        t = vmin2(t, as_v2(B[j]));
        t = vmin2(t, splat2(P2));
        Ln[j] = as_u32(t + as_v2(c[j]));
    }
#pragma unroll
    for (int w = 0; w < NW; w++) ow[w] = pack4(Ln[2 * w], Ln[2 * w + 1]);
    // m = min_k L over the 16-lane row, then normalise the carried state
    u16x2 mm = as_v2(Ln[0]);
#pragma unroll
    for (int j = 1; j < NP; j++) mm = vmin2(mm, as_v2(Ln[j]));
    unsigned m = mm.x < mm.y ? mm.x : mm.y;
    m = row_min_u32(m);
#pragma unroll
    for (int j = 0; j < NP; j++) B[j] = as_u32(as_v2(Ln[j]) - splat2(m));
}

template <int DPL, bool DIAG>
__device__ __forceinline__ void path_line(const uint8_t* __restrict__ C, uint8_t* __restrict__ L,
                                          const PathGeom& g, int rx, int ry, int line, int k) {
    constexpr int NW = DPL / 4, NP = DPL / 2;
    const int W = g.W, H = g.H, D = g.D;
    const unsigned P1 = (unsigned)g.P1, P2 = (unsigned)g.P2;
    const int steps = ry == 0 ? W : H;
    Cursor<DIAG> cc;
    if (ry == 0) { cc.y = line; cc.x = rx > 0 ? 0 : W - 1; }
    else { cc.y = ry > 0 ? 0 : H - 1; cc.x = line; }
    Cursor<DIAG> pc = cc;        // prefetch cursor, clamped at the last step
    int tp = 0;
    const uint8_t* Cb = C + k * DPL;
    uint8_t* Lb = L + k * DPL;

    unsigned B[NP];
#pragma unroll
    for (int j = 0; j < NP; j++) B[j] = 0u;   // L(q) = 0, m = 0  =>  L = C

    Words<NW> ring[PF];
#pragma unroll
    for (int p = 0; p < PF; p++) {
        ring[p] = load_words<NW>(Cb + pc.off(W, D));
        if (tp < steps - 1) { pc.advance(rx, ry, W); tp++; }
    }

    int t = 0;
    for (; t + PF <= steps; t += PF) {
#pragma unroll
        for (int p = 0; p < PF; p++) {
            unsigned cw[NW];
#pragma unroll
            for (int w = 0; w < NW; w++) cw[w] = ring[p].w[w];
            ring[p] = load_words<NW>(Cb + pc.off(W, D));
            if (tp < steps - 1) { pc.advance(rx, ry, W); tp++; }
            unsigned ow[NW];
            sgm_step<DPL>(cw, B, ow, P1, P2);
            store_words<NW>(Lb + cc.off(W, D), ow);
            const bool wrapped = cc.advance(rx, ry, W);
            if constexpr (DIAG) {
                if (wrapped) {
#pragma unroll
                    for (int j = 0; j < NP; j++) B[j] = 0u;
                }
            }
        }
    }
    // tail: fewer than PF steps left, all already in the ring
#pragma unroll
    for (int p = 0; p < PF; p++) {
        if (t + p < steps) {
            unsigned cw[NW];
#pragma unroll
            for (int w = 0; w < NW; w++) cw[w] = ring[p].w[w];
            unsigned ow[NW];
            sgm_step<DPL>(cw, B, ow, P1, P2);
            store_words<NW>(Lb + cc.off(W, D), ow);
            const bool wrapped = cc.advance(rx, ry, W);
            if constexpr (DIAG) {
                if (wrapped) {
#pragma unroll
                    for (int j = 0; j < NP; j++) B[j] = 0u;
                }
            }
        }
    }
}

// Direction table, identical to oracle svo_direction().
__device__ __forceinline__ void dir_of(int r, int& rx, int& ry) {
    constexpr int T[8][2] = {{1, 0}, {-1, 0}, {0, 1}, {0, -1}, {1, 1}, {-1, -1}, {-1, 1}, {1, -1}};
    rx = T[r][0];
    ry = T[r][1];
}

template <int DPL>
__global__ __launch_bounds__(PATH_BLOCK) void sgm_paths_kernel(const uint8_t* __restrict__ C,
                                                               uint8_t* __restrict__ L8,
                                                               PathGeom g) {
    // Horizontal directions (W steps per line, the longest) get the lowest
    // block ids so they are dispatched first; the rest follow.
    int b = blockIdx.x, r, lb;
    if (b < 2 * g.blk_h) {
        r = b / g.blk_h;
        lb = b - r * g.blk_h;
    } else {
        b -= 2 * g.blk_h;
        r = 2 + b / g.blk_w;
        lb = b - (r - 2) * g.blk_w;
    }
    const int line = lb * LINES_PER_BLOCK + (threadIdx.x >> 4);
    const int k = threadIdx.x & 15;
    const int nlines = r < 2 ? g.H : g.W;
    if (line >= nlines) return;  // whole 16-lane row leaves together
    int rx, ry;
    dir_of(r, rx, ry);
    uint8_t* L = L8 + (size_t)r * g.vol;
    if (r >= 4) path_line<DPL, true>(C, L, g, rx, ry, line, k);
    else path_line<DPL, false>(C, L, g, rx, ry, line, k);
}

}  // namespace

bool paths_supported(int D) { return D == 64 || D == 128 || D == 192 || D == 256; }

hipError_t launch_paths(Ctx& c, const uint8_t* C, int W, int H, int D, int P1, int P2,
                        uint8_t* L8) {
    ScopedKernelTimer t(c, "sgm_paths");
    PathGeom g;
    g.W = W; g.H = H; g.D = D; g.P1 = P1; g.P2 = P2;
    g.blk_h = (H + LINES_PER_BLOCK - 1) / LINES_PER_BLOCK;
    g.blk_w = (W + LINES_PER_BLOCK - 1) / LINES_PER_BLOCK;
    g.vol = (size_t)W * H * D;
    dim3 grid(2 * g.blk_h + 6 * g.blk_w);
    switch (D) {
        case 64: hipLaunchKernelGGL(sgm_paths_kernel<4>, grid, dim3(PATH_BLOCK), 0, c.stream, C, L8, g); break;
        case 128: hipLaunchKernelGGL(sgm_paths_kernel<8>, grid, dim3(PATH_BLOCK), 0, c.stream, C, L8, g); break;
        case 192: hipLaunchKernelGGL(sgm_paths_kernel<12>, grid, dim3(PATH_BLOCK), 0, c.stream, C, L8, g); break;
        case 256: hipLaunchKernelGGL(sgm_paths_kernel<16>, grid, dim3(PATH_BLOCK), 0, c.stream, C, L8, g); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace sva
