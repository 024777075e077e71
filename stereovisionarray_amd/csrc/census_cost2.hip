// census_cost2.hip -- 9x7 Census + Hamming cost volume in one kernel for the
// 2-D matching steps of camera-array pairs (SURVEY.md
// §8a rows A10 + A11), with the Hamming distances on the matrix cores.
//
// Same C bytes as census9x7 x2 -> hamming_cost2_kernel:
//   C[(y*W + x)*D + d] = popcount(CL(q) ^ CR(q + off(dmin + d))), 62 where the
//   matched pixel leaves the image, off = step_offset(., bx, by).
// Steps whose primitive form (bx, by) has |by| = 1 and M = max(|bx|, 1) <= 3:
// vertical (0, +-1), the diagonals (+-1, +-1) and (+-2, +-1), (+-3, +-1) --
// every baseline of the reference's 5x5 rig (getCameraPairs,
// functions.cpp:148-213) and of the 2x4 grid of BASELINE config 4.
//
// Lattice lines.  Pixel q + r*v (v = (bx, by)) matched at distance s reads the
// pixel q matches at s + r*M, since rounding commutes with adding an integer
// (off(s + r*M) = off(s) + r*v).  So along one lattice line q0 + r*v the
// problem is the 1-D one of census_cost.hip, with the right operands taken
// along the Bresenham path q0 + off(t) (path position t = r*M + s):
//   * pixel r = c + K n + 16 K sp (class c < K, lane n < 16, span sp < 4/K)
//     sits at path position M r, so in an N-tile of one (c, sp) the tile row
//     R <-> t = dmin + M c + 16 K M sp + R gives d = R - (K M) n;
//   * K M is a multiple of 4 (K = 4, 2, 4 for M = 1, 2, 3), so each lane's
//     four results are four consecutive disparities starting at a multiple
//     of 4: one u8x4 word of the cost volume, as in the 1-D kernel;
//   * T = ceil((15 K M + D) / 16) tiles cover every pixel's D disparities
//     (M = 3 pays 20 tiles at D=128 where M <= 2 pays 12).
// A workgroup owns XB adjacent lattice lines (adjacent columns at every row,
// since |by| = 1) x 64 positions r = 64 image rows.  The image around all of
// them is staged once into two sheared LDS patches -- patch row rho holds
// image row Y0 + by*rho from column X0 + bx*rho - E -- so every census window
// is 7 rows of 9 bytes at a per-row byte offset (census_bytes_at).  Then per
// line, between two barriers:
//   A  the census windows of its 64 pixels and of the 63 M + D path pixels
//      they match become 64-byte operand rows; the previous line's staged
//      costs leave as whole 128-byte lines (nt stores);
//   B  each wave multiplies its 16-pixel N-tile by the T path tiles on
//      v_mfma_i32_16x16x64_i8 and packs the results into the staging rows.
// HBM bytes: 1 B/disparity written + the images (L2-served re-reads).
// dreal < D (a padded frame): disparities d >= dreal get 255.
#include "census_mma.h"
#include "sva_device.h"
#include "sva_internal.h"
#include "sva_tuning.h"

namespace sva {
namespace {

constexpr int CC2_BLOCK = 256;
constexpr int LINE = 64;                 // pixels per lattice-line chunk (rows)

__device__ __forceinline__ void store16_nt(uint8_t* p, const unsigned (&o)[4]) {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    if constexpr (tune::kCostStoreNT)
        __builtin_nontemporal_store((v4u){o[0], o[1], o[2], o[3]}, (v4u*)p);
    else
        *(v4u*)p = (v4u){o[0], o[1], o[2], o[3]};
}

// Geometry of one (D, M, XB) instance, shared by the kernel and the host.
template <int NC, int M, int XB>
struct CC2Geom {
    static constexpr int D = NC * 16;
    static constexpr int K = M % 4 == 0 ? 1 : (M % 2 == 0 ? 2 : 4);   // classes
    static constexpr int KM = K * M;                                   // a multiple of 4
    static constexpr int S = 4 / K;                                    // spans per class
    static constexpr int T = (15 * KM + D + 15) / 16;                  // tiles per N-tile
    static constexpr int NT = (LINE - 1) * M + D;                      // path pixels per line
    // operand rows the tiles read (rows >= NT only feed dump words)
    static constexpr int NA = M * (K - 1) + 16 * KM * (S - 1) + 16 * T;
    static constexpr int NAP = (NA + 15) / 16 * 16;
    static constexpr int WPT = (LINE + NT + CC2_BLOCK - 1) / CC2_BLOCK;
    // patch: E columns of margin left of the line-0 centre; PW bytes per row,
    // PW / 4 odd so that lanes on consecutive patch rows hit distinct banks
    static constexpr int HALF = (M + 1) / 2;
    static constexpr int E = 3 * M + HALF + 4;
    static constexpr int PW0 = (XB + 11 + 6 * M + 2 * HALF + 3) / 4 * 4;
    static constexpr int PW = (PW0 / 4) % 2 ? PW0 : PW0 + 4;
    static constexpr int LR = LINE + 6;                                 // left patch rows
    static constexpr int RR = (NT + M - 1) / M + 8;                     // right patch rows
    static constexpr int S4 = NC * 4 + 7;                               // staging dwords/pixel
    static constexpr int PATCH = (LR + RR) * PW;
};

template <int NC, int M, int XB>
__global__ __launch_bounds__(CC2_BLOCK) void census_cost2_mma_kernel(
    const uint8_t* __restrict__ left, const uint8_t* __restrict__ right, int W, int H,
    size_t pitch, int dmin, int bx, int by, int ngroups, int dreal, uint8_t* __restrict__ C) {
    using G = CC2Geom<NC, M, XB>;
    constexpr int D = G::D, K = G::K, KM = G::KM, S = G::S, T = G::T, NT = G::NT;
    constexpr int NAP = G::NAP, PW = G::PW, E = G::E, LR = G::LR, S4 = G::S4;
    static_assert(KM % 4 == 0 && K * S == 4, "four waves: K classes x S spans");
    __shared__ __attribute__((aligned(16))) uint8_t pat[G::PATCH + 16];   // [left LR | right RR][PW]
    __shared__ __attribute__((aligned(16))) uint8_t opA[4 * NAP * 16];     // [K quarter][path t][16]
    __shared__ __attribute__((aligned(16))) uint8_t opB[4 * LINE * 16];    // [K quarter][slot][16]
    __shared__ unsigned stg[LINE * S4];                                     // [slot][S4]

    const int g = blockIdx.x % ngroups, h = blockIdx.x / ngroups;
    const int t = threadIdx.x;
    const int sx = bx > 0 ? 1 : (bx < 0 ? -1 : 0);
    const int Y0 = by > 0 ? LINE * h : H - 1 - LINE * h;
    const int X0 = g * XB - (LINE - 1) * (bx > 0 ? bx : 0);      // line j: origin (X0 + j, Y0)
    // minor-axis (row) component of the path: b(t) = round_half_up(t / M)
    auto bt = [](int u) { return M == 1 ? u : (2 * u + M) / (2 * M); };
    const int rhoR0 = bt(dmin) - 3;                                // first right patch row
    const int rowstep = by * PW - bx * by;                         // window row r -> r + 1

    // ---- stage both patches (image rows Y0 + by*rho, sheared by bx per row)
    {
        constexpr int NL = (G::PATCH + CC2_BLOCK - 1) / CC2_BLOCK;
        constexpr int CH = 8;
#pragma unroll
        for (int k0 = 0; k0 < NL; k0 += CH) {
            uint8_t v[CH];
#pragma unroll
            for (int k = 0; k < CH; k++) {
                const int i = t + (k0 + k) * CC2_BLOCK;
                const bool isR = i >= LR * PW;
                const int q = isR ? i - LR * PW : i;
                const int pr = q / PW, cb = q - pr * PW;
                const int rho = isR ? rhoR0 + pr : pr - 3;
                const int yy = Y0 + by * rho, xx = X0 + bx * rho - E + cb;
                const uint8_t* img = isR ? right : left;
                v[k] = (k0 + k < NL && i < G::PATCH && (unsigned)yy < (unsigned)H &&
                        (unsigned)xx < (unsigned)W)
                           ? img[(size_t)yy * pitch + xx] : 0;
            }
#pragma unroll
            for (int k = 0; k < CH; k++) {
                const int i = t + (k0 + k) * CC2_BLOCK;
                if (k0 + k < NL && i < G::PATCH) pat[i] = v[k];
            }
        }
    }
    const uint8_t* patL = pat;
    const uint8_t* patR = pat + LR * PW;
    __syncthreads();

    const int wv = t >> 6, l = t & 63, ln = l & 15, lq = l >> 4;
    // slot b = 16 w + n (wave w = c S + sp) <-> pixel r = c + K n + 16 K sp
    auto slot_r = [](int b) {
        const int w = b >> 4, n = b & 15;
        return (w / S) + K * n + 16 * K * (w % S);
    };
    for (int j = 0; j <= XB; j++) {
        // ---- census of line j into the operand rows; store of line j - 1
        if (j < XB) {
#pragma unroll
            for (int k = 0; k < G::WPT; k++) {
                const int w = t + k * CC2_BLOCK;
                unsigned d[16];
                if (w < LINE) {
                    const int r = slot_r(w);
                    const int x = X0 + j + bx * r, y = Y0 + by * r;
                    if (y >= 3 && y < H - 3 && x >= 4 && x < W - 4) {
                        const int a0 = (r - 3 * by + 3) * PW + j - 4 + E + 3 * bx * by;
                        census_bytes_at<true>(patL, a0, rowstep, d);
                    } else {
                        census_zero<true>(d);              // census word 0 (or not stored)
                    }
                    put_operand_row(opB, LINE, w, d);
                } else if (w < LINE + NT) {
                    const int i = w - LINE, u = dmin + i, b = bt(u);
                    const int x = X0 + j + sx * u, y = Y0 + by * b;
                    if ((unsigned)x >= (unsigned)W || (unsigned)y >= (unsigned)H) {
                        census_outside(d);                 // cost 62
                    } else if (y >= 3 && y < H - 3 && x >= 4 && x < W - 4) {
                        const int a0 = (b - 3 * by - rhoR0) * PW + j + sx * u - bx * b - 4 + E +
                                       3 * bx * by;
                        census_bytes_at<false>(patR, a0, rowstep, d);
                    } else {
                        census_zero<false>(d);             // census word 0
                    }
                    put_operand_row(opA, NAP, i, d);
                }
            }
        }
        if (j > 0) {
#pragma unroll
            for (int k = 0; k < LINE * NC / CC2_BLOCK; k++) {
                const int ch = t + k * CC2_BLOCK;
                const int b = ch / NC, ci = ch % NC, r = slot_r(b);
                const int x = X0 + (j - 1) + bx * r, y = Y0 + by * r;
                if ((unsigned)x >= (unsigned)W || (unsigned)y >= (unsigned)H) continue;
                const unsigned* src = &stg[b * S4 + 4 * ci];
                unsigned out[4] = {src[0], src[1], src[2], src[3]};
                if (dreal < D) {                 // padded disparities: cost 255
#pragma unroll
                    for (int q = 0; q < 4; q++) out[q] |= pad_bytes(16 * ci + 4 * q, dreal);
                }
                store16_nt(C + ((size_t)y * W + x) * D + 16 * ci, out);
            }
        }
        __syncthreads();
        // ---- the costs of line j on the matrix cores, into the staging rows
        if (j < XB) {
            const int c = wv / S, sp = wv % S;
            const v4i zero = {0, 0, 0, 0};
            const v4i bf = *reinterpret_cast<const v4i*>(&opB[(lq * LINE + 16 * wv + ln) * 16]);
            unsigned* dst = &stg[(16 * wv + ln) * S4];
            const int base = M * c + 16 * KM * sp;
            constexpr int GT = 4;
#pragma unroll
            for (int gt = 0; gt < T; gt += GT) {
                v4i acc[GT];
#pragma unroll
                for (int i = 0; i < GT && gt + i < T; i++) {
                    const int idx = base + 16 * (gt + i) + ln;
                    const v4i af = *reinterpret_cast<const v4i*>(&opA[(lq * NAP + idx) * 16]);
                    acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af, bf, zero, 0, 0, 0);
                }
#pragma unroll
                for (int i = 0; i < GT && gt + i < T; i++) {
                    // rows 16 (gt + i) + 4 lq + e of pixel lane ln: d = that - KM ln
                    const int jw = 4 * (gt + i) + lq - (KM / 4) * ln;
                    unsigned wd = (unsigned)acc[i][0] | ((unsigned)acc[i][1] << 8);
                    wd |= ((unsigned)acc[i][2] << 16) | ((unsigned)acc[i][3] << 24);
                    dst[(unsigned)jw < (unsigned)(NC * 4) ? jw : NC * 4 + lq] = wd;   // else: dump
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        __syncthreads();
    }
}

// primitive form of (sx, sy)
void reduce_step(int sx, int sy, int* bx, int* by) {
    int a = sx < 0 ? -sx : sx, b = sy < 0 ? -sy : sy;
    while (b) { const int r = a % b; a = b; b = r; }
    *bx = sx / a;
    *by = sy / a;
}

}  // namespace

bool census_cost2_supported(int D, int sx, int sy) {
    if (!(D == 64 || D == 128 || D == 192 || D == 256) || sy == 0) return false;
    int bx, by;
    reduce_step(sx, sy, &bx, &by);
    const int abx = bx < 0 ? -bx : bx;
    return (by == 1 || by == -1) && abx <= 3;
}

hipError_t launch_census_cost2(Ctx& c, const uint8_t* left, const uint8_t* right, int W, int H,
                               size_t pitch, int D, int dmin, int sx, int sy, uint8_t* C,
                               int dreal) {
    if (!census_cost2_supported(D, sx, sy)) return hipErrorInvalidValue;
    if (dreal <= 0) dreal = D;
    ScopedKernelTimer tm(c, "cost");
    int bx, by;
    reduce_step(sx, sy, &bx, &by);
    const int abx = bx < 0 ? -bx : bx, M = abx > 1 ? abx : 1;
    constexpr int XB = tune::kCensusCost2Lines;
    const int ngroups = (W + (LINE - 1) * abx + XB - 1) / XB;
    const long long nchunks = (H + LINE - 1) / LINE;
    const dim3 grid((unsigned)(ngroups * nchunks));
#define SVA_CC2(NC_, M_)                                                                          \
    hipLaunchKernelGGL((census_cost2_mma_kernel<NC_, M_, XB>), grid, dim3(CC2_BLOCK), 0, c.stream, \
                       left, right, W, H, pitch, dmin, bx, by, ngroups, dreal, C)
#define SVA_CC2_D(M_)                        \
    switch (D) {                             \
        case 64: SVA_CC2(4, M_); break;      \
        case 128: SVA_CC2(8, M_); break;     \
        case 192: SVA_CC2(12, M_); break;    \
        default: SVA_CC2(16, M_); break;     \
    }
    switch (M) {
        case 1: SVA_CC2_D(1) break;
        case 2: SVA_CC2_D(2) break;
        default: SVA_CC2_D(3) break;
    }
#undef SVA_CC2_D
#undef SVA_CC2
    return hipGetLastError();
}

}  // namespace sva
