// sgm_common.h -- device pieces shared by the two 8-path aggregation kernels
// (sgm_paths.hip reads a materialised cost volume; sgm_fused.hip computes the
// Hamming costs from the census maps on the fly).  DESIGN.md §4.3 / §4.5.
#pragma once

#include <utility>

#include "sva_device.h"
#include "sva_internal.h"

namespace sva {
namespace sgm {

// f(integral_constant<int, 0>), ..., f(integral_constant<int, N-1>): a
// compile-time unrolled loop whose index can select registers.
template <class F, int... S>
__device__ __forceinline__ void for_seq_impl(std::integer_sequence<int, S...>, F&& f) {
    (f(std::integral_constant<int, S>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void for_seq(F&& f) {
    for_seq_impl(std::make_integer_sequence<int, N>{}, static_cast<F&&>(f));
}

constexpr unsigned INF2 = 0x7fff7fffu;       // neighbour beyond d range

struct PathGeom {
    int W, H, D;
    int P1, P2;
    int blk_h;    // blocks per horizontal direction (H lines)
    int blk_w;    // blocks per vertical / diagonal direction (W lines)
    size_t vol;   // bytes of one direction volume (W*H*D)
    int store_aux; // cache-policy bits for the path stores (0 = default)
};

typedef __amdgpu_buffer_rsrc_t rsrc_t;

// Path volumes are written non-temporally (buffer aux bit nt = 2).  Measured
// A/B (1080p D=128, interleaved runs, ablation variants 0/13): sgm_paths
// 0.826-0.829 -> 0.747-0.774 ms, and the following wta 0.38 -> 0.35 ms.  With
// default write-back stores the 2.1 GB of L_r lines compete in L2/MALL with
// the 265 MB cost volume that all eight directions re-read.
constexpr int kStoreNT = 2;

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, size_t bytes) {
    // raw buffer: 32-bit byte offsets (every volume is < 4 GiB), hardware
    // range check drops anything at or past `bytes`.
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                             (int)(unsigned)bytes, 0x00020000);
}

template <int NW>
struct Words {
    unsigned w[NW];
};

template <int NW>
// Cache-policy bits of the C loads.  A/B (full frame, in-process): nt (2)
// +8 %, sc0+nt (3) +8 %; sc0 (1), sc0+sc1 (17), 8, 16 within the +-2 % noise.
#ifndef SVA_C_LOAD_AUX
#define SVA_C_LOAD_AUX 0
#endif
__device__ __forceinline__ Words<NW> bload(rsrc_t r, unsigned off) {
    Words<NW> o;
    if constexpr (NW == 1) {
        o.w[0] = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, SVA_C_LOAD_AUX);
    } else if constexpr (NW == 2) {
        auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, SVA_C_LOAD_AUX);
        o.w[0] = v[0]; o.w[1] = v[1];
    } else if constexpr (NW == 3) {
        auto v = __builtin_amdgcn_raw_buffer_load_b96(r, off, 0, SVA_C_LOAD_AUX);
        o.w[0] = v[0]; o.w[1] = v[1]; o.w[2] = v[2];
    } else {
        auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, SVA_C_LOAD_AUX);
        o.w[0] = v[0]; o.w[1] = v[1]; o.w[2] = v[2]; o.w[3] = v[3];
    }
    return o;
}

// VAR (ablation builds only, -DSVA_PATHS_ABLATION): 2 = no stores,
// 3 = no loads, 4 = neither.  Production code is VAR = 0.
template <int NW, int VAR>
__device__ __forceinline__ void bstore(rsrc_t r, unsigned off, const unsigned (&w)[NW], int aux) {
    if constexpr (VAR == 2 || VAR == 4) {
#pragma unroll
        for (int i = 0; i < NW; i++) asm volatile("" ::"v"(w[i]));
    } else if constexpr (VAR == 9) {
        typedef unsigned v2u __attribute__((ext_vector_type(2)));
        switch (aux) {
            case 2: __builtin_amdgcn_raw_buffer_store_b64((v2u){w[0], w[1]}, r, off, 0, 2); break;
            case 16: __builtin_amdgcn_raw_buffer_store_b64((v2u){w[0], w[1]}, r, off, 0, 16); break;
            case 18: __builtin_amdgcn_raw_buffer_store_b64((v2u){w[0], w[1]}, r, off, 0, 18); break;
            case 17: __builtin_amdgcn_raw_buffer_store_b64((v2u){w[0], w[1]}, r, off, 0, 17); break;
            default: __builtin_amdgcn_raw_buffer_store_b64((v2u){w[0], w[1]}, r, off, 0, 0); break;
        }
    } else if constexpr (NW == 1) {
        __builtin_amdgcn_raw_buffer_store_b32(w[0], r, off, 0, kStoreNT);
    } else if constexpr (NW == 2) {
        typedef unsigned v2u __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64((v2u){w[0], w[1]}, r, off, 0, kStoreNT);
    } else if constexpr (NW == 3) {
        typedef unsigned v3u __attribute__((ext_vector_type(3)));
        __builtin_amdgcn_raw_buffer_store_b96((v3u){w[0], w[1], w[2]}, r, off, 0, kStoreNT);
    } else {
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128((v4u){w[0], w[1], w[2], w[3]}, r, off, 0, kStoreNT);
    }
}

__device__ __forceinline__ unsigned add3(unsigned a, unsigned b, unsigned c) {
    unsigned r;
    asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// Cursor over one path line: x and the byte offset of (x, y) in any
// [H][W][D] volume (C and every L_r share the layout, so one offset serves
// both the cost load and the path store).  Offsets advance by a constant
// stride; DIAG lines wrap in x (offset -/+ W*D) and report the wrap.
template <bool DIAG>
struct Cursor {
    int x;
    unsigned off;
    __device__ __forceinline__ bool advance(int rx, unsigned stride, int W, unsigned WD) {
        off += stride;
        if constexpr (DIAG) {
            x += rx;
            const bool hi = x >= W, lo = x < 0;
            x = hi ? x - W : (lo ? x + W : x);
            off = hi ? off - WD : (lo ? off + WD : off);
            return hi || lo;
        }
        return false;
    }
};

// One recurrence step for the lane's DPL disparities.  State A = L(q, .)
// (unnormalised u16 pairs), m = min_k L(q, k) broadcast over the row.
//   u      = min(min(A(d-1), A(d+1)) + P1, A(d), m + P2)      (all >= m)
//   L(p,d) = u + C(p,d) - m  = v_add3_u32(u, c, -(m * 0x10001))
// The add3 is exact per 16-bit half: u_lo >= m makes the low half carry
// exactly once, which the high half's (0xffff - m) absorbs.
template <int DPL>
__device__ __forceinline__ void sgm_step_c(const unsigned (&c)[DPL / 2], unsigned (&A)[DPL / 2],
                                           unsigned& m, unsigned (&ow)[DPL / 4], unsigned P1,
                                           unsigned P2) {
    constexpr int NW = DPL / 4, NP = DPL / 2;
    // neighbours: X = lane k-1's last pair, Y = lane k+1's first pair
    const unsigned X = row_shr1(A[NP - 1], INF2);
    const unsigned Y = row_shl1(A[0], INF2);
    unsigned M[NP];
    M[0] = __builtin_amdgcn_alignbit(A[0], X, 16);
#pragma unroll
    for (int j = 1; j < NP; j++) M[j] = __builtin_amdgcn_alignbit(A[j], A[j - 1], 16);
    const unsigned Qlast = __builtin_amdgcn_alignbit(Y, A[NP - 1], 16);
    const unsigned mP2 = m + P2;
    const unsigned K = 0u - (m | (m << 16));
#pragma unroll
    for (int j = 0; j < NP; j++) {
        const u16x2 q = as_v2(j < NP - 1 ? M[j + 1] : Qlast);
        u16x2 t = vmin2(as_v2(M[j]), q) + splat2(P1);
        t = vmin2(t, as_v2(A[j]));
        t = vmin2(t, splat2(mP2));
        A[j] = add3(as_u32(t), c[j], K);
    }
#pragma unroll
    for (int w = 0; w < NW; w++) ow[w] = pack4(A[2 * w], A[2 * w + 1]);
    u16x2 mm = as_v2(A[0]);
#pragma unroll
    for (int j = 1; j < NP; j++) mm = vmin2(mm, as_v2(A[j]));
    m = row_min_u32(mm.x < mm.y ? mm.x : mm.y);
}

// The same step on u8-packed cost words (DPL/4 dwords of 4 disparities).
template <int DPL>
__device__ __forceinline__ void sgm_step(const unsigned (&cw)[DPL / 4], unsigned (&A)[DPL / 2],
                                         unsigned& m, unsigned (&ow)[DPL / 4], unsigned P1,
                                         unsigned P2) {
    unsigned c[DPL / 2];
#pragma unroll
    for (int w = 0; w < DPL / 4; w++) unpack4(cw[w], c[2 * w], c[2 * w + 1]);
    sgm_step_c<DPL>(c, A, m, ow, P1, P2);
}

// Direction table, identical to oracle svo_direction().
__device__ __forceinline__ void dir_of(int r, int& rx, int& ry) {
    constexpr int T[8][2] = {{1, 0}, {-1, 0}, {0, 1}, {0, -1}, {1, 1}, {-1, -1}, {-1, 1}, {1, -1}};
    rx = T[r][0];
    ry = T[r][1];
}

}  // namespace sgm
}  // namespace sva
