// sgm_common.h -- device pieces of the 8-path aggregation shared by the path
// kernel (sgm_paths.hip) and the tile recompute + WTA kernel (wta_hv.hip).
// DESIGN.md §4.3 / §4.9.
#pragma once

#include <utility>

#include "sva_device.h"
#include "sva_internal.h"
#include "sva_tuning.h"

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
    int ckpt;     // 2: the tile pipeline's checkpoints (below); 0: eight volumes
    int ns;       // horizontal checkpoint segments per row, ceil(W / seg)
    size_t ckvol; // bytes of one horizontal checkpoint plane (H*ns*D)
    int nsy;      // vertical checkpoint segments per column, ceil(H / seg)
    size_t ckvvol; // bytes of one vertical checkpoint plane (nsy*W*D)
    // batched launch: npair frames of the same shape, frame
    // f's buffers at C + f*cstr, L8 + f*lstr, CK + f*ckstr, CKV + f*ckvstr
    int npair;
    size_t cstr, lstr, ckstr, ckvstr;
};

// Tile-pipeline checkpoints.  With g.ckpt set, the
// horizontal and vertical directions write no L_r volume: direction 0 (left
// to right) stores L(x) at the last column of every seg-wide segment but the
// row's last, direction 1 (right to left) at the first column of every
// segment but the first ([2][H][ns][D] u8), and the vertical directions the
// same along their columns ([2][nsy][W][D] u8).  wta_hv.hip re-runs all four
// recurrences tile by tile from these states, so their L_r bytes never reach
// HBM.

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

// Cache-policy bits of the C loads (tune::kCLoadAux).
template <int NW, int AUX = tune::kCLoadAux>
__device__ __forceinline__ Words<NW> bload(rsrc_t r, unsigned off) {
    Words<NW> o;
    if constexpr (NW == 1) {
        o.w[0] = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, AUX);
    } else if constexpr (NW == 2) {
        auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, AUX);
        o.w[0] = v[0]; o.w[1] = v[1];
    } else if constexpr (NW == 3) {
        auto v = __builtin_amdgcn_raw_buffer_load_b96(r, off, 0, AUX);
        o.w[0] = v[0]; o.w[1] = v[1]; o.w[2] = v[2];
    } else {
        auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
        o.w[0] = v[0]; o.w[1] = v[1]; o.w[2] = v[2]; o.w[3] = v[3];
    }
    return o;
}

// AUX = cache-policy bits of the store (kStoreNT for the streamed L_r volumes).
template <int NW, int AUX = kStoreNT>
__device__ __forceinline__ void bstore(rsrc_t r, unsigned off, const unsigned (&w)[NW]) {
    if constexpr (NW == 1) {
        __builtin_amdgcn_raw_buffer_store_b32(w[0], r, off, 0, AUX);
    } else if constexpr (NW == 2) {
        typedef unsigned v2u __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64((v2u){w[0], w[1]}, r, off, 0, AUX);
    } else if constexpr (NW == 3) {
        typedef unsigned v3u __attribute__((ext_vector_type(3)));
        __builtin_amdgcn_raw_buffer_store_b96((v3u){w[0], w[1], w[2]}, r, off, 0, AUX);
    } else {
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128((v4u){w[0], w[1], w[2], w[3]}, r, off, 0, AUX);
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

// Three-input packed u16 min through gfx950's v_pk_minimum3_f16.  Exact for
// this kernel's operands: non-negative integers below 1024 (L <= 254, m + P2
// <= 447), i.e. f16 zero/denormal bit patterns, which order like the
// integers (kernels keep f16 denormals: .amdhsa_float_denorm_mode_16_64 3).
// INF (0x7fff, a NaN pattern) never reaches it: the row-end neighbour only
// enters through the integer v_pk_min_u16 with a real neighbour.
__device__ __forceinline__ unsigned min3_u16x2(unsigned a, unsigned b, unsigned c) {
    unsigned r;
    asm("v_pk_minimum3_f16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// Minimum over the 2*NP u16 halves of A (values below 1024): a tree of
// three-input packed mins, then the two halves.
template <int NP>
__device__ __forceinline__ unsigned lane_min_u16(const unsigned (&A)[NP]) {
    unsigned mm[NP];
#pragma unroll
    for (int j = 0; j < NP; j++) mm[j] = A[j];
    int n = NP;
#pragma unroll
    for (int it = 0; it < 4; it++) {
        if (n > 1) {
            int o = 0, i = 0;
#pragma unroll
            for (int q = 0; q < 8; q++) {
                if (i + 2 < n) { mm[o++] = min3_u16x2(mm[i], mm[i + 1], mm[i + 2]); i += 3; }
                else if (i + 1 < n) { mm[o++] = as_u32(vmin2(as_v2(mm[i]), as_v2(mm[i + 1]))); i += 2; }
                else if (i < n) { mm[o++] = mm[i]; i += 1; }
            }
            n = o;
        }
    }
    const u16x2 mf = as_v2(mm[0]);
    return mf.x < mf.y ? mf.x : mf.y;
}

// ---- pair layout of the recurrence state (tune::kSplitPairs, §4.14) -------
// Lane k holds its DPL disparities as NP = DPL/2 packed u16 pairs.  Local
// disparity e (0 <= e < DPL) sits in pair pair_of(e), half half_of(e);
// pair_d(j, h) is the inverse.  Split: pair j = (e = j, e = j + NP).
// Adjacent: pair j = (2j, 2j + 1).
template <int DPL> __host__ __device__ constexpr int pair_d(int j, int h) {
    return tune::kSplitPairs ? j + h * (DPL / 2) : 2 * j + h;
}
template <int DPL> __host__ __device__ constexpr int pair_of(int e) {
    return tune::kSplitPairs ? e % (DPL / 2) : e >> 1;
}
template <int DPL> __host__ __device__ constexpr int half_of(int e) {
    return tune::kSplitPairs ? e / (DPL / 2) : e & 1;
}

// d-ordered u8 words (C, L_r volumes, checkpoints) -> state-layout pairs:
// one v_perm per pair in both layouts.
template <int DPL>
__device__ __forceinline__ void words_to_pairs(const unsigned (&w)[DPL / 4], unsigned (&A)[DPL / 2]) {
    constexpr int NW = DPL / 4, NP = DPL / 2;
    if constexpr (tune::kSplitPairs != 0) {
#pragma unroll
        for (int j = 0; j < NP; j++) {
            constexpr unsigned Z = 0x0cu;     // v_perm selector: zero byte
            const int el = j, eh = j + NP;
            const unsigned sel = (unsigned)(el & 3) | (Z << 8) | ((4u + (unsigned)(eh & 3)) << 16) | (Z << 24);
            A[j] = __builtin_amdgcn_perm(w[eh >> 2], w[el >> 2], sel);
        }
    } else {
#pragma unroll
        for (int q = 0; q < NW; q++) unpack4(w[q], A[2 * q], A[2 * q + 1]);
    }
}

// State-layout pairs (values < 256) -> d-ordered u8 words.  Split: pairs
// (2i, 2i + 1) first merge into T_i = (A_2i.lo, A_2i+1.lo, A_2i.hi,
// A_2i+1.hi) bytes, then each word takes two byte pairs of two T's.
template <int DPL>
__device__ __forceinline__ void pairs_to_words(const unsigned (&A)[DPL / 2], unsigned (&ow)[DPL / 4]) {
    constexpr int NW = DPL / 4, NP = DPL / 2;
    if constexpr (tune::kSplitPairs != 0) {
        unsigned T[NP / 2];
#pragma unroll
        for (int i = 0; i < NP / 2; i++) T[i] = __builtin_amdgcn_perm(A[2 * i + 1], A[2 * i], 0x06020400u);
        if constexpr (NP == 2) {
            ow[0] = T[0];                     // (d0, d2), (d1, d3) -> d0 d1 d2 d3
        } else {
#pragma unroll
            for (int q = 0; q < NW; q++) {
                const int e0 = 4 * q, e2 = 4 * q + 2;
                const int a = (e0 % NP) / 2, ha = e0 / NP, b = (e2 % NP) / 2, hb = e2 / NP;
                const unsigned sel = (unsigned)(2 * ha) | ((unsigned)(2 * ha + 1) << 8) |
                                     ((unsigned)(4 + 2 * hb) << 16) | ((unsigned)(5 + 2 * hb) << 24);
                ow[q] = __builtin_amdgcn_perm(T[b], T[a], sel);
            }
        }
    } else {
#pragma unroll
        for (int w = 0; w < NW; w++) ow[w] = pack4(A[2 * w], A[2 * w + 1]);
    }
}

// One recurrence step for the lane's DPL disparities.  State A = L(q, .)
// (unnormalised u16 pairs), m = min_k L(q, k) broadcast over the row.
//   u      = min(min(A(d-1), A(d+1)) + P1, A(d), m + P2)      (all >= m)
//   L(p,d) = u + C(p,d) - m  = v_add3_u32(u, c, -(m * 0x10001))
// The add3 is exact per 16-bit half: u_lo >= m makes the low half carry
// exactly once, which the high half's (0xffff - m) absorbs.
// Row-edge registers of the d-1 / d+1 neighbour shifts.  A DPP row shift
// leaves the lane without a source (lane 0 for row_shr, 15 for row_shl) at
// its old value, so registers that start as INF keep INF there for the whole
// line when each step's shift takes the previous step's register as its old
// value: no INF re-materialisation per step.
struct Edges {
    unsigned X = INF2, Y = INF2;
};

template <int DPL, bool PIN = false>
__device__ __forceinline__ void sgm_step_c(const unsigned (&c)[DPL / 2], unsigned (&A)[DPL / 2],
                                           unsigned& m, unsigned (&ow)[DPL / 4], unsigned P1,
                                           unsigned P2, Edges& e) {
    constexpr int NP = DPL / 2;
    // neighbours: X = lane k-1's last pair, Y = lane k+1's first pair (its
    // high half holds L(d0 - 1) and its low half L(d0 + DPL) in both layouts)
    e.X = row_shr1(A[NP - 1], e.X);
    e.Y = row_shl1(A[0], e.Y);
    const unsigned X = e.X, Y = e.Y;
    // lo[j] / hi[j]: the pairs whose min is pair j's min(A(d-1), A(d+1))
    unsigned lo[NP], hi[NP];
    if constexpr (tune::kSplitPairs != 0) {
        // pair j = (j, j + NP): its d-1 pair is pair j-1 and its d+1 pair is
        // pair j+1, whole registers, except (X.hi, A[NP-1].lo) for j = 0 and
        // (A[0].hi, Y.lo) for j = NP-1
#pragma unroll
        for (int j = 0; j < NP; j++) {
            lo[j] = j == 0 ? __builtin_amdgcn_alignbit(A[NP - 1], X, 16) : A[j - 1];
            hi[j] = j == NP - 1 ? __builtin_amdgcn_alignbit(Y, A[0], 16) : A[j + 1];
        }
    } else {
        // pair j = (2j, 2j+1): d-1 is (A[j-1].hi, A[j].lo), d+1 the next one
        unsigned M[NP];
        M[0] = __builtin_amdgcn_alignbit(A[0], X, 16);
#pragma unroll
        for (int j = 1; j < NP; j++) M[j] = __builtin_amdgcn_alignbit(A[j], A[j - 1], 16);
        const unsigned Qlast = __builtin_amdgcn_alignbit(Y, A[NP - 1], 16);
#pragma unroll
        for (int j = 0; j < NP; j++) {
            lo[j] = M[j];
            hi[j] = j < NP - 1 ? M[j + 1] : Qlast;
        }
    }
    // K = -(m * 0x10001) in one v_mul_i32_i24 (m < 2^10; the literal's low 24
    // bits are -65537), and m + P2 in both halves = P2 * 0x10001 - K: two VALU
    // where m | m << 16, its negation and the sum took three plus a copy of P2
    unsigned K, mP2;
    asm("v_mul_i32_i24_e32 %0, 0xfffeffff, %1" : "=v"(K) : "v"(m));
    if constexpr (tune::kStepMadP2 != 0) {
        // m + P2 in both halves straight from m (v_mad_u32_u24: m * 0x10001 +
        // P2 * 0x10001, beside K instead of after it): one dependent
        // instruction less on the step's critical path m -> min3 -> add3
        // (asm: in plain C the compiler splits m * 0x10001 into a shift-add;
        // here it re-materialises the uniform P2 * 0x10001 with one v_mov
        // per step, off the critical path)
        asm("v_mad_u32_u24 %0, %1, %2, %3" : "=&v"(mP2) : "v"(m), "s"(0x10001u), "v"(P2 * 0x10001u));
    } else {
        mP2 = P2 * 0x10001u - K;
    }
    // Stage-major over the NP independent pairs, and a min TREE below: each
    // packed op's result is consumed one pair later, not by the next
    // instruction (gfx950 puts an s_nop between dependent VOP3P ops).
    u16x2 t[NP];
#pragma unroll
    for (int j = 0; j < NP; j++) t[j] = vmin2(as_v2(lo[j]), as_v2(hi[j]));
    unsigned tp[NP];
    if constexpr (tune::kStepAddU32 != 0) {
        // + P1 in both halves as ONE 32-bit add (VOP2, full issue rate; the
        // packed v_pk_add_u16 is a 64-bit VOP3P encoding that issues at half
        // rate, profiles/r06_v1/microbench_valu.txt): t <= 448 + 193 per half
        // (INF never reaches t, see min3_u16x2), so the low half never carries
        const unsigned P1x2 = P1 * 0x10001u;
#pragma unroll
        for (int j = 0; j < NP; j++) tp[j] = as_u32(t[j]) + P1x2;
    } else {
#pragma unroll
        for (int j = 0; j < NP; j++) tp[j] = as_u32(t[j] + splat2(P1));
    }
#pragma unroll
    for (int j = 0; j < NP; j++) A[j] = add3(min3_u16x2(tp[j], A[j], mP2), c[j], K);
    pairs_to_words<DPL>(A, ow);
    m = row_min_u32<PIN>(lane_min_u16<NP>(A));
}

template <int DPL>
__device__ __forceinline__ void sgm_step_c(const unsigned (&c)[DPL / 2], unsigned (&A)[DPL / 2],
                                           unsigned& m, unsigned (&ow)[DPL / 4], unsigned P1,
                                           unsigned P2) {
    Edges e;
    sgm_step_c<DPL>(c, A, m, ow, P1, P2, e);
}

// The same step on u8-packed cost words (DPL/4 dwords of 4 disparities).
template <int DPL, bool PIN = false>
__device__ __forceinline__ void sgm_step(const unsigned (&cw)[DPL / 4], unsigned (&A)[DPL / 2],
                                         unsigned& m, unsigned (&ow)[DPL / 4], unsigned P1,
                                         unsigned P2, Edges& e) {
    unsigned c[DPL / 2];
    words_to_pairs<DPL>(cw, c);
    sgm_step_c<DPL, PIN>(c, A, m, ow, P1, P2, e);
}

// Direction table, identical to oracle svo_direction().
__device__ __forceinline__ void dir_of(int r, int& rx, int& ry) {
    constexpr int T[8][2] = {{1, 0}, {-1, 0}, {0, 1}, {0, -1}, {1, 1}, {-1, -1}, {-1, 1}, {1, -1}};
    rx = T[r][0];
    ry = T[r][1];
}

// Prefetch depth in steps, per line kind (tune::kPf*, with the A/B that
// chose each value).
template <int DPL> constexpr int pf_h() {
    return DPL == 4 ? tune::kPfH4 : DPL == 8 ? tune::kPfH8 : DPL == 12 ? tune::kPfH12 : tune::kPfH16;
}
template <int DPL> constexpr int pf_v() {
    return DPL == 4 ? tune::kPfV4 : DPL == 8 ? tune::kPfV8 : DPL == 12 ? tune::kPfV12 : tune::kPfV16;
}


// One path line over a materialised cost volume C.  CKPT
// 1 (horizontal lines) / 2 (vertical lines) / 3 (down-diagonal lines): store
// checkpoints every 2^SL pixels (rows for 2 and 3) to rCK instead of the full
// L_r line to rL (SL is a template parameter: a runtime segment test cost the
// latency-bound lines of small frames 20 %).
template <int DPL, bool DIAG, int PF, int CKPT = 0, int SL = 0>
__device__ __forceinline__ void path_line(rsrc_t rC, rsrc_t rL, const PathGeom& g, int rx, int ry,
                                          int line, int k, rsrc_t rCK) {
    constexpr int NW = DPL / 4, NP = DPL / 2;
    const int W = g.W, H = g.H, D = g.D;
    const unsigned P1 = (unsigned)g.P1, P2 = (unsigned)g.P2;
    const int steps = ry == 0 ? W : H;
    const unsigned WD = (unsigned)W * (unsigned)D;
    const unsigned stride = (unsigned)((ry * W + rx) * D);
    int x0, y0;
    if (ry == 0) { y0 = line; x0 = rx > 0 ? 0 : W - 1; }
    else { y0 = ry > 0 ? 0 : H - 1; x0 = line; }
    Cursor<false> cc;
    cc.x = x0;
    cc.off = ((unsigned)y0 * (unsigned)W + (unsigned)x0) * (unsigned)D + (unsigned)(k * DPL);
    // Prefetch cursor: runs PF steps ahead and may run past the line's end;
    // those loads land in-range garbage or, past the volume, the buffer range
    // check returns 0 -- never consumed either way.
    Cursor<false> pc = cc;
    // Checkpoint stores at compile-time step positions (tune::kStaticCkptHits):
    // with PF a multiple of the segment, step p of every PF-step iteration
    // sits at the same place in the segment grid once the line is preceded by
    // `lead` steps (0 for lines that run with x or y, (-W or -H) mod SEG for
    // the others).  A lead step sees cost 0 from zero state, and zero state
    // with cost 0 stays zero (u = min(P1, 0, P2) = 0), so the line's first
    // real pixel still starts from L = C.  The runtime test this replaces put
    // a taken branch on every step (640x480: horizontal lines alone 0.065 ->
    // 0.050 ms with static positions, profiles/r05_v5/ckpt_hits/).  Only the
    // D = 64 kernel takes it (tune::kStaticCkptHitsMaxDpl).
    constexpr bool STATIC_HITS = DPL <= tune::kStaticCkptHitsMaxDpl && (CKPT == 1 || CKPT == 2) &&
                                 SL > 0 && PF % (1 << SL) == 0;
    int lead = 0;
    if constexpr (STATIC_HITS) {
        constexpr int SEG = 1 << SL;
        lead = CKPT == 1 ? (rx > 0 ? 0 : (SEG - W % SEG) % SEG) : (ry > 0 ? 0 : (SEG - H % SEG) % SEG);
        pc.off -= (unsigned)lead * stride;
    }
    const int nsteps = steps + lead;
    // Diagonal lines wrap without per-step x tracking.  Line l visits
    // x = (l + rx*t) mod W and wraps between pixels s and s+1 when s + 1 =
    // W - l (rx = +1) or l + 1 (rx = -1), then every W steps: tw* hold each
    // lane's next wrap pixel for the compute and prefetch cursors.  A wave's
    // four lines are consecutive, so their wraps fall in one 4-step window per
    // period that starts at the wave-uniform pixel T*; only window steps pay
    // per-lane work (one uniform branch), the others a scalar compare.  (The
    // x tracking had cost ~29 VALU per diagonal step: 78 against 49 for a
    // vertical step.)  Images narrower than 4 columns check every step.
    int twc = 0, twp = 0, Tc = 0, Tp = 0;
    if constexpr (DIAG) {
        const int j = (int)((threadIdx.x >> 4) & 3);          // row of the line in its wave
        const int l0 = __builtin_amdgcn_readfirstlane(line - j);
        twc = twp = rx > 0 ? W - line : line + 1;
        Tc = Tp = rx > 0 ? W - l0 - 3 : l0 + 1;
    }
    const bool narrow = W < 4;

    unsigned A[NP];
#pragma unroll
    for (int j = 0; j < NP; j++) A[j] = 0u;   // L(q) = 0, m = 0  =>  L = C
    unsigned m = 0u;
    Edges edges;

    Words<NW> ring[PF];
#pragma unroll
    for (int p = 0; p < PF; p++) {
        ring[p] = bload<NW>(rC, pc.off);
        if constexpr (STATIC_HITS) {   // lead steps: cost 0 (lead < SEG <= PF)
#pragma unroll
            for (int w = 0; w < NW; w++) ring[p].w[w] = p < lead ? 0u : ring[p].w[w];
        }
        pc.off += stride;
        if constexpr (DIAG) {   // the advance past pixel PF-1 is checked by step 0
            if (p < PF - 1) {
                const bool w = p + 1 == twp;
                const unsigned fixed = rx > 0 ? pc.off - WD : pc.off + WD;
                pc.off = w ? fixed : pc.off;
                twp = w ? twp + W : twp;
            }
        }
    }
    if constexpr (DIAG) {       // prefetch windows the prologue has fully handled
        while (Tp + 3 < PF) Tp += W;
    }

    // One step consumes ring slot p in place (loaded PF steps ago) and only
    // then refills that slot with the load for step t+PF, so the old and new
    // values never overlap and the slot keeps its registers: no copies, and
    // every wait is for a load issued ~PF steps earlier.  (Refilling first
    // made hipcc copy the whole ring at the loop head behind vmcnt(1..3).)
    auto step = [&](int p, bool refill, int ts) {
        unsigned cw[NW];
#pragma unroll
        for (int w = 0; w < NW; w++) cw[w] = ring[p].w[w];
        unsigned ow[NW];
        sgm_step<DPL>(cw, A, m, ow, P1, P2, edges);
        if constexpr (CKPT == 1 && STATIC_HITS) {
            // the last pixel of a segment (rx > 0) or its first (rx < 0) is at
            // step p = SEG - 1 of every SEG steps (lead above); not the row's
            // last / first column
            constexpr int SEG = 1 << SL;
            if ((p & (SEG - 1)) == SEG - 1) {
                const int x = rx > 0 ? ts : W - 1 - (ts - lead);
                if (rx > 0 ? x + 1 < W : x > 0)
                    bstore<NW, tune::kCkptStoreAux>(rCK, ((unsigned)(y0 * g.ns + (x >> SL)) * (unsigned)D +
                                             (unsigned)(k * DPL)), ow);
            }
        } else if constexpr (CKPT == 2 && STATIC_HITS) {
            constexpr int SEG = 1 << SL;
            if ((p & (SEG - 1)) == SEG - 1) {
                const int y = ry > 0 ? ts : H - 1 - (ts - lead);
                if (ry > 0 ? y + 1 < H : y > 0)
                    bstore<NW, tune::kCkptStoreAux>(rCK, ((unsigned)((y >> SL) * W + x0) * (unsigned)D +
                                             (unsigned)(k * DPL)), ow);
            }
        } else if constexpr (CKPT == 1) {
            // ts is the (wave-uniform) step index; x the pixel just computed
            const int x = rx > 0 ? ts : W - 1 - ts;
            constexpr int SEG = 1 << SL;
            const bool hit = rx > 0 ? (((x + 1) & (SEG - 1)) == 0 && x + 1 < W)
                                    : ((x & (SEG - 1)) == 0 && x > 0);
            // out of line (the common step falls through; 640x480 / 960x540 D=128
            // -3 %, 1080p within 0.2 %, profiles/r05_v5/slot_order/he_*)
            if (__builtin_expect(hit, 0))   // default policy (tune::kCkptStoreAux): the WTA kernel reads these back soon
                bstore<NW, tune::kCkptStoreAux>(rCK, ((unsigned)(y0 * g.ns + (x >> SL)) * (unsigned)D +
                                         (unsigned)(k * DPL)), ow);
        } else if constexpr (CKPT == 3) {
            // diagonal line with row checkpoints: a down
            // line (ry = +1) keeps the last row of every row segment but the
            // image's last, an up line (ry = -1) the first row of every
            // segment but the first, in the row checkpoint plane [nsy][W][D]
            // at this pixel's column: the pixel's volume offset minus the
            // rows the plane does not hold
            const int y = ry > 0 ? ts : H - 1 - ts;
            constexpr int SEG = 1 << SL;
            const bool hit = ry > 0 ? (((y + 1) & (SEG - 1)) == 0 && y + 1 < H)
                                    : ((y & (SEG - 1)) == 0 && y > 0);
            if (__builtin_expect(hit, 0))
                bstore<NW, tune::kCkptStoreAux>(rCK, cc.off - (unsigned)(y - (y >> SL)) * WD, ow);
        } else if constexpr (CKPT == 2) {
            // vertical line x0: direction 2 (down) keeps the last row of every
            // row segment but the column's last, direction 3 (up) the first row
            // of every segment but the first; [nsy][W][D] per direction
            const int y = ry > 0 ? ts : H - 1 - ts;
            constexpr int SEG = 1 << SL;
            const bool hit = ry > 0 ? (((y + 1) & (SEG - 1)) == 0 && y + 1 < H)
                                    : ((y & (SEG - 1)) == 0 && y > 0);
            if (__builtin_expect(hit, 0))
                bstore<NW, tune::kCkptStoreAux>(rCK, ((unsigned)((y >> SL) * W + x0) * (unsigned)D +
                                         (unsigned)(k * DPL)), ow);
        } else {
            bstore<NW>(rL, cc.off, ow);
        }
        cc.off += stride;
        if constexpr (DIAG) {
            // One uniform branch, taken only on the steps of a wrap window of
            // either cursor: the compute cursor restarts where x wraps (L = C),
            // and the prefetch cursor's previous advance (past pixel
            // ts + PF - 1) is corrected before its next load.
            const int ec = ts + 1 - Tc;
            const int ep = ts + PF - Tp;
            const bool cev = narrow || (unsigned)ec < 4u;
            const bool pev = refill && (narrow || (unsigned)ep < 4u);
            // (laid out of line: the common step falls through instead of
            // taking a branch around the block; tile-entry A/B, 640x480 D=64
            // -1.6 %, 1080p D=128 -0.4 %, profiles/r05_v5/slot_order/ex_*)
            if (__builtin_expect(cev || pev, 0)) {
                if (cev) {
                    const bool wrapped = ts + 1 == twc;
                    const unsigned fixed = rx > 0 ? cc.off - WD : cc.off + WD;
                    cc.off = wrapped ? fixed : cc.off;
                    twc = wrapped ? twc + W : twc;
#pragma unroll
                    for (int j = 0; j < NP; j++) A[j] = wrapped ? 0u : A[j];
                    m = wrapped ? 0u : m;
                    if (ec == 3) Tc += W;
                }
                if (pev) {
                    const bool wrapped = ts + PF == twp;
                    const unsigned fixed = rx > 0 ? pc.off - WD : pc.off + WD;
                    pc.off = wrapped ? fixed : pc.off;
                    twp = wrapped ? twp + W : twp;
                    if (ep == 3) Tp += W;
                }
            }
        }
        if (refill) {
            __builtin_amdgcn_sched_barrier(0);
            ring[p] = bload<NW>(rC, pc.off);
            pc.off += stride;                // wrap corrected by the next step
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    int t = 0;
    for (; t + PF <= nsteps; t += PF) {
#pragma unroll
        for (int p = 0; p < PF; p++) step(p, true, t + p);
    }
    // tail: fewer than PF steps left, all already in the ring
#pragma unroll
    for (int p = 0; p < PF; p++)
        if (t + p < nsteps) step(p, false, t + p);
}


// ---- shared by the final kernels (wta.hip, wta_hv.hip) ---------------------

// S += the d-ordered u8 words w, in the state's pair layout.
template <int NW>
__device__ __forceinline__ void unpack_add(const unsigned (&w)[NW], unsigned (&S)[2 * NW]) {
    unsigned a[2 * NW];
    words_to_pairs<4 * NW>(w, a);
#pragma unroll
    for (int j = 0; j < 2 * NW; j++) S[j] += a[j];   // packed add: S <= 8 * 255 < 2^16 per half, no carry
}

// Path state from a u8 checkpoint: A = L(q) as packed pairs, m = min_k L(q).
// Padded disparities (PAD) held L >= 255 in the path kernel, which the u8
// checkpoint truncated; they restart at 255.  Every real disparity evolves
// the same from 255 as from the true value: a padded neighbour enters only
// as A + P1 >= 255 >= m + P2 (m <= 62), and never sets the row minimum.
template <int DPL, bool PAD, bool PIN = false>
__device__ __forceinline__ void state_from_words(const Words<DPL / 4>& w, unsigned (&A)[DPL / 2],
                                                 unsigned& m, const unsigned (&padm)[DPL / 2]) {
    constexpr int NP = DPL / 2;
    words_to_pairs<DPL>(w.w, A);
    if constexpr (PAD) {
#pragma unroll
        for (int j = 0; j < NP; j++) A[j] |= padm[j] & 0x00ff00ffu;   // A < 256: OR = max
    }
    if constexpr (tune::kStateMinTree) {
        m = row_min_u32<PIN>(lane_min_u16<NP>(A));
    } else {
        unsigned mm = 0xffffffffu;
#pragma unroll
        for (int j = 0; j < NP; j++) {
            const unsigned lo = A[j] & 0xffffu, hi = A[j] >> 16;
            mm = mm < lo ? mm : lo;
            mm = mm < hi ? mm : hi;
        }
        m = row_min_u32<PIN>(mm);
    }
}
template <int DPL, bool PAD, bool PIN = false>
__device__ __forceinline__ void load_state(rsrc_t r, unsigned off, unsigned (&A)[DPL / 2],
                                           unsigned& m, const unsigned (&padm)[DPL / 2]) {
    state_from_words<DPL, PAD, PIN>(bload<DPL / 4>(r, off), A, m, padm);
}

}  // namespace sgm
}  // namespace sva
