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
//     lanes -- no LDS, no barrier.
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
//
// Two output modes (g.ckpt):
//   0  every direction writes its u8 volume, [8][H][W][D] (sva_paths_d, the
//      stage API the parity tests read): 8 C reads + 8 L writes per disparity.
//   2  the frame route, the tile pipeline: the four
//      diagonal directions write volumes, [4][H][W][D] (directions 4..7 in
//      slots 0..3); horizontal lines store checkpoints every seg columns
//      ([2][H][nsx][D]) and vertical lines every seg rows ([2][nsy][W][D];
//      seg = 2^tile_geom().seg_log2), and wta_hv.hip recomputes those four
//      per tile: 8 C reads + 4 L writes.  (The measured §4.11 experiment,
//      tune::kTileDiagDown / kTileDiagUp = 1, also recomputes a diagonal pair
//      per tile from extra row-checkpoint planes; both constants are 0 in the
//      product.)
//   (Mode 1, the round-2 route of DESIGN.md §4.6 -- six volumes, horizontal
//   checkpoints only, finished by wta_h.hip -- was removed in ABI v5.)
#include "sgm_common.h"
#include "sva_tuning.h"

namespace sva {
namespace {

using namespace sgm;

constexpr int PATH_BLOCK = 256;
constexpr int LINES_PER_BLOCK = PATH_BLOCK / 16;

template <int DPL>
__global__ __launch_bounds__(PATH_BLOCK) void sgm_paths_kernel(const uint8_t* __restrict__ C,
                                                               uint8_t* __restrict__ L8,
                                                               uint8_t* __restrict__ CK,
                                                               uint8_t* __restrict__ CKV,
                                                               PathGeom g) {
    // Horizontal directions (W steps per line, the longest) get the lowest
    // block ids -- every frame's of a batch before any vertical / diagonal
    // block -- and issue priority so they are never the tail.
    int b = blockIdx.x, r, lb, f;
    if (b < 2 * g.blk_h * g.npair) {
        f = b / (2 * g.blk_h);
        b -= f * 2 * g.blk_h;
        r = b / g.blk_h;
        lb = b - r * g.blk_h;
        __builtin_amdgcn_s_setprio(1);
    } else {
        // band-major: the six vertical / diagonal directions of a 16-line band
        // are adjacent in dispatch order, so the waves that read a cost row
        // (its vertical band and the diagonal bands crossing it) start
        // together and progress at a similar pace: more of the second and
        // third reads of a row come from the caches.  A/B in-process at 1080p
        // D=128 (profiles/r03_v3): kernel 0.616-0.622 -> 0.594-0.599 ms, frame
        // 261-263K -> 266-267K Mdisp/s; direction-major had the first-dispatched
        // direction hundreds of steps ahead.
        // (a batch's frames follow one another, each band-major)
        b -= 2 * g.blk_h * g.npair;
        f = b / (6 * g.blk_w);
        b -= f * 6 * g.blk_w;
        r = 2 + b % 6;
        lb = b / 6;
    }
    C += (size_t)f * g.cstr;
    L8 += (size_t)f * g.lstr;
    if (g.ckpt) {
        CK += (size_t)f * g.ckstr;
        CKV += (size_t)f * g.ckvstr;
    }
    const int line = lb * LINES_PER_BLOCK + (threadIdx.x >> 4);
    const int k = threadIdx.x & 15;
    const int nlines = r < 2 ? g.H : g.W;
    if (line >= nlines) return;  // whole 16-lane row leaves together
    int rx, ry;
    dir_of(r, rx, ry);
    const rsrc_t rC = make_rsrc(C, g.vol);
    // the tile pipeline's checkpoint segment (§4.9), rows and columns
    constexpr int SL = DPL <= 8 ? tune::kWtahvTileLog2 : tune::kWtahvTileLog2Wide;
    constexpr bool DOWN = diag_ckpt_down(DPL), UP = diag_ckpt_up(DPL);
    if (r >= 4 && g.ckpt && (ry > 0 ? DOWN : UP)) {
        // tile pipeline, diagonals recomputed per tile: row
        // checkpoints only, in the vertical checkpoint block after the two
        // vertical planes: the down pair (4, 6), then the up pair (5, 7)
        const int plane = ry > 0 ? 2 + (r == 4 ? 0 : 1) : 2 + (DOWN ? 2 : 0) + (r == 5 ? 0 : 1);
        const rsrc_t rCK = make_rsrc(CKV + (size_t)plane * g.ckvvol, g.ckvvol);
        path_line<DPL, true, pf_v<DPL>(), 3, SL>(rC, rC, g, rx, ry, line, k, rCK);
    } else if (r >= 4) {
        // volume slot: every direction (8 volumes), or the tile pipeline's
        // diagonals that stay volumes, in direction order
        const int slot = !g.ckpt ? r
                       : DOWN ? (r == 5 ? 0 : 1)          // 5, 7 (UP is then off here)
                       : UP ? (r == 4 ? 0 : 1)            // 4, 6
                       : r - 4;
        const rsrc_t rL = make_rsrc(L8 + (size_t)slot * g.vol, g.vol);
        path_line<DPL, true, pf_v<DPL>()>(rC, rL, g, rx, ry, line, k, rL);
    } else if (r >= 2 && g.ckpt) {
        const rsrc_t rCK = make_rsrc(CKV + (size_t)(r - 2) * g.ckvvol, g.ckvvol);
        path_line<DPL, false, pf_v<DPL>(), 2, SL>(rC, rC, g, rx, ry, line, k, rCK);
    } else if (r >= 2) {
        const rsrc_t rL = make_rsrc(L8 + (size_t)r * g.vol, g.vol);
        path_line<DPL, false, pf_v<DPL>()>(rC, rL, g, rx, ry, line, k, rL);
    } else if (g.ckpt) {
        const rsrc_t rCK = make_rsrc(CK + (size_t)r * g.ckvol, g.ckvol);
        path_line<DPL, false, pf_h<DPL>(), 1, SL>(rC, rC, g, rx, ry, line, k, rCK);
    } else {
        const rsrc_t rL = make_rsrc(L8 + (size_t)r * g.vol, g.vol);
        path_line<DPL, false, pf_h<DPL>()>(rC, rL, g, rx, ry, line, k, rL);
    }
}

}  // namespace

bool paths_supported(int D) { return D == 64 || D == 128 || D == 192 || D == 256; }

TileGeom tile_geom(int W, int H, int D) {
    TileGeom t;
    t.seg_log2 = D <= 128 ? tune::kWtahvTileLog2 : tune::kWtahvTileLog2Wide;
    const int seg = 1 << t.seg_log2;
    t.ntx = (W + 15) >> 4;
    t.nty = (H + seg - 1) >> t.seg_log2;
    t.nsx = (W + seg - 1) >> t.seg_log2;
    t.hck_bytes = 2 * (size_t)H * t.nsx * D;
    t.vck_bytes = 2 * (size_t)t.nty * W * D;
    const int dpl = D / 16;
    const int ndp = (diag_ckpt_down(dpl) ? 2 : 0) + (diag_ckpt_up(dpl) ? 2 : 0);
    t.dck_bytes = (size_t)ndp / 2 * t.vck_bytes;   // one plane per recomputed diagonal
    t.nvol = 4 - ndp;
    return t;
}

hipError_t launch_paths(Ctx& c, const uint8_t* C, int W, int H, int D, int P1, int P2,
                        uint8_t* L8, uint8_t* CK, uint8_t* CKV, int npair) {
    DispatchTimer t(c, "sgm_paths");
    PathGeom g;
    g.W = W; g.H = H; g.D = D; g.P1 = P1; g.P2 = P2;
    g.blk_h = (H + LINES_PER_BLOCK - 1) / LINES_PER_BLOCK;
    g.blk_w = (W + LINES_PER_BLOCK - 1) / LINES_PER_BLOCK;
    g.vol = (size_t)W * H * D;
    if ((CK == nullptr) != (CKV == nullptr)) return hipErrorInvalidValue;
    g.ckpt = CK ? 2 : 0;
    const TileGeom tg = tile_geom(W, H, D);
    g.nsy = tg.nty;
    g.ckvvol = tg.vck_bytes / 2;        // one row-checkpoint plane
    g.ns = tg.nsx;
    g.ckvol = tg.hck_bytes / 2;
    if (g.vol >= (size_t)1 << 32) return hipErrorInvalidValue;  // 32-bit buffer offsets
    // a batch: npair frames, each with its buffers packed one after another
    if (npair < 1 || (npair > 1 && !CK)) return hipErrorInvalidValue;
    g.npair = npair;
    g.cstr = g.vol;
    g.lstr = (size_t)tg.nvol * g.vol;
    g.ckstr = tg.hck_bytes;
    g.ckvstr = tg.vck_bytes + tg.dck_bytes;
    dim3 grid((unsigned)((2 * g.blk_h + 6 * g.blk_w) * npair));
#define SVA_PATHS_LAUNCH(DPL_)                                                               \
    hipExtLaunchKernelGGL(sgm_paths_kernel<DPL_>, grid, dim3(PATH_BLOCK), 0, c.stream, t.start, \
                          t.stop, 0, C, L8, CK, CKV, g);                                    \
    t.used = true
    switch (D) {
        case 64: SVA_PATHS_LAUNCH(4); break;
        case 128: SVA_PATHS_LAUNCH(8); break;
        case 192: SVA_PATHS_LAUNCH(12); break;
        case 256: SVA_PATHS_LAUNCH(16); break;
        default: return hipErrorInvalidValue;
    }
#undef SVA_PATHS_LAUNCH
    return hipGetLastError();
}

}  // namespace sva
