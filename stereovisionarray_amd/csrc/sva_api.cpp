// sva_api.cpp -- the C-ABI of libsva.so (declared in include/sva.h).
//
// Host C++ only: argument validation, per-context device/stream/workspace
// management, host<->device staging for the host-pointer entry points, the
// hipEvent kernel timer and the multi-context batch driver.  Every compute
// step is one of the HIP kernels in this directory; there is no CPU path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <functional>
#include <thread>
#include <vector>

#include "sva_internal.h"
#include "sva_tuning.h"

using namespace sva;

// ------------------------------------------------------------ internals --
namespace sva {

hipEvent_t KernelTimer::get_event() {
    if (!pool.empty()) {
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

void KernelTimer::begin(hipStream_t s, const char*, hipEvent_t* start_out) {
    hipEvent_t e = get_event();
    if (e && hipEventRecord(e, s) == hipSuccess) *start_out = e;
    else *start_out = nullptr;
}

void KernelTimer::end(hipStream_t s, const char* name, hipEvent_t start) {
    hipEvent_t e = get_event();
    if (!e) return;
    if (hipEventRecord(e, s) != hipSuccess) { pool.push_back(e); return; }
    pending.push_back(Pending{name, start, e});
}

hipError_t KernelTimer::resolve() {
    hipError_t st = hipSuccess;
    for (auto& p : pending) {
        float ms = 0.f;
        hipError_t e = hipEventSynchronize(p.stop);
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, p.start, p.stop);
        if (e != hipSuccess) st = e;
        auto& t = totals[p.name];
        t.first += ms;
        t.second += 1;
        pool.push_back(p.start);
        pool.push_back(p.stop);
    }
    pending.clear();
    return st;
}

void KernelTimer::release_all() {
    for (auto& p : pending) {
        (void)hipEventDestroy(p.start);
        (void)hipEventDestroy(p.stop);
    }
    pending.clear();
    for (auto e : pool) (void)hipEventDestroy(e);
    pool.clear();
}

hipError_t DevBuf::ensure(size_t n) {
    if (n <= bytes && ptr) return hipSuccess;
    if (ptr) {
        (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
    size_t want = std::max<size_t>(n, 256);
    hipError_t e = flags ? hipExtMallocWithFlags(&ptr, want, flags) : hipMalloc(&ptr, want);
    if (e != hipSuccess) {
        ptr = nullptr;
        return e;
    }
    bytes = want;
    return hipSuccess;
}

void DevBuf::release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
}

}  // namespace sva

namespace {

Ctx* as_ctx(void* p) { return static_cast<Ctx*>(p); }

int fail(Ctx* c, int code, const std::string& msg) {
    if (c) c->last_error = msg;
    return code;
}

int hip_fail(Ctx* c, hipError_t e, const char* what) {
    std::string m = std::string(what) + ": " + hipGetErrorString(e);
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation)
        return fail(c, SVA_ERR_OUT_OF_MEMORY, m);
    return fail(c, SVA_ERR_DEVICE, m);
}

#define SVA_HIP(c, expr, what)                           \
    do {                                                 \
        hipError_t _e = (expr);                          \
        if (_e != hipSuccess) return hip_fail(c, _e, what); \
    } while (0)

#define SVA_CHECK_CTX(c)                                                       \
    do {                                                                       \
        if (!(c)) return SVA_ERR_INVALID_ARG;                                  \
        if (hipSetDevice((c)->device) != hipSuccess)                           \
            return fail(c, SVA_ERR_DEVICE, "hipSetDevice failed");             \
    } while (0)

int check_image(Ctx* c, const void* a, int W, int H, size_t pitch) {
    if (!a) return fail(c, SVA_ERR_INVALID_ARG, "null image pointer");
    if (W <= 0 || H <= 0) return fail(c, SVA_ERR_INVALID_ARG, "image size must be positive");
    if (pitch < (size_t)W) return fail(c, SVA_ERR_INVALID_ARG, "pitch smaller than width");
    if ((long long)W * H > (1ll << 31) - 1) return fail(c, SVA_ERR_INVALID_ARG, "image too large");
    return SVA_OK;
}

// Shape limits are checked here, before any workspace is allocated: kernels
// launch with gridDim.y = H (lr_check, refine's gathers), which caps H at
// 65535, and every path volume is addressed with 32-bit buffer offsets.
// Whole-frame entry points take any D in 1..256 (run at the padded native
// width); the stage entry points (native = true) read and
// write [..][D] volumes and take D in {64, 128, 192, 256}.
int check_sgm(Ctx* c, const sva_sgm_params* p, int W, int H, bool native = false) {
    if (!p) return fail(c, SVA_ERR_INVALID_ARG, "null params");
    if (p->D <= 0) return fail(c, SVA_ERR_INVALID_ARG, "D must be positive");
    const int Dp = padded_D(p->D);
    if (!Dp) return fail(c, SVA_ERR_UNSUPPORTED, "GPU path built for D in 1..256");
    if (native && !paths_supported(p->D))
        return fail(c, SVA_ERR_UNSUPPORTED,
                    "stage entry points take D in {64,128,192,256} (whole frames: any D <= 256)");
    if (p->dir < -255 || p->dir > 255 || p->dir_y < -255 || p->dir_y > 255 ||
        (p->dir == 0 && p->dir_y == 0))
        return fail(c, SVA_ERR_INVALID_ARG, "(dir, dir_y) must be a nonzero step, |comp| <= 255");
    if (p->dmin < 0) return fail(c, SVA_ERR_INVALID_ARG, "dmin must be >= 0");
    if (p->dmin + p->D > 65535)
        return fail(c, SVA_ERR_INVALID_ARG, "dmin + D must fit the u16 disparity map");
    if (p->P1 < 0 || p->P2 < 0 || p->P1 > 193 || p->P2 > 193)
        return fail(c, SVA_ERR_INVALID_ARG, "penalties must satisfy 0 <= P1, P2 <= 193");
    if (p->lr_check && p->lr_max_diff < 0)
        return fail(c, SVA_ERR_INVALID_ARG, "lr_max_diff must be >= 0");
    if (H > 65535) return fail(c, SVA_ERR_UNSUPPORTED, "H must be <= 65535");
    if (W > 0 && H > 0 && (unsigned long long)W * (unsigned long long)H * (unsigned)Dp >=
                              (1ull << 32))
        return fail(c, SVA_ERR_UNSUPPORTED, "W*H*D must be < 2^32 (32-bit volume offsets)");
    return SVA_OK;
}

// Paths + WTA of the frame pipeline, the tile pipeline: the
// path kernel writes the four diagonal volumes plus horizontal and vertical
// checkpoints, and wta_hv recomputes the other four directions per tile and
// picks d*.  Dp is the native volume width, p->D <= Dp the caller's
// disparities (§4.7).  (The round-2 route of §4.6 -- six volumes, finished
// by wta_h -- was slower at every frame size measured and left in ABI v5.)
int paths_wta(Ctx* c, const uint8_t* C, int W, int H, const sva_sgm_params* p, int Dp,
              uint16_t* disp, float* sub) {
    if (!wta_hv_supported(Dp)) return fail(c, SVA_ERR_UNSUPPORTED, "no tile pipeline for this D");
    const size_t nv = (size_t)W * H * (size_t)Dp;
    const TileGeom tg = tile_geom(W, H, Dp);
    SVA_HIP(c, c->paths.ensure(nv * tg.nvol), "path workspace");
    SVA_HIP(c, c->ckpt.ensure(tg.hck_bytes + tg.vck_bytes + tg.dck_bytes), "checkpoint workspace");
    uint8_t* L4 = (uint8_t*)c->paths.ptr;
    uint8_t* CK = (uint8_t*)c->ckpt.ptr;
    uint8_t* CKV = CK + tg.hck_bytes;
    SVA_HIP(c, launch_paths(*c, C, W, H, Dp, p->P1, p->P2, L4, CK, CKV), "paths launch");
    SVA_HIP(c, launch_wta_hv(*c, C, L4, CK, CKV, W, H, Dp, p->P1, p->P2, p->dmin, disp, sub, p->D),
            "wta launch");
    return SVA_OK;
}

// Buffer sizes of the tile-pipeline stages (sva_tile_layout).
sva_tile_layout tile_layout(int W, int H, int D) {
    sva_tile_layout l;
    std::memset(&l, 0, sizeof(l));
    const TileGeom tg = tile_geom(W, H, D);
    l.seg = 1 << tg.seg_log2;
    l.nsx = tg.nsx;
    l.nsy = tg.nty;
    l.cost_bytes = (size_t)W * H * (size_t)D;
    l.diag_volumes = tg.nvol;
    l.diag_bytes = (size_t)tg.nvol * l.cost_bytes;
    l.hckpt_bytes = tg.hck_bytes;
    l.vckpt_bytes = tg.vck_bytes + tg.dck_bytes;
    return l;
}

// Caller buffers of the tile stages against the layout: every buffer present
// and at least as large as its plane, so that a sizing slip is an argument
// error before anything reaches the device.
int check_tile_buffers(Ctx* c, int W, int H, int D, const void* C, size_t C_bytes,
                       const void* diag, size_t diag_bytes, const void* hck, size_t hck_bytes,
                       const void* vck, size_t vck_bytes) {
    const sva_tile_layout l = tile_layout(W, H, D);
    if (!C || (!diag && l.diag_bytes) || !hck || !vck)
        return fail(c, SVA_ERR_INVALID_ARG, "null stage buffer");
    if (C_bytes < l.cost_bytes) return fail(c, SVA_ERR_INVALID_ARG, "cost buffer smaller than [H][W][D]");
    if (diag_bytes < l.diag_bytes)
        return fail(c, SVA_ERR_INVALID_ARG, "diagonal volume buffer smaller than [nvol][H][W][D]");
    if (hck_bytes < l.hckpt_bytes)
        return fail(c, SVA_ERR_INVALID_ARG, "horizontal checkpoint buffer smaller than [2][H][nsx][D]");
    if (vck_bytes < l.vckpt_bytes)
        return fail(c, SVA_ERR_INVALID_ARG, "row checkpoint buffer smaller than [np][nsy][W][D]");
    return SVA_OK;
}

// Mode S on device buffers: census -> cost -> 8 paths -> WTA (-> L/R check).
// Any D in 1..256 runs at the native width Dp = padded_D(D): the cost kernels
// write 255 at d >= D and the WTA ignores those disparities.
int run_sgm_device(Ctx* c, const uint8_t* left, const uint8_t* right, int W, int H, size_t pitch,
                   const sva_sgm_params* p, uint16_t* disp, float* sub) {
    const int Dp = padded_D(p->D);
    const size_t np = (size_t)W * H, nv = np * (size_t)Dp;
    int s;
    SVA_HIP(c, c->cost.ensure(nv), "cost workspace");
    uint8_t* C = (uint8_t*)c->cost.ptr;
    uint16_t* dr = nullptr;
    if (p->lr_check) {
        SVA_HIP(c, c->disp_r.ensure(np * 2), "lr workspace");
        dr = (uint16_t*)c->disp_r.ptr;
    }
    if (p->dir_y == 0 && Dp >= tune::kCensusCostMinD && census_cost_supported(Dp)) {
        // census maps stay on chip: one census+cost kernel (census_cost.hip),
        // once per matching role when the L/R check runs.
        SVA_HIP(c, launch_census_cost(*c, left, right, W, H, pitch, Dp, p->dmin, p->dir, C, p->D),
                "cost launch");
        if ((s = paths_wta(c, C, W, H, p, Dp, disp, sub))) return s;
        if (p->lr_check) {
            // right image as reference: the images swap roles, the step flips
            SVA_HIP(c, launch_census_cost(*c, right, left, W, H, pitch, Dp, p->dmin, -p->dir, C,
                                          p->D),
                    "cost launch");
            if ((s = paths_wta(c, C, W, H, p, Dp, dr, nullptr))) return s;
            SVA_HIP(c, launch_lr_check(*c, disp, dr, sub, W, H, p->dir, 0, p->lr_max_diff,
                                       p->invalid),
                    "lr launch");
        }
        return SVA_OK;
    }
    if (census_cost2_supported(Dp, p->dir, p->dir_y)) {
        // 2-D array steps with |by| = 1 (every rig baseline of getCameraPairs
        // and of BASELINE config 4): census + cost on the matrix cores in one
        // kernel (census_cost2.hip)
        SVA_HIP(c, launch_census_cost2(*c, left, right, W, H, pitch, Dp, p->dmin, p->dir,
                                       p->dir_y, C, p->D),
                "cost launch");
        if ((s = paths_wta(c, C, W, H, p, Dp, disp, sub))) return s;
        if (p->lr_check) {
            SVA_HIP(c, launch_census_cost2(*c, right, left, W, H, pitch, Dp, p->dmin, -p->dir,
                                           -p->dir_y, C, p->D),
                    "cost launch");
            if ((s = paths_wta(c, C, W, H, p, Dp, dr, nullptr))) return s;
            SVA_HIP(c, launch_lr_check(*c, disp, dr, sub, W, H, p->dir, p->dir_y, p->lr_max_diff,
                                       p->invalid),
                    "lr launch");
        }
        return SVA_OK;
    }
    SVA_HIP(c, c->census_l.ensure(np * 8), "census workspace");
    SVA_HIP(c, c->census_r.ensure(np * 8), "census workspace");
    uint64_t* cl = (uint64_t*)c->census_l.ptr;
    uint64_t* cr = (uint64_t*)c->census_r.ptr;
    SVA_HIP(c, launch_census_pair(*c, left, right, W, H, pitch, cl, cr), "census launch");
    SVA_HIP(c, launch_cost2(*c, cl, cr, W, H, Dp, p->dmin, p->dir, p->dir_y, C, p->D),
            "cost launch");
    if ((s = paths_wta(c, C, W, H, p, Dp, disp, sub))) return s;
    if (p->lr_check) {
        // right image as reference: roles of the census maps swap, the step flips
        SVA_HIP(c, launch_cost2(*c, cr, cl, W, H, Dp, p->dmin, -p->dir, -p->dir_y, C, p->D),
                "cost launch");
        if ((s = paths_wta(c, C, W, H, p, Dp, dr, nullptr))) return s;
        SVA_HIP(c, launch_lr_check(*c, disp, dr, sub, W, H, p->dir, p->dir_y, p->lr_max_diff,
                                   p->invalid),
                "lr launch");
    }
    return SVA_OK;
}

// A batch of frames of one shape through few launches of each aggregation
// kernel: the cost volume of every frame (census + cost per
// frame, each along its own step), then sgm_paths and wta_hv once per
// sub-batch of tune::kBatchSubFrames frames.  The frames' census + cost
// kernels run on up to tune::kBatchCostStreams side streams forked from the
// context stream, in frame order per stream; the context stream starts a
// sub-batch's aggregation as soon as that sub-batch's costs are done, so the
// next sub-batches' (VALU-bound, small) cost kernels overlap the current
// (HBM-bound) aggregation.  jobs[0..n) share D, dmin, P1, P2 and subpixel
// (checked by the entry point); maps / sub hold n planes of W*H.
int run_sgm_batch(Ctx* c, const sva_pair_d* jobs, int n, int W, int H, size_t pitch,
                  uint16_t* maps, float* sub) {
    const sva_sgm_params* p = &jobs[0].params;
    const int Dp = padded_D(p->D);
    const size_t np = (size_t)W * H, nv = np * (size_t)Dp;
    const TileGeom tg = tile_geom(W, H, Dp);
    const size_t ckb = tg.hck_bytes + tg.vck_bytes + tg.dck_bytes;
    const int sb = tune::kBatchSubFrames > 0 ? std::min(n, tune::kBatchSubFrames) : n;
    const int nsub = (n + sb - 1) / sb;
    SVA_HIP(c, c->cost.ensure(nv * n), "cost workspace");
    // the aggregation workspaces serve one sub-batch at a time (same stream)
    SVA_HIP(c, c->paths.ensure(nv * tg.nvol * sb), "path workspace");
    SVA_HIP(c, c->ckpt.ensure(ckb * sb), "checkpoint workspace");
    uint8_t* C = (uint8_t*)c->cost.ptr;
    const int ns = std::min(n, tune::kBatchCostStreams);
    if (ns > 1) {
        while ((int)c->side.size() < ns) {
            hipStream_t s = nullptr;
            SVA_HIP(c, hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "side stream");
            c->side.push_back(s);
        }
        // one event per (sub-batch, side stream): "this stream's frames of
        // sub-batch j have their cost volumes"
        while ((int)c->side_done.size() < ns * nsub) {
            hipEvent_t e = nullptr;
            SVA_HIP(c, hipEventCreateWithFlags(&e, hipEventDisableTiming), "side stream event");
            c->side_done.push_back(e);
        }
        if (!c->fork) SVA_HIP(c, hipEventCreateWithFlags(&c->fork, hipEventDisableTiming), "fork event");
        SVA_HIP(c, hipEventRecord(c->fork, c->stream), "fork");
        for (int s = 0; s < ns; s++) SVA_HIP(c, hipStreamWaitEvent(c->side[s], c->fork, 0), "fork");
    }
    SVA_HIP(c, c->census_side.ensure(np * 16 * (size_t)std::max(ns, 1)), "census workspace");
    const hipStream_t own = c->stream;
    // fault injection (SVA_DEBUG_FAIL_COST_AT): this call's n-th cost launch fails
    const int fail_at = c->dbg_fail_cost_at;
    c->dbg_fail_cost_at = 0;
    int st = SVA_OK;
    for (int i = 0; i < n && st == SVA_OK; i++) {
        const sva_sgm_params* q = &jobs[i].params;
        uint8_t* Ci = C + (size_t)i * nv;
        if (ns > 1) c->stream = c->side[i % ns];
        hipError_t e;
        if (i + 1 == fail_at) {
            e = hipErrorLaunchFailure;
        } else if (q->dir_y == 0 && Dp >= tune::kCensusCostMinD && census_cost_supported(Dp)) {
            e = launch_census_cost(*c, jobs[i].left, jobs[i].right, W, H, pitch, Dp, q->dmin, q->dir,
                                   Ci, q->D);
        } else if (census_cost2_supported(Dp, q->dir, q->dir_y)) {
            e = launch_census_cost2(*c, jobs[i].left, jobs[i].right, W, H, pitch, Dp, q->dmin,
                                    q->dir, q->dir_y, Ci, q->D);
        } else {
            uint64_t* cl = (uint64_t*)c->census_side.ptr + (size_t)(i % std::max(ns, 1)) * 2 * np;
            uint64_t* cr = cl + np;
            e = launch_census_pair(*c, jobs[i].left, jobs[i].right, W, H, pitch, cl, cr);
            if (e == hipSuccess)
                e = launch_cost2(*c, cl, cr, W, H, Dp, q->dmin, q->dir, q->dir_y, Ci, q->D);
        }
        // the last frame of a sub-batch on this side stream (or of the batch)
        if (e == hipSuccess && ns > 1 && (i + ns >= n || (i + ns) / sb != i / sb))
            e = hipEventRecord(c->side_done[(size_t)(i / sb) * ns + i % ns], c->stream);
        c->stream = own;
        if (e != hipSuccess) st = hip_fail(c, e, "cost launch");
    }
    // Aggregation per sub-batch on the context stream, after its costs.
    for (int j = 0; j < nsub && st == SVA_OK; j++) {
        const int i0 = j * sb, m = std::min(sb, n - i0);
        hipError_t e = hipSuccess;
        if (ns > 1) {
            for (int s = 0; s < ns && s < n && e == hipSuccess; s++) {
                // side stream s holds frames of sub-batch j: its event recorded
                // after the last of them
                bool has = false;
                for (int i = i0; i < i0 + m; i++) has = has || i % ns == s;
                if (has) e = hipStreamWaitEvent(c->stream, c->side_done[(size_t)j * ns + s], 0);
            }
        }
        if (e != hipSuccess) { st = hip_fail(c, e, "join"); break; }
        uint8_t* L4 = (uint8_t*)c->paths.ptr;
        uint8_t* CK = (uint8_t*)c->ckpt.ptr;
        // horizontal planes of the sub-batch's frames, then their vertical planes
        uint8_t* CKV = CK + tg.hck_bytes * m;
        const uint8_t* Cj = C + (size_t)i0 * nv;
        if ((e = launch_paths(*c, Cj, W, H, Dp, p->P1, p->P2, L4, CK, CKV, m)) != hipSuccess) {
            st = hip_fail(c, e, "paths launch");
            break;
        }
        if ((e = launch_wta_hv(*c, Cj, L4, CK, CKV, W, H, Dp, p->P1, p->P2, p->dmin,
                               maps + (size_t)i0 * np, p->subpixel ? sub + (size_t)i0 * np : nullptr,
                               p->D, m)) != hipSuccess) {
            st = hip_fail(c, e, "wta launch");
            break;
        }
    }
    if (st != SVA_OK && ns > 1) {
        // A failed launch skipped later sub-batches' joins, so the context
        // stream may not be ordered after cost kernels already queued on the
        // side streams.  Join every side stream with a fresh record before
        // returning: the caller may free or reuse the images and the cost
        // workspace as soon as the context stream has drained.  (side_done[s]
        // is free for this: nothing later in this call waits on it.)
        for (int s = 0; s < ns; s++) {
            if (hipEventRecord(c->side_done[s], c->side[s]) != hipSuccess ||
                hipStreamWaitEvent(c->stream, c->side_done[s], 0) != hipSuccess)
                (void)hipStreamSynchronize(c->side[s]);   // last resort: order on the host
        }
    }
    return st;
}

int check_camera(Ctx* c, const sva_camera* cam) {
    if (!cam) return fail(c, SVA_ERR_INVALID_ARG, "null camera");
    return SVA_OK;
}

int run_ref_device(Ctx* c, const uint8_t* ref, const uint8_t* other, int W, int H, size_t pitch,
                   const uint8_t* mask, const sva_camera* cref, const sva_camera* coth, int k,
                   double t_near, double t_far, uint8_t* d8, uint16_t* d16, uint8_t* valid) {
    const size_t np = (size_t)W * H;
    SVA_HIP(c, c->census_l.ensure(np * 16), "endpoint workspace");
    SVA_HIP(c, c->census_r.ensure(np), "endpoint workspace");
    int32_t* ends = (int32_t*)c->census_l.ptr;
    uint8_t* ok = (uint8_t*)c->census_r.ptr;
    SVA_HIP(c, launch_ref_endpoints(*c, W, H, *cref, *coth, k, t_near, t_far, ends, ok),
            "endpoint launch");
    SVA_HIP(c, launch_ref_match(*c, ref, other, W, H, pitch, mask, ends, ok, k, d8, d16, valid),
            "match launch");
    return SVA_OK;
}

int check_ref_args(Ctx* c, int W, int H, int k, double t_near, double t_far) {
    if (k < 1) return fail(c, SVA_ERR_INVALID_ARG, "kernel half-size k must be >= 1");
    if (2LL * k >= W || 2LL * k >= H) return fail(c, SVA_ERR_INVALID_ARG, "image smaller than window");
    if (!(t_near > 0.0) || !(t_far > 0.0))
        return fail(c, SVA_ERR_INVALID_ARG, "ray parameters must be positive");
    // the plane kernel packs line geometry in 16-bit fields (refpath.hip)
    if (W > 32767 || H > 32767)
        return fail(c, SVA_ERR_UNSUPPORTED, "Mode R supports W, H <= 32767");
    return SVA_OK;
}

// refinement / 3-D helpers

int check_planes(Ctx* c, int W, int H, size_t pitch) {
    if (W <= 0 || H <= 0) return fail(c, SVA_ERR_INVALID_ARG, "image size must be positive");
    if (pitch < (size_t)W) return fail(c, SVA_ERR_INVALID_ARG, "pitch smaller than width");
    if ((long long)W * H > (1ll << 31) - 1) return fail(c, SVA_ERR_INVALID_ARG, "image too large");
    if (H > 65535) return fail(c, SVA_ERR_UNSUPPORTED, "H must be <= 65535 (gridDim.y)");
    return SVA_OK;
}

int check_window(Ctx* c, int window_size) {
    if (window_size < 1 || (window_size - 1) / 2 > 32)
        return fail(c, SVA_ERR_UNSUPPORTED, "window_size must give kernelSize (w-1)/2 in 0..32");
    return SVA_OK;
}

// improveWithDisparity on device planes; images = n device pointers.
int run_improve(Ctx* c, const uint8_t* disp, const uint8_t* center, const uint8_t* const* images,
                const sva_camera* cams, int n, int W, int H, size_t pitch, const uint8_t* mask,
                int window_size, int strict, uint8_t* out,
                const std::function<int(int, const uint8_t**)>& fetch) {
    const size_t bytes = (size_t)H * pitch;
    SVA_HIP(c, c->shifted.ensure(bytes), "shift workspace");
    SVA_HIP(c, c->total.ensure(sizeof(long long)), "fault flag");
    int* fault = (int*)c->total.ptr;
    SVA_HIP(c, hipMemsetAsync(fault, 0, sizeof(int), c->stream), "memset");
    uint8_t* sh = (uint8_t*)c->shifted.ptr;
    const int k = (window_size - 1) / 2;
    for (int i = 0; i < n; i++) {
        const uint8_t* img = images ? images[i] : nullptr;
        int s;
        if (fetch && (s = fetch(i, &img))) return s;
        // the reference's shifted Mat is uninitialised; DESIGN.md §2.7 fixes it to 0
        // (zero_fill: the shift kernel writes the 0 of every untouched pixel)
        SVA_HIP(c, launch_shift_perspective(*c, cams[2 * i], cams[2 * i + 1], disp, img, W, H,
                                            pitch, sh, true), "shift launch");
        SVA_HIP(c, launch_refine(*c, disp, center, sh, mask, W, H, pitch, k, cams[2 * i],
                                 cams[2 * i + 1], out, fault), "refine launch");
    }
    if (strict) {
        int f = 0;
        SVA_HIP(c, hipMemcpyAsync(&f, fault, sizeof(int), hipMemcpyDeviceToHost, c->stream),
                "download");
        SVA_HIP(c, hipStreamSynchronize(c->stream), "sync");
        if (f)
            return fail(c, SVA_ERR_INVALID_ARG,
                        "a masked pixel's window leaves the image (the reference's ROI throws)");
    }
    return SVA_OK;
}

}  // namespace

// ------------------------------------------------------------------ ABI --
extern "C" {

void sva_sgm_params_default(sva_sgm_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->D = 128;
    p->dmin = 0;
    p->dir = -1;
    p->P1 = 10;
    p->P2 = 120;
    p->subpixel = 0;
    p->lr_check = 0;
    p->lr_max_diff = 1;
    p->invalid = 0xffff;
}

int sva_abi_version(void) { return SVA_ABI_VERSION; }

int sva_device_count(int* count) {
    if (!count) return SVA_ERR_INVALID_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return SVA_OK;
}

const char* sva_status_string(int s) {
    switch (s) {
        case SVA_OK: return "ok";
        case SVA_ERR_INVALID_ARG: return "invalid argument";
        case SVA_ERR_UNSUPPORTED: return "unsupported configuration";
        case SVA_ERR_DEVICE: return "device error";
        case SVA_ERR_OUT_OF_MEMORY: return "out of device memory";
        case SVA_ERR_NO_DEVICE: return "no usable HIP device";
        default: return "unknown status";
    }
}

int sva_create(int device, void** out) {
    if (!out) return SVA_ERR_INVALID_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return SVA_ERR_NO_DEVICE;
    if (device < 0 || device >= n) return SVA_ERR_INVALID_ARG;
    if (hipSetDevice(device) != hipSuccess) return SVA_ERR_DEVICE;
    Ctx* c = new (std::nothrow) Ctx();
    if (!c) return SVA_ERR_OUT_OF_MEMORY;
    c->device = device;
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return SVA_ERR_DEVICE;
    }
    c->stream = c->own_stream;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->cu_count = prop.multiProcessorCount;
    *out = c;
    return SVA_OK;
}

int sva_destroy(void* ctx) {
    Ctx* c = as_ctx(ctx);
    if (!c) return SVA_ERR_INVALID_ARG;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    c->batch_lane.reset();   // its streams and staging (multi.cpp), before the context's own
    for (hipStream_t s : c->side) {
        (void)hipStreamSynchronize(s);
        (void)hipStreamDestroy(s);
    }
    for (hipEvent_t e : c->side_done) (void)hipEventDestroy(e);
    if (c->fork) (void)hipEventDestroy(c->fork);
    c->census_side.release();
    for (DevBuf* b : {&c->census_l, &c->census_r, &c->cost, &c->paths, &c->ckpt, &c->scratch_u16,
                      &c->disp_r, &c->in_a, &c->in_b, &c->in_mask, &c->out_a, &c->out_b,
                      &c->out_c, &c->in_c, &c->shifted, &c->keys, &c->counts, &c->total, &c->ref_keys})
        b->release();
    c->timer.release_all();
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
    return SVA_OK;
}

int sva_set_stream(void* ctx, void* stream) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    c->stream = stream ? (hipStream_t)stream : c->own_stream;
    return SVA_OK;
}

int sva_synchronize(void* ctx) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    SVA_HIP(c, hipStreamSynchronize(c->stream), "hipStreamSynchronize");
    return SVA_OK;
}

const char* sva_last_error(void* ctx) {
    Ctx* c = as_ctx(ctx);
    return c ? c->last_error.c_str() : "null context";
}

namespace {

// The path kernel's time (ns, best of 3 after one warm-up launch) on the
// context's current cost / path / checkpoint buffers.  The volumes hold
// whatever they hold: the kernel's work does not depend on the values.
int time_stage_set(Ctx* c, int W, int H, int D, int64_t* ns) {
    const TileGeom tg = tile_geom(W, H, D);
    const uint8_t* C = (const uint8_t*)c->cost.ptr;
    uint8_t* L4 = (uint8_t*)c->paths.ptr;
    uint8_t* CK = (uint8_t*)c->ckpt.ptr;
    hipEvent_t a = nullptr, b = nullptr;
    SVA_HIP(c, hipEventCreate(&a), "placement event");
    if (hipEventCreate(&b) != hipSuccess) {
        (void)hipEventDestroy(a);
        return fail(c, SVA_ERR_DEVICE, "placement event");
    }
    hipError_t e = hipSuccess;
    float best = 0.f;
    for (int r = 0; r < 4 && e == hipSuccess; r++) {
        e = hipEventRecord(a, c->stream);
        if (e == hipSuccess) e = launch_paths(*c, C, W, H, D, 10, 120, L4, CK, CK + tg.hck_bytes);
        if (e == hipSuccess) e = hipEventRecord(b, c->stream);
        if (e == hipSuccess) e = hipEventSynchronize(b);
        float ms = 0.f;
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, a, b);
        if (e == hipSuccess && r > 0) best = r == 1 ? ms : std::min(best, ms);
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    if (e != hipSuccess) return hip_fail(c, e, "placement timing");
    *ns = (int64_t)((double)best * 1e6);
    return SVA_OK;
}

// sva_reserve's placement check (include/sva.h): keep the
// fastest of `trials` allocations of the stage buffers.  Every trial set stays
// allocated until the choice is made, so each one lands on pages no earlier
// set holds; a trial is taken only while the device keeps a quarter of its
// memory (at least 16 GiB) free beside it.
int place_stage_buffers(Ctx* c, int W, int H, int D, int trials) {
    struct Set {
        DevBuf cost, paths, ckpt;
        int64_t ns = 0;
    };
    const bool timing = c->timer.enabled;
    c->timer.enabled = false;                 // the trials are not the caller's launches
    std::vector<Set> sets(1);
    int rc = time_stage_set(c, W, H, D, &sets[0].ns);
    const size_t set_bytes = c->cost.bytes + c->paths.bytes + c->ckpt.bytes;
    for (int t = 1; rc == SVA_OK && t < trials; t++) {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) break;
        const size_t keep = std::max(total_b / 4, (size_t)16 << 30);
        if (free_b < set_bytes + keep) break;
        Set n;
        n.cost.flags = c->cost.flags;
        n.paths.flags = c->paths.flags;
        n.ckpt.flags = c->ckpt.flags;
        if (n.cost.ensure(c->cost.bytes) != hipSuccess || n.paths.ensure(c->paths.bytes) != hipSuccess ||
            n.ckpt.ensure(c->ckpt.bytes) != hipSuccess) {
            n.cost.release();                 // no room for another set: stop here
            n.paths.release();
            n.ckpt.release();
            (void)hipGetLastError();
            break;
        }
        // time the new set in the context's slots; sets[0] keeps the first set
        std::swap(c->cost, n.cost);
        std::swap(c->paths, n.paths);
        std::swap(c->ckpt, n.ckpt);
        rc = time_stage_set(c, W, H, D, &n.ns);
        std::swap(c->cost, n.cost);
        std::swap(c->paths, n.paths);
        std::swap(c->ckpt, n.ckpt);
        sets.push_back(n);
    }
    c->timer.enabled = timing;
    size_t best = 0;
    int64_t worst = sets[0].ns;
    for (size_t i = 1; i < sets.size(); i++) {
        if (sets[i].ns < sets[best].ns) best = i;
        worst = std::max(worst, sets[i].ns);
    }
    if (rc == SVA_OK && best != 0) {          // the context takes the fastest set
        std::swap(c->cost, sets[best].cost);
        std::swap(c->paths, sets[best].paths);
        std::swap(c->ckpt, sets[best].ckpt);
    }
    const int64_t kept = sets[rc == SVA_OK ? best : 0].ns;
    for (size_t i = 1; i < sets.size(); i++) {  // every other set (the old slots included)
        sets[i].cost.release();
        sets[i].paths.release();
        sets[i].ckpt.release();
    }
    if (rc != SVA_OK) return rc;
    c->placement_ns = kept;
    c->placement_worst_ns = worst;
    c->placement_paths = c->paths.ptr;
    return SVA_OK;
}

}  // namespace

int sva_reserve(void* ctx, int W, int H, int D) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    if (W <= 0 || H <= 0 || D <= 0) return fail(c, SVA_ERR_INVALID_ARG, "bad reserve size");
    if (padded_D(D)) D = padded_D(D);     // a frame's volumes use the native width (§4.7)
    const size_t np = (size_t)W * H, nv = np * (size_t)D;
    SVA_HIP(c, c->census_l.ensure(np * 8), "reserve");
    SVA_HIP(c, c->census_r.ensure(np * 8), "reserve");
    SVA_HIP(c, c->cost.ensure(nv), "reserve");
    // the frame route's path volumes: the 4 diagonal directions (tile pipeline)
    const TileGeom tg = tile_geom(W, H, D);
    const size_t ckb = tg.hck_bytes + tg.vck_bytes + tg.dck_bytes;
    SVA_HIP(c, c->paths.ensure(nv * tg.nvol), "reserve");
    SVA_HIP(c, c->ckpt.ensure(ckb), "reserve");
    // (once per allocation: a repeated reserve of a size the buffers already
    // hold keeps the set the last check chose)
    const int trials = c->placement_trials > 0 ? c->placement_trials : tune::kPlacementTrials;
    if (trials > 1 && wta_hv_supported(D) && nv < ((size_t)1 << 32) &&
        nv + nv * tg.nvol + ckb >= tune::kPlacementMinBytes && c->paths.ptr != c->placement_paths)
        return place_stage_buffers(c, W, H, D, trials);
    return SVA_OK;
}

int sva_set_path_kernel(void* ctx, int kernel) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    if (kernel == SVA_PATH_KERNEL_FUSED)
        return fail(c, SVA_ERR_UNSUPPORTED,
                    "the census-fused path kernel was removed in ABI v4 (DESIGN.md §4.5)");
    if (kernel != SVA_PATH_KERNEL_COST_VOLUME && kernel != SVA_PATH_KERNEL_AUTO)
        return fail(c, SVA_ERR_INVALID_ARG, "unknown path kernel");
    return SVA_OK;
}

int sva_set_timing(void* ctx, int enable) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    if (enable < 0 || enable > SVA_TIMING_AGG)
        return fail(c, SVA_ERR_INVALID_ARG, "timing mode must be 0, 1, 2 or 3");
    c->timer.enabled = enable != 0;
    c->timer.mode = enable;
    return SVA_OK;
}

int sva_reset_timing(void* ctx) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    hipError_t e = c->timer.resolve();
    c->timer.totals.clear();
    if (e != hipSuccess) return hip_fail(c, e, "timer resolve");
    return SVA_OK;
}

int sva_set_debug(void* ctx, int key, int64_t value) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    switch (key) {
        case SVA_DEBUG_PLANE_SPLIT:
            if (value < 0 || value > 16) return fail(c, SVA_ERR_INVALID_ARG, "plane split must be 0..16");
            c->dbg_plane_split = (int)value;
            return SVA_OK;
        case SVA_DEBUG_FAIL_COST_AT:
            if (value < 0 || value > (1 << 30)) return fail(c, SVA_ERR_INVALID_ARG, "bad frame index");
            c->dbg_fail_cost_at = (int)value;
            return SVA_OK;
        case SVA_DEBUG_PLACEMENT_TRIALS:
            if (value < 0 || value > 8) return fail(c, SVA_ERR_INVALID_ARG, "placement trials must be 0..8");
            c->placement_trials = (int)value;
            return SVA_OK;
        default:
            return fail(c, SVA_ERR_INVALID_ARG, "unknown or read-only debug key");
    }
}

int sva_get_debug(void* ctx, int key, int64_t* value) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    if (!value) return fail(c, SVA_ERR_INVALID_ARG, "null value");
    switch (key) {
        case SVA_DEBUG_PLANE_SPLIT: *value = c->dbg_plane_split; return SVA_OK;
        case SVA_DEBUG_FAIL_COST_AT: *value = c->dbg_fail_cost_at; return SVA_OK;
        case SVA_DEBUG_PLACEMENT_TRIALS: *value = c->placement_trials; return SVA_OK;
        case SVA_DEBUG_PLACEMENT_NS: *value = c->placement_ns; return SVA_OK;
        case SVA_DEBUG_PLACEMENT_WORST_NS: *value = c->placement_worst_ns; return SVA_OK;
        case SVA_DEBUG_SIDE_IDLE: {
            bool idle = true;
            for (hipStream_t s : c->side) {
                const hipError_t e = hipStreamQuery(s);
                if (e == hipErrorNotReady) idle = false;
                else if (e != hipSuccess) return hip_fail(c, e, "side stream query");
            }
            *value = idle ? 1 : 0;
            return SVA_OK;
        }
        default:
            return fail(c, SVA_ERR_INVALID_ARG, "unknown debug key");
    }
}

int sva_kernel_time(void* ctx, const char* name, double* total_ms, int64_t* count) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    if (!name || !total_ms || !count) return fail(c, SVA_ERR_INVALID_ARG, "null argument");
    hipError_t e = c->timer.resolve();
    if (e != hipSuccess) return hip_fail(c, e, "timer resolve");
    auto it = c->timer.totals.find(name);
    *total_ms = it == c->timer.totals.end() ? 0.0 : it->second.first;
    *count = it == c->timer.totals.end() ? 0 : it->second.second;
    return SVA_OK;
}

// ---------------------------------------------------------------- Mode S --
int sva_disparity_sgm_d(void* ctx, const uint8_t* left, const uint8_t* right, int W, int H,
                        size_t pitch, const sva_sgm_params* p, uint16_t* disp, float* sub) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_image(c, left, W, H, pitch)) || (s = check_image(c, right, W, H, pitch)) ||
        (s = check_sgm(c, p, W, H)))
        return s;
    if (!disp) return fail(c, SVA_ERR_INVALID_ARG, "null disparity output");
    return run_sgm_device(c, left, right, W, H, pitch, p, disp, p->subpixel ? sub : nullptr);
}

int sva_disparity_sgm_batch_d(void* ctx, const sva_pair_d* jobs, int n, int W, int H,
                              size_t pitch, uint16_t* maps, float* sub) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    if (!jobs || n <= 0 || !maps) return fail(c, SVA_ERR_INVALID_ARG, "bad batch argument");
    int s;
    const sva_sgm_params* p0 = &jobs[0].params;
    for (int i = 0; i < n; i++) {
        const sva_sgm_params* q = &jobs[i].params;
        if ((s = check_image(c, jobs[i].left, W, H, pitch)) ||
            (s = check_image(c, jobs[i].right, W, H, pitch)) || (s = check_sgm(c, q, W, H)))
            return s;
        if (q->D != p0->D || q->dmin != p0->dmin || q->P1 != p0->P1 || q->P2 != p0->P2 ||
            q->subpixel != p0->subpixel)
            return fail(c, SVA_ERR_INVALID_ARG,
                        "a batch's pairs must share D, dmin, P1, P2 and subpixel");
        if (q->lr_check) return fail(c, SVA_ERR_UNSUPPORTED, "the batch route has no L/R check");
    }
    if (!wta_hv_supported(padded_D(p0->D)))
        return fail(c, SVA_ERR_UNSUPPORTED, "no tile pipeline for this D");
    // chunks of at most tune::kBatchMaxPairs frames, whose workspaces stay
    // under tune::kBatchMaxBytes
    const int Dp = padded_D(p0->D);
    const TileGeom tg = tile_geom(W, H, Dp);
    const size_t per = (size_t)W * H * (size_t)Dp * (1 + tg.nvol) + tg.hck_bytes + tg.vck_bytes +
                       tg.dck_bytes;
    int chunk = tune::kBatchMaxPairs;
    while (chunk > 1 && per * (size_t)chunk > tune::kBatchMaxBytes) chunk--;
    const size_t np = (size_t)W * H;
    for (int i0 = 0; i0 < n; i0 += chunk) {
        const int m = std::min(chunk, n - i0);
        if ((s = run_sgm_batch(c, jobs + i0, m, W, H, pitch, maps + (size_t)i0 * np,
                               sub ? sub + (size_t)i0 * np : nullptr)))
            return s;
    }
    return SVA_OK;
}

int sva_disparity_sgm(void* ctx, const uint8_t* left, const uint8_t* right, int W, int H,
                      size_t pitch, const sva_sgm_params* p, uint16_t* disp, float* sub) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_image(c, left, W, H, pitch)) || (s = check_image(c, right, W, H, pitch)) ||
        (s = check_sgm(c, p, W, H)))
        return s;
    if (!disp) return fail(c, SVA_ERR_INVALID_ARG, "null disparity output");
    const bool want_sub = p->subpixel && sub;
    const size_t np = (size_t)W * H;
    SVA_HIP(c, c->in_a.ensure(np), "staging");
    SVA_HIP(c, c->in_b.ensure(np), "staging");
    SVA_HIP(c, c->out_a.ensure(np * 2), "staging");
    if (want_sub) SVA_HIP(c, c->out_b.ensure(np * 4), "staging");
    SVA_HIP(c, hipMemcpy2DAsync(c->in_a.ptr, W, left, pitch, W, H, hipMemcpyHostToDevice, c->stream),
            "upload");
    SVA_HIP(c, hipMemcpy2DAsync(c->in_b.ptr, W, right, pitch, W, H, hipMemcpyHostToDevice, c->stream),
            "upload");
    if ((s = run_sgm_device(c, (uint8_t*)c->in_a.ptr, (uint8_t*)c->in_b.ptr, W, H, W, p,
                            (uint16_t*)c->out_a.ptr, want_sub ? (float*)c->out_b.ptr : nullptr)))
        return s;
    SVA_HIP(c, hipMemcpyAsync(disp, c->out_a.ptr, np * 2, hipMemcpyDeviceToHost, c->stream),
            "download");
    if (want_sub)
        SVA_HIP(c, hipMemcpyAsync(sub, c->out_b.ptr, np * 4, hipMemcpyDeviceToHost, c->stream),
                "download");
    SVA_HIP(c, hipStreamSynchronize(c->stream), "sync");
    return SVA_OK;
}

int sva_census_d(void* ctx, const uint8_t* img, int W, int H, size_t pitch, uint64_t* census) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_image(c, img, W, H, pitch))) return s;
    if (!census) return fail(c, SVA_ERR_INVALID_ARG, "null census output");
    SVA_HIP(c, launch_census(*c, img, W, H, pitch, census), "census launch");
    return SVA_OK;
}

int sva_cost_d(void* ctx, const uint64_t* cl, const uint64_t* cr, int W, int H,
               const sva_sgm_params* p, uint8_t* C) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_sgm(c, p, W, H, true))) return s;
    if (!cl || !cr || !C || W <= 0 || H <= 0) return fail(c, SVA_ERR_INVALID_ARG, "bad argument");
    SVA_HIP(c, launch_cost2(*c, cl, cr, W, H, p->D, p->dmin, p->dir, p->dir_y, C), "cost launch");
    return SVA_OK;
}

int sva_census_cost_d(void* ctx, const uint8_t* left, const uint8_t* right, int W, int H,
                      size_t pitch, const sva_sgm_params* p, uint8_t* C) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_sgm(c, p, W, H, true))) return s;
    if ((s = check_image(c, left, W, H, pitch))) return s;
    if ((s = check_image(c, right, W, H, pitch))) return s;
    if (!C) return fail(c, SVA_ERR_INVALID_ARG, "null cost output");
    if (p->dir_y == 0 && census_cost_supported(p->D)) {
        SVA_HIP(c, launch_census_cost(*c, left, right, W, H, pitch, p->D, p->dmin, p->dir, C),
                "cost launch");
        return SVA_OK;
    }
    if (!census_cost2_supported(p->D, p->dir, p->dir_y))
        return fail(c, SVA_ERR_UNSUPPORTED,
                    "census+cost kernel: D in {64,128,192,256}, 1-D steps or 2-D steps whose "
                    "primitive form has |dir_y| = 1 and |dir| <= 3");
    SVA_HIP(c, launch_census_cost2(*c, left, right, W, H, pitch, p->D, p->dmin, p->dir, p->dir_y, C),
            "cost launch");
    return SVA_OK;
}

int sva_paths_d(void* ctx, const uint8_t* C, int W, int H, const sva_sgm_params* p, uint8_t* L8) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_sgm(c, p, W, H, true))) return s;
    if (!C || !L8 || W <= 0 || H <= 0) return fail(c, SVA_ERR_INVALID_ARG, "bad argument");
    SVA_HIP(c, launch_paths(*c, C, W, H, p->D, p->P1, p->P2, L8), "paths launch");
    return SVA_OK;
}

int sva_aggregate_d(void* ctx, const uint8_t* C, int W, int H, const sva_sgm_params* p,
                    uint16_t* S) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_sgm(c, p, W, H, true))) return s;
    if (!C || !S || W <= 0 || H <= 0) return fail(c, SVA_ERR_INVALID_ARG, "bad argument");
    const size_t nv = (size_t)W * H * (size_t)p->D;
    SVA_HIP(c, c->paths.ensure(nv * 8), "path workspace");
    uint8_t* L8 = (uint8_t*)c->paths.ptr;
    SVA_HIP(c, launch_paths(*c, C, W, H, p->D, p->P1, p->P2, L8), "paths launch");
    SVA_HIP(c, launch_sum(*c, L8, W, H, p->D, S), "sum launch");
    return SVA_OK;
}

int sva_tile_layout_of(int W, int H, int D, sva_tile_layout* out) {
    if (!out || W <= 0 || H <= 0 || !paths_supported(D)) return SVA_ERR_INVALID_ARG;
    *out = tile_layout(W, H, D);
    return SVA_OK;
}

int sva_tile_check(int W, int H, int D, size_t C_bytes, size_t diag_bytes, size_t hckpt_bytes,
                   size_t vckpt_bytes) {
    if (W <= 0 || H <= 0 || !paths_supported(D)) return SVA_ERR_INVALID_ARG;
    const char one = 0;   // any non-null address: sizes only
    return check_tile_buffers(nullptr, W, H, D, &one, C_bytes, &one, diag_bytes, &one, hckpt_bytes,
                              &one, vckpt_bytes);
}

int sva_paths_tile_d(void* ctx, const uint8_t* C, size_t C_bytes, int W, int H,
                     const sva_sgm_params* p, uint8_t* diag, size_t diag_bytes, uint8_t* hckpt,
                     size_t hckpt_bytes, uint8_t* vckpt, size_t vckpt_bytes) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_sgm(c, p, W, H, true))) return s;
    if ((s = check_tile_buffers(c, W, H, p->D, C, C_bytes, diag, diag_bytes, hckpt, hckpt_bytes,
                                vckpt, vckpt_bytes)))
        return s;
    SVA_HIP(c, launch_paths(*c, C, W, H, p->D, p->P1, p->P2, diag, hckpt, vckpt), "paths launch");
    return SVA_OK;
}

int sva_wta_hv_d(void* ctx, const uint8_t* C, size_t C_bytes, const uint8_t* diag,
                 size_t diag_bytes, const uint8_t* hckpt, size_t hckpt_bytes, const uint8_t* vckpt,
                 size_t vckpt_bytes, int W, int H, const sva_sgm_params* p, uint16_t* disp,
                 float* sub) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_sgm(c, p, W, H, true))) return s;
    if ((s = check_tile_buffers(c, W, H, p->D, C, C_bytes, diag, diag_bytes, hckpt, hckpt_bytes,
                                vckpt, vckpt_bytes)))
        return s;
    if (!disp) return fail(c, SVA_ERR_INVALID_ARG, "null disparity output");
    SVA_HIP(c, launch_wta_hv(*c, C, diag, hckpt, vckpt, W, H, p->D, p->P1, p->P2, p->dmin, disp,
                             p->subpixel ? sub : nullptr),
            "wta launch");
    return SVA_OK;
}

int sva_wta_d(void* ctx, const uint16_t* S, int W, int H, const sva_sgm_params* p, uint16_t* disp,
              float* sub) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_sgm(c, p, W, H, true))) return s;
    if (!S || !disp || W <= 0 || H <= 0) return fail(c, SVA_ERR_INVALID_ARG, "bad argument");
    SVA_HIP(c, launch_wta_from_sum(*c, S, W, H, p->D, p->dmin, disp, p->subpixel ? sub : nullptr),
            "wta launch");
    return SVA_OK;
}

// ---------------------------------------------------------------- Mode R --
int sva_ref_endpoints_d(void* ctx, int W, int H, const sva_camera* cref, const sva_camera* coth,
                        int k, double t_near, double t_far, int32_t* ends, uint8_t* valid) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_camera(c, cref)) || (s = check_camera(c, coth)) ||
        (s = check_ref_args(c, W, H, k, t_near, t_far)))
        return s;
    if (!ends || !valid) return fail(c, SVA_ERR_INVALID_ARG, "null output");
    SVA_HIP(c, launch_ref_endpoints(*c, W, H, *cref, *coth, k, t_near, t_far, ends, valid),
            "endpoint launch");
    return SVA_OK;
}

int sva_disparity_ref_d(void* ctx, const uint8_t* ref, const uint8_t* other, int W, int H,
                        size_t pitch, const uint8_t* mask, const sva_camera* cref,
                        const sva_camera* coth, int k, double t_near, double t_far, uint8_t* d8,
                        uint16_t* d16, uint8_t* valid) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_image(c, ref, W, H, pitch)) || (s = check_image(c, other, W, H, pitch)) ||
        (s = check_camera(c, cref)) || (s = check_camera(c, coth)) ||
        (s = check_ref_args(c, W, H, k, t_near, t_far)))
        return s;
    if (!d8) return fail(c, SVA_ERR_INVALID_ARG, "null disparity output");
    return run_ref_device(c, ref, other, W, H, pitch, mask, cref, coth, k, t_near, t_far, d8, d16,
                          valid);
}

int sva_disparity_ref(void* ctx, const uint8_t* ref, const uint8_t* other, int W, int H,
                      size_t pitch, const uint8_t* mask, const sva_camera* cref,
                      const sva_camera* coth, int k, double t_near, double t_far, uint8_t* d8,
                      uint16_t* d16, uint8_t* valid) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_image(c, ref, W, H, pitch)) || (s = check_image(c, other, W, H, pitch)) ||
        (s = check_camera(c, cref)) || (s = check_camera(c, coth)) ||
        (s = check_ref_args(c, W, H, k, t_near, t_far)))
        return s;
    if (!d8) return fail(c, SVA_ERR_INVALID_ARG, "null disparity output");
    const size_t np = (size_t)W * H;
    SVA_HIP(c, c->in_a.ensure(np), "staging");
    SVA_HIP(c, c->in_b.ensure(np), "staging");
    SVA_HIP(c, c->out_a.ensure(np), "staging");
    if (mask) SVA_HIP(c, c->in_mask.ensure(np), "staging");
    if (d16) SVA_HIP(c, c->out_b.ensure(np * 2), "staging");
    if (valid) SVA_HIP(c, c->out_c.ensure(np), "staging");
    hipStream_t st = c->stream;
    SVA_HIP(c, hipMemcpy2DAsync(c->in_a.ptr, W, ref, pitch, W, H, hipMemcpyHostToDevice, st), "upload");
    SVA_HIP(c, hipMemcpy2DAsync(c->in_b.ptr, W, other, pitch, W, H, hipMemcpyHostToDevice, st), "upload");
    if (mask) SVA_HIP(c, hipMemcpyAsync(c->in_mask.ptr, mask, np, hipMemcpyHostToDevice, st), "upload");
    // untouched pixels keep the caller's values (CameraStereoVision.cpp:46,55)
    SVA_HIP(c, hipMemcpyAsync(c->out_a.ptr, d8, np, hipMemcpyHostToDevice, st), "upload");
    if (d16) SVA_HIP(c, hipMemcpyAsync(c->out_b.ptr, d16, np * 2, hipMemcpyHostToDevice, st), "upload");
    if (valid) SVA_HIP(c, hipMemcpyAsync(c->out_c.ptr, valid, np, hipMemcpyHostToDevice, st), "upload");
    if ((s = run_ref_device(c, (uint8_t*)c->in_a.ptr, (uint8_t*)c->in_b.ptr, W, H, W,
                            mask ? (uint8_t*)c->in_mask.ptr : nullptr, cref, coth, k, t_near,
                            t_far, (uint8_t*)c->out_a.ptr, d16 ? (uint16_t*)c->out_b.ptr : nullptr,
                            valid ? (uint8_t*)c->out_c.ptr : nullptr)))
        return s;
    SVA_HIP(c, hipMemcpyAsync(d8, c->out_a.ptr, np, hipMemcpyDeviceToHost, st), "download");
    if (d16) SVA_HIP(c, hipMemcpyAsync(d16, c->out_b.ptr, np * 2, hipMemcpyDeviceToHost, st), "download");
    if (valid) SVA_HIP(c, hipMemcpyAsync(valid, c->out_c.ptr, np, hipMemcpyDeviceToHost, st), "download");
    SVA_HIP(c, hipStreamSynchronize(st), "sync");
    return SVA_OK;
}

int sva_disparity_to_depth_d(void* ctx, const uint8_t* disp, int n, double cam_distance,
                             double f, double pixel_size, double* depth) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    if (!disp || !depth || n < 0) return fail(c, SVA_ERR_INVALID_ARG, "bad argument");
    if (n == 0) return SVA_OK;
    SVA_HIP(c, launch_disp_to_depth(*c, disp, n, cam_distance, f, pixel_size, depth), "depth launch");
    return SVA_OK;
}

int sva_disparity_to_depth(void* ctx, const uint8_t* disp, int n, double cam_distance, double f,
                           double pixel_size, double* depth) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    if (!disp || !depth || n < 0) return fail(c, SVA_ERR_INVALID_ARG, "bad argument");
    if (n == 0) return SVA_OK;
    SVA_HIP(c, c->in_a.ensure((size_t)n), "staging");
    SVA_HIP(c, c->out_a.ensure((size_t)n * 8), "staging");
    SVA_HIP(c, hipMemcpyAsync(c->in_a.ptr, disp, (size_t)n, hipMemcpyHostToDevice, c->stream),
            "upload");
    SVA_HIP(c, launch_disp_to_depth(*c, (uint8_t*)c->in_a.ptr, n, cam_distance, f, pixel_size,
                                    (double*)c->out_a.ptr), "depth launch");
    SVA_HIP(c, hipMemcpyAsync(depth, c->out_a.ptr, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream),
            "download");
    SVA_HIP(c, hipStreamSynchronize(c->stream), "sync");
    return SVA_OK;
}

int check_fuse(Ctx* c, const uint16_t* disps, int n_maps, int W, int H, const double* b,
               const double* depth) {
    if (!disps || !b || !depth) return fail(c, SVA_ERR_INVALID_ARG, "null pointer");
    if (n_maps < 1 || n_maps > 32) return fail(c, SVA_ERR_UNSUPPORTED, "n_maps must be 1..32");
    if (W <= 0 || H <= 0) return fail(c, SVA_ERR_INVALID_ARG, "image size must be positive");
    return SVA_OK;
}

int sva_fuse_depth_d(void* ctx, const uint16_t* disps, int n_maps, int W, int H,
                     const double* baselines, double f, double pixel_size, uint16_t invalid,
                     double* depth, uint8_t* n_valid) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_fuse(c, disps, n_maps, W, H, baselines, depth))) return s;
    double num[32];
    for (int i = 0; i < n_maps; i++) num[i] = baselines[i] * f;
    SVA_HIP(c, launch_fuse_depth(*c, disps, n_maps, (size_t)W * H, num, pixel_size, invalid,
                                 depth, n_valid), "fuse launch");
    return SVA_OK;
}

int sva_fuse_depth(void* ctx, const uint16_t* disps, int n_maps, int W, int H,
                   const double* baselines, double f, double pixel_size, uint16_t invalid,
                   double* depth, uint8_t* n_valid) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_fuse(c, disps, n_maps, W, H, baselines, depth))) return s;
    const size_t np = (size_t)W * H, in_bytes = np * 2 * (size_t)n_maps;
    double num[32];
    for (int i = 0; i < n_maps; i++) num[i] = baselines[i] * f;
    SVA_HIP(c, c->in_a.ensure(in_bytes), "staging");
    SVA_HIP(c, c->out_a.ensure(np * 8), "staging");
    SVA_HIP(c, c->out_b.ensure(np), "staging");
    SVA_HIP(c, hipMemcpyAsync(c->in_a.ptr, disps, in_bytes, hipMemcpyHostToDevice, c->stream),
            "upload");
    SVA_HIP(c, launch_fuse_depth(*c, (const uint16_t*)c->in_a.ptr, n_maps, np, num, pixel_size,
                                 invalid, (double*)c->out_a.ptr, (uint8_t*)c->out_b.ptr),
            "fuse launch");
    SVA_HIP(c, hipMemcpyAsync(depth, c->out_a.ptr, np * 8, hipMemcpyDeviceToHost, c->stream),
            "download");
    if (n_valid)
        SVA_HIP(c, hipMemcpyAsync(n_valid, c->out_b.ptr, np, hipMemcpyDeviceToHost, c->stream),
                "download");
    SVA_HIP(c, hipStreamSynchronize(c->stream), "sync");
    return SVA_OK;
}

// ------------------------------------------ refinement / 3-D --
int sva_shift_perspective_d(void* ctx, const sva_camera* in_cam, const sva_camera* out_cam,
                            const uint8_t* disparity, const uint8_t* image, int W, int H,
                            size_t pitch, uint8_t* shifted) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_planes(c, W, H, pitch)) || (s = check_camera(c, in_cam)) ||
        (s = check_camera(c, out_cam)))
        return s;
    if (!disparity || !image || !shifted) return fail(c, SVA_ERR_INVALID_ARG, "null plane");
    SVA_HIP(c, launch_shift_perspective(*c, *in_cam, *out_cam, disparity, image, W, H, pitch,
                                        shifted), "shift launch");
    return SVA_OK;
}

int sva_shift_perspective(void* ctx, const sva_camera* in_cam, const sva_camera* out_cam,
                          const uint8_t* disparity, const uint8_t* image, int W, int H,
                          size_t pitch, uint8_t* shifted) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_planes(c, W, H, pitch)) || (s = check_camera(c, in_cam)) ||
        (s = check_camera(c, out_cam)))
        return s;
    if (!disparity || !image || !shifted) return fail(c, SVA_ERR_INVALID_ARG, "null plane");
    const size_t bytes = (size_t)H * pitch;
    SVA_HIP(c, c->in_a.ensure(bytes), "staging");
    SVA_HIP(c, c->in_b.ensure(bytes), "staging");
    SVA_HIP(c, c->out_a.ensure(bytes), "staging");
    hipStream_t st = c->stream;
    SVA_HIP(c, hipMemcpyAsync(c->in_a.ptr, disparity, bytes, hipMemcpyHostToDevice, st), "upload");
    SVA_HIP(c, hipMemcpyAsync(c->in_b.ptr, image, bytes, hipMemcpyHostToDevice, st), "upload");
    SVA_HIP(c, hipMemcpyAsync(c->out_a.ptr, shifted, bytes, hipMemcpyHostToDevice, st), "upload");
    SVA_HIP(c, launch_shift_perspective(*c, *in_cam, *out_cam, (uint8_t*)c->in_a.ptr,
                                        (uint8_t*)c->in_b.ptr, W, H, pitch,
                                        (uint8_t*)c->out_a.ptr), "shift launch");
    SVA_HIP(c, hipMemcpyAsync(shifted, c->out_a.ptr, bytes, hipMemcpyDeviceToHost, st), "download");
    SVA_HIP(c, hipStreamSynchronize(st), "sync");
    return SVA_OK;
}

int sva_improve_with_disparity_d(void* ctx, const uint8_t* disparity, const uint8_t* center,
                                 const uint8_t* const* images, const sva_camera* cam_pairs,
                                 int n_pairs, int W, int H, size_t pitch, const uint8_t* mask,
                                 int window_size, int strict, uint8_t* out) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_planes(c, W, H, pitch)) || (s = check_window(c, window_size))) return s;
    if (n_pairs < 0 || (n_pairs > 0 && (!images || !cam_pairs)))
        return fail(c, SVA_ERR_INVALID_ARG, "bad pair list");
    if (!disparity || !center || !out) return fail(c, SVA_ERR_INVALID_ARG, "null plane");
    for (int i = 0; i < n_pairs; i++)
        if (!images[i]) return fail(c, SVA_ERR_INVALID_ARG, "null pair image");
    return run_improve(c, disparity, center, images, cam_pairs, n_pairs, W, H, pitch, mask,
                       window_size, strict, out, nullptr);
}

int sva_improve_with_disparity(void* ctx, const uint8_t* disparity, const uint8_t* center,
                               const uint8_t* const* images, const sva_camera* cam_pairs,
                               int n_pairs, int W, int H, size_t pitch, const uint8_t* mask,
                               int window_size, int strict, uint8_t* out) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_planes(c, W, H, pitch)) || (s = check_window(c, window_size))) return s;
    if (n_pairs < 0 || (n_pairs > 0 && (!images || !cam_pairs)))
        return fail(c, SVA_ERR_INVALID_ARG, "bad pair list");
    if (!disparity || !center || !out) return fail(c, SVA_ERR_INVALID_ARG, "null plane");
    for (int i = 0; i < n_pairs; i++)
        if (!images[i]) return fail(c, SVA_ERR_INVALID_ARG, "null pair image");
    const size_t bytes = (size_t)H * pitch;
    SVA_HIP(c, c->in_a.ensure(bytes), "staging");
    SVA_HIP(c, c->in_b.ensure(bytes), "staging");
    SVA_HIP(c, c->in_c.ensure(bytes), "staging");
    SVA_HIP(c, c->out_a.ensure(bytes), "staging");
    if (mask) SVA_HIP(c, c->in_mask.ensure(bytes), "staging");
    hipStream_t st = c->stream;
    SVA_HIP(c, hipMemcpyAsync(c->in_a.ptr, disparity, bytes, hipMemcpyHostToDevice, st), "upload");
    SVA_HIP(c, hipMemcpyAsync(c->in_b.ptr, center, bytes, hipMemcpyHostToDevice, st), "upload");
    if (mask) SVA_HIP(c, hipMemcpyAsync(c->in_mask.ptr, mask, bytes, hipMemcpyHostToDevice, st), "upload");
    // pixels the refinement does not reach keep the caller's values
    SVA_HIP(c, hipMemcpyAsync(c->out_a.ptr, out, bytes, hipMemcpyHostToDevice, st), "upload");
    uint8_t* dimg = (uint8_t*)c->in_c.ptr;
    auto fetch = [&](int i, const uint8_t** img) -> int {
        // one staging buffer reused per pair: stream order keeps the upload
        // of pair i behind pair i-1's kernels
        SVA_HIP(c, hipMemcpyAsync(dimg, images[i], bytes, hipMemcpyHostToDevice, st), "upload");
        *img = dimg;
        return SVA_OK;
    };
    if ((s = run_improve(c, (uint8_t*)c->in_a.ptr, (uint8_t*)c->in_b.ptr, nullptr, cam_pairs,
                         n_pairs, W, H, pitch, mask ? (uint8_t*)c->in_mask.ptr : nullptr,
                         window_size, strict, (uint8_t*)c->out_a.ptr, fetch)))
        return s;
    SVA_HIP(c, hipMemcpyAsync(out, c->out_a.ptr, bytes, hipMemcpyDeviceToHost, st), "download");
    SVA_HIP(c, hipStreamSynchronize(st), "sync");
    return SVA_OK;
}

int sva_shift_perspective2_d(void* ctx, const sva_camera* in_cam, const sva_camera* out_cam,
                             const double* depth, int W, int H, double* shifted) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_planes(c, W, H, (size_t)W)) || (s = check_camera(c, in_cam)) ||
        (s = check_camera(c, out_cam)))
        return s;
    if (!depth || !shifted) return fail(c, SVA_ERR_INVALID_ARG, "null plane");
    SVA_HIP(c, c->keys.ensure((size_t)W * H * 4), "key workspace");
    SVA_HIP(c, launch_shift_perspective2(*c, *in_cam, *out_cam, depth, W, H,
                                         (unsigned*)c->keys.ptr, shifted), "shift2 launch");
    return SVA_OK;
}

int sva_shift_perspective2(void* ctx, const sva_camera* in_cam, const sva_camera* out_cam,
                           const double* depth, int W, int H, double* shifted) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_planes(c, W, H, (size_t)W)) || (s = check_camera(c, in_cam)) ||
        (s = check_camera(c, out_cam)))
        return s;
    if (!depth || !shifted) return fail(c, SVA_ERR_INVALID_ARG, "null plane");
    const size_t bytes = (size_t)W * H * 8;
    SVA_HIP(c, c->in_a.ensure(bytes), "staging");
    SVA_HIP(c, c->out_a.ensure(bytes), "staging");
    SVA_HIP(c, c->keys.ensure((size_t)W * H * 4), "key workspace");
    hipStream_t st = c->stream;
    SVA_HIP(c, hipMemcpyAsync(c->in_a.ptr, depth, bytes, hipMemcpyHostToDevice, st), "upload");
    SVA_HIP(c, hipMemcpyAsync(c->out_a.ptr, shifted, bytes, hipMemcpyHostToDevice, st), "upload");
    SVA_HIP(c, launch_shift_perspective2(*c, *in_cam, *out_cam, (double*)c->in_a.ptr, W, H,
                                         (unsigned*)c->keys.ptr, (double*)c->out_a.ptr),
            "shift2 launch");
    SVA_HIP(c, hipMemcpyAsync(shifted, c->out_a.ptr, bytes, hipMemcpyDeviceToHost, st), "download");
    SVA_HIP(c, hipStreamSynchronize(st), "sync");
    return SVA_OK;
}

int sva_points_to_depth_d(void* ctx, const double* points, int64_t n_points,
                          const sva_camera* cam, int W, int H, double* depth) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_planes(c, W, H, (size_t)W)) || (s = check_camera(c, cam))) return s;
    if (n_points < 0 || n_points > 0xfffffffell || (n_points > 0 && !points) || !depth)
        return fail(c, SVA_ERR_INVALID_ARG, "bad point list");
    SVA_HIP(c, c->keys.ensure((size_t)W * H * 4), "key workspace");
    SVA_HIP(c, launch_points_to_depth(*c, points, n_points, *cam, W, H, (unsigned*)c->keys.ptr,
                                      depth), "points launch");
    return SVA_OK;
}

int sva_points_to_depth(void* ctx, const double* points, int64_t n_points, const sva_camera* cam,
                        int W, int H, double* depth) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_planes(c, W, H, (size_t)W)) || (s = check_camera(c, cam))) return s;
    if (n_points < 0 || n_points > 0xfffffffell || (n_points > 0 && !points) || !depth)
        return fail(c, SVA_ERR_INVALID_ARG, "bad point list");
    const size_t pbytes = (size_t)n_points * 24, dbytes = (size_t)W * H * 8;
    SVA_HIP(c, c->in_a.ensure(pbytes ? pbytes : 8), "staging");
    SVA_HIP(c, c->out_a.ensure(dbytes), "staging");
    SVA_HIP(c, c->keys.ensure((size_t)W * H * 4), "key workspace");
    hipStream_t st = c->stream;
    if (pbytes)
        SVA_HIP(c, hipMemcpyAsync(c->in_a.ptr, points, pbytes, hipMemcpyHostToDevice, st), "upload");
    SVA_HIP(c, hipMemcpyAsync(c->out_a.ptr, depth, dbytes, hipMemcpyHostToDevice, st), "upload");
    SVA_HIP(c, launch_points_to_depth(*c, (double*)c->in_a.ptr, n_points, *cam, W, H,
                                      (unsigned*)c->keys.ptr, (double*)c->out_a.ptr),
            "points launch");
    SVA_HIP(c, hipMemcpyAsync(depth, c->out_a.ptr, dbytes, hipMemcpyDeviceToHost, st), "download");
    SVA_HIP(c, hipStreamSynchronize(st), "sync");
    return SVA_OK;
}

int sva_depth_to_points_d(void* ctx, const double* depth, int W, int H, const sva_camera* cam,
                          double* points, int64_t* n_points) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_planes(c, W, H, (size_t)W)) || (s = check_camera(c, cam))) return s;
    if (!depth || !points || !n_points) return fail(c, SVA_ERR_INVALID_ARG, "null argument");
    SVA_HIP(c, c->counts.ensure(d2p_units(W, H) * 4), "count workspace");
    SVA_HIP(c, c->total.ensure(sizeof(long long)), "count workspace");
    SVA_HIP(c, launch_depth_to_points(*c, depth, W, H, *cam, (unsigned*)c->counts.ptr,
                                      (long long*)c->total.ptr, points), "d2p launch");
    long long n = 0;
    SVA_HIP(c, hipMemcpyAsync(&n, c->total.ptr, sizeof(n), hipMemcpyDeviceToHost, c->stream),
            "download");
    SVA_HIP(c, hipStreamSynchronize(c->stream), "sync");
    *n_points = n;
    return SVA_OK;
}

int sva_depth_to_points(void* ctx, const double* depth, int W, int H, const sva_camera* cam,
                        double* points, int64_t* n_points) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_planes(c, W, H, (size_t)W)) || (s = check_camera(c, cam))) return s;
    if (!depth || !points || !n_points) return fail(c, SVA_ERR_INVALID_ARG, "null argument");
    const size_t np = (size_t)W * H;
    SVA_HIP(c, c->in_a.ensure(np * 8), "staging");
    SVA_HIP(c, c->out_a.ensure(np * 24), "staging");
    SVA_HIP(c, c->counts.ensure(d2p_units(W, H) * 4), "count workspace");
    SVA_HIP(c, c->total.ensure(sizeof(long long)), "count workspace");
    hipStream_t st = c->stream;
    SVA_HIP(c, hipMemcpyAsync(c->in_a.ptr, depth, np * 8, hipMemcpyHostToDevice, st), "upload");
    SVA_HIP(c, launch_depth_to_points(*c, (double*)c->in_a.ptr, W, H, *cam,
                                      (unsigned*)c->counts.ptr, (long long*)c->total.ptr,
                                      (double*)c->out_a.ptr), "d2p launch");
    long long n = 0;
    SVA_HIP(c, hipMemcpyAsync(&n, c->total.ptr, sizeof(n), hipMemcpyDeviceToHost, st), "download");
    SVA_HIP(c, hipStreamSynchronize(st), "sync");
    if (n > 0)
        SVA_HIP(c, hipMemcpyAsync(points, c->out_a.ptr, (size_t)n * 24, hipMemcpyDeviceToHost, st),
                "download");
    SVA_HIP(c, hipStreamSynchronize(st), "sync");
    *n_points = n;
    return SVA_OK;
}

// ---------------------------------------------------- ingestion (§8f 4) --
int sva_resize_half_size(int W, int H, int* out_w, int* out_h) {
    if (W < 0 || H < 0 || !out_w || !out_h) return SVA_ERR_INVALID_ARG;
    resize_half_size(W, H, out_w, out_h);
    return SVA_OK;
}

int sva_resize_half_d(void* ctx, const uint8_t* src, int W, int H, size_t pitch, uint8_t* dst,
                      size_t dst_pitch) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s, dw, dh;
    if ((s = check_planes(c, W, H, pitch))) return s;
    resize_half_size(W, H, &dw, &dh);
    if (!src || (!dst && dw > 0 && dh > 0) || dst_pitch < (size_t)dw)
        return fail(c, SVA_ERR_INVALID_ARG, "bad resize argument");
    SVA_HIP(c, launch_resize_half(*c, src, W, H, pitch, dst, dst_pitch), "resize launch");
    return SVA_OK;
}

int sva_resize_half(void* ctx, const uint8_t* src, int W, int H, size_t pitch, uint8_t* dst,
                    size_t dst_pitch) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s, dw, dh;
    if ((s = check_planes(c, W, H, pitch))) return s;
    resize_half_size(W, H, &dw, &dh);
    if (!src || (!dst && dw > 0 && dh > 0) || dst_pitch < (size_t)dw)
        return fail(c, SVA_ERR_INVALID_ARG, "bad resize argument");
    if (dw == 0 || dh == 0) return SVA_OK;
    const size_t sb = (size_t)H * pitch, db = (size_t)dh * dst_pitch;
    SVA_HIP(c, c->in_a.ensure(sb), "staging");
    SVA_HIP(c, c->out_a.ensure(db), "staging");
    hipStream_t st = c->stream;
    SVA_HIP(c, hipMemcpyAsync(c->in_a.ptr, src, sb, hipMemcpyHostToDevice, st), "upload");
    SVA_HIP(c, launch_resize_half(*c, (uint8_t*)c->in_a.ptr, W, H, pitch, (uint8_t*)c->out_a.ptr,
                                  dst_pitch), "resize launch");
    SVA_HIP(c, hipMemcpyAsync(dst, c->out_a.ptr, db, hipMemcpyDeviceToHost, st), "download");
    SVA_HIP(c, hipStreamSynchronize(st), "sync");
    return SVA_OK;
}

// ----------------------------------------------------------- evaluation --
namespace {
int check_dims(Ctx* c, int w, int h) {
    if (w <= 0 || h <= 0 || (size_t)w * h > ((size_t)1 << 31))
        return fail(c, SVA_ERR_INVALID_ARG, "matrix dimensions must be positive (< 2^31 elements)");
    return SVA_OK;
}

// Host-buffer form of the resize / error entry points: upload, run, download.
int host_resize(Ctx* c, const double* src, int sw, int sh, const double* ref, int dw, int dh,
                double scale, double* dst) {
    const size_t sb = (size_t)sw * sh * 8, db = (size_t)dw * dh * 8;
    SVA_HIP(c, c->in_a.ensure(sb), "staging");
    SVA_HIP(c, c->out_a.ensure(db), "staging");
    if (ref) SVA_HIP(c, c->in_b.ensure(db), "staging");
    hipStream_t st = c->stream;
    SVA_HIP(c, hipMemcpyAsync(c->in_a.ptr, src, sb, hipMemcpyHostToDevice, st), "upload");
    if (ref) SVA_HIP(c, hipMemcpyAsync(c->in_b.ptr, ref, db, hipMemcpyHostToDevice, st), "upload");
    SVA_HIP(c, launch_resize_linear(*c, (double*)c->in_a.ptr, sw, sh, (double*)c->out_a.ptr, dw, dh,
                                    ref ? (double*)c->in_b.ptr : nullptr, scale), "resize launch");
    SVA_HIP(c, hipMemcpyAsync(dst, c->out_a.ptr, db, hipMemcpyDeviceToHost, st), "download");
    SVA_HIP(c, hipStreamSynchronize(st), "sync");
    return SVA_OK;
}
}  // namespace

int sva_resize_linear_f64_d(void* ctx, const double* src, int sw, int sh, double* dst, int dw,
                            int dh) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_dims(c, sw, sh)) || (s = check_dims(c, dw, dh))) return s;
    if (!src || !dst) return fail(c, SVA_ERR_INVALID_ARG, "null matrix");
    SVA_HIP(c, launch_resize_linear(*c, src, sw, sh, dst, dw, dh, nullptr, 0.0), "resize launch");
    return SVA_OK;
}

int sva_resize_linear_f64(void* ctx, const double* src, int sw, int sh, double* dst, int dw,
                          int dh) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_dims(c, sw, sh)) || (s = check_dims(c, dw, dh))) return s;
    if (!src || !dst) return fail(c, SVA_ERR_INVALID_ARG, "null matrix");
    return host_resize(c, src, sw, sh, nullptr, dw, dh, 0.0, dst);
}

int sva_ref_error_d(void* ctx, const double* depth, int w, int h, const double* ref, int rw,
                    int rh, double scale, double* error) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_dims(c, w, h)) || (s = check_dims(c, rw, rh))) return s;
    if (!depth || !ref || !error) return fail(c, SVA_ERR_INVALID_ARG, "null matrix");
    SVA_HIP(c, launch_resize_linear(*c, depth, w, h, error, rw, rh, ref, scale), "resize launch");
    return SVA_OK;
}

int sva_ref_error(void* ctx, const double* depth, int w, int h, const double* ref, int rw, int rh,
                  double scale, double* error) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_dims(c, w, h)) || (s = check_dims(c, rw, rh))) return s;
    if (!depth || !ref || !error) return fail(c, SVA_ERR_INVALID_ARG, "null matrix");
    return host_resize(c, depth, w, h, ref, rw, rh, scale, error);
}

int sva_masked_mean_d(void* ctx, const double* image, const uint8_t* mask, int w, int h,
                      double* mean) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_dims(c, w, h))) return s;
    if (!image || !mean) return fail(c, SVA_ERR_INVALID_ARG, "null argument");
    SVA_HIP(c, c->scratch_u16.ensure(masked_mean_workspace()), "reduction workspace");
    double* dmean = (double*)((char*)c->scratch_u16.ptr + masked_mean_workspace() - sizeof(double));
    SVA_HIP(c, launch_masked_mean(*c, image, mask, (size_t)w * h, c->scratch_u16.ptr, dmean),
            "mean launch");
    SVA_HIP(c, hipMemcpyAsync(mean, dmean, sizeof(double), hipMemcpyDeviceToHost, c->stream),
            "download");
    SVA_HIP(c, hipStreamSynchronize(c->stream), "sync");
    return SVA_OK;
}

int sva_masked_mean(void* ctx, const double* image, const uint8_t* mask, int w, int h,
                    double* mean) {
    Ctx* c = as_ctx(ctx);
    SVA_CHECK_CTX(c);
    int s;
    if ((s = check_dims(c, w, h))) return s;
    if (!image || !mean) return fail(c, SVA_ERR_INVALID_ARG, "null argument");
    const size_t n = (size_t)w * h;
    SVA_HIP(c, c->in_a.ensure(n * 8), "staging");
    SVA_HIP(c, c->in_mask.ensure(mask ? n : 1), "staging");
    hipStream_t st = c->stream;
    SVA_HIP(c, hipMemcpyAsync(c->in_a.ptr, image, n * 8, hipMemcpyHostToDevice, st), "upload");
    if (mask) SVA_HIP(c, hipMemcpyAsync(c->in_mask.ptr, mask, n, hipMemcpyHostToDevice, st), "upload");
    return sva_masked_mean_d(ctx, (double*)c->in_a.ptr, mask ? (uint8_t*)c->in_mask.ptr : nullptr, w,
                             h, mean);
}

}  // extern "C"
