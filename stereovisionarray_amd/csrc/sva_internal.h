// sva_internal.h -- context, workspace and kernel-launcher declarations shared
// by the C-ABI (sva_api.cpp) and the HIP kernel translation units.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "sva.h"
#include "sva_tuning.h"

namespace sva {

// Host-side status carrier: every launcher returns hipError_t, the API maps it.
struct Status {
    int code = SVA_OK;
    std::string msg;
};

// Per-kernel hipEvent timing on the context stream.  Events are only recorded
// while timing is enabled; resolution happens lazily in kernel_time().
struct KernelTimer {
    bool enabled = false;
    int mode = 0;              // SVA_TIMING_ALL / _PATHS / _AGG (sva_set_timing)
    struct Pending {
        std::string name;
        hipEvent_t start, stop;
    };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> pool;
    std::map<std::string, std::pair<double, int64_t>> totals;  // ms, count

    hipEvent_t get_event();
    void begin(hipStream_t s, const char* name, hipEvent_t* start_out);
    void end(hipStream_t s, const char* name, hipEvent_t start);
    hipError_t resolve();  // fold pending into totals (synchronises on each stop event)
    void release_all();
};

// Device workspace grown on demand (never shrinks within a context).
struct DevBuf {
    void* ptr = nullptr;
    size_t bytes = 0;
    unsigned flags = 0;   // hipExtMallocWithFlags flags (0 = hipMalloc)
    hipError_t ensure(size_t n);
    void release();
};

struct Ctx {
    int device = -1;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string last_error;
    KernelTimer timer;
    // Mode S workspace
    DevBuf census_l, census_r, cost, paths, ckpt, scratch_u16, disp_r;
    // host-pointer staging
    DevBuf in_a, in_b, in_mask, out_a, out_b, out_c;
    // refinement / 3-D workspace (refine.hip)
    DevBuf in_c, shifted, keys, counts, total;
    // Mode R's split plane loop: one first-minimum key per pixel (refpath.hip).
    // ref_finalize_kernel puts every key it reads back to all-ones, so after
    // the first call only a grown buffer needs the memset: ref_keys_clean =
    // leading bytes known to be all-ones (of allocation ref_keys_alloc)
    DevBuf ref_keys;
    size_t ref_keys_clean = 0;
    const void* ref_keys_alloc = nullptr;
    int cu_count = 256;
    // sva_batch_sgm's per-context pipeline (copy streams, events, pinned and
    // device staging), created on first use and kept for later calls
    std::shared_ptr<void> batch_lane;
    // sva_disparity_sgm_batch_d: side streams for the frames' census + cost
    // (fork / join through events on `stream`), their census workspaces
    std::vector<hipStream_t> side;
    std::vector<hipEvent_t> side_done;
    hipEvent_t fork = nullptr;
    DevBuf census_side;
    // sva_set_debug switches (include/sva.h SVA_DEBUG_*): Mode R shares per
    // tile forced (0 = automatic), and the batch route's injected cost-launch
    // failure (1-based frame of the next call, 0 = off)
    int dbg_plane_split = 0;
    int dbg_fail_cost_at = 0;
    // sva_reserve's placement check: sets to time (0 = tune::kPlacementTrials),
    // and the kept / slowest set's path-kernel time of the last check (ns)
    int placement_trials = 0;
    int64_t placement_ns = 0, placement_worst_ns = 0;
    const void* placement_paths = nullptr;   // the path buffer the last check chose
};

// Which launches a timing mode records: SVA_TIMING_ALL every one,
// SVA_TIMING_PATHS only the path-aggregation launch "sgm_paths" (the
// roofline-graded kernel), SVA_TIMING_AGG that one and the kernel that
// finishes the aggregation, "wta_hv" (bench.py's aggregation roofline).
inline bool timer_wants(const KernelTimer& t, const char* name) {
    if (!t.enabled) return false;
    if (t.mode == SVA_TIMING_ALL) return true;
    if (std::strcmp(name, "sgm_paths") == 0) return true;
    return t.mode == SVA_TIMING_AGG && std::strcmp(name, "wta_hv") == 0;
}

// RAII helper: records timing events around one launch when enabled.
struct ScopedKernelTimer {
    Ctx& c;
    const char* name;
    hipEvent_t start = nullptr;
    ScopedKernelTimer(Ctx& ctx, const char* n) : c(ctx), name(n) {
        if (timer_wants(c.timer, name)) c.timer.begin(c.stream, name, &start);
    }
    ~ScopedKernelTimer() {
        if (c.timer.enabled && start) c.timer.end(c.stream, name, start);
    }
};

// Timing of one launch through hipExtLaunchKernelGGL's start/stop events: the
// runtime stamps them from the kernel's own dispatch, so no separate event
// packets enter the stream (used for the two aggregation kernels, the ones
// bench.py times inside its timed region).  start/stop stay null when timing
// is off.
struct DispatchTimer {
    Ctx& c;
    const char* name;
    hipEvent_t start = nullptr, stop = nullptr;
    bool used = false;   // set by the launch that received start/stop
    DispatchTimer(Ctx& ctx, const char* n) : c(ctx), name(n) {
        if (timer_wants(c.timer, name)) {
            start = c.timer.get_event();
            stop = start ? c.timer.get_event() : nullptr;
            if (!stop && start) { c.timer.pool.push_back(start); start = nullptr; }
        }
    }
    ~DispatchTimer() {
        if (start && stop && used)
            c.timer.pending.push_back(KernelTimer::Pending{name, start, stop});
        else if (start && stop) {
            c.timer.pool.push_back(start);
            c.timer.pool.push_back(stop);
        }
    }
};

// ------------------------------------------------------------- launchers --
// All launchers enqueue on ctx.stream and return the launch status.

// census.hip
hipError_t launch_census(Ctx& c, const uint8_t* img, int W, int H, size_t pitch, uint64_t* out);
hipError_t launch_census_pair(Ctx& c, const uint8_t* left, const uint8_t* right, int W, int H,
                              size_t pitch, uint64_t* out_l, uint64_t* out_r);
// cost.hip
// Census + cost in one kernel (census_cost.hip), 1-D steps (dir = +-1).
bool census_cost_supported(int D);
// D is the native volume width (64/128/192/256); dreal <= D the caller's
// disparity count: d >= dreal gets cost 255 (0 = D).
hipError_t launch_census_cost(Ctx& c, const uint8_t* left, const uint8_t* right, int W, int H,
                              size_t pitch, int D, int dmin, int dir, uint8_t* C, int dreal = 0);
// Census + cost in one kernel for 2-D steps (census_cost2.hip): steps whose
// primitive form has |by| = 1 and |bx| <= 3, native D.
bool census_cost2_supported(int D, int sx, int sy);
hipError_t launch_census_cost2(Ctx& c, const uint8_t* left, const uint8_t* right, int W, int H,
                               size_t pitch, int D, int dmin, int sx, int sy, uint8_t* C,
                               int dreal = 0);
hipError_t launch_cost(Ctx& c, const uint64_t* cl, const uint64_t* cr, int W, int H, int D,
                       int dmin, int dir, uint8_t* C, int dreal = 0);
// sgm_paths.hip -- all 8 directions in one launch.  CK == CKV == nullptr:
// L8 = [8][H][W][D] u8.  CK and CKV set (the tile pipeline, DESIGN.md §4.9,
// §4.11): L8 = [nvol][H][W][D] (directions 5, 7, or 4..7), CK = [2][H][nsx][D]
// and CKV = the vertical then the down-diagonal row checkpoints,
// vck_bytes + dck_bytes (tile_geom below).  npair > 1 (tile pipeline only): a
// batch of frames in one launch, each buffer holding npair such planes back
// to back.
hipError_t launch_paths(Ctx& c, const uint8_t* C, int W, int H, int D, int P1, int P2,
                        uint8_t* L8, uint8_t* CK = nullptr, uint8_t* CKV = nullptr,
                        int npair = 1);
// Tile pipeline geometry: tiles of 16 columns x seg rows (seg = 2^seg_log2),
// checkpoints every seg columns (horizontal lines) and every seg rows
// (vertical lines).
struct TileGeom {
    int seg_log2;
    int ntx, nty;             // tiles per row / per column (nty = vertical segments)
    int nsx;                  // horizontal segments per row
    size_t hck_bytes;         // [2][H][nsx][D]
    size_t vck_bytes;         // [2][nty][W][D]: directions 2, 3
    size_t dck_bytes;         // [2][nty][W][D]: directions 4, 6 (0 when they are volumes)
    int nvol;                 // diagonal volumes the path kernel writes: 2 (5, 7) or 4
};
TileGeom tile_geom(int W, int H, int D);
// Which diagonal pairs the path kernel leaves as row checkpoints instead of
// volumes, per lane width DPL = D / 16: all four on the strip route (D <= 128,
// tune::kStripRoute), else the §4.11 experiment's switches.
constexpr bool diag_ckpt_down(int dpl) {
    return (tune::kStripRoute != 0 && dpl <= 8) || tune::kTileDiagDown != 0;
}
constexpr bool diag_ckpt_up(int dpl) {
    return (tune::kStripRoute != 0 && dpl <= 8) || tune::kTileDiagUp != 0;
}
// wta_strip.hip -- the strip route's final kernel (all eight directions per
// tile from the checkpoints of launch_paths at D <= 128, no volume)
bool wta_strip_supported(int D);
hipError_t launch_wta_strip(Ctx& c, const uint8_t* C, const uint8_t* CK, const uint8_t* CKV, int W,
                            int H, int D, int P1, int P2, int dmin, uint16_t* disp, float* sub,
                            int dreal = 0, int npair = 1);
bool paths_supported(int D);
// Native volume width of a frame with D disparities: 64, 128, 192 or 256
// (the smallest >= D), 0 when D is outside 1..256.
inline int padded_D(int D) {
    return D <= 0 ? 0 : D <= 64 ? 64 : D <= 128 ? 128 : D <= 192 ? 192 : D <= 256 ? 256 : 0;
}
// wta_hv.hip -- the tile pipeline's final kernel: horizontal + vertical
// recompute from the checkpoints of launch_paths(.., CK, CKV), sum with the
// four diagonal volumes L4, WTA.  dreal < D: a padded frame (DESIGN.md
// §4.7), WTA over d < dreal only.
bool wta_hv_supported(int D);
hipError_t launch_wta_hv(Ctx& c, const uint8_t* C, const uint8_t* L4, const uint8_t* CK,
                         const uint8_t* CKV, int W, int H, int D, int P1, int P2, int dmin,
                         uint16_t* disp, float* sub, int dreal = 0, int npair = 1);
// wta.hip
hipError_t launch_sum(Ctx& c, const uint8_t* L8, int W, int H, int D, uint16_t* S);
hipError_t launch_wta_from_sum(Ctx& c, const uint16_t* S, int W, int H, int D, int dmin,
                               uint16_t* disp, float* sub);
hipError_t launch_lr_check(Ctx& c, uint16_t* disp_l, const uint16_t* disp_r, float* sub, int W, int H,
                           int sx, int sy, int max_diff, uint16_t invalid);
// 2-D matching step (sy != 0); sy == 0 forwards to launch_cost(dir = sx).
hipError_t launch_cost2(Ctx& c, const uint64_t* cl, const uint64_t* cr, int W, int H, int D,
                        int dmin, int sx, int sy, uint8_t* C, int dreal = 0);
// Median depth fusion over n_maps <= 32 u16 maps.
// num[i] = baseline_i * f (host-computed, same f64 product as the oracle).
hipError_t launch_fuse_depth(Ctx& c, const uint16_t* disps, int n_maps, size_t np,
                             const double* num, double pixel_size, uint16_t invalid,
                             double* depth, uint8_t* n_valid);
// refpath.hip
hipError_t launch_ref_endpoints(Ctx& c, int W, int H, const sva_camera& cref,
                                const sva_camera& coth, int k, double t_near, double t_far,
                                int32_t* ends, uint8_t* valid);
hipError_t launch_ref_match(Ctx& c, const uint8_t* ref, const uint8_t* other, int W, int H,
                            size_t pitch, const uint8_t* mask, const int32_t* ends,
                            const uint8_t* valid_in, int k, uint8_t* disp_u8,
                            uint16_t* disp_u16, uint8_t* valid_out);
// depth.hip
// refine.hip
hipError_t launch_shift_perspective(Ctx& c, const sva_camera& in, const sva_camera& out,
                                    const uint8_t* disp, const uint8_t* img, int W, int H,
                                    size_t pitch, uint8_t* shifted, bool zero_fill = false);
hipError_t launch_refine(Ctx& c, const uint8_t* disp, const uint8_t* center,
                         const uint8_t* shifted, const uint8_t* mask, int W, int H, size_t pitch,
                         int k, const sva_camera& c0, const sva_camera& c1, uint8_t* out,
                         int* fault);
hipError_t launch_shift_perspective2(Ctx& c, const sva_camera& in, const sva_camera& out,
                                     const double* depth, int W, int H, unsigned* keys,
                                     double* shifted);
hipError_t launch_points_to_depth(Ctx& c, const double* pts, long long n, const sva_camera& cam,
                                  int W, int H, unsigned* keys, double* depth);
size_t d2p_units(int W, int H);
hipError_t launch_depth_to_points(Ctx& c, const double* depth, int W, int H,
                                  const sva_camera& cam, unsigned* counts, long long* total,
                                  double* pts);
// ingest.hip
void resize_half_size(int W, int H, int* dw, int* dh);
// evaluation (evaluate.hip): resize(src, dst, Size(dw, dh)) INTER_LINEAR on
// dense f64; with ref non-null dst = resized * scale + ref * -scale + 0.
hipError_t launch_resize_linear(Ctx& c, const double* src, int sw, int sh, double* dst, int dw,
                                int dh, const double* ref, double scale);
size_t masked_mean_workspace();
hipError_t launch_masked_mean(Ctx& c, const double* img, const uint8_t* mask, size_t n,
                              void* ws, double* mean);
hipError_t launch_resize_half(Ctx& c, const uint8_t* src, int W, int H, size_t pitch,
                              uint8_t* dst, size_t dpitch);
hipError_t launch_disp_to_depth(Ctx& c, const uint8_t* disp, int n, double cam_distance,
                                double f, double pixel_size, double* depth);

}  // namespace sva
