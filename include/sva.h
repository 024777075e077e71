/*
 * sva.h -- C-ABI of libsva.so, the MI355X-native stereo disparity engine.
 *
 * This is the drop-in boundary for the reference's array-stereo cost-volume
 * path.  The reference (Nahuel-M/StereoVisionArray) has no plugin API: its hot
 * loop is written inline in main() (src/CameraStereoVision.cpp:44-95) and
 * reaches helpers through include/functions.h and include/Camera.h.  Each
 * entry point below names the reference code it replaces.
 *
 * Conventions
 *   - extern "C", plain pointers and sizes, no C++/torch types.
 *   - Every function returns an int status: SVA_OK (0) or an SVA_ERR_* code.
 *     No exception crosses the ABI.  sva_last_error() gives the message of the
 *     last failing call on that context.
 *   - Functions without suffix take HOST buffers and are synchronous.
 *     Functions with suffix _d take DEVICE buffers (hipMalloc'd on the
 *     context's device) and are asynchronous on the context's stream; call
 *     sva_synchronize() (or synchronise the stream yourself) before reading.
 *   - Images are 8-bit grayscale, row-major, row pitch in bytes (>= width).
 *     Every other array is dense (pitch = width).
 *   - A context owns one device and one stream and is not re-entrant; calls on
 *     different contexts may run concurrently from different host threads.
 *   - There is no CPU fallback: if no HIP device is usable every compute call
 *     fails with SVA_ERR_NO_DEVICE.
 */
#ifndef SVA_H
#define SVA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SVA_ABI_VERSION 6

enum {
    SVA_OK = 0,
    SVA_ERR_INVALID_ARG = 1,   /* bad size / pointer / parameter            */
    SVA_ERR_UNSUPPORTED = 2,   /* parameter combination not built           */
    SVA_ERR_DEVICE = 3,        /* HIP runtime error                         */
    SVA_ERR_OUT_OF_MEMORY = 4, /* workspace allocation failed               */
    SVA_ERR_NO_DEVICE = 5      /* no usable HIP device                      */
};

/* Mirrors class Camera (include/Camera.h:6-21): public f, pos3D, pixel_size. */
typedef struct sva_camera {
    double f;
    double pos[3];
    double pixel_size;
} sva_camera;

/* Mode S parameters.  Use sva_sgm_params_default(). */
typedef struct sva_sgm_params {
    int32_t D;           /* disparity count, 1..256 (whole-frame entry points; the
                            stage entry points take 64, 128, 192 or 256).  Other
                            D run at the next of those widths with the extra
                            disparities masked out              */
    int32_t dmin;        /* first disparity                                        */
    int32_t dir;         /* x component of the match step: +1: x+(dmin+d) in the
                            other image, -1: x-(dmin+d) (rectified horizontal);
                            see dir_y for array baselines                          */
    int32_t P1;          /* small-jump penalty (default 10)                        */
    int32_t P2;          /* large-jump penalty (default 120); 0 <= P1, P2 <= 193    */
    int32_t subpixel;    /* 1: also write the f32 parabola sub-pixel map          */
    int32_t lr_check;    /* 1: left/right consistency check       */
    int32_t lr_max_diff; /* max |dL - dR| kept by the check (default 1)            */
    uint16_t invalid;    /* disparity written for pixels the check rejects         */
    uint16_t _pad;
    int32_t dir_y;       /* y component (default 0).  (dir, dir_y) = integer
                            baseline direction of an array pair, |comp| <= 255:
                            disparity s = dmin+d counts pixels along the major
                            axis, the minor offset is round_half_up(s*m/M)
                            (DESIGN.md §2.2); (+-1,0), (0,+-1), (+-1,+-1) are the
                            horizontal / vertical / 45-degree cases              */
} sva_sgm_params;

/* One stereo pair for the batch API. */
typedef struct sva_pair_job {
    const uint8_t* left;  /* host, reference image                  */
    const uint8_t* right; /* host, matched image                    */
    int32_t width, height;
    size_t pitch;
    uint16_t* disp;       /* host, width*height                     */
    float* subpix;        /* host, width*height or NULL             */
} sva_pair_job;

/* ------------------------------------------------------------ context --- */
void sva_sgm_params_default(sva_sgm_params* p);
int sva_abi_version(void);
int sva_device_count(int* count);
int sva_create(int device, void** ctx_out);          /* sva_ctx* as void*   */
int sva_destroy(void* ctx);
/* Adopt an external hipStream_t (NULL = the context's own stream). */
int sva_set_stream(void* ctx, void* hip_stream);
int sva_synchronize(void* ctx);
const char* sva_last_error(void* ctx);
const char* sva_status_string(int status);
/* Pre-size the workspace for W x H x D (optional; calls grow it on demand).
 * When the frame's stage buffers (cost volume, diagonal path volumes,
 * checkpoints) reach 4 GiB, reserve also checks their placement: it times the
 * path kernel on the buffers it got and on up to five further allocations of
 * them (all held until it chooses, while a quarter of the device memory stays
 * free), keeps the fastest set and frees the others (at 4K
 * D=256 the kernel's rate depends on which physical pages the 10.6 GB of
 * volumes land on, 4.3-4.9 ms, and not on anything else measured).  About
 * 0.2 s at 4K D=256, once per allocation; the call then returns after the
 * trial launches have finished on the context stream (work queued on that
 * stream before it runs first).  SVA_DEBUG_PLACEMENT_TRIALS sets the count
 * (1 = off). */
int sva_reserve(void* ctx, int width, int height, int D);

/* Path-aggregation route of sva_disparity_sgm*.  COST_VOLUME (= AUTO, the
 * default): census -> W*H*D u8 cost volume -> 8-path kernel writing the four
 * diagonal volumes and the horizontal / vertical checkpoints -> per-tile
 * recompute of those four directions + WTA (the tile pipeline, DESIGN.md
 * §4.9).  FUSED (the
 * census-fused path kernel of ABI v1-v3, slower at every D once the
 * checkpoint route existed) was removed in ABI v4: selecting it returns
 * SVA_ERR_UNSUPPORTED. */
#define SVA_PATH_KERNEL_COST_VOLUME 0
#define SVA_PATH_KERNEL_FUSED 1
#define SVA_PATH_KERNEL_AUTO 2
int sva_set_path_kernel(void* ctx, int kernel);

/* Kernel timing with hipEvents on the context stream (measurement only).
 * enable: SVA_TIMING_OFF, SVA_TIMING_ALL (every launch), SVA_TIMING_PATHS
 * (only the path-aggregation launch "sgm_paths") or SVA_TIMING_AGG
 * ("sgm_paths" and "wta_hv", the two kernels of the aggregation).  The
 * aggregation kernels are timed by their own dispatch's start/stop events;
 * each timed launch still costs a few microseconds of stream time. */
#define SVA_TIMING_OFF 0
#define SVA_TIMING_ALL 1
#define SVA_TIMING_PATHS 2
#define SVA_TIMING_AGG 3
int sva_set_timing(void* ctx, int enable);
int sva_reset_timing(void* ctx);
/* Total milliseconds and launch count of kernel `name` since the last reset. */
int sva_kernel_time(void* ctx, const char* name, double* total_ms, int64_t* count);

/* Per-context test and debug switches (ABI v6; they replace the round-5
 * SVA_PLANE_SPLIT environment variable, so the environment never changes
 * how production work is dispatched).  Every key defaults to 0 = off.
 *   SVA_DEBUG_PLANE_SPLIT    set: split every Mode R tile into 1..16 workgroup
 *                            shares (0 = the automatic count, refpath.hip
 *                            plane_shares), so the parity tests cover every
 *                            share count at every size.
 *   SVA_DEBUG_FAIL_COST_AT   set: the next sva_disparity_sgm_batch_d call fails
 *                            its n-th cost launch (1-based) with
 *                            SVA_ERR_DEVICE, without launching it; the switch
 *                            then resets to 0 (fault injection for the
 *                            side-stream join test).
 *   SVA_DEBUG_SIDE_IDLE      get: 1 if every side stream of the batch route
 *                            has finished its queued work (hipStreamQuery),
 *                            else 0.
 *   SVA_DEBUG_PLACEMENT_TRIALS  set: buffer sets sva_reserve's placement check
 *                            times (1..8; 1 = no check; 0 = the default, 6).
 *   SVA_DEBUG_PLACEMENT_NS   get: the path kernel's time on the set the last
 *                            check kept, ns (0: no check ran).
 *   SVA_DEBUG_PLACEMENT_WORST_NS  get: the slowest set that check timed, ns. */
#define SVA_DEBUG_PLANE_SPLIT 1
#define SVA_DEBUG_FAIL_COST_AT 2
#define SVA_DEBUG_SIDE_IDLE 3
#define SVA_DEBUG_PLACEMENT_TRIALS 4
#define SVA_DEBUG_PLACEMENT_NS 5
#define SVA_DEBUG_PLACEMENT_WORST_NS 6
int sva_set_debug(void* ctx, int key, int64_t value);
int sva_get_debug(void* ctx, int key, int64_t* value);

/* ------------------------------------------------------ Mode S (SGM) --- */
/* Whole path: census -> Hamming cost -> 8-path SGM -> WTA (+ sub-pixel).
 * Replaces the inline hot loop CameraStereoVision.cpp:44-95 with the
 * north_star SGM matcher.  disp: W*H u16 (dmin + d*); subpix: W*H f32 or NULL.
 * Size limits (SVA_ERR_UNSUPPORTED beyond them): H <= 65535, and W*H*Dn < 2^32
 * where Dn is D rounded up to 64, 128, 192 or 256 -- every volume is addressed
 * with 32-bit byte offsets (e.g. 4K at D = 256 is 2.1e9, within the limit;
 * 8K x 4K at D = 256 is not). */
int sva_disparity_sgm(void* ctx, const uint8_t* left, const uint8_t* right, int width,
                      int height, size_t pitch, const sva_sgm_params* p, uint16_t* disp,
                      float* subpix);
int sva_disparity_sgm_d(void* ctx, const uint8_t* left, const uint8_t* right, int width,
                        int height, size_t pitch, const sva_sgm_params* p, uint16_t* disp,
                        float* subpix);

/* A batch of device-resident frames of one shape on this context's stream:
 * pair j matches jobs[j].left against jobs[j].right along its own step
 * (params.dir, params.dir_y), and every frame's cost volume then goes through
 * ONE sgm_paths and ONE wta_hv launch (up to 8 frames per launch), so small
 * frames fill the chip (the reference's half-size renders,
 * CameraStereoVision.cpp:17-18, at the pair loop of :55).  The jobs must share
 * D, dmin, P1, P2 and subpixel (SVA_ERR_INVALID_ARG otherwise) and may not set
 * lr_check (SVA_ERR_UNSUPPORTED).  maps: [n][H][W] u16 device; subpix:
 * [n][H][W] f32 device or NULL.  Results equal sva_disparity_sgm_d per pair.
 * sva_pair_d is declared with the multi-GPU engine below. */
struct sva_pair_d;
int sva_disparity_sgm_batch_d(void* ctx, const struct sva_pair_d* jobs, int n_jobs, int width,
                              int height, size_t pitch, uint16_t* maps, float* subpix);

/* Stage entry points (device buffers).  Layouts: census W*H u64; C, L
 * [y][x][d] u8; S [y][x][d] u16; L volumes [8][y][x][d] (direction table in
 * DESIGN.md §2.3).  Each buffer must hold exactly its documented shape for
 * the (width, height, D) passed; the tile stages below take byte sizes. */
int sva_census_d(void* ctx, const uint8_t* img, int width, int height, size_t pitch,
                 uint64_t* census);
int sva_cost_d(void* ctx, const uint64_t* census_l, const uint64_t* census_r, int width,
               int height, const sva_sgm_params* p, uint8_t* C);
/* Census of both images and the cost volume in one kernel, the one
 * sva_disparity_sgm* runs: 1-D steps (dir_y = 0), and 2-D steps whose
 * primitive form has |dir_y| = 1 and |dir| <= 3 (every baseline of the
 * reference's 5x5 rig, functions.cpp:148-213, and of a 2x4 grid); other
 * steps return SVA_ERR_UNSUPPORTED.  Same C bytes as sva_census_d x2 ->
 * sva_cost_d; the census maps stay on chip. */
int sva_census_cost_d(void* ctx, const uint8_t* left, const uint8_t* right, int width,
                      int height, size_t pitch, const sva_sgm_params* p, uint8_t* C);
int sva_paths_d(void* ctx, const uint8_t* C, int width, int height, const sva_sgm_params* p,
                uint8_t* L8);
int sva_aggregate_d(void* ctx, const uint8_t* C, int width, int height,
                    const sva_sgm_params* p, uint16_t* S);
/* The two stages of the frame route, the tile pipeline (DESIGN.md §4.9,
 * §4.11).
 *   sva_paths_tile_d: diag = [diag_volumes][H][W][D] u8, the diagonal
 *     volumes (diag_volumes = 4 in this build: directions 4..7, the values of
 *     those slots of sva_paths_d); hckpt = [2][H][nsx][D] u8, hckpt[0][y][s]
 *     = L_0(s*seg + seg - 1, y) and hckpt[1][y][s] = L_1(s*seg, y); vckpt =
 *     [6 - diag_volumes][nsy][W][D] u8, vckpt[0][s][x] = L_2(x, s*seg + seg
 *     - 1), vckpt[1][s][x] = L_3(x, s*seg) (entries with no such column / row
 *     are not written).  Experiment builds that recompute diagonals per tile
 *     (measured slower and not shipped) report
 *     diag_volumes 2 or 0 and carry those diagonals' row checkpoints in
 *     vckpt planes 2.. instead; size every buffer from sva_tile_layout_of.
 *   sva_wta_hv_d: recomputes the checkpointed directions per 16 x seg tile,
 *     sums S with the diagonal volumes, picks d* (+ sub-pixel).
 * Every buffer comes with its size in bytes: a buffer smaller than its plane
 * returns SVA_ERR_INVALID_ARG before anything is launched.  seg, nsx, nsy and
 * the plane sizes come from sva_tile_layout_of (no device needed);
 * sva_tile_check applies the entry points' size test alone. */
typedef struct sva_tile_layout {
    int32_t seg;          /* checkpoint spacing, columns and rows            */
    int32_t nsx, nsy;     /* ceil(W / seg), ceil(H / seg)                    */
    int32_t diag_volumes; /* 4: directions 4..7 (2 or 0: §4.11 builds)     */
    size_t cost_bytes;    /* C      [H][W][D]                                */
    size_t diag_bytes;    /* diag   [diag_volumes][H][W][D]                  */
    size_t hckpt_bytes;   /* hckpt  [2][H][nsx][D]                           */
    size_t vckpt_bytes;   /* vckpt  [6 - diag_volumes][nsy][W][D]            */
} sva_tile_layout;
int sva_tile_layout_of(int width, int height, int D, sva_tile_layout* out);
int sva_tile_check(int width, int height, int D, size_t C_bytes, size_t diag_bytes,
                   size_t hckpt_bytes, size_t vckpt_bytes);
int sva_paths_tile_d(void* ctx, const uint8_t* C, size_t C_bytes, int width, int height,
                     const sva_sgm_params* p, uint8_t* diag, size_t diag_bytes, uint8_t* hckpt,
                     size_t hckpt_bytes, uint8_t* vckpt, size_t vckpt_bytes);
int sva_wta_hv_d(void* ctx, const uint8_t* C, size_t C_bytes, const uint8_t* diag,
                 size_t diag_bytes, const uint8_t* hckpt, size_t hckpt_bytes,
                 const uint8_t* vckpt, size_t vckpt_bytes, int width, int height,
                 const sva_sgm_params* p, uint16_t* disp, float* subpix);
int sva_wta_d(void* ctx, const uint16_t* S, int width, int height, const sva_sgm_params* p,
              uint16_t* disp, float* subpix);

/* -------------------------------------------- Mode R (reference parity) --- */
/* The reference's own path, bit-exact: per pixel the t_near/t_far ray ends
 * (CameraStereoVision.cpp:60-64, Camera.cpp:15-34), bounds check (:66-71),
 * Bresenham candidates (functions.cpp:253-321), 2k x 2k SAD (getAbsDiff,
 * functions.cpp:215-218), first-minimum WTA (:85), (uchar)(int)norm (:89).
 * mask: W*H u8 or NULL (all selected, :53).  Writes only pixels the pair keeps
 * (multi-pair callers overwrite in order, :55); disp_u16 / valid nullable.
 * The context keeps a W*H key buffer (u32; u64 when a line can hold 4,096
 * or more candidates, i.e. W or H >= 4096; grown on demand, freed by
 * sva_destroy) where a tile's workgroups merge their first minima.
 * Limits: 1 <= k, 2k < W and 2k < H (the reference's own window bounds,
 * CameraStereoVision.cpp:49-51); W, H <= 32767.  k <= 32 runs the
 * offset-plane kernel, larger k one wave per pixel. */
int sva_disparity_ref(void* ctx, const uint8_t* ref_img, const uint8_t* other_img, int width,
                      int height, size_t pitch, const uint8_t* mask,
                      const sva_camera* ref_cam, const sva_camera* other_cam, int k,
                      double t_near, double t_far, uint8_t* disp_u8, uint16_t* disp_u16,
                      uint8_t* valid);
int sva_disparity_ref_d(void* ctx, const uint8_t* ref_img, const uint8_t* other_img,
                        int width, int height, size_t pitch, const uint8_t* mask,
                        const sva_camera* ref_cam, const sva_camera* other_cam, int k,
                        double t_near, double t_far, uint8_t* disp_u8, uint16_t* disp_u16,
                        uint8_t* valid);
/* Stage: per-pixel ray endpoints (CameraStereoVision.cpp:60-71).
 * ends: W*H*4 int32 (p1x, p1y, p2x, p2y); valid: W*H u8. */
int sva_ref_endpoints_d(void* ctx, int width, int height, const sva_camera* ref_cam,
                        const sva_camera* other_cam, int k, double t_near, double t_far,
                        int32_t* ends, uint8_t* valid);

/* ---------------------- refinement and 3-D output --
 * Semantics of the reference's undefined corners: DESIGN.md §2.7.  Every
 * u8 plane of a call shares `pitch`; depth planes are dense W*H f64.  Pixels a
 * routine does not write keep the caller's buffer contents (the reference
 * leaves them uninitialised). */

/* shiftPerspectiveWithDisparity (functions.cpp:55-77): shifted(x, y) =
 * image((int)(d*preX + x), (int)(d*preY + y)) for d = disparity(x, y) != 0,
 * pre = (in.pos - out.pos) / |in.pos - out.pos|. */
int sva_shift_perspective_d(void* ctx, const sva_camera* in_cam, const sva_camera* out_cam,
                            const uint8_t* disparity, const uint8_t* image, int width, int height,
                            size_t pitch, uint8_t* shifted);
int sva_shift_perspective(void* ctx, const sva_camera* in_cam, const sva_camera* out_cam,
                          const uint8_t* disparity, const uint8_t* image, int width, int height,
                          size_t pitch, uint8_t* shifted);

/* improveWithDisparity (functions.cpp:11-52): for each pair i (cam_pairs[2i],
 * cam_pairs[2i+1], paired image images[i]) shift the image by the disparity,
 * then re-search 11 candidates along the 0/1 direction with 2k x 2k SADs,
 * k = (window_size-1)/2 <= 32; the last pair wins.  mask nullable (= the
 * reference's getFaceMask, :13).  strict: fail with SVA_ERR_INVALID_ARG if a
 * masked pixel's window leaves the image (the reference's ROI throws);
 * otherwise such pixels are skipped.  _d: images is a HOST array of device
 * pointers; the host form takes host pointers. */
int sva_improve_with_disparity_d(void* ctx, const uint8_t* disparity, const uint8_t* center,
                                 const uint8_t* const* images, const sva_camera* cam_pairs,
                                 int n_pairs, int width, int height, size_t pitch,
                                 const uint8_t* mask, int window_size, int strict, uint8_t* out);
int sva_improve_with_disparity(void* ctx, const uint8_t* disparity, const uint8_t* center,
                               const uint8_t* const* images, const sva_camera* cam_pairs,
                               int n_pairs, int width, int height, size_t pitch,
                               const uint8_t* mask, int window_size, int strict, uint8_t* out);

/* shiftPerspective2 (functions.cpp:79-103): depth >= 0.5 scattered to
 * (x + (int)(preX/depth), y + (int)(preY/depth)), pre = (in.pos - out.pos)*f/ps;
 * collisions resolve to the last write of the reference's x-major loop. */
int sva_shift_perspective2_d(void* ctx, const sva_camera* in_cam, const sva_camera* out_cam,
                             const double* depth, int width, int height, double* shifted);
int sva_shift_perspective2(void* ctx, const sva_camera* in_cam, const sva_camera* out_cam,
                           const double* depth, int width, int height, double* shifted);

/* Points3DToDepthMap (functions.cpp:118-132): points [n][3] f64 projected
 * with Camera::project + W/2, H/2; depth = z - cam.z; the last point wins. */
int sva_points_to_depth_d(void* ctx, const double* points, int64_t n_points,
                          const sva_camera* cam, int width, int height, double* depth);
int sva_points_to_depth(void* ctx, const double* points, int64_t n_points,
                        const sva_camera* cam, int width, int height, double* depth);

/* DepthMapToPoints3D (functions.cpp:134-146): every pixel with depth > 0.1,
 * in the reference's column-major order, to pos + inv_project(pixel - half)
 * * depth.  points: capacity width*height*3 f64; *n_points (host) = count. */
int sva_depth_to_points_d(void* ctx, const double* depth, int width, int height,
                          const sva_camera* cam, double* points, int64_t* n_points);
int sva_depth_to_points(void* ctx, const double* depth, int width, int height,
                        const sva_camera* cam, double* points, int64_t* n_points);

/* ------------------------------------------ ingestion --
 * resize(img, img, Size(), 0.5, 0.5) with the default INTER_LINEAR
 * (CameraStereoVision.cpp:18): OpenCV 4.2's exact-2x area path -- output
 * (cvRound(W/2), cvRound(H/2)) (half to even), full 2x2 blocks
 * (sum + 2) >> 2, partial edge blocks cvRound(sum / count).  u8 planes. */
int sva_resize_half_size(int width, int height, int* out_width, int* out_height);
int sva_resize_half_d(void* ctx, const uint8_t* src, int width, int height, size_t pitch,
                      uint8_t* dst, size_t dst_pitch);
int sva_resize_half(void* ctx, const uint8_t* src, int width, int height, size_t pitch,
                    uint8_t* dst, size_t dst_pitch);

/* ------------------------------------------ evaluation --
 * The reference's ground-truth comparison (CameraStereoVision.cpp:107-110,
 * 118-119) and calculateAverageError (functions.cpp:348-354), on dense
 * row-major f64 matrices.  OpenCV 4.2 semantics restated (DESIGN.md §2.8;
 * OpenCV absent: parity unpinned):
 *   sva_resize_linear_f64: resize(src, dst, Size(dw, dh)), INTER_LINEAR --
 *     copy at equal size, the area path at exactly 2x, else float-coefficient
 *     bilinear taps (x clamped, y rows clipped).
 *   sva_ref_error: error = (resize(depth, ref.size()) - ref) * scale,
 *     evaluated as OpenCV's addWeighted: a * scale + b * (-scale) + 0.
 *   sva_masked_mean: cv::mean(image, mask)[0]; mask nullable (= all pixels);
 *     0 for an empty mask.  *mean is a HOST pointer in both forms (the _d form
 *     synchronises the context stream). */
int sva_resize_linear_f64_d(void* ctx, const double* src, int src_w, int src_h, double* dst,
                            int dst_w, int dst_h);
int sva_resize_linear_f64(void* ctx, const double* src, int src_w, int src_h, double* dst,
                          int dst_w, int dst_h);
int sva_ref_error_d(void* ctx, const double* depth, int width, int height, const double* ref,
                    int ref_w, int ref_h, double scale, double* error);
int sva_ref_error(void* ctx, const double* depth, int width, int height, const double* ref,
                  int ref_w, int ref_h, double scale, double* error);
int sva_masked_mean_d(void* ctx, const double* image, const uint8_t* mask, int width, int height,
                      double* mean);
int sva_masked_mean(void* ctx, const double* image, const uint8_t* mask, int width, int height,
                    double* mean);

/* Multi-pair depth fusion on the root: per
 * pixel the median of baseline_i * f / (disp_i * pixel_size) over the maps
 * with disp_i != invalid and disp_i > 0 (mean of the middle two for an even
 * count), 0 if none.  disps: [n_maps][H][W] u16 (device / host), baselines:
 * HOST array of n_maps per-axis baselines (m), n_maps <= 32; n_valid nullable. */
int sva_fuse_depth_d(void* ctx, const uint16_t* disps, int n_maps, int width, int height,
                     const double* baselines, double f, double pixel_size, uint16_t invalid,
                     double* depth, uint8_t* n_valid);
int sva_fuse_depth(void* ctx, const uint16_t* disps, int n_maps, int width, int height,
                   const double* baselines, double f, double pixel_size, uint16_t invalid,
                   double* depth, uint8_t* n_valid);

/* Disparity -> depth, CameraStereoVision.cpp:47,98-100 (f64; 0 where disp 0). */
int sva_disparity_to_depth_d(void* ctx, const uint8_t* disp, int n, double cam_distance,
                             double f, double pixel_size, double* depth);
int sva_disparity_to_depth(void* ctx, const uint8_t* disp, int n, double cam_distance,
                           double f, double pixel_size, double* depth);

/* -------------------------------------------------- multi-pair batch --- */
/* Independent pairs round-robin over the given contexts (one per device),
 * one host thread per context.  Replaces the `for (auto pair : pairs)` loop
 * (CameraStereoVision.cpp:55) for whole-image Mode S matching on HOST images.
 * Per context, the upload of pair j+1 and the download of pair j-1 overlap
 * the compute of pair j (pinned staging, separate copy streams).  A failing
 * pair does not stop the others: job_status (nullable, n_jobs entries)
 * receives each pair's status and the call returns the first failure. */
int sva_batch_sgm(void** ctxs, int n_ctx, const sva_pair_job* jobs, int n_jobs,
                  const sva_sgm_params* p, int* job_status);

/* ----------------------------------- multi-GPU engine --- */
/* One process drives several GPUs of a node: pairs are the shard unit (pair j
 * -> device j mod n_devices, and round-robin over that device's streams), each
 * device keeps its own cost and path volumes, and the only exchange is the
 * gather of the finished u16 disparity maps (and f32 sub-pixel maps) to
 * devices[0] over xGMI -- an RCCL grouped send/recv on a single-process
 * communicator (ncclCommInitAll, librccl loaded at sva_multi_create), or peer
 * copies with SVA_MULTI_GATHER_PEER.  north_star / BASELINE configs 4-5;
 * replaces the pair loop at CameraStereoVision.cpp:55 with the pair tables of
 * functions.cpp:148-213 (sva.hpp getCameraPairs). */
#define SVA_MULTI_GATHER_RCCL 0   /* default */
#define SVA_MULTI_GATHER_PEER 1
#define SVA_MULTI_GATHER_ALL 2    /* flag: route device 0's own maps through the
                                     gather too (exercises the exchange on one GPU) */
int sva_multi_create(const int* devices, int n_devices, int streams_per_device, int flags,
                     void** multi_out);
int sva_multi_destroy(void* multi);
/* Block until every queued batch has finished on every device. */
int sva_multi_synchronize(void* multi);
const char* sva_multi_last_error(void* multi);
/* The shard plan, a pure function (no device needed): for job j,
 * device_index[j] = j mod n_devices and context_index[j] = (j / n_devices) mod
 * streams_per_device (nullable outputs); slot_index[j] = rank of j among the
 * jobs of its context (nullable). */
int sva_multi_plan(int n_devices, int streams_per_device, int n_jobs, int32_t* device_index,
                   int32_t* context_index, int32_t* slot_index);
/* The context behind (device_index, stream_index), e.g. for sva_set_timing. */
int sva_multi_context(void* multi, int device_index, int stream_index, void** ctx_out);

/* One device-resident pair: left/right live on device
 * devices[j mod n_devices] (see sva_multi_plan), pitch in bytes. */
typedef struct sva_pair_d {
    const uint8_t* left;
    const uint8_t* right;
    sva_sgm_params params;
} sva_pair_d;
/* Every pair's Mode S map, gathered into maps (device memory on devices[0],
 * [n_jobs][H][W] u16) and, when subpix is non-NULL, the f32 maps of the jobs
 * that set params.subpixel into subpix ([n_jobs][H][W] on devices[0]; the
 * planes of the other jobs are not written).  Asynchronous: the results are
 * complete on devices[0]'s first stream (stream_index 0) once the call returns
 * SVA_OK and that stream has run; sva_multi_synchronize waits for everything.
 * Work the caller queues on that stream after a call (e.g. reading maps) is
 * ordered before the next call writes maps / subpix. */
int sva_batch_sgm_d(void* multi, const sva_pair_d* jobs, int n_jobs, int width, int height,
                    size_t pitch, uint16_t* maps, float* subpix);

/* A camera-array frame from HOST images: pair j matches images[pairs[j].ref]
 * against images[pairs[j].other] with its own params (the 2-D step of its
 * baseline) on device j mod n_devices; the maps are gathered to devices[0],
 * which fuses group g = pairs [group_start[g], group_start[g+1]) (one
 * reference camera, DESIGN.md §2.6, with pairs[j].baseline) into depth[g].
 * Uploads run on per-device copy streams and each pair waits only for its two
 * images, so transfers overlap compute; the fused maps download as each group
 * finishes.  depth: host [n_groups][H][W] f64; n_valid (nullable) host u8,
 * same shape; maps (nullable) host [n_pairs][H][W] u16.  Synchronous.  The
 * pairs of one group must share params.invalid (SVA_ERR_INVALID_ARG). */
typedef struct sva_array_pair {
    int32_t ref;              /* index into images[]: the reference view      */
    int32_t other;            /* index into images[]: the matched view        */
    sva_sgm_params params;    /* D, dmin, (dir, dir_y) = this pair's step     */
    double baseline;          /* major-axis baseline (m) for the fusion       */
} sva_array_pair;
int sva_array_depth(void* multi, const uint8_t* const* images, int n_images, int width,
                    int height, size_t pitch, const sva_array_pair* pairs, int n_pairs,
                    const int32_t* group_start, int n_groups, double f, double pixel_size,
                    double* depth, uint8_t* n_valid, uint16_t* maps);

#ifdef __cplusplus
}
#endif
#endif /* SVA_H */
