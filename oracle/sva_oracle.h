/*
 * sva_oracle.h -- CPU ORACLE for the stereovisionarray_amd hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load liboracle.so, and only as the checker
 * or the timed CPU baseline.  The product library (libsva.so) never links,
 * loads or calls anything in this directory.
 *
 * PARITY STATUS: "parity unpinned".
 *   - The reference (Nahuel-M/StereoVisionArray) ships no tests, no golden
 *     vectors and no fixtures.
 *   - The reference's hot-path translation units (src/Camera.cpp,
 *     src/functions.cpp) need OpenCV 4.2 headers/libraries that are absent from
 *     this image; building them would require writing stand-in headers, which
 *     this project does not do.  The reference is therefore unbuildable here and
 *     there is no oracle/_ref.
 *   - Mode S (Census / Hamming / 8-path SGM / WTA) does not exist in the
 *     reference at all; its spec is frozen in DESIGN.md §2.
 *   What pins this oracle instead: hand-derived known-answer tests in
 *   tests/test_oracle_kat.py (hand-expanded Bresenham traces of
 *   functions.cpp:253-321, hand-computed Camera.cpp:15-34 projections, census
 *   words, 1-D SGM recurrences, shifted-texture disparities).
 *
 * Mode R functions restate the reference path line by line
 * (src/CameraStereoVision.cpp:44-95, src/Camera.cpp:15-34,
 * src/functions.cpp:215-218,253-321).  Mode S functions restate DESIGN.md §2.
 */
#ifndef SVA_ORACLE_H
#define SVA_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- Mode R -- */

/* Mirrors class Camera (include/Camera.h:6-21): public f, pos3D, pixel_size. */
typedef struct {
    double f;
    double pos[3];
    double pixel_size;
} svo_camera;

/* Camera::project (src/Camera.cpp:15-21). out = (int) truncation toward 0. */
void svo_cam_project(const svo_camera* cam, const double P[3], int out[2]);

/* Camera::inv_project (src/Camera.cpp:25-33). */
void svo_cam_inv_project(const svo_camera* cam, int px, int py, double out[3]);

/* bresenham(pixel1, pixel2) as called at CameraStereoVision.cpp:73
 * (definition functions.cpp:299-321 names its first parameter point2).
 * Writes at most cap points; returns the full point count. */
int svo_bresenham(int p1x, int p1y, int p2x, int p2y, int* xs, int* ys, int cap);

/* getAbsDiff (functions.cpp:215-218): sum |a-b| over a w x h window. */
int64_t svo_sad(const uint8_t* a, ptrdiff_t pitch_a, const uint8_t* b, ptrdiff_t pitch_b,
                int w, int h);

/* Per-pixel endpoint geometry of CameraStereoVision.cpp:60-71.
 * Returns 1 if the pixel survives the bounds check (:66-71), else 0. */
int svo_ref_endpoints(const svo_camera* cref, const svo_camera* coth, int W, int H, int k,
                      double t_near, double t_far, int x, int y, int p1[2], int p2[2]);

/* The hot loop CameraStereoVision.cpp:49-95 for ONE camera pair.
 * Writes only pixels the pair does not skip (last pair overwrites, :55):
 *   disp_u8[y*W+x]  = (uchar)(int)norm(best - (x,y))      (:89, wraps mod 256)
 *   disp_u16[y*W+x] = (int)norm(best - (x,y))              (unwrapped; nullable)
 *   valid[y*W+x]    = 1                                    (nullable)
 * mask: nullable (NULL = every pixel selected, :53).
 * Returns the number of SAD evaluations performed. */
int64_t svo_ref_pair(const uint8_t* ref, const uint8_t* other, int W, int H, ptrdiff_t pitch,
                     const uint8_t* mask, const svo_camera* cref, const svo_camera* coth,
                     int k, double t_near, double t_far,
                     uint8_t* disp_u8, uint16_t* disp_u16, uint8_t* valid);

/* Disparity -> depth (CameraStereoVision.cpp:47,98-100):
 * depth = (‖c0-c1‖·f) / ((double)disp · pixel_size); 0 where disp == 0. */
void svo_disp_to_depth(const uint8_t* disp, int n, double cam_distance, double f,
                       double pixel_size, double* depth);

/* ---------------------------------------------------------------- Mode S -- */

/* Census 9x7.  Bit order row-major over the window, centre
 * skipped, first window element is bit 61; bit = I(q) < I(p).  0 where the
 * window leaves the image (x<4, x>=W-4, y<3, y>=H-3). */
void svo_census(const uint8_t* img, int W, int H, ptrdiff_t pitch, uint64_t* out);

/* Hamming cost: C[(y*W+x)*D+d] = popcount(CL(x,y) ^ CR(x+dir*(dmin+d), y)),
 * 62 when the matched column leaves the image. */
void svo_cost(const uint64_t* cl, const uint64_t* cr, int W, int H, int D, int dmin, int dir,
              uint8_t* C);

/* 2-D matching step.  (sx, sy) = integer baseline direction
 * (bx, by), not both 0; with s = dmin + d the matched pixel is (x, y) +
 * svo_step_offset(s, bx, by): s pixels along the major axis (|bx| >= |by|: x),
 * round_half_up(s*m/M) along the minor one (m, M = minor/major |component|),
 * each with the sign of its component.  Unit steps (+-1, 0), (0, +-1),
 * (+-1, +-1) are the axis / 45-degree cases; by = 0 is svo_cost(dir = sign bx).
 * Array pairs (parallel optical axes, equal f) have exactly this epipolar
 * geometry; the rounding is the closed form of the reference's Bresenham
 * (functions.cpp:299-321). */
void svo_step_offset(int s, int bx, int by, int* ox, int* oy);
void svo_cost2(const uint64_t* cl, const uint64_t* cr, int W, int H, int D, int dmin, int sx,
               int sy, uint8_t* C);

/* One SGM path direction: step vector (rx, ry); L u8 volume. */
void svo_path(const uint8_t* C, int W, int H, int D, int rx, int ry, int P1, int P2, uint8_t* L);

/* Direction table used by every implementation: r = 0..7. */
void svo_direction(int r, int* rx, int* ry);

/* S = sum of the 8 path volumes (u16).  threads <= 1: serial. */
void svo_aggregate(const uint8_t* C, int W, int H, int D, int P1, int P2, uint16_t* S,
                   int threads);

/* WTA + sub-pixel.  sub nullable. */
void svo_wta(const uint16_t* S, int W, int H, int D, int dmin, uint16_t* disp, float* sub);

/* Whole Mode S pipeline; threads <= 1: serial.  sub nullable. */
void svo_sgm(const uint8_t* left, const uint8_t* right, int W, int H, ptrdiff_t pitch, int D,
             int dmin, int dir, int P1, int P2, uint16_t* disp, float* sub, int threads);

/* Mode S on a 2-D matching step (svo_cost2); threads <= 1: serial. */
void svo_sgm2(const uint8_t* left, const uint8_t* right, int W, int H, ptrdiff_t pitch, int D,
              int dmin, int sx, int sy, int P1, int P2, uint16_t* disp, float* sub,
              int threads);

/* Left/right consistency check.  disp_r is the disparity map
 * computed with the roles of the images swapped (dir negated); pixels whose
 * |dL - dR(matched)| > max_diff are set to invalid. */
void svo_lr_check(uint16_t* disp_l, const uint16_t* disp_r, int W, int H, int dir,
                  int max_diff, uint16_t invalid);
/* The f32 sub-pixel map after the check: NaN wherever disp == invalid. */
void svo_lr_sub(const uint16_t* disp, float* sub, size_t n, uint16_t invalid);
/* 2-D form: the right-reference map was computed with (-sx, -sy); the left
 * disparity d is followed to (x, y) + svo_step_offset(d, sx, sy). */
void svo_lr_check2(uint16_t* disp_l, const uint16_t* disp_r, int W, int H, int sx, int sy,
                   int max_diff, uint16_t invalid);

/* Multi-pair depth fusion: per pixel, depth_i =
 * (baseline_i * f) / ((double)disp_i * pixel_size) for every map i with
 * disp_i != invalid and disp_i > 0; output the median (mean of the two middle
 * values for an even count, f64), 0 where no map is valid.  n_valid nullable. */
void svo_fuse_depth(const uint16_t* disps, int n_maps, int W, int H, const double* baseline,
                    double f, double pixel_size, uint16_t invalid, double* depth,
                    uint8_t* n_valid);

/* --------------------------------------- refinement / 3-D -- */
/* Semantics for the reference's undefined corners: refine_oracle.c header,
 * DESIGN.md §2.7.  Pixels a loop skips keep the caller's buffer contents. */

/* shiftPerspectiveWithDisparity (functions.cpp:55-77): gather. */
void svo_shift_perspective(const svo_camera* in, const svo_camera* out, const uint8_t* disp,
                           const uint8_t* img, int W, int H, ptrdiff_t pitch, uint8_t* shifted);

/* improveWithDisparity (functions.cpp:11-52); cams = [n][2]; returns 0, or -1
 * when strict and a masked pixel's window leaves the image (reference throws). */
int svo_improve_with_disparity(const uint8_t* disp, const uint8_t* center,
                               const uint8_t* const* images, const svo_camera* cams, int n,
                               int W, int H, ptrdiff_t pitch, const uint8_t* mask, int window,
                               int strict, uint8_t* out);

/* shiftPerspective2 (functions.cpp:79-103): scatter, last write in x-major order wins. */
void svo_shift_perspective2(const svo_camera* in, const svo_camera* out, const double* depth,
                            int W, int H, double* shifted);

/* Points3DToDepthMap (functions.cpp:118-132): pts [n][3], last point wins. */
void svo_points_to_depth(const double* pts, int64_t n, const svo_camera* cam, int W, int H,
                         double* depth);

/* DepthMapToPoints3D (functions.cpp:134-146): column-major, depth > 0.1;
 * pts capacity W*H*3; returns the count. */
int64_t svo_depth_to_points(const double* depth, int W, int H, const svo_camera* cam,
                            double* pts);

/* Ingestion: resize(..., 0.5, 0.5) INTER_LINEAR as OpenCV
 * 4.2's exact-2x area path (refine_oracle.c; parity unpinned, OpenCV absent). */
void svo_resize_half_size(int W, int H, int* dw, int* dh);
void svo_resize_half(const uint8_t* src, int W, int H, ptrdiff_t pitch, uint8_t* dst,
                     ptrdiff_t dpitch);

/* Evaluation (eval_oracle.c, OpenCV restated, parity
 * unpinned): resize(src, dst, Size(dw, dh)) INTER_LINEAR on dense f64,
 * error = resize(depth, ref.size()) * scale + ref * -scale + 0, and
 * cv::mean(image, mask)[0] (mask nullable = all). */
void svo_resize_linear_f64(const double* src, int sw, int sh, double* dst, int dw, int dh);
void svo_ref_error(const double* depth, int w, int h, const double* ref, int rw, int rh,
                   double scale, double* error);
double svo_masked_mean(const double* image, const uint8_t* mask, int w, int h);

#ifdef __cplusplus
}
#endif
#endif
