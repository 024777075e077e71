/*
 * refine_oracle.c -- CPU ORACLE (test infrastructure only, see sva_oracle.h)
 * for the SURVEY.md §8f rows 1-2: disparity refinement and depth <-> 3-D
 * points.  Each function restates the reference loop it cites; the
 * reference's undefined / non-deterministic corners get one fixed meaning,
 * listed in DESIGN.md §2.7 and repeated here:
 *   - pixels a loop skips are left as the caller's buffer had them (the
 *     reference leaves them uninitialised);
 *   - the refinement's intermediate shifted image starts zeroed (the
 *     reference's `Mat{size,type}` is uninitialised);
 *   - a double -> int conversion whose value is NaN or outside int range
 *     skips the pixel/point (x86 gives INT_MIN there, which the reference's
 *     bounds check then rejects);
 *   - the refined value double -> uchar wraps mod 256 ((uchar)(int)v, x86).
 * All f64 arithmetic in the reference's operand order, built with
 * -ffp-contract=off.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "sva_oracle.h"

static double norm3(const double a[3], const double b[3]) {
    double x = a[0] - b[0], y = a[1] - b[1], z = a[2] - b[2];
    return sqrt(x * x + y * y + z * z);
}

/* (int) of a double with the skip rule above; returns 0 if not representable. */
static int to_int(double v, long long* out) {
    if (!(v > -2147483649.0 && v < 2147483648.0)) return 0;   /* NaN fails too */
    *out = (long long)(int)v;
    return 1;
}

/* shiftPerspectiveWithDisparity (functions.cpp:55-77). */
void svo_shift_perspective(const svo_camera* in, const svo_camera* out, const uint8_t* disp,
                           const uint8_t* img, int W, int H, ptrdiff_t pitch, uint8_t* shifted) {
    double n = norm3(in->pos, out->pos);
    double preX = (in->pos[0] - out->pos[0]) / n;
    double preY = (in->pos[1] - out->pos[1]) / n;
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            double d = disp[(size_t)y * pitch + x];
            if (d == 0) continue;
            long long sx, sy;
            if (!to_int(d * preX + x, &sx) || !to_int(d * preY + y, &sy)) continue;
            if (sy >= H || sy < 0 || sx >= W || sx < 0) continue;
            shifted[(size_t)y * pitch + x] = img[(size_t)sy * pitch + sx];
        }
}

/* 0/1 direction of functions.cpp:23-25: v / norm(v) && (v > 0.001). */
static int unit01(double v) { return v > 0.001 ? 1 : 0; }

static int64_t sad_win(const uint8_t* a, const uint8_t* b, ptrdiff_t pitch, int w) {
    int64_t s = 0;
    for (int v = 0; v < w; v++)
        for (int u = 0; u < w; u++) {
            int d = (int)a[(size_t)v * pitch + u] - (int)b[(size_t)v * pitch + u];
            s += d < 0 ? -d : d;
        }
    return s;
}

/* improveWithDisparity (functions.cpp:11-52).  cams = [n][2] (cam[0], cam[1]
 * of each pair), images[c] = the image paired with the centre view.  strict:
 * return -1 at the first masked pixel whose window leaves the image (the
 * reference's cv::Mat ROI throws there); otherwise such pixels are skipped.
 * out: pixels written by the last pair that reached them (last wins). */
int svo_improve_with_disparity(const uint8_t* disp, const uint8_t* center,
                               const uint8_t* const* images, const svo_camera* cams, int n,
                               int W, int H, ptrdiff_t pitch, const uint8_t* mask, int window,
                               int strict, uint8_t* out) {
    int k = (window - 1) / 2;
    uint8_t* shifted = (uint8_t*)malloc((size_t)H * pitch);
    if (!shifted) return -2;
    for (int c = 0; c < n; c++) {
        const svo_camera* c0 = &cams[2 * c];
        const svo_camera* c1 = &cams[2 * c + 1];
        memset(shifted, 0, (size_t)H * pitch);
        svo_shift_perspective(c0, c1, disp, images[c], W, H, pitch, shifted);
        int ddx = unit01(c0->pos[0] - c1->pos[0]);
        int ddy = unit01(c0->pos[1] - c1->pos[1]);
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++) {
                if (mask && mask[(size_t)y * pitch + x] == 0) continue;
                /* every window [p-k, p+k)^2 must lie inside the image */
                int ok = x - k >= 0 && x + k <= W && y - k >= 0 && y + k <= H;
                int lo = -5, hi = 5;
                ok = ok && x + lo * ddx - k >= 0 && x + hi * ddx + k <= W &&
                     y + lo * ddy - k >= 0 && y + hi * ddy + k <= H;
                if (!ok) {
                    if (strict) { free(shifted); return -1; }
                    continue;
                }
                const uint8_t* win = center + (size_t)(y - k) * pitch + (x - k);
                int64_t best = 0;
                int bi = 0;
                for (int p = 0; p <= 10; p++) {
                    int nx = x + ddx * (p - 5), ny = y + ddy * (p - 5);
                    int64_t e = sad_win(shifted + (size_t)(ny - k) * pitch + (nx - k), win, pitch,
                                        2 * k);
                    if (p == 0 || e < best) { best = e; bi = p; }
                }
                double v = (double)disp[(size_t)y * pitch + x] + (double)(bi - 5) * (double)(ddx + ddy);
                out[(size_t)y * pitch + x] = (uint8_t)(int)v;
            }
    }
    free(shifted);
    return 0;
}

/* shiftPerspective2 (functions.cpp:79-103): scatter, x-major loop, last write
 * wins; depth < 0.5 skipped. */
void svo_shift_perspective2(const svo_camera* in, const svo_camera* out, const double* depth,
                            int W, int H, double* shifted) {
    double preX = (in->pos[0] - out->pos[0]) * in->f / in->pixel_size;
    double preY = (in->pos[1] - out->pos[1]) * in->f / in->pixel_size;
    for (int x = 0; x < W; x++)
        for (int y = 0; y < H; y++) {
            double d = depth[(size_t)y * W + x];
            if (d < 0.5) continue;
            long long tx, ty;
            if (!to_int(preX / d, &tx) || !to_int(preY / d, &ty)) continue;
            long long sx = tx + x, sy = ty + y;
            if (sy >= H || sy < 0 || sx >= W || sx < 0) continue;
            shifted[(size_t)sy * W + sx] = d;
        }
}

/* Camera::project (Camera.cpp:15-21) with the skip rule; 0 = not representable. */
static int project_pt(const svo_camera* cam, const double P[3], long long* px, long long* py) {
    double mult = cam->f / (P[2] - cam->pos[2]) / cam->pixel_size;
    return to_int((P[0] - cam->pos[0]) * mult, px) && to_int((P[1] - cam->pos[1]) * mult, py);
}

/* Points3DToDepthMap (functions.cpp:118-132): point order, last wins. */
void svo_points_to_depth(const double* pts, int64_t n, const svo_camera* cam, int W, int H,
                         double* depth) {
    int hx = W / 2, hy = H / 2;
    for (int64_t i = 0; i < n; i++) {
        long long px, py;
        if (!project_pt(cam, pts + 3 * i, &px, &py)) continue;
        px += hx;
        py += hy;
        if (px >= 0 && px < W && py >= 0 && py < H)
            depth[(size_t)py * W + px] = pts[3 * i + 2] - cam->pos[2];
    }
}

/* DepthMapToPoints3D (functions.cpp:134-146): column-major order, depth > 0.1.
 * pts capacity W*H*3; returns the point count. */
int64_t svo_depth_to_points(const double* depth, int W, int H, const svo_camera* cam,
                            double* pts) {
    int hx = W / 2, hy = H / 2;
    int64_t n = 0;
    for (int u = 0; u < W; u++)
        for (int v = 0; v < H; v++) {
            double d = depth[(size_t)v * W + u];
            if (!(d > 0.1)) continue;
            double r[3];
            svo_cam_inv_project(cam, u - hx, v - hy, r);
            pts[3 * n + 0] = cam->pos[0] + r[0] * d;
            pts[3 * n + 1] = cam->pos[1] + r[1] * d;
            pts[3 * n + 2] = cam->pos[2] + r[2] * d;
            n++;
        }
    return n;
}

/* ---- ingestion: resize(img, img, Size(), 0.5, 0.5) -----
 * CameraStereoVision.cpp:18 with the default INTER_LINEAR.  OpenCV 4.2 routes
 * an exact 2x INTER_LINEAR reduction to its fast INTER_AREA path (third-party,
 * absent here: parity unpinned; restated from its published algorithm):
 *   dsize = (cvRound(W * 0.5), cvRound(H * 0.5))      (round half to even)
 *   full 2x2 block:    dst = (s00 + s01 + s10 + s11 + 2) >> 2
 *   partial block (the last row/column when cvRound rounded up):
 *                      dst = cvRound(sum / count) over the in-image pixels   */
static int cv_round_half_even(double v) {
    double r = floor(v + 0.5);
    if (r - v == 0.5 && fmod(r, 2.0) != 0.0) r -= 1.0;   /* exact .5: to even */
    return (int)r;
}

void svo_resize_half_size(int W, int H, int* dw, int* dh) {
    *dw = cv_round_half_even(W * 0.5);
    *dh = cv_round_half_even(H * 0.5);
}

void svo_resize_half(const uint8_t* src, int W, int H, ptrdiff_t pitch, uint8_t* dst,
                     ptrdiff_t dpitch) {
    int dw, dh;
    svo_resize_half_size(W, H, &dw, &dh);
    for (int y = 0; y < dh; y++)
        for (int x = 0; x < dw; x++) {
            int sx = 2 * x, sy = 2 * y, sum = 0, cnt = 0;
            for (int v = 0; v < 2; v++)
                for (int u = 0; u < 2; u++)
                    if (sx + u < W && sy + v < H) {
                        sum += src[(size_t)(sy + v) * pitch + sx + u];
                        cnt++;
                    }
            dst[(size_t)y * dpitch + x] =
                cnt == 4 ? (uint8_t)((sum + 2) >> 2) : (uint8_t)cv_round_half_even((double)sum / cnt);
        }
}
