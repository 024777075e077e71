/*
 * refpath_oracle.c -- CPU ORACLE, Mode R ("reference parity" path).
 * TEST INFRASTRUCTURE ONLY (see sva_oracle.h).  Parity unpinned: the
 * reference is unbuildable here (needs OpenCV); see DESIGN.md §5.
 *
 * Each function restates one reference function.  Floating-point expressions
 * keep the reference's operand order; this file is compiled with
 * -ffp-contract=off so no FMA contraction changes a rounding.
 */
#include "sva_oracle.h"

#include <math.h>
#include <stdlib.h>

/* Camera::project -- src/Camera.cpp:15-21
 *   double mult = f / (Pos3D.z - this->pos3D.z) / pixel_size;
 *   pixel.x = int((Pos3D.x - this->pos3D.x) * mult);  (same for y)          */
void svo_cam_project(const svo_camera* c, const double P[3], int out[2]) {
    double mult = c->f / (P[2] - c->pos[2]) / c->pixel_size;
    out[0] = (int)((P[0] - c->pos[0]) * mult);
    out[1] = (int)((P[1] - c->pos[1]) * mult);
}

/* Camera::inv_project -- src/Camera.cpp:25-33
 *   Point3d vector{pixel.x*pixel_size, pixel.y*pixel_size, f};
 *   return vector / norm(vector);
 * cv::norm(Point3d) = sqrt(x*x + y*y + z*z) (left to right); Point3_ / double
 * divides each component (OpenCV 4.2 operator/=).                            */
void svo_cam_inv_project(const svo_camera* c, int px, int py, double out[3]) {
    double v0 = (double)px * c->pixel_size;
    double v1 = (double)py * c->pixel_size;
    double v2 = c->f;
    double n = sqrt(v0 * v0 + v1 * v1 + v2 * v2);
    out[0] = v0 / n;
    out[1] = v1 / n;
    out[2] = v2 / n;
}

/* plotLineLow -- functions.cpp:253-274 */
static int plot_line_low(int x0, int y0, int x1, int y1, int* xs, int* ys, int cap) {
    int dx = x1 - x0, dy = y1 - y0, yi = 1, n = 0;
    if (dy < 0) { yi = -1; dy = -dy; }
    int D = 2 * dy - dx, y = y0;
    for (int x = x0; x <= x1; x++) {
        if (n < cap) { xs[n] = x; ys[n] = y; }
        n++;
        if (D > 0) { y = y + yi; D = D - 2 * dx; }
        D = D + 2 * dy;
    }
    return n;
}

/* plotLineHigh -- functions.cpp:276-297 */
static int plot_line_high(int x0, int y0, int x1, int y1, int* xs, int* ys, int cap) {
    int dx = x1 - x0, dy = y1 - y0, xi = 1, n = 0;
    if (dx < 0) { xi = -1; dx = -dx; }
    int D = 2 * dx - dy, x = x0;
    for (int y = y0; y <= y1; y++) {
        if (n < cap) { xs[n] = x; ys[n] = y; }
        n++;
        if (D > 0) { x = x + xi; D = D - 2 * dy; }
        D = D + 2 * dx;
    }
    return n;
}

/* bresenham(Point2i point2, Point2i point1) -- functions.cpp:299-321, called
 * as bresenham(pixel1, pixel2) at CameraStereoVision.cpp:73, so point2 is the
 * caller's pixel1 (the t_near endpoint).                                      */
int svo_bresenham(int p1x, int p1y, int p2x, int p2y, int* xs, int* ys, int cap) {
    const int ax = p1x, ay = p1y; /* point2 */
    const int bx = p2x, by = p2y; /* point1 */
    if (abs(ay - by) < abs(ax - bx)) {
        if (bx > ax) return plot_line_low(ax, ay, bx, by, xs, ys, cap);
        return plot_line_low(bx, by, ax, ay, xs, ys, cap);
    }
    if (by > ay) return plot_line_high(ax, ay, bx, by, xs, ys, cap);
    return plot_line_high(bx, by, ax, ay, xs, ys, cap);
}

/* getAbsDiff -- functions.cpp:215-218: sum(abs(m1 - m2))[0].  OpenCV 4.2
 * turns abs(A-B) of two Mats into absdiff, so this is the exact integer
 * sum |a-b| (returned as double by the reference; exact below 2^53).        */
int64_t svo_sad(const uint8_t* a, ptrdiff_t pa, const uint8_t* b, ptrdiff_t pb, int w, int h) {
    int64_t s = 0;
    for (int v = 0; v < h; v++)
        for (int u = 0; u < w; u++) {
            int d = (int)a[v * pa + u] - (int)b[v * pb + u];
            s += d < 0 ? -d : d;
        }
    return s;
}

/* CameraStereoVision.cpp:28 (halfRes = resolution / 2, integer division),
 * :60-64 (ray endpoints), :66-71 (bounds check, note '>' not '>=').         */
int svo_ref_endpoints(const svo_camera* cref, const svo_camera* coth, int W, int H, int k,
                      double t_near, double t_far, int x, int y, int p1[2], int p2[2]) {
    const int hx = W / 2, hy = H / 2;
    double vec[3], P[3];
    svo_cam_inv_project(cref, x - hx, y - hy, vec);
    /* p1 = pos3D + (vec * 0.5); p2 = pos3D + vec  (vec*1.0 == vec exactly) */
    for (int i = 0; i < 3; i++) P[i] = cref->pos[i] + vec[i] * t_near;
    svo_cam_project(coth, P, p1);
    for (int i = 0; i < 3; i++) P[i] = cref->pos[i] + vec[i] * t_far;
    svo_cam_project(coth, P, p2);
    p1[0] += hx; p1[1] += hy;
    p2[0] += hx; p2[1] += hy;
    if (p1[0] < k || p1[1] < k || p1[0] > W - k || p1[1] > H - k) return 0;
    if (p2[0] < k || p2[1] < k || p2[0] > W - k || p2[1] > H - k) return 0;
    return 1;
}

/* The hot loop, CameraStereoVision.cpp:49-95, for one pair. */
int64_t svo_ref_pair(const uint8_t* ref, const uint8_t* other, int W, int H, ptrdiff_t pitch,
                     const uint8_t* mask, const svo_camera* cref, const svo_camera* coth,
                     int k, double t_near, double t_far,
                     uint8_t* disp_u8, uint16_t* disp_u16, uint8_t* valid) {
    int cap = 4 * (W + H) + 8;
    int* xs = (int*)malloc(sizeof(int) * (size_t)cap);
    int* ys = (int*)malloc(sizeof(int) * (size_t)cap);
    int64_t evals = 0;
    for (int y = k; y < H - k; y++) {
        for (int x = k; x < W - k; x++) {
            if (mask && mask[(size_t)y * W + x] == 0) continue;               /* :53 */
            int p1[2], p2[2];
            if (!svo_ref_endpoints(cref, coth, W, H, k, t_near, t_far, x, y, p1, p2))
                continue;                                                       /* :66-71 */
            int n = svo_bresenham(p1[0], p1[1], p2[0], p2[1], xs, ys, cap);     /* :73 */
            const uint8_t* kern = ref + (ptrdiff_t)(y - k) * pitch + (x - k);  /* :57 */
            int64_t best = -1;
            int bi = 0;
            for (int i = 0; i < n; i++) {                                       /* :76-83 */
                const uint8_t* sel = other + (ptrdiff_t)(ys[i] - k) * pitch + (xs[i] - k);
                int64_t e = svo_sad(sel, pitch, kern, pitch, 2 * k, 2 * k);
                if (best < 0 || e < best) { best = e; bi = i; }                 /* :85 first min */
            }
            evals += n;
            double ddx = (double)(xs[bi] - x), ddy = (double)(ys[bi] - y);
            int dn = (int)sqrt(ddx * ddx + ddy * ddy);                           /* :89 */
            disp_u8[(size_t)y * W + x] = (uint8_t)dn;
            if (disp_u16) disp_u16[(size_t)y * W + x] = (uint16_t)dn;
            if (valid) valid[(size_t)y * W + x] = 1;
        }
    }
    free(xs);
    free(ys);
    return evals;
}

/* CameraStereoVision.cpp:98-100:
 *   multiply(disparity, pixelSize, pixSizeDisp, 1, 6);   (CV_64F)
 *   depth = camDistance * f / (pixSizeDisp);             (0 where divisor 0) */
void svo_disp_to_depth(const uint8_t* disp, int n, double cam_distance, double f,
                       double pixel_size, double* depth) {
    double num = cam_distance * f;
    for (int i = 0; i < n; i++) {
        double den = (double)disp[i] * pixel_size;
        depth[i] = den != 0.0 ? num / den : 0.0;
    }
}
