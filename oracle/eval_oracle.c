/* eval_oracle.c -- TEST INFRASTRUCTURE ONLY (see sva_oracle.h): CPU
 * restatement of the reference's evaluation step, SURVEY.md §8f row 4:
 *
 *   Mat ref = getIdealRef();                      functions.cpp:323-329
 *   resize(depth, depth2, ref.size());            CameraStereoVision.cpp:108,118
 *   Mat error = (depth2 - ref) * 50;              CameraStereoVision.cpp:109,119
 *   cv::mean(image, mask)[0]                      functions.cpp:348-354
 *
 * The arithmetic lives in OpenCV 4.2.0 (third-party, absent here: parity
 * unpinned).  What follows restates its published algorithm for a
 * single-channel CV_64F matrix:
 *
 * resize, default INTER_LINEAR (imgproc/src/resize.cpp):
 *   dsize == ssize                 -> copy
 *   inv = dw / sw, scale = 1 / inv (both f64, per axis)
 *   scale exactly 2 on both axes   -> the INTER_AREA fast path:
 *        dst = (0 + ((s00 + s01) + s10) + s11) * 0.25
 *   otherwise resizeGeneric_ with float coefficients:
 *     x: fx = (float)((dx + 0.5) * scale_x - 0.5); sx = floor(fx); fx -= sx
 *        sx < 0       -> sx = 0, fx = 0
 *        sx >= sw - 1 -> dst row value S[sw - 1]          (the "xmax" tail)
 *        else            h = S[sx] * (double)(1.f - fx) + S[sx + 1] * (double)fx
 *     y: fy likewise but NOT zeroed at the borders; the two source rows are
 *        clip(sy) and clip(sy + 1) to [0, sh - 1]:
 *        dst = h(r0) * (double)(1.f - fy) + h(r1) * (double)fy
 * (MatExpr) (A - B) * s is addWeighted(A, s, B, -s, 0): a * s + b * (-s) + 0.
 * cv::mean(src, mask): sum over mask != 0 (row-major), divided by the count;
 * 0 when the mask is empty.
 * Compiled with -ffp-contract=off (no FMA), like the GPU side. */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "sva_oracle.h"

void svo_resize_linear_f64(const double* src, int sw, int sh, double* dst, int dw, int dh) {
    if (sw == dw && sh == dh) {
        memcpy(dst, src, (size_t)sw * sh * sizeof(double));
        return;
    }
    const double sx_scale = 1.0 / ((double)dw / sw), sy_scale = 1.0 / ((double)dh / sh);
    if (sx_scale == 2.0 && sy_scale == 2.0) {
        for (int y = 0; y < dh; y++)
            for (int x = 0; x < dw; x++) {
                const double* s0 = src + (size_t)(2 * y) * sw + 2 * x;
                const double* s1 = s0 + sw;
                double sum = 0;
                sum += s0[0] + s0[1] + s1[0] + s1[1];
                dst[(size_t)y * dw + x] = sum * 0.25;
            }
        return;
    }
    for (int y = 0; y < dh; y++) {
        float fy = (float)((y + 0.5) * sy_scale - 0.5);
        int sy = (int)floorf(fy);
        fy -= (float)sy;
        const int r0 = sy < 0 ? 0 : (sy >= sh ? sh - 1 : sy);
        const int r1 = sy + 1 < 0 ? 0 : (sy + 1 >= sh ? sh - 1 : sy + 1);
        const double b0 = (double)(1.f - fy), b1 = (double)fy;
        for (int x = 0; x < dw; x++) {
            float fx = (float)((x + 0.5) * sx_scale - 0.5);
            int sx = (int)floorf(fx);
            fx -= (float)sx;
            if (sx < 0) { sx = 0; fx = 0.f; }
            double h0, h1;
            const double* S0 = src + (size_t)r0 * sw;
            const double* S1 = src + (size_t)r1 * sw;
            if (sx >= sw - 1) {
                h0 = S0[sw - 1];
                h1 = S1[sw - 1];
            } else {
                const double a0 = (double)(1.f - fx), a1 = (double)fx;
                h0 = S0[sx] * a0 + S0[sx + 1] * a1;
                h1 = S1[sx] * a0 + S1[sx + 1] * a1;
            }
            dst[(size_t)y * dw + x] = h0 * b0 + h1 * b1;
        }
    }
}

void svo_ref_error(const double* depth, int w, int h, const double* ref, int rw, int rh,
                   double scale, double* error) {
    svo_resize_linear_f64(depth, w, h, error, rw, rh);
    for (size_t i = 0; i < (size_t)rw * rh; i++) error[i] = error[i] * scale + ref[i] * -scale + 0.0;
}

double svo_masked_mean(const double* image, const uint8_t* mask, int w, int h) {
    double s = 0;
    size_t n = 0;
    for (size_t i = 0; i < (size_t)w * h; i++)
        if (!mask || mask[i]) {
            s += image[i];
            n++;
        }
    return n ? s / (double)n : 0.0;
}
