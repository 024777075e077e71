/* Host sanitizer driver: every oracle entry point on small
 * seeded inputs, including ragged sizes, images smaller than the census
 * window, 2-D steps, the threaded pipeline, scatters with collisions and the
 * evaluation helpers.  Built with -fsanitize=address,undefined by
 * `make -C oracle asan` and run by tests/test_asan.py; any out-of-bounds
 * access, leak or undefined behaviour aborts with a nonzero status.
 * Test infrastructure only, like the rest of oracle/. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sva_oracle.h"

static unsigned rng = 12345u;
static unsigned nextu(void) {
    rng = rng * 1664525u + 1013904223u;
    return rng >> 8;
}
static uint8_t* tex(int W, int H) {
    uint8_t* p = malloc((size_t)W * H);
    for (size_t i = 0; i < (size_t)W * H; i++) p[i] = (uint8_t)nextu();
    return p;
}

static void mode_s(int W, int H, int D, int dmin, int dir, int sx, int sy, int threads) {
    uint8_t* L = tex(W, H);
    uint8_t* R = tex(W, H);
    size_t np = (size_t)W * H, nv = np * (size_t)D;
    uint64_t* cl = malloc(np * 8);
    uint64_t* cr = malloc(np * 8);
    uint8_t* C = malloc(nv);
    uint8_t* Lr = malloc(nv);
    uint16_t* S = malloc(nv * 2);
    uint16_t* d = malloc(np * 2);
    uint16_t* d2 = malloc(np * 2);
    float* sub = malloc(np * 4);
    svo_census(L, W, H, W, cl);
    svo_census(R, W, H, W, cr);
    if (sy == 0) svo_cost(cl, cr, W, H, D, dmin, dir, C);
    else svo_cost2(cl, cr, W, H, D, dmin, sx, sy, C);
    for (int r = 0; r < 8; r++) {
        int rx, ry;
        svo_direction(r, &rx, &ry);
        svo_path(C, W, H, D, rx, ry, 10, 120, Lr);
    }
    svo_aggregate(C, W, H, D, 10, 120, S, threads);
    svo_wta(S, W, H, D, dmin, d, sub);
    svo_sgm(L, R, W, H, W, D, dmin, dir, 10, 120, d2, sub, threads);
    svo_sgm(R, L, W, H, W, D, dmin, -dir, 10, 120, d, NULL, threads);
    if (sy == 0) svo_lr_check(d2, d, W, H, dir, 1, 0xFFFF);
    else svo_lr_check2(d2, d, W, H, sx, sy, 1, 0xFFFF);
    svo_lr_sub(d2, sub, np, 0xFFFF);
    double b[3] = {0.05, 0.1, 0.0707};
    uint16_t* maps = malloc(np * 2 * 3);
    for (int i = 0; i < 3; i++) memcpy(maps + np * i, i == 1 ? d : d2, np * 2);
    double* z = malloc(np * 8);
    uint8_t* nvd = malloc(np);
    svo_fuse_depth(maps, 3, W, H, b, 0.05, 0.036 / W, 0xFFFF, z, nvd);
    free(L); free(R); free(cl); free(cr); free(C); free(Lr); free(S); free(d); free(d2);
    free(sub); free(maps); free(z); free(nvd);
}

static void mode_r(int W, int H, int k) {
    svo_camera cams[25];
    const double ps = 0.036 / W;
    for (int i = 0; i < 25; i++) {
        cams[i].f = 0.05;
        cams[i].pos[0] = -0.1 + (i % 5) * 0.05;
        cams[i].pos[1] = -0.1 + (i / 5) * 0.05;
        cams[i].pos[2] = -0.75;
        cams[i].pixel_size = ps;
    }
    uint8_t* ref = tex(W, H);
    uint8_t* oth = tex(W, H);
    uint8_t* mask = tex(W, H);
    size_t np = (size_t)W * H;
    uint8_t* d8 = calloc(np, 1);
    uint16_t* d16 = calloc(np, 2);
    uint8_t* valid = calloc(np, 1);
    const int others[4] = {11, 7, 18, 6};
    for (int i = 0; i < 4; i++)
        svo_ref_pair(ref, oth, W, H, W, i == 0 ? NULL : mask, &cams[12], &cams[others[i]], k,
                     0.5, 1.0, d8, d16, valid);
    int xs[512], ys[512];
    svo_bresenham(3, 9, 40, 2, xs, ys, 512);
    svo_bresenham(5, 5, 5, 5, xs, ys, 512);
    svo_bresenham(0, 0, 10, 600, xs, ys, 512);   /* more points than cap */
    double* depth = malloc(np * 8);
    svo_disp_to_depth(d8, (int)np, 0.05, 0.05, ps, depth);
    /* refinement and 3-D output */
    uint8_t* shifted = calloc(np, 1);
    svo_shift_perspective(&cams[12], &cams[13], d8, oth, W, H, W, shifted);
    const uint8_t* imgs[2] = {oth, ref};
    svo_camera pairs[4] = {cams[12], cams[13], cams[12], cams[17]};
    uint8_t* out = calloc(np, 1);
    svo_improve_with_disparity(d8, ref, imgs, pairs, 2, W, H, W, mask, 2 * k + 1, 0, out);
    double* sh = calloc(np, 8);
    svo_shift_perspective2(&cams[12], &cams[13], depth, W, H, sh);
    double* pts = malloc(np * 3 * 8);
    int64_t n = svo_depth_to_points(depth, W, H, &cams[12], pts);
    double* back = calloc(np, 8);
    svo_points_to_depth(pts, n, &cams[12], W, H, back);
    /* ingestion + evaluation */
    int dw, dh;
    svo_resize_half_size(W, H, &dw, &dh);
    uint8_t* half = malloc((size_t)dw * dh);
    svo_resize_half(ref, W, H, W, half, dw);
    double* up = malloc(np * 8);
    double* err = malloc(np * 8);
    svo_resize_linear_f64(depth, W, H, up, W, H);
    double* small = malloc((size_t)dw * dh * 8);
    svo_resize_linear_f64(depth, W, H, small, dw, dh);
    svo_ref_error(small, dw, dh, depth, W, H, 50.0, err);
    volatile double m = svo_masked_mean(err, mask, W, H) + svo_masked_mean(err, NULL, W, H);
    (void)m;
    free(ref); free(oth); free(mask); free(d8); free(d16); free(valid); free(depth);
    free(shifted); free(out); free(sh); free(pts); free(back); free(half); free(up); free(err);
    free(small);
}

int main(void) {
    const int sizes[][2] = {{1, 1}, {2, 3}, {9, 7}, {8, 6}, {17, 5}, {5, 40}, {63, 33}, {70, 1}};
    for (size_t i = 0; i < sizeof sizes / sizeof sizes[0]; i++) {
        mode_s(sizes[i][0], sizes[i][1], 64, 0, -1, -1, 0, 1);
        mode_s(sizes[i][0], sizes[i][1], 64, 3, 1, 1, 0, 1);
    }
    mode_s(96, 40, 128, 5, -1, -1, 0, 4);
    mode_s(60, 50, 64, 0, 0, -2, 1, 2);
    mode_s(50, 60, 64, 0, 0, 1, 1, 1);
    mode_s(40, 70, 64, 2, 0, 0, -1, 1);
    mode_r(120, 90, 8);
    mode_r(160, 120, 20);
    printf("asan driver ok\n");
    return 0;
}
