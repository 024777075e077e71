/*
 * sgm_oracle.c -- CPU ORACLE, Mode S (Census 9x7 -> Hamming cost volume ->
 * 8-path SGM -> winner-take-all + sub-pixel).
 * TEST INFRASTRUCTURE ONLY (see sva_oracle.h).
 *
 * The reference has no Census/Hamming/SGM, so this file follows
 * the frozen spec in DESIGN.md §2.  The WTA
 * tie-break (first minimum in index order) mirrors the reference's
 * std::min_element at src/CameraStereoVision.cpp:85.  Parity unpinned.
 *
 * Written for clarity, not speed: plain int arithmetic, one direction at a
 * time.  The optional OpenMP threads only split independent path lines.
 */
#include "sva_oracle.h"

/* Threads for the row-parallel stage loops (census, cost, WTA): 1 except
 * inside a threaded svo_sgm call (the CPU baseline's all-cores leg).  The
 * arithmetic is the same either way. */
static int g_threads = 1;

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* DESIGN.md §2.1 -- census 9 wide x 7 high. */
void svo_census(const uint8_t* img, int W, int H, ptrdiff_t pitch, uint64_t* out) {
    #ifdef _OPENMP
#pragma omp parallel for num_threads(g_threads) schedule(static)
#endif
    for (int y = 0; y < H; y++) {
        for (int x = 0; x < W; x++) {
            uint64_t w = 0;
            if (x >= 4 && x < W - 4 && y >= 3 && y < H - 3) {
                int c = img[(ptrdiff_t)y * pitch + x];
                for (int dy = -3; dy <= 3; dy++)
                    for (int dx = -4; dx <= 4; dx++) {
                        if (dx == 0 && dy == 0) continue;
                        int q = img[(ptrdiff_t)(y + dy) * pitch + (x + dx)];
                        w = (w << 1) | (uint64_t)(q < c);
                    }
            }
            out[(size_t)y * W + x] = w;
        }
    }
}

static int popcount64(uint64_t v) { return __builtin_popcountll(v); }

/* DESIGN.md §2.2 -- Hamming matching cost, D-contiguous u8. */
void svo_cost(const uint64_t* cl, const uint64_t* cr, int W, int H, int D, int dmin, int dir,
              uint8_t* C) {
    #ifdef _OPENMP
#pragma omp parallel for num_threads(g_threads) schedule(static)
#endif
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++)
            for (int d = 0; d < D; d++) {
                int xr = x + dir * (dmin + d);
                int c = 62;
                if (xr >= 0 && xr < W)
                    c = popcount64(cl[(size_t)y * W + x] ^ cr[(size_t)y * W + xr]);
                C[((size_t)y * W + x) * D + d] = (uint8_t)c;
            }
}

/* DESIGN.md §2.2 -- 2-D matching step. */
void svo_step_offset(int s, int bx, int by, int* ox, int* oy) {
    int ax = bx < 0 ? -bx : bx, ay = by < 0 ? -by : by;
    int M = ax > ay ? ax : ay, m = ax > ay ? ay : ax;
    int major = s, minor = (2 * s * m + M) / (2 * M);   /* round half up, s >= 0 */
    int mx = ax >= ay ? major : minor, my = ax >= ay ? minor : major;
    *ox = bx < 0 ? -mx : (bx > 0 ? mx : 0);
    *oy = by < 0 ? -my : (by > 0 ? my : 0);
}

void svo_cost2(const uint64_t* cl, const uint64_t* cr, int W, int H, int D, int dmin, int sx,
               int sy, uint8_t* C) {
    int* ox = (int*)malloc((size_t)D * sizeof(int));
    int* oy = (int*)malloc((size_t)D * sizeof(int));
    for (int d = 0; d < D; d++) svo_step_offset(dmin + d, sx, sy, &ox[d], &oy[d]);
    #ifdef _OPENMP
#pragma omp parallel for num_threads(g_threads) schedule(static)
#endif
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++)
            for (int d = 0; d < D; d++) {
                int xr = x + ox[d], yr = y + oy[d];
                int c = 62;
                if (xr >= 0 && xr < W && yr >= 0 && yr < H)
                    c = popcount64(cl[(size_t)y * W + x] ^ cr[(size_t)yr * W + xr]);
                C[((size_t)y * W + x) * D + d] = (uint8_t)c;
            }
    free(ox);
    free(oy);
}

/* DESIGN.md §2.3 -- direction table r = 0..7 (step vectors p = q + r). */
void svo_direction(int r, int* rx, int* ry) {
    static const int T[8][2] = {{1, 0}, {-1, 0}, {0, 1}, {0, -1},
                                {1, 1}, {-1, -1}, {-1, 1}, {1, -1}};
    *rx = T[r & 7][0];
    *ry = T[r & 7][1];
}

/* L_r(p,d) = C(p,d) + min(L(q,d), L(q,d-1)+P1, L(q,d+1)+P1, m+P2) - m,
 * m = min_k L(q,k), q = p - r; L = C where q is outside the image.
 * Visiting order: rows in the direction of ry (top-down if ry >= 0), columns
 * in the direction of rx, so q is always finished before p.                 */
void svo_path(const uint8_t* C, int W, int H, int D, int rx, int ry, int P1, int P2,
              uint8_t* L) {
    for (int yi = 0; yi < H; yi++) {
        int y = ry >= 0 ? yi : H - 1 - yi;
        for (int xi = 0; xi < W; xi++) {
            int x = rx >= 0 ? xi : W - 1 - xi;
            const uint8_t* c = C + ((size_t)y * W + x) * D;
            uint8_t* l = L + ((size_t)y * W + x) * D;
            int qx = x - rx, qy = y - ry;
            if (qx < 0 || qx >= W || qy < 0 || qy >= H) {
                memcpy(l, c, (size_t)D);
                continue;
            }
            const uint8_t* lq = L + ((size_t)qy * W + qx) * D;
            int m = lq[0];
            for (int k = 1; k < D; k++) if (lq[k] < m) m = lq[k];
            for (int d = 0; d < D; d++) {
                int best = lq[d];
                if (d > 0 && lq[d - 1] + P1 < best) best = lq[d - 1] + P1;
                if (d < D - 1 && lq[d + 1] + P1 < best) best = lq[d + 1] + P1;
                if (m + P2 < best) best = m + P2;
                l[d] = (uint8_t)(c[d] + best - m);
            }
        }
    }
}

/* DESIGN.md §2.4 -- first-minimum WTA (mirrors CameraStereoVision.cpp:85)
 * and parabola sub-pixel in f32. */
void svo_wta(const uint16_t* S, int W, int H, int D, int dmin, uint16_t* disp, float* sub) {
    #ifdef _OPENMP
#pragma omp parallel for num_threads(g_threads) schedule(static)
#endif
    for (size_t p = 0; p < (size_t)W * H; p++) {
        const uint16_t* s = S + p * D;
        int best = 0;
        for (int d = 1; d < D; d++) if (s[d] < s[best]) best = d;
        disp[p] = (uint16_t)(dmin + best);
        if (sub) {
            float v = (float)(dmin + best);
            if (best > 0 && best < D - 1) {
                int a = s[best - 1], b = s[best], c = s[best + 1];
                int den = a - 2 * b + c;
                if (den > 0) v = v + (float)(a - c) / (float)(2 * den);
            }
            sub[p] = v;
        }
    }
}

/* Path-parallel variant of svo_path used only to speed up the CPU baseline:
 * lines of one direction are independent, so the image is split into the
 * lines the direction sweeps.  Same arithmetic as svo_path. */
static void path_line_step(const uint8_t* C, uint8_t* L, int W, int H, int D, int x, int y,
                           int rx, int ry, int P1, int P2) {
    const uint8_t* c = C + ((size_t)y * W + x) * D;
    uint8_t* l = L + ((size_t)y * W + x) * D;
    int qx = x - rx, qy = y - ry;
    if (qx < 0 || qx >= W || qy < 0 || qy >= H) {
        memcpy(l, c, (size_t)D);
        return;
    }
    const uint8_t* lq = L + ((size_t)qy * W + qx) * D;
    int m = lq[0];
    for (int k = 1; k < D; k++) if (lq[k] < m) m = lq[k];
    for (int d = 0; d < D; d++) {
        int best = lq[d];
        if (d > 0 && lq[d - 1] + P1 < best) best = lq[d - 1] + P1;
        if (d < D - 1 && lq[d + 1] + P1 < best) best = lq[d + 1] + P1;
        if (m + P2 < best) best = m + P2;
        l[d] = (uint8_t)(c[d] + best - m);
    }
}

static void svo_path_threaded(const uint8_t* C, int W, int H, int D, int rx, int ry, int P1,
                              int P2, uint8_t* L, int threads) {
    /* Lines are independent: every pixel whose predecessor p - r leaves the
     * image starts one, and one thread walks each line in path order.
     * Entry pixels: the entry row (ry != 0) and the entry column (rx != 0),
     * the corner counted once. */
    const int y0 = ry > 0 ? 0 : H - 1, x0 = rx > 0 ? 0 : W - 1;
    const int nrow = ry != 0 ? W : 0;
    const int ncol = rx == 0 ? 0 : (ry != 0 ? H - 1 : H);
#ifdef _OPENMP
#pragma omp parallel for num_threads(threads) schedule(dynamic, 16)
#endif
    for (int e = 0; e < nrow + ncol; e++) {
        int x, y;
        if (e < nrow) {
            x = e;
            y = y0;
        } else {
            int i = e - nrow;                       /* i-th entry-column pixel */
            x = x0;
            if (ry == 0) y = i;
            else y = ry > 0 ? 1 + i : H - 2 - i;    /* skip the corner on the entry row */
        }
        for (; x >= 0 && x < W && y >= 0 && y < H; x += rx, y += ry)
            path_line_step(C, L, W, H, D, x, y, rx, ry, P1, P2);
    }
}

/* S = sum of the 8 path volumes; threads > 1 walks each direction's lines in
 * parallel (svo_path_threaded), same arithmetic as the serial svo_path. */
void svo_aggregate(const uint8_t* C, int W, int H, int D, int P1, int P2, uint16_t* S,
                   int threads) {
    size_t n = (size_t)W * H * D;
    memset(S, 0, n * sizeof(uint16_t));
    uint8_t* L = (uint8_t*)malloc(n);
    for (int r = 0; r < 8; r++) {
        int rx, ry;
        svo_direction(r, &rx, &ry);
        if (threads > 1) svo_path_threaded(C, W, H, D, rx, ry, P1, P2, L, threads);
        else svo_path(C, W, H, D, rx, ry, P1, P2, L);
#ifdef _OPENMP
#pragma omp parallel for num_threads(threads > 1 ? threads : 1) schedule(static)
#endif
        for (long long i = 0; i < (long long)n; i++) S[i] = (uint16_t)(S[i] + L[i]);
    }
    free(L);
}

/* Whole Mode S pipeline on a 2-D matching step: census ->
 * svo_cost2 -> 8 paths -> WTA; threads <= 1: serial. */
void svo_sgm2(const uint8_t* left, const uint8_t* right, int W, int H, ptrdiff_t pitch, int D,
              int dmin, int sx, int sy, int P1, int P2, uint16_t* disp, float* sub,
              int threads) {
    size_t np = (size_t)W * H, n = np * D;
    uint64_t* cl = (uint64_t*)malloc(np * 8);
    uint64_t* cr = (uint64_t*)malloc(np * 8);
    uint8_t* C = (uint8_t*)malloc(n);
    uint16_t* S = (uint16_t*)malloc(n * 2);
    g_threads = threads > 1 ? threads : 1;
    svo_census(left, W, H, pitch, cl);
    svo_census(right, W, H, pitch, cr);
    svo_cost2(cl, cr, W, H, D, dmin, sx, sy, C);
    svo_aggregate(C, W, H, D, P1, P2, S, threads);
    svo_wta(S, W, H, D, dmin, disp, sub);
    g_threads = 1;
    free(cl);
    free(cr);
    free(C);
    free(S);
}

void svo_sgm(const uint8_t* left, const uint8_t* right, int W, int H, ptrdiff_t pitch, int D,
             int dmin, int dir, int P1, int P2, uint16_t* disp, float* sub, int threads) {
    size_t np = (size_t)W * H, n = np * D;
    uint64_t* cl = (uint64_t*)malloc(np * 8);
    uint64_t* cr = (uint64_t*)malloc(np * 8);
    uint8_t* C = (uint8_t*)malloc(n);
    uint16_t* S = (uint16_t*)malloc(n * 2);
    g_threads = threads > 1 ? threads : 1;
    svo_census(left, W, H, pitch, cl);
    svo_census(right, W, H, pitch, cr);
    svo_cost(cl, cr, W, H, D, dmin, dir, C);
    if (threads > 1) {
        uint8_t* L = (uint8_t*)malloc(n);
        memset(S, 0, n * 2);
        for (int r = 0; r < 8; r++) {
            int rx, ry;
            svo_direction(r, &rx, &ry);
            svo_path_threaded(C, W, H, D, rx, ry, P1, P2, L, threads);
#ifdef _OPENMP
#pragma omp parallel for num_threads(threads) schedule(static)
#endif
            for (long long i = 0; i < (long long)n; i++) S[i] = (uint16_t)(S[i] + L[i]);
        }
        free(L);
    } else {
        svo_aggregate(C, W, H, D, P1, P2, S, 1);
    }
    svo_wta(S, W, H, D, dmin, disp, sub);
    g_threads = 1;
    free(cl);
    free(cr);
    free(C);
    free(S);
}

/* DESIGN.md §2.5 -- left/right consistency. */
void svo_lr_check(uint16_t* disp_l, const uint16_t* disp_r, int W, int H, int dir,
                  int max_diff, uint16_t invalid) {
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            uint16_t* dl = disp_l + (size_t)y * W + x;
            if (*dl == invalid) continue;
            int xr = x + dir * (int)*dl;
            if (xr < 0 || xr >= W) { *dl = invalid; continue; }
            int dr = disp_r[(size_t)y * W + xr];
            int diff = (int)*dl - dr;
            if (diff < 0) diff = -diff;
            if (dr == invalid || diff > max_diff) *dl = invalid;
        }
}

void svo_lr_check2(uint16_t* disp_l, const uint16_t* disp_r, int W, int H, int sx, int sy,
                   int max_diff, uint16_t invalid) {
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            uint16_t* dl = disp_l + (size_t)y * W + x;
            if (*dl == invalid) continue;
            int ox, oy;
            svo_step_offset((int)*dl, sx, sy, &ox, &oy);
            int xr = x + ox, yr = y + oy;
            if (xr < 0 || xr >= W || yr < 0 || yr >= H) { *dl = invalid; continue; }
            int dr = disp_r[(size_t)yr * W + xr];
            int diff = (int)*dl - dr;
            if (diff < 0) diff = -diff;
            if (dr == invalid || diff > max_diff) *dl = invalid;
        }
}

/* DESIGN.md §2.5 -- the sub-pixel map follows the check: NaN wherever the
 * disparity is `invalid` after it (a caller building depth from
 * the f32 map must not see a parabola value for a rejected pixel). */
void svo_lr_sub(const uint16_t* disp, float* sub, size_t n, uint16_t invalid) {
    for (size_t i = 0; i < n; i++)
        if (disp[i] == invalid) sub[i] = NAN;
}

/* DESIGN.md §2.6 -- median depth over the valid maps (insertion sort). */
void svo_fuse_depth(const uint16_t* disps, int n_maps, int W, int H, const double* baseline,
                    double f, double pixel_size, uint16_t invalid, double* depth,
                    uint8_t* n_valid) {
    double v[64];
    for (size_t p = 0; p < (size_t)W * H; p++) {
        int n = 0;
        for (int i = 0; i < n_maps && i < 64; i++) {
            uint16_t d = disps[(size_t)i * W * H + p];
            if (d == invalid || d == 0) continue;
            double z = (baseline[i] * f) / ((double)d * pixel_size);
            int j = n++;
            while (j > 0 && v[j - 1] > z) { v[j] = v[j - 1]; j--; }
            v[j] = z;
        }
        double out = 0.0;
        if (n > 0) out = (n & 1) ? v[n / 2] : (v[n / 2 - 1] + v[n / 2]) * 0.5;
        depth[p] = out;
        if (n_valid) n_valid[p] = (uint8_t)n;
    }
}
