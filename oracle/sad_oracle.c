/*
 * sad_oracle.c -- CPU ORACLE (test infrastructure only; see usv_oracle.h).
 *
 * Spec restated (the reference has no block matcher,
 * SURVEY.md §0.1, so this spec is the build's own and this file IS its
 * definition):
 *
 *   r = (w-1)/2,  cx(x) = clamp(x, 0, W-1),  cy(y) = clamp(y, 0, H-1)
 *   term(a,b) = |a-b|            (SAD; u8 absdiff, no wrap -- the semantics of
 *                                 OpenCV absdiff as used at P/Main.cpp:304)
 *             = (a-b)^2          (SSD)
 *   cost(y,x,d) = sum_{dy,dx in [-r,r]} term(L[cy(y+dy)][cx(x+dx)],
 *                                            R[cy(y+dy)][cx(x+dx-d)])
 *   disp(y,x) = argmin_{d in [0,D)} cost(y,x,d), smallest d on ties, stored u8.
 *
 * The border clamps apply to the L column and the R column independently, so
 * the window of a border pixel is NOT a replicated copy of its neighbour's.
 */
#include "usv_oracle.h"
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

static int check_args(const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int D,
                      int w, int metric, const uint8_t* disp, int disp_pitch) {
    if (!L || !R || !disp) return -1;
    if (W <= 0 || H <= 0 || pitch < W || disp_pitch < W) return -2;
    if (D < 1 || D > 256) return -3;
    if (w < 1 || (w & 1) == 0 || w > 63) return -4;
    if (metric != USV_ORACLE_SAD && metric != USV_ORACLE_SSD) return -5;
    return 0;
}

int usv_oracle_sad_naive(const uint8_t* L, const uint8_t* R, int W, int H, int pitch,
                         int D, int w, int metric, uint8_t* disp, int disp_pitch) {
    int rc = check_args(L, R, W, H, pitch, D, w, metric, disp, disp_pitch);
    if (rc) return rc;
    const int r = (w - 1) / 2;
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W; ++x) {
            uint32_t best = 0xFFFFFFFFu;
            int best_d = 0;
            for (int d = 0; d < D; ++d) {
                uint32_t cost = 0;
                for (int dy = -r; dy <= r; ++dy) {
                    const uint8_t* lrow = L + (size_t)clampi(y + dy, 0, H - 1) * pitch;
                    const uint8_t* rrow = R + (size_t)clampi(y + dy, 0, H - 1) * pitch;
                    for (int dx = -r; dx <= r; ++dx) {
                        int a = lrow[clampi(x + dx, 0, W - 1)];
                        int b = rrow[clampi(x + dx - d, 0, W - 1)];
                        int t = a - b;
                        cost += (uint32_t)(metric == USV_ORACLE_SAD ? (t < 0 ? -t : t) : t * t);
                    }
                }
                if (cost < best) { best = cost; best_d = d; }  /* strict: smallest d wins ties */
            }
            disp[(size_t)y * disp_pitch + x] = (uint8_t)best_d;
        }
    }
    return 0;
}

/* ---- separable running-sum variant ------------------------------------- */

typedef struct {
    const uint8_t *L, *R;
    int W, H, pitch, D, w, metric;
    uint8_t* disp;
    int disp_pitch;
    int y0, y1; /* output rows of this band */
    int rc;
} band_job;

/* e(y', x', d) for the extended column x' in [-r, W-1+r], row y' already clamped. */
static inline uint32_t term(const uint8_t* lrow, const uint8_t* rrow, int W, int xe, int d,
                            int metric) {
    int a = lrow[clampi(xe, 0, W - 1)];
    int b = rrow[clampi(xe - d, 0, W - 1)];
    int t = a - b;
    return (uint32_t)(metric == USV_ORACLE_SAD ? (t < 0 ? -t : t) : t * t);
}

static void* band_worker(void* arg) {
    band_job* j = (band_job*)arg;
    const int W = j->W, H = j->H, r = (j->w - 1) / 2, We = W + 2 * r;
    const int nrows = j->y1 - j->y0;
    uint32_t* col = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)We);
    uint32_t* best = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)W * nrows);
    uint8_t* bestd = (uint8_t*)calloc((size_t)W * nrows, 1);
    if (!col || !best || !bestd) {
        j->rc = -10;
        free(col); free(best); free(bestd);
        return NULL;
    }
    for (size_t i = 0; i < (size_t)W * nrows; ++i) best[i] = 0xFFFFFFFFu;

    for (int d = 0; d < j->D; ++d) {
        /* column sums for the first output row of the band */
        memset(col, 0, sizeof(uint32_t) * (size_t)We);
        for (int dy = -r; dy <= r; ++dy) {
            int yy = clampi(j->y0 + dy, 0, H - 1);
            const uint8_t* lrow = j->L + (size_t)yy * j->pitch;
            const uint8_t* rrow = j->R + (size_t)yy * j->pitch;
            for (int xe = 0; xe < We; ++xe) col[xe] += term(lrow, rrow, W, xe - r, d, j->metric);
        }
        for (int y = j->y0; y < j->y1; ++y) {
            if (y > j->y0) { /* slide the window down one row */
                int yin = clampi(y + r, 0, H - 1), yout = clampi(y - r - 1, 0, H - 1);
                const uint8_t* li = j->L + (size_t)yin * j->pitch;
                const uint8_t* ri = j->R + (size_t)yin * j->pitch;
                const uint8_t* lo = j->L + (size_t)yout * j->pitch;
                const uint8_t* ro = j->R + (size_t)yout * j->pitch;
                for (int xe = 0; xe < We; ++xe)
                    col[xe] += term(li, ri, W, xe - r, d, j->metric) -
                               term(lo, ro, W, xe - r, d, j->metric);
            }
            uint32_t s = 0;
            for (int k = 0; k < j->w; ++k) s += col[k]; /* x = 0 covers xe 0..w-1 */
            uint32_t* brow = best + (size_t)(y - j->y0) * W;
            uint8_t* drow = bestd + (size_t)(y - j->y0) * W;
            for (int x = 0; x < W; ++x) {
                if (x > 0) s += col[x + 2 * r] - col[x - 1];
                if (s < brow[x]) { brow[x] = s; drow[x] = (uint8_t)d; }
            }
        }
    }
    for (int y = j->y0; y < j->y1; ++y)
        memcpy(j->disp + (size_t)y * j->disp_pitch, bestd + (size_t)(y - j->y0) * W, (size_t)W);
    free(col); free(best); free(bestd);
    j->rc = 0;
    return NULL;
}

int usv_oracle_sad_sliding_rows(const uint8_t* L, const uint8_t* R, int W, int H, int pitch,
                                int D, int w, int metric, uint8_t* disp, int disp_pitch,
                                int y0, int y1, int n_threads) {
    int rc = check_args(L, R, W, H, pitch, D, w, metric, disp, disp_pitch);
    if (rc) return rc;
    if (y0 < 0) y0 = 0;
    if (y1 > H) y1 = H;
    if (y1 <= y0) return 0;
    if (n_threads <= 0) {
        long n = sysconf(_SC_NPROCESSORS_ONLN);
        n_threads = n > 0 ? (int)n : 1;
    }
    int rows = y1 - y0;
    if (n_threads > rows) n_threads = rows;
    band_job* jobs = (band_job*)calloc((size_t)n_threads, sizeof(band_job));
    pthread_t* th = (pthread_t*)calloc((size_t)n_threads, sizeof(pthread_t));
    if (!jobs || !th) { free(jobs); free(th); return -10; }
    for (int t = 0; t < n_threads; ++t) {
        band_job* j = &jobs[t];
        j->L = L; j->R = R; j->W = W; j->H = H; j->pitch = pitch; j->D = D; j->w = w;
        j->metric = metric; j->disp = disp; j->disp_pitch = disp_pitch;
        j->y0 = y0 + (int)((long)rows * t / n_threads);
        j->y1 = y0 + (int)((long)rows * (t + 1) / n_threads);
        j->rc = -11;
    }
    for (int t = 1; t < n_threads; ++t) pthread_create(&th[t], NULL, band_worker, &jobs[t]);
    band_worker(&jobs[0]);
    for (int t = 1; t < n_threads; ++t) pthread_join(th[t], NULL);
    rc = 0;
    for (int t = 0; t < n_threads; ++t) if (jobs[t].rc) rc = jobs[t].rc;
    free(jobs); free(th);
    return rc;
}

int usv_oracle_sad_sliding(const uint8_t* L, const uint8_t* R, int W, int H, int pitch,
                           int D, int w, int metric, uint8_t* disp, int disp_pitch,
                           int n_threads) {
    return usv_oracle_sad_sliding_rows(L, R, W, H, pitch, D, w, metric, disp, disp_pitch, 0, H,
                                       n_threads);
}
