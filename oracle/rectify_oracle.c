/*
 * rectify_oracle.c -- CPU ORACLE (test infrastructure only; see usv_oracle.h).
 *
 * the rectification that produces the input the block
 * matcher assumes.  The reference calls, per frame and per camera
 * (P/Main.cpp:351-359):
 *     initUndistortRectifyMap(intrinsic, distCoeffs, RectificationTransformMat,
 *                             ProjectionMat, size, CV_16SC2, map1, map2);
 *     remap(src, dst, map1, map2, INTER_LINEAR, BORDER_CONSTANT, Scalar());
 * OpenCV 3.0.0 is not in this image and the reference has no tests or
 * fixtures for it: PARITY UNPINNED against OpenCV.  What follows restates the
 * published OpenCV 3.0 algorithms (imgproc/undistort.cpp, imgproc/imgwarp.cpp,
 * core/lapack.cpp invert) operation by operation; the GPU path must equal this
 * restatement bit for bit, and tests/test_rectify.py pins it with known
 * answers (identity and integer-shift calibrations reproduce the source,
 * half-pixel shifts give the rounded neighbour mean).
 *
 * Map (CV_16SC2 + CV_16UC1, INTER_BITS = 5, INTER_TAB_SIZE = 32):
 *   iR = inverse(P[:, 0:3] * Rrect)            (3x3 double; adjugate / det,
 *                                                the n <= 3 path of cv::invert)
 *   per row i:  _x = i*ir[1] + ir[2], _y = i*ir[4] + ir[5], _w = i*ir[7] + ir[8]
 *   per column j (then _x += ir[0], _y += ir[3], _w += ir[6], sequentially):
 *     w = 1/_w, x = _x*w, y = _y*w, x2 = x*x, y2 = y*y, r2 = x2 + y2, _2xy = 2*x*y
 *     kr = (1 + ((k3*r2 + k2)*r2 + k1)*r2) / (1 + ((k6*r2 + k5)*r2 + k4)*r2)
 *     u = fx*(x*kr + p1*_2xy + p2*(r2 + 2*x2) + s1*r2 + s2*r2*r2) + u0
 *     v = fy*(y*kr + p1*(r2 + 2*y2) + p2*_2xy + s3*r2 + s4*r2*r2) + v0
 *     iu = round_half_even(u*32), iv = round_half_even(v*32)  (saturating to int)
 *     map1 = ((short)(iu >> 5), (short)(iv >> 5)),
 *     map2 = (iv & 31)*32 + (iu & 31)
 *   (fx, fy, u0, v0 from the camera matrix; k1 k2 p1 p2 [k3 [k4 k5 k6 [s1 s2 s3 s4]]]
 *    from distCoeffs of length 4, 5, 8 or 12, missing terms 0.)
 * Remap (INTER_LINEAR, fixed point INTER_REMAP_COEF_BITS = 15, BORDER_CONSTANT 0):
 *   sx, sy = map1; ty = map2 >> 5, tx = map2 & 31;
 *   w = {(32-ty)(32-tx), (32-ty)tx, ty(32-tx), ty tx} * 32   (the bilinear table:
 *        every product of the float taps is exact, so the table's sum is
 *        exactly 32768 and its rounding fix-up never fires)
 *   if sx >= W || sx+1 < 0 || sy >= H || sy+1 < 0:  dst = 0 (all channels)
 *   else taps outside the image read 0 and
 *        dst = clamp((S00*w0 + S01*w1 + S10*w2 + S11*w3 + (1 << 14)) >> 15, 0, 255)
 */
#include "usv_oracle.h"

#include <math.h>
#include <stddef.h>
#include <stdint.h>

/* cv::invert, DECOMP_LU, n == 3: adjugate over the determinant (det3 as OpenCV writes it). */
int usv_oracle_invert3(const double* m, double* out) {
#define M(i, j) m[(i) * 3 + (j)]
    double d = M(0, 0) * (M(1, 1) * M(2, 2) - M(1, 2) * M(2, 1)) -
               M(0, 1) * (M(1, 0) * M(2, 2) - M(1, 2) * M(2, 0)) +
               M(0, 2) * (M(1, 0) * M(2, 1) - M(1, 1) * M(2, 0));
    if (d == 0.) return 0;
    d = 1. / d;
    out[0] = (M(1, 1) * M(2, 2) - M(1, 2) * M(2, 1)) * d;
    out[1] = (M(0, 2) * M(2, 1) - M(0, 1) * M(2, 2)) * d;
    out[2] = (M(0, 1) * M(1, 2) - M(0, 2) * M(1, 1)) * d;
    out[3] = (M(1, 2) * M(2, 0) - M(1, 0) * M(2, 2)) * d;
    out[4] = (M(0, 0) * M(2, 2) - M(0, 2) * M(2, 0)) * d;
    out[5] = (M(0, 2) * M(1, 0) - M(0, 0) * M(1, 2)) * d;
    out[6] = (M(1, 0) * M(2, 1) - M(1, 1) * M(2, 0)) * d;
    out[7] = (M(0, 1) * M(2, 0) - M(0, 0) * M(2, 1)) * d;
    out[8] = (M(0, 0) * M(1, 1) - M(0, 1) * M(1, 0)) * d;
#undef M
    return 1;
}

/* cvRound of a double into int with saturation (OpenCV saturate_cast<int>(double)). */
static int sat_round(double v) {
    if (!(v > -2147483648.0)) return (int)0x80000000; /* NaN lands here too, as the x86 cvRound */
    if (v >= 2147483647.0) return 0x7FFFFFFF;
    return (int)lrint(v);
}

int usv_oracle_rectify_params(const double* K, const double* dist, int n_dist, const double* Rrect,
                              const double* P, int p_cols, double* params) {
    /* params: ir[9], fx, fy, u0, v0, k1 k2 p1 p2 k3 k4 k5 k6 s1 s2 s3 s4  (25 doubles) */
    if (!K || !P || (p_cols != 3 && p_cols != 4) || !params) return -1;
    if (!(n_dist == 0 || n_dist == 4 || n_dist == 5 || n_dist == 8 || n_dist == 12)) return -2;
    if (n_dist && !dist) return -1;
    double Rm[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    if (Rrect)
        for (int i = 0; i < 9; ++i) Rm[i] = Rrect[i];
    double A[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            A[i * 3 + j] = P[i * p_cols + 0] * Rm[0 * 3 + j] + P[i * p_cols + 1] * Rm[1 * 3 + j] +
                           P[i * p_cols + 2] * Rm[2 * 3 + j];
    if (!usv_oracle_invert3(A, params)) return -3;
    params[9] = K[0];   /* fx */
    params[10] = K[4];  /* fy */
    params[11] = K[2];  /* u0 */
    params[12] = K[5];  /* v0 */
    double k[12] = {0};
    for (int i = 0; i < n_dist; ++i) k[i] = dist[i];
    for (int i = 0; i < 12; ++i) params[13 + i] = k[i]; /* k1 k2 p1 p2 k3 k4 k5 k6 s1 s2 s3 s4 */
    return 0;
}

int usv_oracle_rectify_map(const double* params, int W, int H, int16_t* map1, uint16_t* map2) {
    if (!params || W <= 0 || H <= 0 || !map1 || !map2) return -1;
    const double* ir = params;
    const double fx = params[9], fy = params[10], u0 = params[11], v0 = params[12];
    const double k1 = params[13], k2 = params[14], p1 = params[15], p2 = params[16], k3 = params[17];
    const double k4 = params[18], k5 = params[19], k6 = params[20];
    const double s1 = params[21], s2 = params[22], s3 = params[23], s4 = params[24];
    for (int i = 0; i < H; ++i) {
        double _x = i * ir[1] + ir[2], _y = i * ir[4] + ir[5], _w = i * ir[7] + ir[8];
        int16_t* m1 = map1 + (size_t)i * W * 2;
        uint16_t* m2 = map2 + (size_t)i * W;
        for (int j = 0; j < W; ++j, _x += ir[0], _y += ir[3], _w += ir[6]) {
            const double w = 1. / _w, x = _x * w, y = _y * w;
            const double x2 = x * x, y2 = y * y;
            const double r2 = x2 + y2, _2xy = 2 * x * y;
            const double kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2);
            const double u = fx * (x * kr + p1 * _2xy + p2 * (r2 + 2 * x2) + s1 * r2 + s2 * r2 * r2) + u0;
            const double v = fy * (y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy + s3 * r2 + s4 * r2 * r2) + v0;
            const int iu = sat_round(u * 32), iv = sat_round(v * 32);
            m1[j * 2] = (int16_t)(iu >> 5);
            m1[j * 2 + 1] = (int16_t)(iv >> 5);
            m2[j] = (uint16_t)((iv & 31) * 32 + (iu & 31));
        }
    }
    return 0;
}

int usv_oracle_remap_linear(const uint8_t* src, int sW, int sH, int spitch, int cn, const int16_t* map1,
                            const uint16_t* map2, int W, int H, uint8_t* dst, int dpitch) {
    if (!src || !map1 || !map2 || !dst || cn < 1 || cn > 4 || sW <= 0 || sH <= 0 || W <= 0 || H <= 0)
        return -1;
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W; ++x) {
            const size_t m = (size_t)y * W + x;
            const int sx = map1[2 * m], sy = map1[2 * m + 1];
            const int ty = map2[m] >> 5, tx = map2[m] & 31;
            const int w0 = (32 - ty) * (32 - tx) * 32, w1 = (32 - ty) * tx * 32;
            const int w2 = ty * (32 - tx) * 32, w3 = ty * tx * 32;
            uint8_t* d = dst + (size_t)y * dpitch + (size_t)x * cn;
            if (sx >= sW || sx + 1 < 0 || sy >= sH || sy + 1 < 0) {
                for (int k = 0; k < cn; ++k) d[k] = 0;
                continue;
            }
            const int x0ok = sx >= 0, x1ok = sx + 1 < sW, y0ok = sy >= 0, y1ok = sy + 1 < sH;
            for (int k = 0; k < cn; ++k) {
                const int v0 = (x0ok && y0ok) ? src[(size_t)sy * spitch + (size_t)sx * cn + k] : 0;
                const int v1 = (x1ok && y0ok) ? src[(size_t)sy * spitch + (size_t)(sx + 1) * cn + k] : 0;
                const int v2 = (x0ok && y1ok) ? src[(size_t)(sy + 1) * spitch + (size_t)sx * cn + k] : 0;
                const int v3 = (x1ok && y1ok) ? src[(size_t)(sy + 1) * spitch + (size_t)(sx + 1) * cn + k] : 0;
                const int t = (v0 * w0 + v1 * w1 + v2 * w2 + v3 * w3 + (1 << 14)) >> 15;
                d[k] = (uint8_t)(t < 0 ? 0 : (t > 255 ? 255 : t));
            }
        }
    }
    return 0;
}
