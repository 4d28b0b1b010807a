// usv_contours.hip -- batched contour matcher on gfx950.
//
// The reference scores every (i, j) contour pair with
//   v = matchShapes(L_i, R_j, CONTOURS_MATCH_I1, 0) + |(A_i - A_j) / ((A_i + A_j) / 2)|
// recomputing both contours' Hu moments and four contourArea calls per pair
// (P/Main.cpp:408-424, O(N·M·K)).  Here the per-contour part runs once per
// contour (contour_desc_kernel: one lane walks one contour's points in order,
// the same f64 operation sequence as csrc/host/matching.cpp, so Hu invariants
// and areas are bit-identical to the host path), and the N×M pair scores are
// one lane per pair over 8-double descriptors (pair_score_kernel).  The only
// transcendental, log10 of each |Hu| invariant, is taken once per contour.
//
// Work is tiny (tens..hundreds of contours of tens..hundreds of points): both
// kernels are latency-bound single waves; the point is to keep the matcher on
// the device next to the frame data, not throughput.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>

#include "usv.h"

namespace usv {
namespace {

constexpr int kDesc = 8;  // 7 I1 terms (1 / (sign(h) log10|h|), NaN when |h| <= 1e-5) + |area|

__global__ void __launch_bounds__(64) contour_desc_kernel(const int* __restrict__ pts, const int* __restrict__ off,
                                                          int n, double* __restrict__ desc) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    if (c >= n) return;
    const int b = off[c], e = off[c + 1], np = e - b;
    double h[7] = {0, 0, 0, 0, 0, 0, 0};
    double area = 0;
    if (np > 0) {
        const int* p = pts + 2 * (size_t)b;
        // Green's-theorem polygon moments (host: usv::hu_of, same order of operations)
        double a00 = 0, a10 = 0, a01 = 0, a20 = 0, a11 = 0, a02 = 0, a30 = 0, a21 = 0, a12 = 0, a03 = 0;
        double px = p[2 * (np - 1)], py = p[2 * (np - 1) + 1];
        double px2 = px * px, py2 = py * py;
        // shoelace area in the float-converted points (host: usv::contourAreaAbs)
        double s00 = 0;
        float fx = (float)p[2 * (np - 1)], fy = (float)p[2 * (np - 1) + 1];
        for (int i = 0; i < np; ++i) {
            const double x = p[2 * i], y = p[2 * i + 1];
            const double x2 = x * x, y2 = y * y;
            const double cross = px * y - x * py;
            const double sx = px + x, sy = py + y;
            a00 += cross;
            a10 += cross * sx;
            a01 += cross * sy;
            a20 += cross * (px * sx + x2);
            a11 += cross * (px * (sy + py) + x * (sy + y));
            a02 += cross * (py * sy + y2);
            a30 += cross * sx * (px2 + x2);
            a03 += cross * sy * (py2 + y2);
            a21 += cross * (px2 * (3 * py + y) + 2 * x * px * sy + x2 * (py + 3 * y));
            a12 += cross * (py2 * (3 * px + x) + 2 * y * py * sx + y2 * (px + 3 * x));
            px = x;
            py = y;
            px2 = x2;
            py2 = y2;
            const float gx = (float)p[2 * i], gy = (float)p[2 * i + 1];
            s00 += (double)fx * gy - (double)fy * gx;
            fx = gx;
            fy = gy;
        }
        area = fabs(s00 * 0.5);
        if (fabs(a00) > FLT_EPSILON) {
            const double sgn = a00 > 0 ? 1.0 : -1.0;
            const double m00 = a00 * (sgn * 0.5), m10 = a10 * (sgn / 6), m01 = a01 * (sgn / 6);
            const double m20 = a20 * (sgn / 12), m11 = a11 * (sgn / 24), m02 = a02 * (sgn / 12);
            const double m30 = a30 * (sgn / 20), m21 = a21 * (sgn / 60), m12 = a12 * (sgn / 60);
            const double m03 = a03 * (sgn / 20);
            double cx = 0, cy = 0, inv_m00 = 0;
            if (fabs(m00) > DBL_EPSILON) {
                inv_m00 = 1. / m00;
                cx = m10 * inv_m00;
                cy = m01 * inv_m00;
            }
            const double mu20 = m20 - m10 * cx, mu11 = m11 - m10 * cy, mu02 = m02 - m01 * cy;
            const double mu30 = m30 - cx * (3 * mu20 + cx * m10);
            const double mu21 = m21 - cx * (2 * mu11 + cx * m01) - cy * mu20;
            const double mu12 = m12 - cy * (2 * mu11 + cy * m10) - cx * mu02;
            const double mu03 = m03 - cy * (3 * mu02 + cy * m01);
            const double s2 = inv_m00 * inv_m00, s3 = s2 * sqrt(fabs(inv_m00));
            const double n20 = mu20 * s2, n11 = mu11 * s2, n02 = mu02 * s2;
            const double n30 = mu30 * s3, n21 = mu21 * s3, n12 = mu12 * s3, n03 = mu03 * s3;
            double t0 = n30 + n12, t1 = n21 + n03;
            double q0 = t0 * t0, q1 = t1 * t1;
            const double n4 = 4 * n11, s = n20 + n02, d = n20 - n02;
            h[0] = s;
            h[1] = d * d + n4 * n11;
            h[3] = q0 + q1;
            h[5] = d * (q0 - q1) + n4 * t0 * t1;
            t0 *= q0 - 3 * q1;
            t1 *= 3 * q0 - q1;
            q0 = n30 - 3 * n12;
            q1 = 3 * n21 - n03;
            h[2] = q0 * q0 + q1 * q1;
            h[4] = q0 * t0 + q1 * t1;
            h[6] = q1 * t0 - q0 * t1;
        }
    }
    double* o = desc + (size_t)c * kDesc;
    for (int k = 0; k < 7; ++k) {
        const double a = fabs(h[k]);
        const double sg = h[k] > 0 ? 1.0 : (h[k] < 0 ? -1.0 : 0.0);
        o[k] = a > 1.e-5 ? 1. / (sg * log10(a)) : __builtin_nan("");
    }
    o[7] = area;
}

// scores[i * n_b + j] = I1(i, j) + |(A_i - A_j) / ((A_i + A_j) / 2)|; i-major like the reference's loops.
__global__ void __launch_bounds__(256) pair_score_kernel(const double* __restrict__ da, int n_a,
                                                         const double* __restrict__ db, int n_b,
                                                         double* __restrict__ scores) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)n_a * n_b) return;
    const int i = (int)(t / n_b), j = (int)(t - (int64_t)i * n_b);
    const double* a = da + (size_t)i * kDesc;
    const double* b = db + (size_t)j * kDesc;
    double v = 0;
    for (int k = 0; k < 7; ++k) {
        const double ma = a[k], mb = b[k];
        if (!__builtin_isnan(ma) && !__builtin_isnan(mb)) v += fabs(-ma + mb);
    }
    v += fabs((a[7] - b[7]) / ((a[7] + b[7]) / 2));
    scores[t] = v;
}

usv_status status_of(hipError_t e) { return e == hipSuccess ? USV_OK : USV_ERR_HIP; }

}  // namespace
}  // namespace usv

extern "C" {

usv_status usv_contour_descriptors(const int* pts, const int* off, int n, double* desc, void* stream) {
    if (n < 0 || (n && (!off || !desc))) return USV_ERR_INVALID_ARG;
    if (n == 0) return USV_OK;
    hipLaunchKernelGGL(usv::contour_desc_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0,
                       static_cast<hipStream_t>(stream), pts, off, n, desc);
    return usv::status_of(hipGetLastError());
}

usv_status usv_contour_pair_scores(const double* desc_a, int n_a, const double* desc_b, int n_b, double* scores,
                                   void* stream) {
    if (n_a < 0 || n_b < 0 || (n_a && n_b && (!desc_a || !desc_b || !scores))) return USV_ERR_INVALID_ARG;
    const int64_t total = (int64_t)n_a * n_b;
    if (total == 0) return USV_OK;
    if (total > (int64_t)1 << 31) return USV_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(usv::pair_score_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), desc_a, n_a, desc_b, n_b, scores);
    return usv::status_of(hipGetLastError());
}

}  // extern "C"
