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
#include <algorithm>
#include <cstring>

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

// GenerateMatchingList's whole selection on the device: one wave per row i of the score matrix walks
// j in chunks of 64 lanes, keeps v < 0.75 (NaN fails the test, as in the reference's `if`), and
// compacts the survivors of each chunk in lane order with a ballot + mbcnt, so row i's matches land at
// out + i * n_b in j order; counts[i] gets the row's count.  i-major, j-minor: the host concatenates
// the rows in order (P/Main.cpp:408-420).
__global__ void __launch_bounds__(256) match_select_kernel(const double* __restrict__ da, int n_a,
                                                           const double* __restrict__ db, int n_b,
                                                           usv_match* __restrict__ out, int* __restrict__ counts) {
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (i >= n_a) return;
    double a[kDesc];
#pragma unroll
    for (int k = 0; k < kDesc; ++k) a[k] = da[(size_t)i * kDesc + k];
    usv_match* row = out + (size_t)i * n_b;
    int n = 0;
    for (int j0 = 0; j0 < n_b; j0 += 64) {
        const int j = j0 + lane;
        bool keep = false;
        double v = 0;
        if (j < n_b) {
            const double* b = db + (size_t)j * kDesc;
            for (int k = 0; k < 7; ++k) {
                const double ma = a[k], mb = b[k];
                if (!__builtin_isnan(ma) && !__builtin_isnan(mb)) v += fabs(-ma + mb);
            }
            v += fabs((a[7] - b[7]) / ((a[7] + b[7]) / 2));
            keep = v < 0.75;
        }
        const uint64_t m = __ballot(keep);
        if (keep) {
            const int slot = n + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            row[slot].left_index = (unsigned)i;
            row[slot].right_index = (unsigned)j;
            row[slot].match_value = v;
        }
        n += __popcll(m);
    }
    if (lane == 0) counts[i] = n;
}

// Exclusive prefix of the row counts (one block): offs[i] = matches before row i, offs[n] = the total.
__global__ void __launch_bounds__(1024) match_offsets_kernel(const int* __restrict__ counts, int n,
                                                             int* __restrict__ offs) {
    __shared__ int part[1024];
    const int t = threadIdx.x;
    int carry = 0;
    for (int base = 0; base < n; base += 1024) {
        const int i = base + t;
        int v = i < n ? counts[i] : 0;
        part[t] = v;
        __syncthreads();
        for (int d = 1; d < 1024; d <<= 1) {  // Hillis-Steele inclusive scan
            const int add = t >= d ? part[t - d] : 0;
            __syncthreads();
            part[t] += add;
            __syncthreads();
        }
        if (i < n) offs[i] = carry + part[t] - v;
        carry += part[1023];
        __syncthreads();
    }
    if (t == 0) offs[n] = carry;
}

// Row i's matches (rows n_b apart) to dense[offs[i] ..]: the whole list in i-major, j-minor order, so one
// copy of `total` entries brings it to the host.  One wave per row.
__global__ void __launch_bounds__(256) match_gather_kernel(const usv_match* __restrict__ rows, int n_a, int n_b,
                                                           const int* __restrict__ counts,
                                                           const int* __restrict__ offs,
                                                           usv_match* __restrict__ dense) {
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (i >= n_a) return;
    const int c = counts[i], o = offs[i];
    for (int k = lane; k < c; k += 64) dense[(size_t)o + k] = rows[(size_t)i * n_b + k];
}

}  // namespace
}  // namespace usv

// Device matcher object: pinned host staging for the two contour sets and the results, device buffers
// sized for max_contours per set and max_points per set, one stream.  One call = one H2D copy of both
// sets, the descriptor launches, the select launch, the row offsets and the gather into one dense list on
// the device, then one D2H of the total and of the list's first `guess` entries (the previous call's
// total, at least 256) and, only when the list is longer, a second D2H of the rest.
struct usv_contour_matcher {
    int max_n = 0, max_pts = 0, device = 0;
    hipStream_t stream = nullptr;
    // host pinned block: off_a[max_n + 1] off_b[max_n + 1] pts_a[2 max_pts] pts_b[2 max_pts] (ints)
    int* h_in = nullptr;
    int* d_in = nullptr;
    double* d_desc = nullptr;   // 2 max_n x kDesc
    usv_match* d_rows = nullptr;  // max_n x max_n
    int* d_counts = nullptr;      // max_n row counts, then max_n + 1 row offsets
    usv_match* d_dense = nullptr; // max_n x max_n: the compacted list
    usv_match* h_rows = nullptr;  // pinned: the list's head (and rest)
    int* h_counts = nullptr;      // pinned: the total
    long long last_total = 256;   // D2H guess for the next call
};

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

usv_status usv_contour_matcher_create(int max_contours, int max_points, usv_contour_matcher** out) {
    if (!out) return USV_ERR_INVALID_ARG;
    *out = nullptr;
    if (max_contours < 1 || max_points < 1 || max_contours > 16384) return USV_ERR_INVALID_ARG;
    auto* m = new usv_contour_matcher;
    m->max_n = max_contours;
    m->max_pts = max_points;
    const size_t n_in = 2 * ((size_t)max_contours + 1) + 4 * (size_t)max_points;
    const size_t rows = (size_t)max_contours * max_contours;
    bool ok = hipGetDevice(&m->device) == hipSuccess &&
              hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking) == hipSuccess &&
              hipHostMalloc(&m->h_in, n_in * sizeof(int), hipHostMallocDefault) == hipSuccess &&
              hipMalloc(&m->d_in, n_in * sizeof(int)) == hipSuccess &&
              hipMalloc(&m->d_desc, 2 * (size_t)max_contours * usv::kDesc * sizeof(double)) == hipSuccess &&
              hipMalloc(&m->d_rows, rows * sizeof(usv_match)) == hipSuccess &&
              hipMalloc(&m->d_counts, (2 * (size_t)max_contours + 1) * sizeof(int)) == hipSuccess &&
              hipMalloc(&m->d_dense, rows * sizeof(usv_match)) == hipSuccess &&
              hipHostMalloc(&m->h_rows, rows * sizeof(usv_match), hipHostMallocDefault) == hipSuccess &&
              hipHostMalloc(&m->h_counts, sizeof(int), hipHostMallocDefault) == hipSuccess;
    if (!ok) {
        usv_contour_matcher_destroy(m);
        return USV_ERR_HIP;
    }
    *out = m;
    return USV_OK;
}

usv_status usv_contour_matcher_destroy(usv_contour_matcher* m) {
    if (!m) return USV_ERR_INVALID_ARG;
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(m->device);
    if (m->stream) (void)hipStreamSynchronize(m->stream);
    (void)hipHostFree(m->h_in);
    (void)hipFree(m->d_in);
    (void)hipFree(m->d_desc);
    (void)hipFree(m->d_rows);
    (void)hipFree(m->d_counts);
    (void)hipFree(m->d_dense);
    (void)hipHostFree(m->h_rows);
    (void)hipHostFree(m->h_counts);
    if (m->stream) (void)hipStreamDestroy(m->stream);
    (void)hipSetDevice(cur);
    delete m;
    return USV_OK;
}

usv_status usv_generate_matching_list_gpu(usv_contour_matcher* m, const int* pts_a, const int* off_a, int n_a,
                                          const int* pts_b, const int* off_b, int n_b, usv_match* out, int cap,
                                          int* n_out) {
    if (!m || !n_out || n_a < 0 || n_b < 0 || cap < 0 || (cap && !out)) return USV_ERR_INVALID_ARG;
    *n_out = 0;
    if (n_a == 0 || n_b == 0) return USV_OK;  // P/Main.cpp:405: an empty set matches nothing
    if (!pts_a || !off_a || !pts_b || !off_b) return USV_ERR_INVALID_ARG;
    if (n_a > m->max_n || n_b > m->max_n) return USV_ERR_UNSUPPORTED;
    const int pa = off_a[n_a], pb = off_b[n_b];
    if (off_a[0] != 0 || off_b[0] != 0 || pa < 0 || pb < 0 || pa > m->max_pts || pb > m->max_pts)
        return USV_ERR_INVALID_ARG;
    for (int i = 0; i < n_a; ++i)
        if (off_a[i + 1] < off_a[i]) return USV_ERR_INVALID_ARG;
    for (int i = 0; i < n_b; ++i)
        if (off_b[i + 1] < off_b[i]) return USV_ERR_INVALID_ARG;
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess || hipSetDevice(m->device) != hipSuccess) return USV_ERR_HIP;
    struct Restore {
        int d;
        ~Restore() { (void)hipSetDevice(d); }
    } restore{cur};
    // one contiguous block: off_a | off_b | pts_a | pts_b
    int* h = m->h_in;
    std::memcpy(h, off_a, (size_t)(n_a + 1) * sizeof(int));
    std::memcpy(h + n_a + 1, off_b, (size_t)(n_b + 1) * sizeof(int));
    std::memcpy(h + n_a + n_b + 2, pts_a, 2 * (size_t)pa * sizeof(int));
    std::memcpy(h + n_a + n_b + 2 + 2 * (size_t)pa, pts_b, 2 * (size_t)pb * sizeof(int));
    const size_t n_in = (size_t)n_a + n_b + 2 + 2 * ((size_t)pa + pb);
    hipStream_t s = m->stream;
    const int* d_off_a = m->d_in;
    const int* d_off_b = m->d_in + n_a + 1;
    const int* d_pts_a = m->d_in + n_a + n_b + 2;
    const int* d_pts_b = d_pts_a + 2 * (size_t)pa;
    double* desc_a = m->d_desc;
    double* desc_b = m->d_desc + (size_t)m->max_n * usv::kDesc;
    auto fail = [&](usv_status st) {
        (void)hipStreamSynchronize(s);
        return st;
    };
    if (hipMemcpyAsync(m->d_in, h, n_in * sizeof(int), hipMemcpyHostToDevice, s) != hipSuccess) return fail(USV_ERR_HIP);
    hipLaunchKernelGGL(usv::contour_desc_kernel, dim3((unsigned)((n_a + 63) / 64)), dim3(64), 0, s, d_pts_a, d_off_a, n_a,
                       desc_a);
    hipLaunchKernelGGL(usv::contour_desc_kernel, dim3((unsigned)((n_b + 63) / 64)), dim3(64), 0, s, d_pts_b, d_off_b, n_b,
                       desc_b);
    hipLaunchKernelGGL(usv::match_select_kernel, dim3((unsigned)((n_a + 3) / 4)), dim3(256), 0, s, desc_a, n_a, desc_b,
                       n_b, m->d_rows, m->d_counts);
    int* d_offs = m->d_counts + m->max_n;
    hipLaunchKernelGGL(usv::match_offsets_kernel, dim3(1), dim3(1024), 0, s, m->d_counts, n_a, d_offs);
    hipLaunchKernelGGL(usv::match_gather_kernel, dim3((unsigned)((n_a + 3) / 4)), dim3(256), 0, s, m->d_rows, n_a,
                       n_b, m->d_counts, d_offs, m->d_dense);
    if (hipGetLastError() != hipSuccess) return fail(USV_ERR_HIP);
    const long long most = (long long)n_a * n_b;
    const long long guess = std::min(most, std::max(256LL, m->last_total));
    if (hipMemcpyAsync(m->h_counts, d_offs + n_a, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(m->h_rows, m->d_dense, (size_t)guess * sizeof(usv_match), hipMemcpyDeviceToHost, s) !=
            hipSuccess)
        return fail(USV_ERR_HIP);
    if (hipStreamSynchronize(s) != hipSuccess) return USV_ERR_HIP;
    const long long total = m->h_counts[0];
    m->last_total = total;
    if (total > cap) return USV_ERR_INVALID_ARG;  // as usv_generate_matching_list: out must hold every match
    if (total > guess) {
        if (hipMemcpyAsync(m->h_rows + guess, m->d_dense + guess, (size_t)(total - guess) * sizeof(usv_match),
                           hipMemcpyDeviceToHost, s) != hipSuccess)
            return fail(USV_ERR_HIP);
        if (hipStreamSynchronize(s) != hipSuccess) return USV_ERR_HIP;
    }
    if (total > 0) std::memcpy(out, m->h_rows, (size_t)total * sizeof(usv_match));
    *n_out = (int)total;
    return USV_OK;
}

}  // extern "C"
