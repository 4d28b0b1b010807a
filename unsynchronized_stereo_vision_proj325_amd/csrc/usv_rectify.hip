// usv_rectify.hip -- stereo rectification on gfx950.
//
// The reference rebuilds the OpenCV rectification map for every frame of
// both cameras and remaps with it (P/Main.cpp:351-359: initUndistortRectifyMap
// CV_16SC2 + remap INTER_LINEAR, BORDER_CONSTANT 0); the calibration struct is
// passed by value, so the map never survives a call.  Here the map is built
// once per calibration on the device (rectify_map_kernel, f64, the OpenCV
// column recurrence replayed exactly) and every frame is one HBM-bound gather
// (remap_kernel): 6 B of map + the output bytes per pixel, the source served
// from L2.  Both cameras go in one launch (grid z).  Semantics restated in
// oracle/rectify_oracle.c; the two agree bit for bit (tests/test_rectify.py).
#include <climits>

#include "usv.h"
#include "usv_kernels.hpp"

namespace usv {
namespace {

struct RectParams {
    double ir[9];
    double fx, fy, u0, v0;
    double k[12];  // k1 k2 p1 p2 k3 k4 k5 k6 s1 s2 s3 s4
};

__device__ __forceinline__ int sat_round(double v) {
    if (!(v > -2147483648.0)) return INT_MIN;
    if (v >= 2147483647.0) return INT_MAX;
    return __double2int_rn(v);
}

constexpr int kMapChunk = 32;  // columns per thread

// One thread per (row, chunk of kMapChunk columns).  OpenCV walks a row with
// _x += ir[0] (etc.) per column, so the thread first replays that recurrence
// from column 0 to its chunk: three dependent f64 adds per skipped column, the
// same rounding sequence as the sequential loop.
__global__ __launch_bounds__(64) void rectify_map_kernel(RectParams p, int W, int H, int16_t* __restrict__ map1,
                                                         uint16_t* __restrict__ map2) {
    const int i = blockIdx.y;
    const int j0 = (blockIdx.x * 64 + threadIdx.x) * kMapChunk;
    if (i >= H || j0 >= W) return;
    const double* ir = p.ir;
    double _x = i * ir[1] + ir[2], _y = i * ir[4] + ir[5], _w = i * ir[7] + ir[8];
    for (int j = 0; j < j0; ++j) {
        _x += ir[0];
        _y += ir[3];
        _w += ir[6];
    }
    const double k1 = p.k[0], k2 = p.k[1], p1 = p.k[2], p2 = p.k[3], k3 = p.k[4], k4 = p.k[5];
    const double k5 = p.k[6], k6 = p.k[7], s1 = p.k[8], s2 = p.k[9], s3 = p.k[10], s4 = p.k[11];
    const int j1 = min(W, j0 + kMapChunk);
    int16_t* m1 = map1 + (size_t)i * W * 2;
    uint16_t* m2 = map2 + (size_t)i * W;
    for (int j = j0; j < j1; ++j, _x += ir[0], _y += ir[3], _w += ir[6]) {
        const double w = 1. / _w, x = _x * w, y = _y * w;
        const double x2 = x * x, y2 = y * y;
        const double r2 = x2 + y2, _2xy = 2 * x * y;
        const double kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2);
        const double u = p.fx * (x * kr + p1 * _2xy + p2 * (r2 + 2 * x2) + s1 * r2 + s2 * r2 * r2) + p.u0;
        const double v = p.fy * (y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy + s3 * r2 + s4 * r2 * r2) + p.v0;
        const int iu = sat_round(u * 32), iv = sat_round(v * 32);
        m1[j * 2] = (int16_t)(iu >> 5);
        m1[j * 2 + 1] = (int16_t)(iv >> 5);
        m2[j] = (uint16_t)((iv & 31) * 32 + (iu & 31));
    }
}

struct RemapJob {
    const uint8_t* src;
    int spitch;
    const int16_t* map1;
    const uint16_t* map2;
    uint8_t* dst;
    int dpitch;
};

// QPT quads (4 output pixels each) per thread over a flat range of quads per camera.  Per thread
// every load is issued before any arithmetic: the maps of all its quads (one 16-B and one 8-B load
// per quad when the rows are 4-pixel aligned), then, for every pixel, the two aligned source reads
// (2 dwords for gray, 3 for BGR per row) at an address clamped into the image, so the reads are
// unconditional straight-line code; a pixel whose taps are not all inside the image (or whose
// aligned read was clamped) is redone afterwards on a per-tap path that reads 0 outside.  The
// result leaves as one 4-B (gray) or one 12-B (BGR) store per quad.
//   * Blocks are numbered XCD-contiguously (block b runs on XCD b % 8, and XCD k takes the k-th
//     contiguous run of quads), so the source rows one output band reads are fetched into one L2.
//   * Fixed point: every weight of OpenCV's bilinear table is a multiple of 32 and the four sum to
//     32768, so (S00 w0 + S01 w1 + S10 w2 + S11 w3 + 2^14) >> 15 = (S00 a0 + ... + 2^9) >> 10 with
//     a = w / 32 <= 1024: products < 2^18, sums < 2^24 and never above 255 after the shift.  The
//     two taps of a row are one u16 pair and their weights another, so each channel is two
//     v_dot2_u32_u16.
//   * Source offsets are 32-bit (sy * pitch + byte, a 24-bit multiply) from the job's base pointer.
typedef unsigned short usv_us2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t dot2(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_udot2(__builtin_bit_cast(usv_us2, a), __builtin_bit_cast(usv_us2, b), c, false);
}

#ifndef USV_REMAP_QPT
#define USV_REMAP_QPT 1  // quads per thread (2: 18.1 us, 4: 24.6 us vs 15.1 us at 1, 1080p BGR pair, one box)
#endif
constexpr int kRemapQPT = USV_REMAP_QPT;

template <int CN>
__global__ __launch_bounds__(256) void remap_kernel(RemapJob j0, RemapJob j1, int sW, int sH, int W, int H,
                                                    unsigned blocks_per_job, int vec_map, int vec_dst, int vec_src) {
    constexpr int QPT = kRemapQPT, NWD = CN == 1 ? 2 : 3;
    const unsigned total = gridDim.x, lin = blockIdx.x;
    const unsigned xcd = lin & 7u, base = total >> 3, rem = total & 7u;
    const unsigned lb = xcd * base + min(xcd, rem) + (lin >> 3);
    const unsigned job = lb >= blocks_per_job ? 1u : 0u;
    const RemapJob& j = job ? j1 : j0;
    const unsigned nq = (unsigned)(W + 3) >> 2, nqt = nq * (unsigned)H;
    const unsigned qb = (lb - job * blocks_per_job) * (256u * QPT) + threadIdx.x;
    int yq[QPT], xq[QPT], nn[QPT];
    int mx[QPT][4], my[QPT][4], mf[QPT][4];
#pragma unroll
    for (int u = 0; u < QPT; ++u) {
        const unsigned q = qb + 256u * u;
        const bool ok = q < nqt;
        const int y = ok ? (int)(q / nq) : 0;
        const int x0 = ok ? 4 * (int)(q - (unsigned)y * nq) : 0;
        yq[u] = y;
        xq[u] = x0;
        nn[u] = ok ? min(4, W - x0) : 0;
        const size_t mrow = (size_t)y * W + x0;
        if (vec_map && nn[u] == 4) {
            const int4 a = *reinterpret_cast<const int4*>(j.map1 + 2 * mrow);
            const uint2 f = *reinterpret_cast<const uint2*>(j.map2 + mrow);
            const int w4[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                mx[u][k] = (int)(int16_t)(w4[k] & 0xFFFF);
                my[u][k] = (int)(int16_t)((unsigned)w4[k] >> 16);
            }
            mf[u][0] = f.x & 0xFFFF;
            mf[u][1] = f.x >> 16;
            mf[u][2] = f.y & 0xFFFF;
            mf[u][3] = f.y >> 16;
        } else {
            for (int k = 0; k < 4; ++k) {
                const int kk = k < nn[u] ? k : 0;
                mx[u][k] = nn[u] ? j.map1[2 * (mrow + kk)] : -2;  // an idle slot: outside, nothing stored
                my[u][k] = nn[u] ? j.map1[2 * (mrow + kk) + 1] : -2;
                mf[u][k] = nn[u] ? j.map2[mrow + kk] : 0;
            }
        }
    }
    // unconditional aligned reads at clamped addresses (rows sy, sy + 1 and bytes a .. a + 4 NWD - 1
    // always inside the source)
    const int amax = (j.spitch - 4 * NWD) & ~3;
    uint32_t u0[QPT][4][NWD], u1[QPT][4][NWD];
    uint32_t good = 0;  // bit (4u + k): the clamped read is the exact one and every tap is inside
#pragma unroll
    for (int u = 0; u < QPT; ++u) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (!vec_src) {  // (uniform) unaligned source: every pixel takes the per-tap path
#pragma unroll
                for (int i = 0; i < NWD; ++i) u0[u][k][i] = u1[u][k][i] = 0;
                continue;
            }
            const int sx = mx[u][k], sy = my[u][k];
            const int a = (sx * CN) & ~3;
            const int ac = min(max(a, 0), amax), yc = min(max(sy, 0), sH - 2 > 0 ? sH - 2 : 0);
            const bool in = sx >= 0 && sx + 1 < sW && sy >= 0 && sy + 1 < sH && a == ac;
            good |= in ? 1u << (4 * u + k) : 0u;
            const uint32_t r0 = __umul24((uint32_t)yc, (uint32_t)j.spitch) + (uint32_t)ac;  // both < 2^24 (launch)
            const uint32_t* q0 = reinterpret_cast<const uint32_t*>(j.src + r0);
            const uint32_t* q1 = reinterpret_cast<const uint32_t*>(j.src + r0 + (uint32_t)(sH > 1 ? j.spitch : 0));
#pragma unroll
            for (int i = 0; i < NWD; ++i) {
                u0[u][k][i] = q0[i];
                u1[u][k][i] = q1[i];
            }
        }
    }
#pragma unroll
    for (int u = 0; u < QPT; ++u) {
        uint32_t out[4 * CN];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t ty = (uint32_t)mf[u][k] >> 5, tx = (uint32_t)mf[u][k] & 31u;
            // row weights as u16 pairs: (32 - tx, tx) scaled by (32 - ty) for row 0, by ty for row 1
            const uint32_t wx = (32u - tx) | (tx << 16);
            const uint32_t wr0 = wx * (32u - ty), wr1 = wx * ty;  // both halves <= 1024: no carry
            const int o = (mx[u][k] * CN) & 3;
            const uint32_t l0 = __builtin_amdgcn_alignbyte(u0[u][k][1], u0[u][k][0], o);  // tap bytes 0..3
            const uint32_t l1 = __builtin_amdgcn_alignbyte(u1[u][k][1], u1[u][k][0], o);
            uint32_t h0 = 0, h1 = 0;
            if constexpr (CN == 3) {
                h0 = __builtin_amdgcn_alignbyte(u0[u][k][2], u0[u][k][1], o);  // tap bytes 4..7
                h1 = __builtin_amdgcn_alignbyte(u1[u][k][2], u1[u][k][1], o);
            }
#pragma unroll
            for (int c = 0; c < CN; ++c) {
                // (left tap | right tap << 16) of each row: byte c and byte CN + c of (h:l); v_perm bytes
                // 0-3 are its second operand, 4-7 its first, 0x0c gives zero
                const uint32_t sel = 0x0c000c00u | (uint32_t)c | ((uint32_t)(CN + c) << 16);
                const uint32_t p0 = __builtin_amdgcn_perm(h0, l0, sel);
                const uint32_t p1 = __builtin_amdgcn_perm(h1, l1, sel);
                out[k * CN + c] = dot2(p0, wr0, dot2(p1, wr1, 1u << 9)) >> 10;
            }
            if (!(good >> (4 * u + k) & 1u)) {
                // border / clamped read: per-tap reads, 0 outside (BORDER_CONSTANT), all four outside -> 0
                const int sx = mx[u][k], sy = my[u][k];
                const bool x0ok = sx >= 0, x1ok = sx + 1 < sW, y0ok = sy >= 0, y1ok = sy + 1 < sH;
                const bool any = sx < sW && sx + 1 >= 0 && sy < sH && sy + 1 >= 0;
                const uint8_t* rp0 = j.src + (ptrdiff_t)sy * j.spitch + (ptrdiff_t)sx * CN;
                const uint8_t* rp1 = rp0 + j.spitch;
                const uint32_t w0 = wr0 & 0xFFFFu, w1 = wr0 >> 16, w2 = wr1 & 0xFFFFu, w3 = wr1 >> 16;
#pragma unroll
                for (int c = 0; c < CN; ++c) {
                    const uint32_t v0 = (any && x0ok && y0ok) ? rp0[c] : 0;
                    const uint32_t v1 = (any && x1ok && y0ok) ? rp0[CN + c] : 0;
                    const uint32_t v2 = (any && x0ok && y1ok) ? rp1[c] : 0;
                    const uint32_t v3 = (any && x1ok && y1ok) ? rp1[CN + c] : 0;
                    out[k * CN + c] =
                        (__umul24(v0, w0) + __umul24(v1, w1) + __umul24(v2, w2) + __umul24(v3, w3) + (1u << 9)) >> 10;
                }
            }
        }
        const int n = nn[u];
        if (n == 0) continue;
        uint8_t* d = j.dst + (size_t)yq[u] * j.dpitch + (size_t)xq[u] * CN;
        if (vec_dst && n == 4) {
            if constexpr (CN == 3) {
                uint3 w;
                w.x = out[0] | (out[1] << 8) | (out[2] << 16) | (out[3] << 24);
                w.y = out[4] | (out[5] << 8) | (out[6] << 16) | (out[7] << 24);
                w.z = out[8] | (out[9] << 8) | (out[10] << 16) | (out[11] << 24);
                *reinterpret_cast<uint3*>(d) = w;
            } else {
                *reinterpret_cast<uint32_t*>(d) = out[0] | (out[1] << 8) | (out[2] << 16) | (out[3] << 24);
            }
        } else {
            for (int b = 0; b < n * CN; ++b) d[b] = (uint8_t)out[b];
        }
    }
}

bool aligned(const void* p, size_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }

usv_status launch_remap(const RemapJob& a, const RemapJob& b, int n_jobs, int cn, int sW, int sH, int W, int H,
                        hipStream_t s) {
    bool vec_map = (W % 4) == 0, vec_dst = true, vec_src = true;
    for (int i = 0; i < n_jobs; ++i) {
        const RemapJob& j = i ? b : a;
        vec_map = vec_map && aligned(j.map1, 16) && aligned(j.map2, 8);
        vec_dst = vec_dst && aligned(j.dst, 4) && (j.dpitch % 4) == 0;
        vec_src = vec_src && aligned(j.src, 4) && (j.spitch % 4) == 0;
    }
    // 32-bit source offsets: sy * spitch + byte stays below 2^32
    if ((long long)(sH + 1) * a.spitch >= (1LL << 32) || (long long)(sH + 1) * b.spitch >= (1LL << 32) ||
        a.spitch >= (1 << 24) || b.spitch >= (1 << 24))
        return USV_ERR_UNSUPPORTED;
    const long long quads = (long long)((W + 3) / 4) * H;
    const long long per_job = (quads + 256 * kRemapQPT - 1) / (256 * kRemapQPT);
    if (a.spitch < 4 * (cn == 1 ? 2 : 3) || b.spitch < 4 * (cn == 1 ? 2 : 3)) vec_src = false;  // rows too short for the aligned reads
    if (per_job * n_jobs > 0x7FFFFFFFLL) return USV_ERR_UNSUPPORTED;
    dim3 grid((unsigned)(per_job * n_jobs)), block(256);
    if (cn == 1)
        hipLaunchKernelGGL(remap_kernel<1>, grid, block, 0, s, a, b, sW, sH, W, H, (unsigned)per_job, (int)vec_map,
                           (int)vec_dst, (int)vec_src);
    else if (cn == 3)
        hipLaunchKernelGGL(remap_kernel<3>, grid, block, 0, s, a, b, sW, sH, W, H, (unsigned)per_job, (int)vec_map,
                           (int)vec_dst, (int)vec_src);
    else
        return USV_ERR_UNSUPPORTED;
    return hipGetLastError() == hipSuccess ? USV_OK : USV_ERR_HIP;
}

bool job_ok(const RemapJob& j, int cn, int sW, int W) {
    return j.src && j.map1 && j.map2 && j.dst && j.spitch >= sW * cn && j.dpitch >= W * cn;
}

}  // namespace
}  // namespace usv

extern "C" {

usv_status usv_rectify_params(const double* K, const double* dist, int n_dist, const double* Rrect,
                              const double* P, int p_cols, double* params) {
    if (!K || !P || !params || (p_cols != 3 && p_cols != 4)) return USV_ERR_INVALID_ARG;
    if (!(n_dist == 0 || n_dist == 4 || n_dist == 5 || n_dist == 8 || n_dist == 12) || (n_dist && !dist))
        return USV_ERR_INVALID_ARG;
    double Rm[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    if (Rrect)
        for (int i = 0; i < 9; ++i) Rm[i] = Rrect[i];
    // Ar.colRange(0,3) * R, then its inverse by adjugate / determinant (cv::invert, n <= 3)
    double A[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            A[i * 3 + j] = P[i * p_cols] * Rm[j] + P[i * p_cols + 1] * Rm[3 + j] + P[i * p_cols + 2] * Rm[6 + j];
    auto m = [&](int i, int j) { return A[i * 3 + j]; };
    double det = m(0, 0) * (m(1, 1) * m(2, 2) - m(1, 2) * m(2, 1)) - m(0, 1) * (m(1, 0) * m(2, 2) - m(1, 2) * m(2, 0)) +
                 m(0, 2) * (m(1, 0) * m(2, 1) - m(1, 1) * m(2, 0));
    if (det == 0.) return USV_ERR_INVALID_ARG;
    det = 1. / det;
    params[0] = (m(1, 1) * m(2, 2) - m(1, 2) * m(2, 1)) * det;
    params[1] = (m(0, 2) * m(2, 1) - m(0, 1) * m(2, 2)) * det;
    params[2] = (m(0, 1) * m(1, 2) - m(0, 2) * m(1, 1)) * det;
    params[3] = (m(1, 2) * m(2, 0) - m(1, 0) * m(2, 2)) * det;
    params[4] = (m(0, 0) * m(2, 2) - m(0, 2) * m(2, 0)) * det;
    params[5] = (m(0, 2) * m(1, 0) - m(0, 0) * m(1, 2)) * det;
    params[6] = (m(1, 0) * m(2, 1) - m(1, 1) * m(2, 0)) * det;
    params[7] = (m(0, 1) * m(2, 0) - m(0, 0) * m(2, 1)) * det;
    params[8] = (m(0, 0) * m(1, 1) - m(0, 1) * m(1, 0)) * det;
    params[9] = K[0];
    params[10] = K[4];
    params[11] = K[2];
    params[12] = K[5];
    for (int i = 0; i < 12; ++i) params[13 + i] = i < n_dist ? dist[i] : 0.;
    return USV_OK;
}

usv_status usv_rectify_map(const double* params, int W, int H, int16_t* map1, uint16_t* map2, void* stream) {
    if (!params || !map1 || !map2 || W <= 0 || H <= 0 || W > 32767 || H > 32767) return USV_ERR_INVALID_ARG;
    usv::RectParams p;
    for (int i = 0; i < 9; ++i) p.ir[i] = params[i];
    p.fx = params[9];
    p.fy = params[10];
    p.u0 = params[11];
    p.v0 = params[12];
    for (int i = 0; i < 12; ++i) p.k[i] = params[13 + i];
    const int chunks = (W + usv::kMapChunk - 1) / usv::kMapChunk;
    dim3 grid((unsigned)((chunks + 63) / 64), (unsigned)H), block(64);
    hipLaunchKernelGGL(usv::rectify_map_kernel, grid, block, 0, static_cast<hipStream_t>(stream), p, W, H, map1,
                       map2);
    return hipGetLastError() == hipSuccess ? USV_OK : USV_ERR_HIP;
}

usv_status usv_remap_linear_u8(const uint8_t* src, int sW, int sH, int spitch, int cn, const int16_t* map1,
                               const uint16_t* map2, int W, int H, uint8_t* dst, int dpitch, void* stream) {
    if (sW <= 0 || sH <= 0 || W <= 0 || H <= 0 || H > 65535) return USV_ERR_INVALID_ARG;
    if (cn != 1 && cn != 3) return USV_ERR_UNSUPPORTED;
    const usv::RemapJob j{src, spitch, map1, map2, dst, dpitch};
    if (!usv::job_ok(j, cn, sW, W)) return USV_ERR_INVALID_ARG;
    return usv::launch_remap(j, j, 1, cn, sW, sH, W, H, static_cast<hipStream_t>(stream));
}

usv_status usv_rectify_pair_u8(const uint8_t* srcL, const uint8_t* srcR, int sW, int sH, int spitch, int cn,
                               const int16_t* map1L, const uint16_t* map2L, const int16_t* map1R,
                               const uint16_t* map2R, int W, int H, uint8_t* dstL, uint8_t* dstR, int dpitch,
                               void* stream) {
    if (sW <= 0 || sH <= 0 || W <= 0 || H <= 0 || H > 65535) return USV_ERR_INVALID_ARG;
    if (cn != 1 && cn != 3) return USV_ERR_UNSUPPORTED;
    const usv::RemapJob a{srcL, spitch, map1L, map2L, dstL, dpitch};
    const usv::RemapJob b{srcR, spitch, map1R, map2R, dstR, dpitch};
    if (!usv::job_ok(a, cn, sW, W) || !usv::job_ok(b, cn, sW, W)) return USV_ERR_INVALID_ARG;
    return usv::launch_remap(a, b, 2, cn, sW, sH, W, H, static_cast<hipStream_t>(stream));
}

}  // extern "C"
