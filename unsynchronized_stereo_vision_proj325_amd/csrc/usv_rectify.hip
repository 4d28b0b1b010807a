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
#include "usv_remap.hpp"

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

// One quad (4 output pixels) per thread over a flat, XCD-contiguous range of quads per camera;
// remap_quad (usv_remap.hpp) computes it, the result leaves as one 4-B (gray) or one 12-B (BGR)
// store.  Measured alternatives, all slower (profiles/probes_r03/ab_remap_gather_r03.txt): two or four
// quads per thread with every load issued first (18.1 / 24.6 vs 15.1 us), and 2 / 4 / 8 quads per thread
// with the next quad's map prefetched during the current quad's gathers (16.5 / 15.0 / 18.9 vs 15.2 us).
// A build with no source reads at all still took 11.4 of 13.7 us: the launch is bound by its per-quad
// VALU (~250 instructions: decode, clamps, alignbytes, 3 x (2 v_perm + 2 v_dot2) per pixel, packing)
// and wants every wave slot, not by the map round trip.
#ifndef USV_REMAP_BLOCK
#define USV_REMAP_BLOCK 256  // threads per block
#endif
#ifndef USV_REMAP_XCD
#define USV_REMAP_XCD 1  // XCD-contiguous block order
#endif
constexpr int kRemapBlock = USV_REMAP_BLOCK;
template <int CN, bool PK>
__global__ __launch_bounds__(kRemapBlock) void remap_kernel(RemapJob j0, RemapJob j1, int sW, int sH, int W, int H,
                                                    unsigned blocks_per_job, int vec_map, int vec_dst, int vec_src) {
    const unsigned lb = USV_REMAP_XCD ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const unsigned job = lb >= blocks_per_job ? 1u : 0u;
    const RemapJob& j = job ? j1 : j0;
    const unsigned nq = (unsigned)(W + 3) >> 2;
    const unsigned q = (lb - job * blocks_per_job) * (unsigned)kRemapBlock + threadIdx.x;
    if (q >= nq * (unsigned)H) return;
    const int y = (int)quad_row(q, nq, quad_row_fast(nq * (unsigned)H, nq));
    const int x0 = 4 * (int)(q - (unsigned)y * nq);
    const int n = min(4, W - x0);
    uint32_t out[4 * CN];
    remap_quad<CN, PK>(j, sW, sH, W, y, x0, n, vec_map, vec_src, out);
    uint8_t* d = j.dst + (size_t)y * j.dpitch + (size_t)x0 * CN;
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

bool aligned(const void* p, size_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }

usv_status launch_remap(const RemapJob& a, const RemapJob& b, int n_jobs, int cn, int sW, int sH, int W, int H,
                        hipStream_t s) {
    const bool pk = a.pmap != nullptr;  // both jobs packed or neither (the entry points check)
    bool vec_map = (W % 4) == 0, vec_dst = true, vec_src = true;
    for (int i = 0; i < n_jobs; ++i) {
        const RemapJob& j = i ? b : a;
        vec_map = vec_map && (pk ? aligned(j.pmap, 16) : aligned(j.map1, 16) && aligned(j.map2, 8));
        vec_dst = vec_dst && aligned(j.dst, 4) && (j.dpitch % 4) == 0;
        vec_src = vec_src && aligned(j.src, 4) && (j.spitch % 4) == 0;
    }
    // 32-bit source offsets: sy * spitch + byte stays below 2^32
    if ((long long)(sH + 1) * a.spitch >= (1LL << 32) || (long long)(sH + 1) * b.spitch >= (1LL << 32) ||
        a.spitch >= (1 << 24) || b.spitch >= (1 << 24))
        return USV_ERR_UNSUPPORTED;
    const long long quads = (long long)((W + 3) / 4) * H;
    const long long per_job = (quads + kRemapBlock - 1) / kRemapBlock;
    if (a.spitch < 4 * (cn == 1 ? 2 : 3) || b.spitch < 4 * (cn == 1 ? 2 : 3)) vec_src = false;  // rows too short for the aligned reads
    if (per_job * n_jobs > 0x7FFFFFFFLL) return USV_ERR_UNSUPPORTED;
    dim3 grid((unsigned)(per_job * n_jobs)), block(kRemapBlock);
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, block, 0, s, a, b, sW, sH, W, H, (unsigned)per_job, (int)vec_map, (int)vec_dst,
                           (int)vec_src);
    };
    if (cn == 1) pk ? go(remap_kernel<1, true>) : go(remap_kernel<1, false>);
    else if (cn == 3) pk ? go(remap_kernel<3, true>) : go(remap_kernel<3, false>);
    else return USV_ERR_UNSUPPORTED;
    return hipGetLastError() == hipSuccess ? USV_OK : USV_ERR_HIP;
}

// map1 / map2 -> the packed word per pixel (usv_remap.hpp pack_map_word); a flat range of pixels.
__global__ __launch_bounds__(256) void pack_map_kernel(const int16_t* __restrict__ map1,
                                                       const uint16_t* __restrict__ map2, long long n, int sW, int sH,
                                                       uint32_t* __restrict__ pmap) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    pmap[i] = pack_map_word(map1[2 * i], map1[2 * i + 1], map2[i], sW, sH);
}

// ---- LDS-tiled remap (packed map): one workgroup per 64 x 16 output tile ----------------------------
// The direct kernel gathers ~24 scattered dwords per quad through the texture path, two dependent
// round trips per wave (map, then source).  Here the source box a tile reads (precomputed once per
// calibration by tile_box_kernel from the packed map) is staged in LDS by coalesced dword loads issued
// together with the map loads -- one round trip -- and each pixel's two source rows are read from LDS;
// a pixel with a tap outside its tile's box (image borders, or a box too large for LDS) takes
// remap_blend's per-tap global path.  Same integer blend: bit-identical results.
constexpr int kTileW = 64, kTileH = 16;      // 16 quads x 16 rows: one quad per thread of 256
constexpr int kBoxMaxDw = 3072;              // 12 KB of LDS per workgroup for the box
// Box word pair per tile: x = bx0 | by0 << 16, y = rowdw | h << 16 (rowdw = LDS dwords per staged row,
// 0 = no box: every pixel of the tile takes the global path).  The staged row covers source bytes
// [(bx0 cn) & ~3, (bx1 + 1) cn) plus two dwords of slack for the aligned three-dword reads.
__global__ __launch_bounds__(256) void tile_box_kernel(const uint32_t* __restrict__ pmap, int W, int H, int sW, int sH,
                                                       int cn, int tiles_x, uint2* __restrict__ boxes) {
    __shared__ int red[4][4];
    const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const int x0 = tx * kTileW + 4 * (threadIdx.x & 15), y = ty * kTileH + (threadIdx.x >> 4);
    int lo_x = INT_MAX, hi_x = INT_MIN, lo_y = INT_MAX, hi_y = INT_MIN;
    if (y < H)
        for (int k = 0; k < 4 && x0 + k < W; ++k) {
            const uint32_t w = pmap[(size_t)y * W + x0 + k];
            const int sx = (int)((w >> 10) & 2047u) - 1, sy = (int)(w >> 21) - 1;
            if (sx < sW && sx + 1 >= 0 && sy < sH && sy + 1 >= 0) {  // some tap in the source
                lo_x = min(lo_x, sx);
                hi_x = max(hi_x, sx + 1);
                lo_y = min(lo_y, sy);
                hi_y = max(hi_y, sy + 1);
            }
        }
    for (int o = 32; o > 0; o >>= 1) {
        lo_x = min(lo_x, __shfl_xor(lo_x, o));
        hi_x = max(hi_x, __shfl_xor(hi_x, o));
        lo_y = min(lo_y, __shfl_xor(lo_y, o));
        hi_y = max(hi_y, __shfl_xor(hi_y, o));
    }
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[wv][0] = lo_x;
        red[wv][1] = hi_x;
        red[wv][2] = lo_y;
        red[wv][3] = hi_y;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    for (int k = 1; k < 4; ++k) {
        lo_x = min(red[0][0], red[k][0]);
        red[0][0] = lo_x;
        red[0][1] = max(red[0][1], red[k][1]);
        red[0][2] = min(red[0][2], red[k][2]);
        red[0][3] = max(red[0][3], red[k][3]);
    }
    const int bx0 = max(red[0][0], 0), bx1 = min(red[0][1], sW - 1);
    const int by0 = max(red[0][2], 0), by1 = min(red[0][3], sH - 1);
    uint2 b = make_uint2(0u, 0u);
    if (red[0][0] != INT_MAX && bx1 > bx0 && by1 > by0) {
        const int rowdw = (((bx1 + 1) * cn + 3) >> 2) - ((bx0 * cn) >> 2) + 2;
        const int h = by1 - by0 + 1;
        if (rowdw <= 256 && rowdw * h <= kBoxMaxDw)
            b = make_uint2((unsigned)bx0 | ((unsigned)by0 << 16), (unsigned)rowdw | ((unsigned)h << 16));
    }
    boxes[blockIdx.x] = b;
}

template <int CN>
__global__ __launch_bounds__(256) void remap_tile_kernel(RemapJob j0, RemapJob j1, int sW, int sH, int W, int H,
                                                         int tiles_x, unsigned tiles_per_job, const uint2* __restrict__ b0,
                                                         const uint2* __restrict__ b1, int vec_dst) {
    constexpr int NWD = CN == 1 ? 2 : 3;
    __shared__ uint32_t box[kBoxMaxDw];
    const unsigned lb = xcd_block(blockIdx.x, gridDim.x);
    const unsigned job = lb >= tiles_per_job ? 1u : 0u;
    const RemapJob& j = job ? j1 : j0;
    const unsigned tile = lb - job * tiles_per_job;
    const uint2 b = (job ? b1 : b0)[tile];
    const int tx = (int)(tile % (unsigned)tiles_x), ty = (int)(tile / (unsigned)tiles_x);
    const int x0 = tx * kTileW + 4 * (int)(threadIdx.x & 15), y = ty * kTileH + (int)(threadIdx.x >> 4);
    const int bx0 = (int)(b.x & 0xFFFFu), by0 = (int)(b.x >> 16), rowdw = (int)(b.y & 0xFFFFu), bh = (int)(b.y >> 16);
    // last column whose bytes are all staged (and in the image: the staged row may run past sW - 1)
    const int bx1 = rowdw ? min((4 * (rowdw - 2) + ((bx0 * CN) & ~3)) / CN - 1, sW - 1) : -1;
    const int by1 = by0 + bh - 1;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(j.src), (short)0, (int)((unsigned)sH * (unsigned)j.spitch), 0x00020000);
    // 1. the box (coalesced dwords) and the map, in flight together.  A dword wholly past the last source
    // byte reads as 0 (never used); the one dword that straddles the end is read byte by byte, since a
    // buffer load returns 0 for a dword that is only partly in range.
    if (rowdw) {
        const int per = 256 / rowdw;
        const int t = (int)threadIdx.x, r0 = t / rowdw, c = t - r0 * rowdw;
        const uint32_t base = (uint32_t)((bx0 * CN) & ~3) + 4u * (uint32_t)c;
        const uint32_t lim = (uint32_t)sH * (uint32_t)j.spitch;
        if (r0 < per)
            for (int r = r0; r < bh; r += per) {
                const uint32_t off = (uint32_t)(by0 + r) * (uint32_t)j.spitch + base;
                uint32_t v;
                if (off + 4u <= lim || off >= lim) {
                    v = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
                } else {
                    v = 0;
                    for (uint32_t q = 0; q < 4u && off + q < lim; ++q) v |= (uint32_t)j.src[off + q] << (8u * q);
                }
                box[r * rowdw + c] = v;
            }
    }
    const bool live = y < H && x0 < W;
    const int n = live ? min(4, W - x0) : 0;
    int mx[4], my[4], mf[4];
    {
        uint32_t w4[4] = {0u, 0u, 0u, 0u};
        if (live) {
            const size_t mrow = (size_t)y * W + x0;
            if (n == 4 && (W & 3) == 0) {
                const uint4 m = *reinterpret_cast<const uint4*>(j.pmap + mrow);
                w4[0] = m.x; w4[1] = m.y; w4[2] = m.z; w4[3] = m.w;
            } else {
                for (int k = 0; k < 4; ++k) w4[k] = j.pmap[mrow + (k < n ? k : 0)];
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            mf[k] = (int)(w4[k] & 1023u);
            mx[k] = (int)((w4[k] >> 10) & 2047u) - 1;
            my[k] = (int)(w4[k] >> 21) - 1;
        }
    }
    __syncthreads();
    if (!live) return;
    // 2. each pixel whose four taps lie in the box reads its two rows' aligned dwords from LDS
    uint32_t u0[4][NWD], u1[4][NWD];
    uint32_t good = 0;
    const int bbase = (bx0 * CN) & ~3;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int sx = mx[k], sy = my[k];
        const bool in = rowdw && sx >= bx0 && sx + 1 <= bx1 && sy >= by0 && sy + 1 <= by1;
        good |= in ? 1u << k : 0u;
        const int r = in ? sy - by0 : 0;
        const int di = in ? r * rowdw + ((((sx * CN) & ~3) - bbase) >> 2) : 0;
#pragma unroll
        for (int i = 0; i < NWD; ++i) {
            u0[k][i] = box[di + i];
            u1[k][i] = box[di + rowdw + i];
        }
    }
    uint32_t out[4 * CN];
    remap_blend<CN>(j, sW, sH, mx, my, mf, u0, u1, good, out);
    uint8_t* d = j.dst + (size_t)y * j.dpitch + (size_t)x0 * CN;
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
        for (int q = 0; q < n * CN; ++q) d[q] = (uint8_t)out[q];
    }
}

usv_status launch_remap_tiled(const RemapJob& a, const RemapJob& b, const uint2* ba, const uint2* bb, int n_jobs,
                              int cn, int sW, int sH, int W, int H, hipStream_t s) {
    bool vec_dst = true;
    for (int i = 0; i < n_jobs; ++i) {
        const RemapJob& j = i ? b : a;
        vec_dst = vec_dst && aligned(j.dst, 4) && (j.dpitch % 4) == 0;
        if (!aligned(j.pmap, 16)) return USV_ERR_INVALID_ARG;
    }
    if ((long long)sH * a.spitch >= (1LL << 31) || (long long)sH * b.spitch >= (1LL << 31)) return USV_ERR_UNSUPPORTED;
    const int tiles_x = (W + kTileW - 1) / kTileW, tiles_y = (H + kTileH - 1) / kTileH;
    const unsigned per_job = (unsigned)tiles_x * (unsigned)tiles_y;
    dim3 grid(per_job * (unsigned)n_jobs), block(256);
    if (cn == 1)
        hipLaunchKernelGGL(remap_tile_kernel<1>, grid, block, 0, s, a, b, sW, sH, W, H, tiles_x, per_job, ba, bb,
                           (int)vec_dst);
    else if (cn == 3)
        hipLaunchKernelGGL(remap_tile_kernel<3>, grid, block, 0, s, a, b, sW, sH, W, H, tiles_x, per_job, ba, bb,
                           (int)vec_dst);
    else
        return USV_ERR_UNSUPPORTED;
    return hipGetLastError() == hipSuccess ? USV_OK : USV_ERR_HIP;
}

bool job_ok(const RemapJob& j, int cn, int sW, int W) {
    return j.src && (j.pmap || (j.map1 && j.map2)) && j.dst && j.spitch >= sW * cn && j.dpitch >= W * cn;
}
// the packed map only describes sources of at most kPackMaxSrc columns and rows
bool packed_ok(int sW, int sH) { return sW <= kPackMaxSrc && sH <= kPackMaxSrc; }

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

usv_status usv_remap_pack_map(const int16_t* map1, const uint16_t* map2, int W, int H, int sW, int sH, uint32_t* pmap,
                              void* stream) {
    if (!map1 || !map2 || !pmap || W <= 0 || H <= 0 || sW <= 0 || sH <= 0) return USV_ERR_INVALID_ARG;
    if (!usv::packed_ok(sW, sH)) return USV_ERR_UNSUPPORTED;
    const long long n = (long long)W * H;
    if ((n + 255) / 256 > 0x7FFFFFFFLL) return USV_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(usv::pack_map_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), map1, map2, n, sW, sH, pmap);
    return hipGetLastError() == hipSuccess ? USV_OK : USV_ERR_HIP;
}

usv_status usv_remap_packed_u8(const uint8_t* src, int sW, int sH, int spitch, int cn, const uint32_t* pmap, int W,
                               int H, uint8_t* dst, int dpitch, void* stream) {
    if (!pmap || sW <= 0 || sH <= 0 || W <= 0 || H <= 0 || H > 65535) return USV_ERR_INVALID_ARG;
    if (cn != 1 && cn != 3) return USV_ERR_UNSUPPORTED;
    if (!usv::packed_ok(sW, sH)) return USV_ERR_UNSUPPORTED;
    usv::RemapJob j{src, spitch, nullptr, nullptr, dst, dpitch, pmap};
    if (!usv::job_ok(j, cn, sW, W)) return USV_ERR_INVALID_ARG;
    return usv::launch_remap(j, j, 1, cn, sW, sH, W, H, static_cast<hipStream_t>(stream));
}

usv_status usv_rectify_pair_packed_u8(const uint8_t* srcL, const uint8_t* srcR, int sW, int sH, int spitch, int cn,
                                      const uint32_t* pmapL, const uint32_t* pmapR, int W, int H, uint8_t* dstL,
                                      uint8_t* dstR, int dpitch, void* stream) {
    if (!pmapL || !pmapR || sW <= 0 || sH <= 0 || W <= 0 || H <= 0 || H > 65535) return USV_ERR_INVALID_ARG;
    if (cn != 1 && cn != 3) return USV_ERR_UNSUPPORTED;
    if (!usv::packed_ok(sW, sH)) return USV_ERR_UNSUPPORTED;
    const usv::RemapJob a{srcL, spitch, nullptr, nullptr, dstL, dpitch, pmapL};
    const usv::RemapJob b{srcR, spitch, nullptr, nullptr, dstR, dpitch, pmapR};
    if (!usv::job_ok(a, cn, sW, W) || !usv::job_ok(b, cn, sW, W)) return USV_ERR_INVALID_ARG;
    return usv::launch_remap(a, b, 2, cn, sW, sH, W, H, static_cast<hipStream_t>(stream));
}

usv_status usv_remap_tile_boxes(const uint32_t* pmap, int W, int H, int sW, int sH, int cn, uint32_t* boxes,
                                void* stream) {
    if (!pmap || !boxes || W <= 0 || H <= 0 || sW <= 0 || sH <= 0) return USV_ERR_INVALID_ARG;
    if (cn != 1 && cn != 3) return USV_ERR_UNSUPPORTED;
    if (!usv::packed_ok(sW, sH) || H > 65535) return USV_ERR_UNSUPPORTED;
    const int tiles_x = (W + usv::kTileW - 1) / usv::kTileW, tiles_y = (H + usv::kTileH - 1) / usv::kTileH;
    hipLaunchKernelGGL(usv::tile_box_kernel, dim3((unsigned)(tiles_x * tiles_y)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), pmap, W, H, sW, sH, cn, tiles_x, reinterpret_cast<uint2*>(boxes));
    return hipGetLastError() == hipSuccess ? USV_OK : USV_ERR_HIP;
}

usv_status usv_remap_packed_tiled_u8(const uint8_t* src, int sW, int sH, int spitch, int cn, const uint32_t* pmap,
                                     const uint32_t* boxes, int W, int H, uint8_t* dst, int dpitch, void* stream) {
    if (!pmap || !boxes || sW <= 0 || sH <= 0 || W <= 0 || H <= 0 || H > 65535) return USV_ERR_INVALID_ARG;
    if (cn != 1 && cn != 3) return USV_ERR_UNSUPPORTED;
    if (!usv::packed_ok(sW, sH)) return USV_ERR_UNSUPPORTED;
    usv::RemapJob j{src, spitch, nullptr, nullptr, dst, dpitch, pmap};
    if (!usv::job_ok(j, cn, sW, W)) return USV_ERR_INVALID_ARG;
    const uint2* b = reinterpret_cast<const uint2*>(boxes);
    return usv::launch_remap_tiled(j, j, b, b, 1, cn, sW, sH, W, H, static_cast<hipStream_t>(stream));
}

usv_status usv_rectify_pair_packed_tiled_u8(const uint8_t* srcL, const uint8_t* srcR, int sW, int sH, int spitch,
                                            int cn, const uint32_t* pmapL, const uint32_t* pmapR,
                                            const uint32_t* boxesL, const uint32_t* boxesR, int W, int H,
                                            uint8_t* dstL, uint8_t* dstR, int dpitch, void* stream) {
    if (!pmapL || !pmapR || !boxesL || !boxesR || sW <= 0 || sH <= 0 || W <= 0 || H <= 0 || H > 65535)
        return USV_ERR_INVALID_ARG;
    if (cn != 1 && cn != 3) return USV_ERR_UNSUPPORTED;
    if (!usv::packed_ok(sW, sH)) return USV_ERR_UNSUPPORTED;
    const usv::RemapJob a{srcL, spitch, nullptr, nullptr, dstL, dpitch, pmapL};
    const usv::RemapJob b{srcR, spitch, nullptr, nullptr, dstR, dpitch, pmapR};
    if (!usv::job_ok(a, cn, sW, W) || !usv::job_ok(b, cn, sW, W)) return USV_ERR_INVALID_ARG;
    return usv::launch_remap_tiled(a, b, reinterpret_cast<const uint2*>(boxesL), reinterpret_cast<const uint2*>(boxesR),
                                   2, cn, sW, sH, W, H, static_cast<hipStream_t>(stream));
}

}  // extern "C"
