// usv_preproc.hip -- per-frame colour chain and masks on gfx950.
//
// What the reference runs on every rectified frame of each camera, OpenCV 3.0
// u8 semantics (restated in oracle/preproc_oracle.c, bit-exact here):
//   hsv_hist_kernel      BGR2HSV (P/Main.cpp:919) + the 256-bin histogram of V
//                        that equalizeHist needs (P/Main.cpp:368)
//   equalize_kernel      equalizeHist LUT (per block, from the histogram), V' =
//                        LUT[V] written back into the HSV image (merge through
//                        the shared Mat, P/Main.cpp:369), HSV2BGR (P/Main.cpp:370)
//                        and BGR2GRAY (P/Main.cpp:921) in one pass
//   v_hist_kernel +      usv_frame_prep_u8 / _pair_u8: the histogram of V = max(B,G,R) (reads only),
//   equalize_kernel<1>   then the pass above recomputing BGR2HSV from the frame (no HSV intermediate)
//   mask_kernel<MODE>    absdiff > 40 (ABSDiffSearch, P/Main.cpp:304-308) or two
//                        inRange + saturating add (ColourSearch, P/Main.cpp:322-324),
//                        then erode + dilate with the 5x5 ellipse
//                        (MorphilogicalFilter, P/Main.cpp:289-292), one LDS tile
// All three are HBM-bound byte streams: no MFMA, integer work
// except the HSV2BGR float path, which follows OpenCV's float operations in
// order (-ffp-contract=off).
#include <algorithm>

#include "usv.h"
#include "usv_colour.hpp"
#include "usv_kernels.hpp"
#include "usv_remap.hpp"

namespace usv {
namespace {

#ifndef USV_PREP_THREADS
#define USV_PREP_THREADS 256  // threads per block of the two frame-prep kernels (512 / 1024 ran slower)
#endif


// Work buffer (include/usv.h USV_FRAME_PREP_WORK_BYTES): per parity (the
// caller alternates it between frames) kHistCopies 256-bin histograms; block
// b adds into copy b % kHistCopies so each bin address takes 1/kHistCopies of
// the blocks' atomics (same-address atomics serialise at the memory side).
constexpr int kWHist = 0, kHistCopies = 8, kParityWords = 256 * kHistCopies;

// 4 interleaved BGR / HSV pixels = 12 bytes = one dwordx3 when the row and x
// are 4-pixel aligned; byte access otherwise.
struct Px4 { int c[12]; };
// Vector path: raw-buffer loads / stores over the image (32-bit offsets y * pitch + 3x, the dword index in
// no register at all) instead of a 64-bit address per quad; the host only sets `vec` when every
// pitch * H < 2^31.  Byte path: size_t pointer arithmetic.
typedef unsigned px_v3u __attribute__((ext_vector_type(3)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t px_rsrc(const uint8_t* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, (int)0xFFFFFFFF, 0x00020000);
}
__device__ __forceinline__ Px4 load_px4(const uint8_t* base, int pitch, int y, int x, bool vec, int n) {
    Px4 r;
    if (vec) {
        const px_v3u w = __builtin_amdgcn_raw_buffer_load_b96(px_rsrc(base), (uint32_t)(y * pitch + 3 * x), 0, 0);
        const uint32_t ww[3] = {w.x, w.y, w.z};
#pragma unroll
        for (int i = 0; i < 12; ++i) r.c[i] = (ww[i >> 2] >> (8 * (i & 3))) & 0xFF;
    } else {
        const uint8_t* p = base + (size_t)y * pitch + 3 * (size_t)x;
#pragma unroll
        for (int i = 0; i < 12; ++i) r.c[i] = i < 3 * n ? p[i] : 0;
    }
    return r;
}
__device__ __forceinline__ void store_px4(uint8_t* base, int pitch, int y, int x, const Px4& v, bool vec, int n) {
    if (vec) {
        px_v3u w;
        w.x = v.c[0] | (v.c[1] << 8) | (v.c[2] << 16) | ((uint32_t)v.c[3] << 24);
        w.y = v.c[4] | (v.c[5] << 8) | (v.c[6] << 16) | ((uint32_t)v.c[7] << 24);
        w.z = v.c[8] | (v.c[9] << 8) | (v.c[10] << 16) | ((uint32_t)v.c[11] << 24);
        __builtin_amdgcn_raw_buffer_store_b96(w, px_rsrc(base), (uint32_t)(y * pitch + 3 * x), 0, 0);
    } else {
        uint8_t* p = base + (size_t)y * pitch + 3 * (size_t)x;
#pragma unroll
        for (int i = 0; i < 12; ++i)  // static indices: a dynamic one would put the array in scratch
            if (i < 3 * n) p[i] = (uint8_t)v.c[i];
    }
}
// host: 32-bit buffer offsets cover every row of an image of H rows at this pitch
static bool fits32(int pitch, int H) { return (long long)pitch * H < (1LL << 31); }

// Pixels are processed as quads (4 interleaved pixels, one dwordx3) over the
// whole image as one flat range: quad q -> row q / nq, column 4 (q % nq).  A
// thread takes kU quads per sweep and issues all their loads before any
// compute, and the grid is sized to one sweep (~4 waves per SIMD at 1080p): the
// row-by-row form with a fixed 256-block grid ran latency-bound.  When W % 4 == 0 and the rows are 4-byte aligned
// every full sweep is straight-line vector code; the rest take a byte path.
#ifndef USV_PREP_KU
#define USV_PREP_KU 2  // quads per thread per sweep (all their loads issued before any compute)
#endif
constexpr int kU = USV_PREP_KU;
// The equalize pass that reads an HSV image (equalize_kernel<false>: the fused rectify + HSV chain and
// usv_equalize_hsv_bgr_gray_u8) runs faster at four quads per thread, the one that recomputes HSV from BGR at two
// (rocprof, three passes: 14.8-15.0 vs 15.6-16.1 us and 14.2-14.5 vs 13.6-13.8 us, profiles/probes_r06/ab_prep_ku_r06.txt).
#ifndef USV_PREP_KU_HSV
#define USV_PREP_KU_HSV 4
#endif
constexpr int kUHsv = USV_PREP_KU_HSV;
constexpr int kPT = USV_PREP_THREADS;  // threads per block (frame prep)
static_assert(kPT % 256 == 0 && kPT <= 1024, "whole 256-bin groups of threads");

// for_each_quad: body(y, x, n, vec, in) handles one quad, load(y, x, n, vec) -> Px4 reads it.  Block
// blk of nblk (a job's share of the grid) sweeps quads blk * kPT * kU + threadIdx.x + u * kPT; the
// first sweep's loads are issued BEFORE prologue() (the block's table / LUT set-up, which ends in a
// barrier every thread reaches), so the two latencies overlap instead of adding.
template <int kU = kU, typename LoadF, typename PrologueF, typename BodyF>
__device__ __forceinline__ void for_each_quad(int W, int H, bool vec4, int blk, int nblk, LoadF load,
                                              PrologueF prologue, BodyF body) {
    const int nq = (W + 3) >> 2;
    const int Q = nq * H;  // W * H <= 2^24
    const int stride = nblk * kPT * kU;
    int base = blk * kPT * kU + threadIdx.x;
    int y[kU], x[kU];
    Px4 in[kU];
    auto full = [&](int b) { return vec4 && b + (kU - 1) * kPT < Q; };
    auto issue = [&](int b) {
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const unsigned q = (unsigned)(b + u * kPT);
            y[u] = (int)quad_row(q, (unsigned)nq, quad_row_fast((unsigned)Q, (unsigned)nq));
            x[u] = 4 * (int)(q - (unsigned)y[u] * (unsigned)nq);
            in[u] = load(y[u], x[u], 4, true);
        }
    };
    if (full(base)) issue(base);
    prologue();
    for (bool first = true; base < Q; base += stride, first = false) {
        if (full(base)) {
            if (!first) issue(base);
#pragma unroll
            for (int u = 0; u < kU; ++u) body(y[u], x[u], 4, true, in[u]);
        } else {
            for (int u = 0; u < kU; ++u) {
                const int q = base + u * kPT;
                if (q >= Q) break;
                const int yy = q / nq, xx = 4 * (q - yy * nq), n = min(4, W - xx);
                const bool v = vec4 && n == 4;
                body(yy, xx, n, v, load(yy, xx, n, v));
            }
        }
    }
}

// BGR2HSV + histogram of V.  Each block accumulates its histogram in LDS and
// adds the occupied bins to histogram `parity` of the work buffer (no-return
// atomics); block 0 also clears histogram 1 - parity, which the previous
// frame used and the next one will fill.  (A single "last block" ticket to
// build the LUT here cost ~40 us: 512 returning atomics on one address.)
struct HistJob {
    const uint8_t* bgr;
    int pitch;
    uint8_t* hsv;
    int hsv_pitch;
    uint32_t* work;
};
__global__ __launch_bounds__(kPT) void hsv_hist_kernel(HistJob j0, HistJob j1, int W, int H, int parity,
                                                       int blocks_per_job, int vec) {
    constexpr int NWV = kPT / 64;
    const int job = (int)blockIdx.x >= blocks_per_job ? 1 : 0;
    const int blk = (int)blockIdx.x - job * blocks_per_job;
    const HistJob& j = job ? j1 : j0;
    const uint8_t* __restrict__ bgr = j.bgr;
    const int pitch = j.pitch, hsv_pitch = j.hsv_pitch;
    uint8_t* __restrict__ hsv = j.hsv;
    uint32_t* __restrict__ work = j.work;
    __shared__ int sdiv[256], hdiv[256];
    __shared__ uint32_t lh[NWV][256];  // one histogram per wave: its atomics never meet another wave's
    const int t = threadIdx.x, wv = t >> 6;
    const bool vec4 = vec && (W & 3) == 0;
    for_each_quad(
        W, H, vec4, blk, blocks_per_job,
        [&](int y, int x, int n, bool v) { return load_px4(bgr, pitch, y, x, v, n); },
        [&] {
            hsv_tables(sdiv, hdiv);
            for (int i = t; i < NWV * 256; i += kPT) (&lh[0][0])[i] = 0;
            if (blk == 0 && t < 256)
                for (int c = 0; c < kHistCopies; ++c) work[kWHist + kParityWords * (1 - parity) + 256 * c + t] = 0;
            __syncthreads();
        },
        [&](int y, int x, int n, bool v, const Px4& in) {
            Px4 out;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                int h, sat, val;
                bgr2hsv_px(in.c[3 * k], in.c[3 * k + 1], in.c[3 * k + 2], sdiv, hdiv, h, sat, val);
                out.c[3 * k] = h;
                out.c[3 * k + 1] = sat;
                out.c[3 * k + 2] = val;
                if (k < n) atomicAdd(&lh[wv][val], 1u);
            }
            store_px4(hsv, hsv_pitch, y, x, out, v, n);
        });
    __syncthreads();
    if (t < 256) {
        uint32_t sum = 0;
#pragma unroll
        for (int w = 0; w < NWV; ++w) sum += lh[w][t];
        if (sum)
            atomicAdd(&work[kWHist + kParityWords * parity + 256 * (blk % kHistCopies) + t], sum);
    }
}

// Quads per thread of the V-histogram pass.  A stand-alone probe of the pass at 1080p (scripts/probes/hist_probe.hip,
// profiles/probes_r05/hist_probe_r05.txt) ran 4.38 us at two quads per thread, 3.68 at four, 3.94 at eight,
// with a no-histogram floor of 3.37 us at four: the LDS atomics are not what binds it, and interleaving copies
// over the banks (32 or 64 per block) was slower.  In the product kernel four quads per thread measured slower
// than two (rocprof 8.3 vs 6.3 us average, 5.9 vs 4.1 us minimum, profiles/r05e vs r05a), so two it stays.
#ifndef USV_HIST_KU
#define USV_HIST_KU 2
#endif
constexpr int kUHist = USV_HIST_KU;

// Histogram of V = max(B, G, R) only (RGB2HSV_b's v; P/Main.cpp:368 equalizes that channel): the
// first pass of usv_frame_prep_u8 / _pair_u8, which reads the frame and writes nothing but the
// workspace histograms (per-wave LDS copies, one global add per occupied bin and block, the other
// parity cleared by block 0, as hsv_hist_kernel).
__global__ __launch_bounds__(kPT) void v_hist_kernel(HistJob j0, HistJob j1, int W, int H, int parity,
                                                     int blocks_per_job, int vec) {
    constexpr int NWV = kPT / 64;
    const int job = (int)blockIdx.x >= blocks_per_job ? 1 : 0;
    const int blk = (int)blockIdx.x - job * blocks_per_job;
    const HistJob& j = job ? j1 : j0;
    uint32_t* __restrict__ work = j.work;
    __shared__ uint32_t lh[NWV][256];
    const int t = threadIdx.x, wv = t >> 6;
    const bool vec4 = vec && (W & 3) == 0;
    for_each_quad<kUHist>(
        W, H, vec4, blk, blocks_per_job,
        [&](int y, int x, int n, bool v) { return load_px4(j.bgr, j.pitch, y, x, v, n); },
        [&] {
            for (int i = t; i < NWV * 256; i += kPT) (&lh[0][0])[i] = 0;
            if (blk == 0 && t < 256)
                for (int c = 0; c < kHistCopies; ++c) work[kWHist + kParityWords * (1 - parity) + 256 * c + t] = 0;
            __syncthreads();
        },
        [&](int, int, int n, bool, const Px4& in) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (k < n) atomicAdd(&lh[wv][max(max(in.c[3 * k], in.c[3 * k + 1]), in.c[3 * k + 2])], 1u);
        });
    __syncthreads();
    if (t < 256) {
        uint32_t sum = 0;
#pragma unroll
        for (int w = 0; w < NWV; ++w) sum += lh[w][t];
        if (sum) atomicAdd(&work[kWHist + kParityWords * parity + 256 * (blk % kHistCopies) + t], sum);
    }
}

// One camera's equalize pass: the histogram it reads and the images it rewrites.
struct EqJob {
    const uint32_t* work;
    uint8_t* hsv;
    int hsv_pitch;
    uint8_t* bgr;
    int bgr_pitch;
    uint8_t* gray;
    int gray_pitch;
    const uint8_t* src = nullptr;  // FROM_BGR: the BGR frame HSV is recomputed from (hsv is output only)
    int src_pitch = 0;
};

// V' = LUT[V] written back into hsv, HSV2BGR, BGR2GRAY; kU quads per thread.  Blocks
// [0, blocks_per_job) take job j0, the rest j1 (both cameras of a pair in one launch).  The
// equalizeHist LUT comes from the job's complete histogram, built by the block's first 256 threads
// while the first sweep's pixel loads are in flight: an inclusive scan within each wave by shuffles
// plus the four wave totals, then OpenCV's float scale and cvRound.
// FROM_BGR (usv_frame_prep_u8 / _pair_u8): the pass reads the BGR frame instead of an HSV image and
// recomputes BGR2HSV (the same integer tables as hsv_hist_kernel), so the first pass only has to
// histogram V = max(B, G, R) (v_hist_kernel) and no HSV intermediate crosses HBM: 13 B per pixel
// instead of 16, outputs bit-identical.
template <bool FROM_BGR>
__global__ __launch_bounds__(kPT) void equalize_kernel(EqJob j0, EqJob j1, int parity, int W, int H,
                                                       int blocks_per_job, int vec) {
    __shared__ int sdiv[FROM_BGR ? 256 : 1], hdiv[FROM_BGR ? 256 : 1];
    __shared__ int scan[256];
    __shared__ int first;
    __shared__ uint8_t lut[256];
    __shared__ int wsum[4], wfirst[4];
    const int job = (int)blockIdx.x >= blocks_per_job ? 1 : 0;
    const EqJob& j = job ? j1 : j0;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    auto build_lut = [&] {
        if constexpr (FROM_BGR) hsv_tables(sdiv, hdiv);  // (read after the barriers below)
        int x = 0;
        if (t < 256) {
            int hv = 0;
#pragma unroll
            for (int c = 0; c < kHistCopies; ++c) hv += (int)j.work[kWHist + kParityWords * parity + 256 * c + t];
            x = hv;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int y = __shfl_up(x, off, 64);
                if (lane >= off) x += y;
            }
            const unsigned long long nz = __ballot(hv != 0);
            if (lane == 63) wsum[wv] = x;
            if (lane == 0) wfirst[wv] = nz ? 64 * wv + __ffsll((long long)nz) - 1 : 256;
        }
        __syncthreads();
        if (t < 256) {
            for (int k = 0; k < wv; ++k) x += wsum[k];
            scan[t] = x;
            if (t == 0) first = min(min(wfirst[0], wfirst[1]), min(wfirst[2], wfirst[3]));
        }
        __syncthreads();
        if (t < 256) {
            const int total = W * H, i0 = first;
            int lv = 0;
            if (i0 < 256) {
                const int h0 = scan[i0] - (i0 ? scan[i0 - 1] : 0);
                if (h0 == total) {
                    lv = t == i0 ? i0 : 0;  // dst.setTo(i0)
                } else if (t > i0) {
                    const float scale = (256 - 1.f) / (total - h0);
                    const int acc = scan[t] - scan[i0];  // hist[i0 + 1 .. t]
                    lv = min(max(__float2int_rn(acc * scale), 0), 255);
                }
            }
            lut[t] = (uint8_t)lv;
        }
        __syncthreads();
    };
    const bool vec4 = vec && (W & 3) == 0;
    for_each_quad<FROM_BGR ? kU : kUHsv>(
        W, H, vec4, (int)blockIdx.x - job * blocks_per_job, blocks_per_job,
        [&](int y, int x, int n, bool v) {
            if constexpr (FROM_BGR) return load_px4(j.src, j.src_pitch, y, x, v, n);
            else return load_px4(j.hsv, j.hsv_pitch, y, x, v, n);
        },
        build_lut,
        [&](int y, int x, int n, bool v, Px4 in) {
            Px4 o;
            uint32_t g4 = 0;
            if constexpr (FROM_BGR) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    int h, sat, val;
                    bgr2hsv_px(in.c[3 * k], in.c[3 * k + 1], in.c[3 * k + 2], sdiv, hdiv, h, sat, val);
                    in.c[3 * k] = h;
                    in.c[3 * k + 1] = sat;
                    in.c[3 * k + 2] = val;
                }
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                in.c[3 * k + 2] = lut[in.c[3 * k + 2]];
                int b, g, r;
                hsv2bgr_px(in.c[3 * k], in.c[3 * k + 1], in.c[3 * k + 2], b, g, r);
                o.c[3 * k] = b;
                o.c[3 * k + 1] = g;
                o.c[3 * k + 2] = r;
                g4 |= (uint32_t)((b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14) << (8 * k);
            }
            store_px4(j.hsv, j.hsv_pitch, y, x, in, v, n);
            store_px4(j.bgr, j.bgr_pitch, y, x, o, v, n);
            uint8_t* go = j.gray + (size_t)y * j.gray_pitch + x;
            if (v) *reinterpret_cast<uint32_t*>(go) = g4;
            else for (int k = 0; k < n; ++k) go[k] = (uint8_t)(g4 >> (8 * k));
        });
}

// Fused first half of the per-frame chain for BOTH cameras (P/Main.cpp:913-919): rectify
// (remap_quad: initUndistortRectifyMap map + remap INTER_LINEAR, P/Main.cpp:351-359), BGR2HSV and
// the histogram of V, without writing the rectified BGR image the reference overwrites anyway
// (LightingCorrection writes its HSV2BGR result back into CalibratedImg, P/Main.cpp:370).  One quad
// per thread per iteration over the job's quads; per-wave LDS histograms, one global add per bin
// and block into copy blockIdx % kHistCopies of the job's workspace (as hsv_hist_kernel).
struct RectPrepJob {
    RemapJob r;  // r.dst / r.dpitch: the HSV image
    uint32_t* work;
};
template <bool PK>
__global__ __launch_bounds__(256) void rectify_hsv_hist_kernel(RectPrepJob j0, RectPrepJob j1, int sW, int sH, int W,
                                                               int H, int blocks_per_job, int vec_map, int vec_src,
                                                               int vec_dst, int parity) {
    __shared__ int sdiv[256], hdiv[256];
    __shared__ uint32_t lh[4][256];
    const unsigned lb = xcd_block(blockIdx.x, gridDim.x);
    const int job = (int)lb >= blocks_per_job ? 1 : 0;
    const RectPrepJob& j = job ? j1 : j0;
    const int blk = (int)lb - job * blocks_per_job;
    const int t = threadIdx.x, wv = t >> 6;
    const int nq = (W + 3) >> 2, Q = nq * H;
    hsv_tables(sdiv, hdiv);
    for (int i = t; i < 4 * 256; i += 256) (&lh[0][0])[i] = 0;
    if (blk == 0)
        for (int c = 0; c < kHistCopies; ++c) j.work[kWHist + kParityWords * (1 - parity) + 256 * c + t] = 0;
    __syncthreads();
    const bool fastq = quad_row_fast((unsigned)Q, (unsigned)nq);
    for (int q = blk * 256 + t; q < Q; q += blocks_per_job * 256) {
        const int y = (int)quad_row((unsigned)q, (unsigned)nq, fastq), x0 = 4 * (q - y * nq), n = min(4, W - x0);
        uint32_t px[12];
        remap_quad<3, PK>(j.r, sW, sH, W, y, x0, n, vec_map, vec_src, px);
        Px4 out;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            int h, sat, val;
            bgr2hsv_px((int)px[3 * k], (int)px[3 * k + 1], (int)px[3 * k + 2], sdiv, hdiv, h, sat, val);
            out.c[3 * k] = h;
            out.c[3 * k + 1] = sat;
            out.c[3 * k + 2] = val;
            if (k < n) atomicAdd(&lh[wv][val], 1u);
        }
        store_px4(j.r.dst, j.r.dpitch, y, x0, out, vec_dst && n == 4, n);
    }
    __syncthreads();
    const uint32_t sum = lh[0][t] + lh[1][t] + lh[2][t] + lh[3][t];
    if (sum) atomicAdd(&j.work[kWHist + kParityWords * parity + 256 * (blockIdx.x % kHistCopies) + t], sum);
}

// ---- masks: threshold / inRange, then erode + dilate (5x5 ellipse) in one tile ----
// Mask pixels are 0 or 255, so min / max are AND / OR and four pixels packed
// in a u32 are processed at once; a shift by k pixels is v_alignbyte over the
// neighbouring word.  The ellipse is rows -2 and +2 (centre only) and rows
// -1..1 (five wide): E = T[-2] & T[+2] & h5(T[-1]) & h5(T[0]) & h5(T[+1]).
#ifndef USV_MASK_TW
#define USV_MASK_TW 64  // output tile width (pixels, multiple of 4); 64 x 16 measured best (profiles/probes_r06/ab_mask_r06.txt)
#endif
#ifndef USV_MASK_TH
#define USV_MASK_TH 16  // output tile height (rows)
#endif
constexpr int kTW = USV_MASK_TW, kTH = USV_MASK_TH;       // output tile (pixels)
constexpr int kR = 2;                                    // ellipse radius
constexpr int kIH = kTH + 4 * kR, kIWW = (kTW + 8 * kR) / 4 + 0;  // input tile rows, words (4 px halo each side -> 80 px = 20 words)
constexpr int kEH = kTH + 2 * kR, kEWW = kIWW - 2;      // eroded tile: 20 rows x 18 words (x0 - 4 .. x0 + 67)
constexpr int kOWW = kTW / 4;                            // 16 output words per row
constexpr int kMT = kTH * kOWW < 256 ? kTH * kOWW : 256;  // threads per tile: one output word each, at most 256

struct MaskArgs {
    const uint8_t* a;  // gray (motion) or hsv (colour)
    const uint8_t* b;  // prev gray (motion)
    int W, H, pitch;
    int thresh;
    int lo1[3], hi1[3], lo2[3], hi2[3];
    uint8_t* mask;
    int mask_pitch;
};

__device__ __forceinline__ uint32_t shl_px(uint32_t lo, uint32_t hi, int k) {  // pixels x + k, k = 1..3
    return __builtin_amdgcn_alignbyte(hi, lo, k);
}
template <bool AND>
__device__ __forceinline__ uint32_t h5(const uint32_t* row, int j) {  // 5-wide AND / OR around word j
    const uint32_t l = row[j - 1], c = row[j], r = row[j + 1];
    const uint32_t m2 = __builtin_amdgcn_alignbyte(c, l, 2), m1 = __builtin_amdgcn_alignbyte(c, l, 3);
    const uint32_t p1 = shl_px(c, r, 1), p2 = shl_px(c, r, 2);
    return AND ? (c & m1 & m2 & p1 & p2) : (c | m1 | m2 | p1 | p2);
}

template <int MODE>  // 0: motion (absdiff > thresh), 1: colour (two inRange, saturating add)
__device__ __forceinline__ int mask_px(const MaskArgs& m, int y, int x) {
    if constexpr (MODE == 0) {
        const int p = m.a[(size_t)y * m.pitch + x], q = m.b[(size_t)y * m.pitch + x];
        return (p > q ? p - q : q - p) > m.thresh ? 255 : 0;
    } else {
        const uint8_t* s = m.a + (size_t)y * m.pitch + 3 * x;
        bool in1 = true, in2 = true;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            in1 = in1 && s[c] >= m.lo1[c] && s[c] <= m.hi1[c];
            in2 = in2 && s[c] >= m.lo2[c] && s[c] <= m.hi2[c];
        }
        return (in1 || in2) ? 255 : 0;
    }
}

template <int MODE>
__global__ __launch_bounds__(kMT) void mask_kernel(MaskArgs m, int vec) {
    __shared__ uint32_t T[kIH][kIWW];  // x0 - 8 .. x0 + 71
    __shared__ uint32_t E[kEH][kEWW];  // word e covers x0 - 4 + 4e
    const int X0 = blockIdx.x * kTW, Y0 = blockIdx.y * kTH;
    // thresholded input, rows Y0-4 .. Y0+19, words x0-8 .. x0+71; outside the image = 255 (never wins the min)
    for (int i = threadIdx.x; i < kIH * kIWW; i += kMT) {
        const int ty = i / kIWW, tw = i - ty * kIWW;
        const int y = Y0 - 2 * kR + ty, x = X0 - 8 + 4 * tw;
        uint32_t w = 0xFFFFFFFFu;
        if (y >= 0 && y < m.H) {
            if (MODE == 0 && vec && x >= 0 && x + 4 <= m.W) {
                const uint32_t p = *reinterpret_cast<const uint32_t*>(m.a + (size_t)y * m.pitch + x);
                const uint32_t q = *reinterpret_cast<const uint32_t*>(m.b + (size_t)y * m.pitch + x);
                w = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int a = (p >> (8 * k)) & 0xFF, b = (q >> (8 * k)) & 0xFF;
                    w |= (uint32_t)((a > b ? a - b : b - a) > m.thresh ? 255 : 0) << (8 * k);
                }
            } else {
                w = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int xx = x + k;
                    const int v = (xx >= 0 && xx < m.W) ? mask_px<MODE>(m, y, xx) : 255;
                    w |= (uint32_t)v << (8 * k);
                }
            }
        }
        T[ty][tw] = w;
    }
    __syncthreads();
    // erode, rows Y0-2 .. Y0+17, words x0-4 .. x0+67; outside the image = 0 (never wins the max)
    for (int i = threadIdx.x; i < kEH * kEWW; i += kMT) {
        const int ey = i / kEWW, ew = i - ey * kEWW;
        const int y = Y0 - kR + ey, x = X0 - 4 + 4 * ew;
        const int tw = ew + 1, ty = ey + kR;
        uint32_t e = T[ty - 2][tw] & T[ty + 2][tw] & h5<true>(T[ty - 1], tw) & h5<true>(T[ty], tw) &
                     h5<true>(T[ty + 1], tw);
        if (y < 0 || y >= m.H) e = 0;
        else if (x < 0 || x + 4 > m.W) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (x + k < 0 || x + k >= m.W) e &= ~(0xFFu << (8 * k));
        }
        E[ey][ew] = e;
    }
    __syncthreads();
    // dilate, one output word (4 pixels) per thread and pass
    static_assert((kTH * kOWW) % kMT == 0, "whole passes of output words");
#pragma unroll
    for (int i = threadIdx.x; i < kTH * kOWW; i += kMT) {
        const int oy = i / kOWW, ow = i - oy * kOWW;
        const int y = Y0 + oy, x = X0 + 4 * ow;
        const int ew = ow + 1, ey = oy + kR;
        const uint32_t d = E[ey - 2][ew] | E[ey + 2][ew] | h5<false>(E[ey - 1], ew) | h5<false>(E[ey], ew) |
                           h5<false>(E[ey + 1], ew);
        if (y < m.H && x < m.W) {
            uint8_t* o = m.mask + (size_t)y * m.mask_pitch + x;
            if (vec && x + 4 <= m.W) *reinterpret_cast<uint32_t*>(o) = d;
            else for (int k = 0; k < 4 && x + k < m.W; ++k) o[k] = (uint8_t)(d >> (8 * k));
        }
    }
}


// one sweep of ku quads per thread, at most 4096 blocks (larger frames loop)
int prep_blocks(int W, int H, int ku = kU) {
    const long long q = (long long)((W + 3) / 4) * H, per = (long long)kPT * ku;
    return (int)std::min<long long>(4096, std::max<long long>(1, (q + per - 1) / per));
}

usv_status st(hipError_t e) { return e == hipSuccess ? USV_OK : USV_ERR_HIP; }

}  // namespace
}  // namespace usv

extern "C" {

static bool al4(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 3) == 0; }

usv_status usv_bgr2hsv_hist_u8(const uint8_t* bgr, int W, int H, int pitch, uint8_t* hsv, int hsv_pitch,
                               void* work, int parity, void* stream) {
    if (!bgr || !hsv || !work || W <= 0 || H <= 0 || pitch < 3 * W || hsv_pitch < 3 * W ||
        (long long)W * H > (1LL << 24) || !al4(work) || (parity != 0 && parity != 1))
        return USV_ERR_INVALID_ARG;
    const int vec = al4(bgr) && al4(hsv) && pitch % 4 == 0 && hsv_pitch % 4 == 0 && usv::fits32(pitch, H) &&
                    usv::fits32(hsv_pitch, H);
    const usv::HistJob j{bgr, pitch, hsv, hsv_pitch, static_cast<uint32_t*>(work)};
    const int nb = usv::prep_blocks(W, H);
    hipLaunchKernelGGL(usv::hsv_hist_kernel, dim3(nb), dim3(usv::kPT), 0, static_cast<hipStream_t>(stream), j, j, W, H,
                       parity, nb, vec);
    return usv::st(hipGetLastError());
}

usv_status usv_equalize_hsv_bgr_gray_u8(const void* work, int parity, uint8_t* hsv, int W, int H, int hsv_pitch,
                                        uint8_t* bgr_out, int bgr_pitch, uint8_t* gray, int gray_pitch,
                                        void* stream) {
    if (!work || !hsv || !bgr_out || !gray || W <= 0 || H <= 0 || hsv_pitch < 3 * W || bgr_pitch < 3 * W ||
        gray_pitch < W || !al4(work) || (parity != 0 && parity != 1) || (long long)W * H > (1LL << 24))
        return USV_ERR_INVALID_ARG;
    const int vec = al4(hsv) && al4(bgr_out) && al4(gray) && hsv_pitch % 4 == 0 && bgr_pitch % 4 == 0 &&
                    gray_pitch % 4 == 0 && usv::fits32(hsv_pitch, H) && usv::fits32(bgr_pitch, H);
    const usv::EqJob j{static_cast<const uint32_t*>(work), hsv, hsv_pitch, bgr_out, bgr_pitch, gray, gray_pitch};
    const int nb = usv::prep_blocks(W, H, usv::kUHsv);
    hipLaunchKernelGGL(usv::equalize_kernel<false>, dim3(nb), dim3(usv::kPT), 0, static_cast<hipStream_t>(stream), j, j,
                       parity, W, H, nb, vec);
    return usv::st(hipGetLastError());
}

usv_status usv_frame_prep_u8(const uint8_t* bgr, int W, int H, int pitch, uint8_t* hsv, int hsv_pitch,
                             uint8_t* bgr_out, int bgr_pitch, uint8_t* gray, int gray_pitch, void* work,
                             int parity, void* stream) {
    // V histogram (reads only), then BGR2HSV + equalize + HSV2BGR + gray from the BGR frame
    if (!bgr || !hsv || !bgr_out || !gray || !work || W <= 0 || H <= 0 || pitch < 3 * W || hsv_pitch < 3 * W ||
        bgr_pitch < 3 * W || gray_pitch < W || !al4(work) || (parity != 0 && parity != 1) ||
        (long long)W * H > (1LL << 24))
        return USV_ERR_INVALID_ARG;
    const int vh = al4(bgr) && pitch % 4 == 0 && usv::fits32(pitch, H);
    const int ve = vh && al4(hsv) && al4(bgr_out) && al4(gray) && hsv_pitch % 4 == 0 && bgr_pitch % 4 == 0 &&
                   gray_pitch % 4 == 0 && usv::fits32(hsv_pitch, H) && usv::fits32(bgr_pitch, H);
    const usv::HistJob hj{bgr, pitch, nullptr, 0, static_cast<uint32_t*>(work)};
    const int nb = usv::prep_blocks(W, H), nbh = usv::prep_blocks(W, H, usv::kUHist);
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(usv::v_hist_kernel, dim3(nbh), dim3(usv::kPT), 0, s, hj, hj, W, H, parity, nbh, vh);
    if (hipGetLastError() != hipSuccess) return USV_ERR_HIP;
    const usv::EqJob ej{static_cast<const uint32_t*>(work), hsv, hsv_pitch, bgr_out, bgr_pitch, gray, gray_pitch,
                        bgr, pitch};
    hipLaunchKernelGGL(usv::equalize_kernel<true>, dim3(nb), dim3(usv::kPT), 0, s, ej, ej, parity, W, H, nb, ve);
    return usv::st(hipGetLastError());
}

usv_status usv_frame_prep_pair_u8(const uint8_t* bgrL, const uint8_t* bgrR, int W, int H, int pitch, uint8_t* hsvL,
                                  uint8_t* hsvR, int hsv_pitch, uint8_t* bgr_outL, uint8_t* bgr_outR, int bgr_pitch,
                                  uint8_t* grayL, uint8_t* grayR, int gray_pitch, void* work, int parity,
                                  void* stream) {
    if (!bgrL || !bgrR || !hsvL || !hsvR || !bgr_outL || !bgr_outR || !grayL || !grayR || !work || W <= 0 ||
        H <= 0 || pitch < 3 * W || hsv_pitch < 3 * W || bgr_pitch < 3 * W || gray_pitch < W || !al4(work) ||
        (parity != 0 && parity != 1) || (long long)W * H > (1LL << 24))
        return USV_ERR_INVALID_ARG;
    uint32_t* wL = static_cast<uint32_t*>(work);
    uint32_t* wR = wL + USV_FRAME_PREP_WORK_BYTES / 4;
    // V histograms (reads only), then BGR2HSV + equalize + HSV2BGR + gray from the BGR frames
    const int vh = al4(bgrL) && al4(bgrR) && pitch % 4 == 0 && usv::fits32(pitch, H);
    const int ve = vh && al4(hsvL) && al4(hsvR) && al4(bgr_outL) && al4(bgr_outR) && al4(grayL) && al4(grayR) &&
                   hsv_pitch % 4 == 0 && bgr_pitch % 4 == 0 && gray_pitch % 4 == 0 && usv::fits32(hsv_pitch, H) &&
                   usv::fits32(bgr_pitch, H);
    const int nb = usv::prep_blocks(W, H), nbh = usv::prep_blocks(W, H, usv::kUHist);
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(usv::v_hist_kernel, dim3(2 * nbh), dim3(usv::kPT), 0, s, usv::HistJob{bgrL, pitch, nullptr, 0, wL},
                       usv::HistJob{bgrR, pitch, nullptr, 0, wR}, W, H, parity, nbh, vh);
    if (hipGetLastError() != hipSuccess) return USV_ERR_HIP;
    hipLaunchKernelGGL(usv::equalize_kernel<true>, dim3(2 * nb), dim3(usv::kPT), 0, s,
                       usv::EqJob{wL, hsvL, hsv_pitch, bgr_outL, bgr_pitch, grayL, gray_pitch, bgrL, pitch},
                       usv::EqJob{wR, hsvR, hsv_pitch, bgr_outR, bgr_pitch, grayR, gray_pitch, bgrR, pitch}, parity, W, H,
                       nb, ve);
    return usv::st(hipGetLastError());
}

// usv_rectify_prep_pair_u8 / _packed_u8: jl.r / jr.r carry either map1 + map2 or pmap.
static usv_status rectify_prep_pair(const usv::RemapJob& jl_r, const usv::RemapJob& jr_r, int sW, int sH, int W, int H,
                                    uint8_t* bgr_outL, uint8_t* bgr_outR, int bgr_pitch, uint8_t* grayL,
                                    uint8_t* grayR, int gray_pitch, void* work, int parity, void* stream) {
    const int spitch = jl_r.spitch, hsv_pitch = jl_r.dpitch;
    uint8_t* hsvL = jl_r.dst;
    uint8_t* hsvR = jr_r.dst;
    if (!jl_r.src || !jr_r.src || !hsvL || !hsvR || !bgr_outL || !bgr_outR || !grayL || !grayR || !work || sW <= 0 ||
        sH <= 0 || W <= 0 || H <= 0 || spitch < 3 * sW || hsv_pitch < 3 * W || bgr_pitch < 3 * W || gray_pitch < W ||
        !al4(work) || (parity != 0 && parity != 1) || (long long)W * H > (1LL << 24))
        return USV_ERR_INVALID_ARG;
    if ((long long)(sH + 1) * spitch >= (1LL << 32) || spitch >= (1 << 24)) return USV_ERR_UNSUPPORTED;
    const bool pk = jl_r.pmap != nullptr;
    if (pk && (sW > usv::kPackMaxSrc || sH > usv::kPackMaxSrc)) return USV_ERR_UNSUPPORTED;
    uint32_t* wL = static_cast<uint32_t*>(work);
    uint32_t* wR = wL + USV_FRAME_PREP_WORK_BYTES / 4;
    auto al = [](const void* p, size_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; };
    const int vec_map = (W % 4) == 0 && (pk ? al(jl_r.pmap, 16) && al(jr_r.pmap, 16)
                                            : al(jl_r.map1, 16) && al(jr_r.map1, 16) && al(jl_r.map2, 8) &&
                                                  al(jr_r.map2, 8));
    const int vec_src = al4(jl_r.src) && al4(jr_r.src) && spitch % 4 == 0 && spitch >= 12;
    const int vec_hsv = al4(hsvL) && al4(hsvR) && hsv_pitch % 4 == 0 && usv::fits32(hsv_pitch, H);
    const int ve = vec_hsv && al4(bgr_outL) && al4(bgr_outR) && al4(grayL) && al4(grayR) && bgr_pitch % 4 == 0 &&
                   gray_pitch % 4 == 0 && usv::fits32(bgr_pitch, H);
    // rectify + HSV + histogram: a quad per thread per iteration, ~4 quads per thread at 1080p
    const long long quads = (long long)((W + 3) / 4) * H;
    const int per_job = (int)std::max<long long>(1, std::min<long long>(1024, (quads + 1023) / 1024));
    hipStream_t s = static_cast<hipStream_t>(stream);
    const usv::RectPrepJob jl{jl_r, wL};
    const usv::RectPrepJob jr{jr_r, wR};
    if (pk)
        hipLaunchKernelGGL(usv::rectify_hsv_hist_kernel<true>, dim3(2 * per_job), dim3(256), 0, s, jl, jr, sW, sH, W, H,
                           per_job, vec_map, vec_src, vec_hsv, parity);
    else
        hipLaunchKernelGGL(usv::rectify_hsv_hist_kernel<false>, dim3(2 * per_job), dim3(256), 0, s, jl, jr, sW, sH, W,
                           H, per_job, vec_map, vec_src, vec_hsv, parity);
    if (hipGetLastError() != hipSuccess) return USV_ERR_HIP;
    const int nb = usv::prep_blocks(W, H, usv::kUHsv);
    hipLaunchKernelGGL(usv::equalize_kernel<false>, dim3(2 * nb), dim3(usv::kPT), 0, s,
                       usv::EqJob{wL, hsvL, hsv_pitch, bgr_outL, bgr_pitch, grayL, gray_pitch},
                       usv::EqJob{wR, hsvR, hsv_pitch, bgr_outR, bgr_pitch, grayR, gray_pitch}, parity, W, H, nb, ve);
    return usv::st(hipGetLastError());
}

usv_status usv_rectify_prep_pair_u8(const uint8_t* srcL, const uint8_t* srcR, int sW, int sH, int spitch,
                                    const int16_t* map1L, const uint16_t* map2L, const int16_t* map1R,
                                    const uint16_t* map2R, int W, int H, uint8_t* hsvL, uint8_t* hsvR, int hsv_pitch,
                                    uint8_t* bgr_outL, uint8_t* bgr_outR, int bgr_pitch, uint8_t* grayL,
                                    uint8_t* grayR, int gray_pitch, void* work, int parity, void* stream) {
    if (!map1L || !map2L || !map1R || !map2R) return USV_ERR_INVALID_ARG;
    return rectify_prep_pair(usv::RemapJob{srcL, spitch, map1L, map2L, hsvL, hsv_pitch},
                             usv::RemapJob{srcR, spitch, map1R, map2R, hsvR, hsv_pitch}, sW, sH, W, H, bgr_outL,
                             bgr_outR, bgr_pitch, grayL, grayR, gray_pitch, work, parity, stream);
}

usv_status usv_rectify_prep_pair_packed_u8(const uint8_t* srcL, const uint8_t* srcR, int sW, int sH, int spitch,
                                           const uint32_t* pmapL, const uint32_t* pmapR, int W, int H, uint8_t* hsvL,
                                           uint8_t* hsvR, int hsv_pitch, uint8_t* bgr_outL, uint8_t* bgr_outR,
                                           int bgr_pitch, uint8_t* grayL, uint8_t* grayR, int gray_pitch, void* work,
                                           int parity, void* stream) {
    if (!pmapL || !pmapR) return USV_ERR_INVALID_ARG;
    return rectify_prep_pair(usv::RemapJob{srcL, spitch, nullptr, nullptr, hsvL, hsv_pitch, pmapL},
                             usv::RemapJob{srcR, spitch, nullptr, nullptr, hsvR, hsv_pitch, pmapR}, sW, sH, W, H,
                             bgr_outL, bgr_outR, bgr_pitch, grayL, grayR, gray_pitch, work, parity, stream);
}

usv_status usv_motion_mask_u8(const uint8_t* gray, const uint8_t* prev, int W, int H, int pitch, int thresh,
                              uint8_t* mask, int mask_pitch, void* stream) {
    if (!gray || !prev || !mask || W <= 0 || H <= 0 || pitch < W || mask_pitch < W) return USV_ERR_INVALID_ARG;
    usv::MaskArgs m{};
    m.a = gray; m.b = prev; m.W = W; m.H = H; m.pitch = pitch; m.thresh = thresh;
    m.mask = mask; m.mask_pitch = mask_pitch;
    dim3 grid((unsigned)((W + usv::kTW - 1) / usv::kTW), (unsigned)((H + usv::kTH - 1) / usv::kTH));
    const int vec = al4(gray) && al4(prev) && al4(mask) && pitch % 4 == 0 && mask_pitch % 4 == 0;
    hipLaunchKernelGGL(usv::mask_kernel<0>, grid, dim3(usv::kMT), 0, static_cast<hipStream_t>(stream), m, vec);
    return usv::st(hipGetLastError());
}

usv_status usv_colour_mask_u8(const uint8_t* hsv, int W, int H, int pitch, const int* lo1, const int* hi1,
                              const int* lo2, const int* hi2, uint8_t* mask, int mask_pitch, void* stream) {
    if (!hsv || !lo1 || !hi1 || !lo2 || !hi2 || !mask || W <= 0 || H <= 0 || pitch < 3 * W || mask_pitch < W)
        return USV_ERR_INVALID_ARG;
    usv::MaskArgs m{};
    m.a = hsv; m.W = W; m.H = H; m.pitch = pitch;
    for (int c = 0; c < 3; ++c) {
        m.lo1[c] = lo1[c]; m.hi1[c] = hi1[c]; m.lo2[c] = lo2[c]; m.hi2[c] = hi2[c];
    }
    m.mask = mask; m.mask_pitch = mask_pitch;
    dim3 grid((unsigned)((W + usv::kTW - 1) / usv::kTW), (unsigned)((H + usv::kTH - 1) / usv::kTH));
    const int vec = al4(mask) && mask_pitch % 4 == 0;
    hipLaunchKernelGGL(usv::mask_kernel<1>, grid, dim3(usv::kMT), 0, static_cast<hipStream_t>(stream), m, vec);
    return usv::st(hipGetLastError());
}

}  // extern "C"
