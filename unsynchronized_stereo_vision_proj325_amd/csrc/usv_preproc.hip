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
//   mask_kernel<MODE>    absdiff > 40 (ABSDiffSearch, P/Main.cpp:304-308) or two
//                        inRange + saturating add (ColourSearch, P/Main.cpp:322-324),
//                        then erode + dilate with the 5x5 ellipse
//                        (MorphilogicalFilter, P/Main.cpp:289-292), one LDS tile
// All three are HBM-bound byte streams: no MFMA, integer work
// except the HSV2BGR float path, which follows OpenCV's float operations in
// order (-ffp-contract=off).
#include "usv.h"
#include "usv_kernels.hpp"

namespace usv {
namespace {

constexpr int kHsvShift = 12;

__device__ __forceinline__ void bgr2hsv_px(int b, int g, int r, const int* sdiv, const int* hdiv, int& h, int& s,
                                           int& v) {
    v = max(max(b, g), r);
    const int vmin = min(min(b, g), r);
    const int diff = v - vmin;
    const int vr = v == r ? -1 : 0, vg = v == g ? -1 : 0;
    s = (diff * sdiv[v] + (1 << (kHsvShift - 1))) >> kHsvShift;
    h = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + ((~vg) & (r - g + 4 * diff))));
    h = (h * hdiv[diff] + (1 << (kHsvShift - 1))) >> kHsvShift;
    h += h < 0 ? 180 : 0;
    h = min(max(h, 0), 255);
}

// RGB2HSV_b tables: cvRound((255 << 12) / i), cvRound((180 << 12) / (6 i)), entry 0 = 0.
__device__ void hsv_tables(int* sdiv, int* hdiv) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
        sdiv[i] = i ? __double2int_rn((255 << kHsvShift) / (1. * i)) : 0;
        hdiv[i] = i ? __double2int_rn((180 << kHsvShift) / (6. * i)) : 0;
    }
}

__device__ __forceinline__ int round_u8(float f) { return min(max(__float2int_rn(f), 0), 255); }

__device__ __forceinline__ void hsv2bgr_px(int H8, int S8, int V8, int& ob, int& og, int& orr) {
    float h = (float)H8, s = S8 * (1.f / 255.f), v = V8 * (1.f / 255.f);
    float b, g, r;
    if (s == 0) {
        b = g = r = v;
    } else {
        const float hscale = 6.f / 180;
        h *= hscale;
        if (h < 0)
            do h += 6; while (h < 0);
        else if (h >= 6)
            do h -= 6; while (h >= 6);
        int sector = (int)floorf(h);
        h -= sector;
        if ((unsigned)sector >= 6u) {
            sector = 0;
            h = 0.f;
        }
        const float t0 = v, t1 = v * (1.f - s), t2 = v * (1.f - s * h), t3 = v * (1.f - s * (1.f - h));
        // sector_data {1,3,0} {1,0,2} {3,0,1} {0,2,1} {0,1,3} {2,1,0} -> (b, g, r) taps
        switch (sector) {
            case 0: b = t1; g = t3; r = t0; break;
            case 1: b = t1; g = t0; r = t2; break;
            case 2: b = t3; g = t0; r = t1; break;
            case 3: b = t0; g = t2; r = t1; break;
            case 4: b = t0; g = t1; r = t3; break;
            default: b = t2; g = t1; r = t0; break;
        }
    }
    ob = round_u8(b * 255.f);
    og = round_u8(g * 255.f);
    orr = round_u8(r * 255.f);
}

// One block per group of rows; per-block LDS histogram flushed with at most
// 256 global atomics.  hist must be zero on entry (the C entry point clears it
// on the same stream).
__global__ __launch_bounds__(256) void hsv_hist_kernel(const uint8_t* __restrict__ bgr, int W, int H, int pitch,
                                                       uint8_t* __restrict__ hsv, int hsv_pitch,
                                                       uint32_t* __restrict__ hist) {
    __shared__ int sdiv[256], hdiv[256];
    __shared__ uint32_t lh[256];
    hsv_tables(sdiv, hdiv);
    lh[threadIdx.x] = 0;
    __syncthreads();
    for (int y = blockIdx.x; y < H; y += gridDim.x) {
        const uint8_t* s = bgr + (size_t)y * pitch;
        uint8_t* d = hsv + (size_t)y * hsv_pitch;
        for (int x = threadIdx.x; x < W; x += 256) {
            int h, sat, v;
            bgr2hsv_px(s[3 * x], s[3 * x + 1], s[3 * x + 2], sdiv, hdiv, h, sat, v);
            d[3 * x] = (uint8_t)h;
            d[3 * x + 1] = (uint8_t)sat;
            d[3 * x + 2] = (uint8_t)v;
            atomicAdd(&lh[v], 1u);
        }
    }
    __syncthreads();
    if (lh[threadIdx.x]) atomicAdd(&hist[threadIdx.x], lh[threadIdx.x]);
}

// equalizeHist's LUT, computed by every block from the 256-bin histogram
// (inclusive scan in LDS; float scale and cvRound exactly as OpenCV), then
// per pixel V' = LUT[V] (written back into hsv), HSV2BGR, BGR2GRAY.
__global__ __launch_bounds__(256) void equalize_kernel(const uint32_t* __restrict__ hist, int W, int H,
                                                       uint8_t* __restrict__ hsv, int hsv_pitch,
                                                       uint8_t* __restrict__ bgr, int bgr_pitch,
                                                       uint8_t* __restrict__ gray, int gray_pitch) {
    __shared__ int scan[256];
    __shared__ int first;
    __shared__ uint8_t lut[256];
    const int t = threadIdx.x;
    const int hv = (int)hist[t];
    if (t == 0) first = 256;
    scan[t] = hv;
    __syncthreads();
    if (hv) atomicMin(&first, t);
    for (int off = 1; off < 256; off <<= 1) {
        const int add = t >= off ? scan[t - off] : 0;
        __syncthreads();
        scan[t] += add;
        __syncthreads();
    }
    const int total = W * H;
    const int i0 = first;
    int lv = 0;
    if (i0 < 256) {
        const int h0 = (int)hist[i0];
        if (h0 == total) {
            lv = t == i0 ? i0 : 0;  // dst.setTo(i0)
        } else if (t > i0) {
            const float scale = (256 - 1.f) / (total - h0);
            const int sum = scan[t] - scan[i0];  // hist[i0 + 1 .. t]
            lv = min(max(__float2int_rn(sum * scale), 0), 255);
        }
    }
    lut[t] = (uint8_t)lv;
    __syncthreads();
    for (int y = blockIdx.x; y < H; y += gridDim.x) {
        uint8_t* hs = hsv + (size_t)y * hsv_pitch;
        uint8_t* bo = bgr + (size_t)y * bgr_pitch;
        uint8_t* go = gray + (size_t)y * gray_pitch;
        for (int x = threadIdx.x; x < W; x += 256) {
            const int H8 = hs[3 * x], S8 = hs[3 * x + 1];
            const int V8 = lut[hs[3 * x + 2]];
            hs[3 * x + 2] = (uint8_t)V8;
            int b, g, r;
            hsv2bgr_px(H8, S8, V8, b, g, r);
            bo[3 * x] = (uint8_t)b;
            bo[3 * x + 1] = (uint8_t)g;
            bo[3 * x + 2] = (uint8_t)r;
            go[x] = (uint8_t)((b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14);
        }
    }
}

// ---- masks: threshold / inRange, then erode + dilate (5x5 ellipse) in one tile ----
constexpr int kTW = 64, kTH = 16;            // output tile
constexpr int kR = 2;                        // ellipse radius
constexpr int kIW = kTW + 4 * kR, kIH = kTH + 4 * kR;  // thresholded input tile (two radii of halo)
constexpr int kEW = kTW + 2 * kR, kEH = kTH + 2 * kR;  // eroded tile (one radius of halo)

struct MaskArgs {
    const uint8_t* a;  // gray (motion) or hsv (colour)
    const uint8_t* b;  // prev gray (motion)
    int W, H, pitch;
    int thresh;
    int lo1[3], hi1[3], lo2[3], hi2[3];
    uint8_t* mask;
    int mask_pitch;
};

// the 17 taps of the 5x5 ellipse: rows -2 and 2 the centre column only
template <bool ERODE>
__device__ __forceinline__ int ellipse5(const uint8_t* t, int stride) {
    // t points at the tap (dy, dx) = (0, 0)
    int acc = t[-2 * stride];
#define USV_TAP(o) acc = ERODE ? min(acc, (int)t[o]) : max(acc, (int)t[o])
    USV_TAP(2 * stride);
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
        for (int dx = -2; dx <= 2; ++dx) USV_TAP(dy * stride + dx);
#undef USV_TAP
    return acc;
}

template <int MODE>  // 0: motion (absdiff > thresh), 1: colour (two inRange, saturating add)
__global__ __launch_bounds__(256) void mask_kernel(MaskArgs m) {
    __shared__ uint8_t T[kIH][kIW];
    __shared__ uint8_t E[kEH][kEW];
    const int X0 = blockIdx.x * kTW, Y0 = blockIdx.y * kTH;
    for (int i = threadIdx.x; i < kIH * kIW; i += 256) {
        const int ty = i / kIW, tx = i - ty * kIW;
        const int y = Y0 - 2 * kR + ty, x = X0 - 2 * kR + tx;
        int v = 255;  // outside the image: never wins the erode min
        if (y >= 0 && y < m.H && x >= 0 && x < m.W) {
            if constexpr (MODE == 0) {
                const int p = m.a[(size_t)y * m.pitch + x], q = m.b[(size_t)y * m.pitch + x];
                v = (p > q ? p - q : q - p) > m.thresh ? 255 : 0;
            } else {
                const uint8_t* s = m.a + (size_t)y * m.pitch + 3 * x;
                bool in1 = true, in2 = true;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    in1 = in1 && s[c] >= m.lo1[c] && s[c] <= m.hi1[c];
                    in2 = in2 && s[c] >= m.lo2[c] && s[c] <= m.hi2[c];
                }
                v = (in1 || in2) ? 255 : 0;
            }
        }
        T[ty][tx] = (uint8_t)v;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kEH * kEW; i += 256) {
        const int ey = i / kEW, ex = i - ey * kEW;
        const int y = Y0 - kR + ey, x = X0 - kR + ex;
        int v = 0;  // outside the image: never wins the dilate max
        if (y >= 0 && y < m.H && x >= 0 && x < m.W) v = ellipse5<true>(&T[ey + kR][ex + kR], kIW);
        E[ey][ex] = (uint8_t)v;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kTH * kTW; i += 256) {
        const int oy = i / kTW, ox = i - oy * kTW;
        const int y = Y0 + oy, x = X0 + ox;
        if (y < m.H && x < m.W) m.mask[(size_t)y * m.mask_pitch + x] = (uint8_t)ellipse5<false>(&E[oy + kR][ox + kR], kEW);
    }
}

int row_blocks(int H) { return H < 1024 ? H : 1024; }

usv_status st(hipError_t e) { return e == hipSuccess ? USV_OK : USV_ERR_HIP; }

}  // namespace
}  // namespace usv

extern "C" {

usv_status usv_bgr2hsv_hist_u8(const uint8_t* bgr, int W, int H, int pitch, uint8_t* hsv, int hsv_pitch,
                               uint32_t* hist256, void* stream) {
    if (!bgr || !hsv || !hist256 || W <= 0 || H <= 0 || pitch < 3 * W || hsv_pitch < 3 * W)
        return USV_ERR_INVALID_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (hipMemsetAsync(hist256, 0, 256 * sizeof(uint32_t), s) != hipSuccess) return USV_ERR_HIP;
    hipLaunchKernelGGL(usv::hsv_hist_kernel, dim3(usv::row_blocks(H)), dim3(256), 0, s, bgr, W, H, pitch, hsv,
                       hsv_pitch, hist256);
    return usv::st(hipGetLastError());
}

usv_status usv_equalize_hsv_bgr_gray_u8(const uint32_t* hist256, uint8_t* hsv, int W, int H, int hsv_pitch,
                                        uint8_t* bgr_out, int bgr_pitch, uint8_t* gray, int gray_pitch,
                                        void* stream) {
    if (!hist256 || !hsv || !bgr_out || !gray || W <= 0 || H <= 0 || hsv_pitch < 3 * W || bgr_pitch < 3 * W ||
        gray_pitch < W || (long long)W * H > (1LL << 24))
        return USV_ERR_INVALID_ARG;
    hipLaunchKernelGGL(usv::equalize_kernel, dim3(usv::row_blocks(H)), dim3(256), 0, static_cast<hipStream_t>(stream),
                       hist256, W, H, hsv, hsv_pitch, bgr_out, bgr_pitch, gray, gray_pitch);
    return usv::st(hipGetLastError());
}

usv_status usv_frame_prep_u8(const uint8_t* bgr, int W, int H, int pitch, uint8_t* hsv, int hsv_pitch,
                             uint8_t* bgr_out, int bgr_pitch, uint8_t* gray, int gray_pitch, uint32_t* hist256,
                             void* stream) {
    usv_status r = usv_bgr2hsv_hist_u8(bgr, W, H, pitch, hsv, hsv_pitch, hist256, stream);
    if (r != USV_OK) return r;
    return usv_equalize_hsv_bgr_gray_u8(hist256, hsv, W, H, hsv_pitch, bgr_out, bgr_pitch, gray, gray_pitch, stream);
}

usv_status usv_motion_mask_u8(const uint8_t* gray, const uint8_t* prev, int W, int H, int pitch, int thresh,
                              uint8_t* mask, int mask_pitch, void* stream) {
    if (!gray || !prev || !mask || W <= 0 || H <= 0 || pitch < W || mask_pitch < W) return USV_ERR_INVALID_ARG;
    usv::MaskArgs m{};
    m.a = gray; m.b = prev; m.W = W; m.H = H; m.pitch = pitch; m.thresh = thresh;
    m.mask = mask; m.mask_pitch = mask_pitch;
    dim3 grid((unsigned)((W + usv::kTW - 1) / usv::kTW), (unsigned)((H + usv::kTH - 1) / usv::kTH));
    hipLaunchKernelGGL(usv::mask_kernel<0>, grid, dim3(256), 0, static_cast<hipStream_t>(stream), m);
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
    hipLaunchKernelGGL(usv::mask_kernel<1>, grid, dim3(256), 0, static_cast<hipStream_t>(stream), m);
    return usv::st(hipGetLastError());
}

}  // extern "C"
