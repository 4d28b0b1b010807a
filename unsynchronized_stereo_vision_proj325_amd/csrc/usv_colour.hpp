// usv_colour.hpp -- OpenCV 3.0 u8 colour conversions shared by the frame-prep
// kernels (usv_preproc.hip): BGR2HSV (RGB2HSV_b, hsv_shift = 12 tables) and
// HSV2BGR (HSV2RGB_f in float, OpenCV's operation order; build with
// -ffp-contract=off).  Restated in oracle/preproc_oracle.c; internal to libusv.so.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

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

// RGB2HSV_b tables: cvRound((255 << 12) / i), cvRound((180 << 12) / (6 i)), entry 0 = 0.  Built at
// compile time (IEEE double division as at run time; no quotient is an exact half, so rounding half
// up equals cvRound's half-to-even here) and copied into LDS per block: the round-2 kernel computed
// 512 f64 divisions per block.
struct HsvTables {
    int sdiv[256], hdiv[256];
};
constexpr HsvTables make_hsv_tables() {
    HsvTables t{};
    for (int i = 1; i < 256; ++i) {
        t.sdiv[i] = (int)((255 << kHsvShift) / (1. * i) + 0.5);
        t.hdiv[i] = (int)((180 << kHsvShift) / (6. * i) + 0.5);
    }
    return t;
}
__constant__ HsvTables c_hsv_tables = make_hsv_tables();
static_assert(make_hsv_tables().sdiv[7] == 149211 && make_hsv_tables().hdiv[7] == 17554, "cvRound values");

__device__ void hsv_tables(int* sdiv, int* hdiv) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
        sdiv[i] = c_hsv_tables.sdiv[i];
        hdiv[i] = c_hsv_tables.hdiv[i];
    }
}

__device__ __forceinline__ int round_u8(float f) { return min(max(__float2int_rn(f), 0), 255); }

// Branchless HSV2BGR (the same float operations and the same selected taps as OpenCV's HSV2RGB_f, so
// bit-identical): a wave holds all six sectors on real frames, and the switch / s == 0 branches ran as
// divergent paths.  With s == 0 every tap equals v exactly (v * (1 - 0 * x) == v), so that branch
// needs no special case; H8 <= 255 puts h in [0, 8.5], so the wrap is one conditional subtraction.
__device__ __forceinline__ void hsv2bgr_px(int H8, int S8, int V8, int& ob, int& og, int& orr) {
    float h = (float)H8 * (6.f / 180), s = S8 * (1.f / 255.f), v = V8 * (1.f / 255.f);
    h = h >= 6 ? h - 6 : h;
    int sector = (int)floorf(h);
    h -= sector;
    const bool bad = (unsigned)sector >= 6u;
    sector = bad ? 0 : sector;
    h = bad ? 0.f : h;
    const float t0 = v, t1 = v * (1.f - s), t2 = v * (1.f - s * h), t3 = v * (1.f - s * (1.f - h));
    // sector_data {1,3,0} {1,0,2} {3,0,1} {0,2,1} {0,1,3} {2,1,0} -> (b, g, r) taps
    const float b = sector <= 1 ? t1 : sector == 2 ? t3 : sector <= 4 ? t0 : t2;
    const float g = sector == 0 ? t3 : sector <= 2 ? t0 : sector == 3 ? t2 : t1;
    const float r = sector == 0 ? t0 : sector == 1 ? t2 : sector <= 3 ? t1 : sector == 4 ? t3 : t0;
    ob = round_u8(b * 255.f);
    og = round_u8(g * 255.f);
    orr = round_u8(r * 255.f);
}

}  // namespace
}  // namespace usv
