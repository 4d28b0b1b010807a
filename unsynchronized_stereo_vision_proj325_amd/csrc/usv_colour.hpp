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

// hsv2bgr_px for two pixels with the float arithmetic on packed f32 pairs (v_pk_mul_f32 /
// v_pk_add_f32: the same IEEE operations in the same order, so the same bytes); the floor, the
// sector selects and the conversions stay per pixel.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void hsv2bgr_px2(const int* H8, const int* S8, const int* V8, int* ob, int* og,
                                            int* orr) {
    f32x2 h = f32x2{(float)H8[0], (float)H8[1]} * (6.f / 180);
    const f32x2 s = f32x2{(float)S8[0], (float)S8[1]} * (1.f / 255.f);
    const f32x2 v = f32x2{(float)V8[0], (float)V8[1]} * (1.f / 255.f);
    const f32x2 hw = h - 6.f;
    h = f32x2{h.x >= 6 ? hw.x : h.x, h.y >= 6 ? hw.y : h.y};
    const f32x2 fl = f32x2{floorf(h.x), floorf(h.y)};
    int sec[2] = {(int)fl.x, (int)fl.y};
    h = h - fl;
#pragma unroll
    for (int i = 0; i < 2; ++i)
        if ((unsigned)sec[i] >= 6u) {
            sec[i] = 0;
            h[i] = 0.f;
        }
    const f32x2 one = 1.f;
    const f32x2 t0 = v, t1 = v * (one - s), t2 = v * (one - s * h), t3 = v * (one - s * (one - h));
    f32x2 b, g, r;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int sector = sec[i];
        b[i] = sector <= 1 ? t1[i] : sector == 2 ? t3[i] : sector <= 4 ? t0[i] : t2[i];
        g[i] = sector == 0 ? t3[i] : sector <= 2 ? t0[i] : sector == 3 ? t2[i] : t1[i];
        r[i] = sector == 0 ? t0[i] : sector == 1 ? t2[i] : sector <= 3 ? t1[i] : sector == 4 ? t3[i] : t0[i];
    }
    b = b * 255.f;
    g = g * 255.f;
    r = r * 255.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        ob[i] = round_u8(b[i]);
        og[i] = round_u8(g[i]);
        orr[i] = round_u8(r[i]);
    }
}

}  // namespace
}  // namespace usv
