// usv_kernels.hpp -- launch-side declarations shared by the .hip kernel files
// and the C ABI (usv_capi.hip).  Internal to libusv.so.
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

// Build kind.  The product library (csrc/Makefile) is built with every tuning knob at its default;
// scripts/build_variant.sh compiles A/B variants with -DUSV_VARIANT_BUILD and knob overrides, and its
// usv_version() says so ("variant build"), so a variant can never pass for the shipped library
// (tests/test_capi.py checks the in-tree libusv.so reports "product build").  This header is
// included before any knob's default is defined, so a knob set on the command line of a product
// build is an error here.
#ifndef USV_VARIANT_BUILD
#if defined(USV_GEN_WEIGHTS) || defined(USV_GROUP_MIN_BAND_ROWS) || defined(USV_GROUP_MIN_BAND_WINS) ||          \
    defined(USV_GROUP_OCC) || defined(USV_GROUP_WEIGHTS) || defined(USV_HIST_KU) ||                              \
    defined(USV_MASK_TH) || defined(USV_MASK_TW) ||                                                              \
    defined(USV_PAIR_GEN_WEIGHTS) || defined(USV_PAIR_GEN_WEIGHTS_NW2) ||                                        \
    defined(USV_PAIR_GEN_WEIGHTS_UNPIPED) || defined(USV_PAIR_M0REUSE) || defined(USV_PAIR_OCC5) ||              \
    defined(USV_PAIR_K16) || defined(USV_PAIR_LEARLY) || defined(USV_PAIR16_GEN_WEIGHTS) ||                      \
    defined(USV_PAIR16_RA) || defined(USV_PAIR16_LEARLY) || defined(USV_PAIR16_MIDT) ||                          \
    defined(USV_PAIR_OCC7) || defined(USV_PAIR_RDASM) || defined(USV_PREP_KU) ||                        \
    defined(USV_PREP_KU_HSV) || defined(USV_PREP_THREADS) ||                                                     \
    defined(USV_REMAP_BLOCK) || defined(USV_REMAP_XCD) || defined(USV_SSD_GEN_WEIGHTS) ||                        \
    defined(USV_SSD_MFMA_MINROWS) || defined(USV_SSD_MFMA_OCC) || defined(USV_SSD_MFMA_WAVES) ||                 \
    defined(USV_STAMPS) || defined(USV_WGTIME)
#error "tuning knobs are variant-build only: use scripts/build_variant.sh (it defines USV_VARIANT_BUILD)"
#endif
#define USV_BUILD_KIND "product build"
#else
#define USV_BUILD_KIND "variant build"
#endif

namespace usv {

// Everything a block-match launch needs; one struct so every kernel variant
// takes the same argument block (batch strides included).
struct MatchArgs {
    const uint8_t* L;
    const uint8_t* R;
    int W, H, pitch;
    int D, w, metric;
    uint8_t* disp;
    int disp_pitch;
    double* dist;  // nullable: fused per-pixel distance map
    int dist_pitch;
    const double* lut;  // 256 doubles (device), required when dist != nullptr
    int batch;
    size_t pair_stride, disp_stride, dist_stride;
};

// Fast path: lane = disparity, running sums, packed-u16 ring (usv_sad_fast.hip).
// Returns hipErrorInvalidValue when the shape is outside the fast path.
bool fast_path_supported(const MatchArgs& a);
hipError_t launch_fast(const MatchArgs& a, hipStream_t s);

// Paired-disparity kernel (usv_sad_pair.hip): SAD, even D > 64, 11 <= w <= 15 (configs C, D, E), on
// shapes fast_path_supported accepts.  hipErrorInvalidValue otherwise.
bool pair_path_supported(const MatchArgs& a);
hipError_t launch_pair(const MatchArgs& a, hipStream_t s);

// SSD kernel (usv_sad_ssd.hip): 11 <= w <= 15, on shapes fast_path_supported accepts.
hipError_t launch_ssd(const MatchArgs& a, hipStream_t s);

// SSD with the window cross term on the matrix cores (usv_ssd_mfma.hip): w = 3 .. 13, D = 32 .. 160 in steps of
// 32, W >= 64, any pitch / alignment.  hipErrorInvalidValue otherwise.
bool ssd_mfma_supported(const MatchArgs& a);
hipError_t launch_ssd_mfma(const MatchArgs& a, hipStream_t s);

// Grouped paired-disparity kernel for small disparity ranges (usv_sad_group.hip): SAD, even
// 16 < D <= 64, 5 <= w <= 9, on shapes fast_path_supported accepts.  hipErrorInvalidValue otherwise.
bool group_path_supported(const MatchArgs& a);
hipError_t launch_group(const MatchArgs& a, hipStream_t s);

// Tiled sliding-window path: SAD or SSD, any W / pitch / alignment, odd w <= 31
// (usv_sad_tiled.hip).  Returns hipErrorInvalidValue outside that range.
bool tiled_path_supported(const MatchArgs& a);
hipError_t launch_tiled(const MatchArgs& a, hipStream_t s);

// Generic direct-window path: any odd w <= 63, SAD or SSD (usv_sad_generic.hip).
hipError_t launch_generic(const MatchArgs& a, hipStream_t s);

// disparity -> distance gather (usv_distance.hip).
hipError_t launch_disp_to_dist(const uint8_t* disp, int W, int H, int disp_pitch,
                               const double* lut, double* out, int out_pitch, hipStream_t s);

}  // namespace usv
