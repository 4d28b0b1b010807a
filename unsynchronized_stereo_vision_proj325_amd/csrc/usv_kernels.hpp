// usv_kernels.hpp -- launch-side declarations shared by the .hip kernel files
// and the C ABI (usv_capi.hip).  Internal to libusv.so.
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

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
