// usv_distance.hip -- per-pixel disparity -> distance.
//
// The reference's distance law P/DistanceCalculator.cpp:84 takes an integer
// disparity, so a per-pixel map is a 256-entry gather: the table is built on
// the host in double with the reference formula (usv_distance_lut_cm) and the
// kernel only moves bytes -- bit-exact by construction and HBM-bound
// (1 B in + 8 B out per pixel).  16 pixels per thread: one 16-B load, eight
// 16-B stores.
#include "usv_kernels.hpp"

namespace usv {
namespace {

__global__ __launch_bounds__(256) void disp_to_dist_kernel(const uint8_t* __restrict__ disp,
                                                           int W, int H, int disp_pitch,
                                                           const double* __restrict__ lut,
                                                           double* __restrict__ out,
                                                           int out_pitch) {
    __shared__ double lut_s[256];
    lut_s[threadIdx.x] = lut[threadIdx.x];
    __syncthreads();
    const int y = blockIdx.y;
    const int x = (blockIdx.x * 256 + threadIdx.x) * 16;
    if (x >= W) return;
    const uint8_t* src = disp + (size_t)y * disp_pitch + x;
    double* dst = out + (size_t)y * out_pitch + x;
    const bool vec_ok = (x + 16 <= W) && ((reinterpret_cast<uintptr_t>(src) & 15) == 0) &&
                        ((reinterpret_cast<uintptr_t>(dst) & 15) == 0);
    if (vec_ok) {
        const uint4 v = *reinterpret_cast<const uint4*>(src);
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            double2 p0, p1;
            p0.x = lut_s[(w4[k] >> 0) & 0xFF];
            p0.y = lut_s[(w4[k] >> 8) & 0xFF];
            p1.x = lut_s[(w4[k] >> 16) & 0xFF];
            p1.y = lut_s[(w4[k] >> 24) & 0xFF];
            reinterpret_cast<double2*>(dst)[2 * k] = p0;
            reinterpret_cast<double2*>(dst)[2 * k + 1] = p1;
        }
    } else {
        for (int k = 0; k < 16 && x + k < W; ++k) dst[k] = lut_s[src[k]];
    }
}

}  // namespace

hipError_t launch_disp_to_dist(const uint8_t* disp, int W, int H, int disp_pitch,
                               const double* lut, double* out, int out_pitch, hipStream_t s) {
    dim3 block(256), grid((W + 256 * 16 - 1) / (256 * 16), H);
    hipLaunchKernelGGL(disp_to_dist_kernel, grid, block, 0, s, disp, W, H, disp_pitch, lut, out,
                       out_pitch);
    return hipGetLastError();
}

}  // namespace usv
