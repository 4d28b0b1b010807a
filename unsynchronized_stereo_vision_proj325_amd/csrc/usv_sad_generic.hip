// usv_sad_generic.hip -- direct-window SAD/SSD block match for gfx950.
//
// The fallback for shapes outside the fast path (SSD, w > 15, unaligned
// pitch).  One thread per output pixel, the window summed directly from
// L1/L2-resident rows; O(D*w^2) per pixel.  Same spec and tie rule as the fast
// kernel and oracle/sad_oracle.c.
#include "usv_kernels.hpp"

namespace usv {
namespace {

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

template <int METRIC>
__global__ __launch_bounds__(256) void sad_generic_kernel(MatchArgs a) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int b = blockIdx.z;
    if (x >= a.W) return;
    const uint8_t* L = a.L + (size_t)b * a.pair_stride;
    const uint8_t* R = a.R + (size_t)b * a.pair_stride;
    const int r = (a.w - 1) / 2;
    uint32_t best = 0xFFFFFFFFu;
    int best_d = 0;
    for (int d = 0; d < a.D; ++d) {
        uint32_t cost = 0;
        for (int dy = -r; dy <= r; ++dy) {
            const int yy = clampi(y + dy, 0, a.H - 1);
            const uint8_t* lr = L + (size_t)yy * a.pitch;
            const uint8_t* rr = R + (size_t)yy * a.pitch;
            for (int dx = -r; dx <= r; ++dx) {
                const int t = (int)lr[clampi(x + dx, 0, a.W - 1)] - (int)rr[clampi(x + dx - d, 0, a.W - 1)];
                cost += METRIC == 0 ? (uint32_t)(t < 0 ? -t : t) : (uint32_t)(t * t);
            }
        }
        if (cost < best) { best = cost; best_d = d; }
    }
    a.disp[(size_t)b * a.disp_stride + (size_t)y * a.disp_pitch + x] = (uint8_t)best_d;
    if (a.dist) a.dist[(size_t)b * a.dist_stride + (size_t)y * a.dist_pitch + x] = a.lut[best_d];
}

}  // namespace

hipError_t launch_generic(const MatchArgs& a, hipStream_t s) {
    dim3 block(256), grid((a.W + 255) / 256, a.H, a.batch);
    if (a.metric == 0)
        hipLaunchKernelGGL(sad_generic_kernel<0>, grid, block, 0, s, a);
    else
        hipLaunchKernelGGL(sad_generic_kernel<1>, grid, block, 0, s, a);
    return hipGetLastError();
}

}  // namespace usv
