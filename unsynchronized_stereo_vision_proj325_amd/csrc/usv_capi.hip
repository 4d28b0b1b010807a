// usv_capi.hip -- C ABI entry points of the GPU path (include/usv.h).
//
// Validates arguments, fills a usv::MatchArgs and dispatches to the fast
// (lane-per-disparity) or generic kernel.  No allocation, no synchronisation:
// everything is enqueued on the caller's stream, so a caller may capture these
// calls in a hipGraph.
#include <string>

#include "usv.h"
#include "usv_kernels.hpp"

namespace {

usv_status to_status(hipError_t e) { return e == hipSuccess ? USV_OK : USV_ERR_HIP; }

usv_status validate(const usv::MatchArgs& a) {
    if (!a.L || !a.R || !a.disp) return USV_ERR_INVALID_ARG;
    if (a.W <= 0 || a.H <= 0 || a.pitch < a.W || a.disp_pitch < a.W || a.batch < 1)
        return USV_ERR_INVALID_ARG;
    if (a.dist && (!a.lut || a.dist_pitch < a.W)) return USV_ERR_INVALID_ARG;
    if (a.D < 1 || a.D > 256) return USV_ERR_UNSUPPORTED;
    if (a.w < 1 || a.w > 63 || (a.w & 1) == 0) return USV_ERR_UNSUPPORTED;
    if (a.metric != USV_METRIC_SAD && a.metric != USV_METRIC_SSD) return USV_ERR_UNSUPPORTED;
    if (a.batch > 1 && (a.pair_stride < (size_t)a.pitch * a.H || a.disp_stride < (size_t)a.disp_pitch * a.H))
        return USV_ERR_INVALID_ARG;
    if (a.batch > 1 && a.dist && a.dist_stride < (size_t)a.dist_pitch * a.H) return USV_ERR_INVALID_ARG;
    if (a.batch > 65535) return USV_ERR_UNSUPPORTED;
    return USV_OK;
}

usv_status dispatch(const usv::MatchArgs& a, int kernel, void* stream) {
    usv_status st = validate(a);
    if (st != USV_OK) return st;
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (kernel) {
        case USV_KERNEL_AUTO:
            return to_status(usv::fast_path_supported(a) ? usv::launch_fast(a, s) : usv::launch_generic(a, s));
        case USV_KERNEL_FAST:
            if (!usv::fast_path_supported(a)) return USV_ERR_UNSUPPORTED;
            return to_status(usv::launch_fast(a, s));
        case USV_KERNEL_GENERIC:
            return to_status(usv::launch_generic(a, s));
        default:
            return USV_ERR_INVALID_ARG;
    }
}

}  // namespace

extern "C" {

const char* usv_version(void) { return "usv-mi355x 0.1.0 (gfx950)"; }

usv_status usv_device_check(int* n_devices) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    if (n_devices) *n_devices = n;
    if (n == 0) return USV_ERR_NO_DEVICE;
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
        return USV_ERR_HIP;
    return std::string(prop.gcnArchName).rfind("gfx950", 0) == 0 ? USV_OK : USV_ERR_NO_DEVICE;
}

usv_status usv_sad_disparity_ex(const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int D,
                                int w, int metric, uint8_t* disp, int disp_pitch, double* dist_cm,
                                int dist_pitch, const double* lut_cm, int kernel, void* stream) {
    usv::MatchArgs a{};
    a.L = L; a.R = R; a.W = W; a.H = H; a.pitch = pitch; a.D = D; a.w = w; a.metric = metric;
    a.disp = disp; a.disp_pitch = disp_pitch; a.dist = dist_cm; a.dist_pitch = dist_pitch;
    a.lut = lut_cm; a.batch = 1;
    return dispatch(a, kernel, stream);
}

usv_status usv_sad_disparity(const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int D, int w,
                             int metric, uint8_t* disp, int disp_pitch, void* stream) {
    return usv_sad_disparity_ex(L, R, W, H, pitch, D, w, metric, disp, disp_pitch, nullptr, 0,
                                nullptr, USV_KERNEL_AUTO, stream);
}

usv_status usv_sad_disparity_batch(const uint8_t* L, const uint8_t* R, int batch, size_t pair_stride,
                                   int W, int H, int pitch, int D, int w, int metric, uint8_t* disp,
                                   size_t disp_stride, int disp_pitch, double* dist_cm,
                                   size_t dist_stride, int dist_pitch, const double* lut_cm,
                                   void* stream) {
    usv::MatchArgs a{};
    a.L = L; a.R = R; a.W = W; a.H = H; a.pitch = pitch; a.D = D; a.w = w; a.metric = metric;
    a.disp = disp; a.disp_pitch = disp_pitch; a.dist = dist_cm; a.dist_pitch = dist_pitch;
    a.lut = lut_cm; a.batch = batch; a.pair_stride = pair_stride; a.disp_stride = disp_stride;
    a.dist_stride = dist_stride;
    return dispatch(a, USV_KERNEL_AUTO, stream);
}

usv_status usv_disparity_to_distance(const uint8_t* disp, int W, int H, int disp_pitch,
                                     const double* lut_cm, double* out, int out_pitch, void* stream) {
    if (!disp || !lut_cm || !out || W <= 0 || H <= 0 || disp_pitch < W || out_pitch < W)
        return USV_ERR_INVALID_ARG;
    return to_status(usv::launch_disp_to_dist(disp, W, H, disp_pitch, lut_cm, out, out_pitch,
                                              static_cast<hipStream_t>(stream)));
}

}  // extern "C"
