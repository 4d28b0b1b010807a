// usv_capi.hip -- C ABI entry points of the GPU path (include/usv.h).
//
// Validates arguments, fills a usv::MatchArgs and dispatches to the fast
// (lane-per-disparity) or generic kernel.  No allocation, no synchronisation:
// everything is enqueued on the caller's stream, so a caller may capture these
// calls in a hipGraph.
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "usv.h"
#include "usv_kernels.hpp"

namespace {

usv_status to_status(hipError_t e) { return e == hipSuccess ? USV_OK : USV_ERR_HIP; }

// ---- distance tables given in host memory -----------------------------------
// The kernels read the 256-entry table on the device.  A caller may pass a
// device pointer (used as is), a pinned/registered host pointer (its device
// alias is used) or ordinary pageable host memory, e.g. the
// `static double lut[256]` that usv_distance_lut_cm fills.
// Pageable tables are copied once per (device, contents) into a library-owned
// device buffer that lives until process exit; later calls with the same
// contents find it by value and enqueue nothing extra.  The first call with a
// new table copies it synchronously (hipMemcpy), so make that call once before
// capturing a hipGraph.  Bounded: at most kMaxHostTables distinct tables.
struct HostTable {
    int device;
    double values[256];
    double* dev;
};
constexpr size_t kMaxHostTables = 64;
std::mutex g_tables_mu;
std::vector<HostTable*> g_tables;

usv_status resolve_lut(const double* lut, const double** dev_lut) {
    *dev_lut = lut;
    if (!lut) return USV_OK;
    hipPointerAttribute_t attr{};
    hipError_t e = hipPointerGetAttributes(&attr, lut);
    // The host copy below dereferences the pointer, so it is taken only for memory positively
    // identified as pageable host memory: hipSuccess with hipMemoryTypeUnregistered, or the
    // invalid-value error older runtimes return for unregistered host pointers.  Anything else the
    // runtime knows is passed through (device, managed, unified, VMM-mapped device memory) or
    // refused (a host type without a device alias).
    bool pageable = false;
    if (e == hipSuccess) {
        switch (attr.type) {
            case hipMemoryTypeUnregistered:
                pageable = true;
                break;
            case hipMemoryTypeHost:
                if (!attr.devicePointer) return USV_ERR_INVALID_ARG;
                *dev_lut = static_cast<const double*>(attr.devicePointer);  // pinned / registered host memory
                return USV_OK;
            default:
                return USV_OK;  // device-accessible as is
        }
    } else if (e == hipErrorInvalidValue) {
        (void)hipGetLastError();  // the failed query left its error behind; clear only that one
        pageable = true;
    } else {
        (void)hipGetLastError();
        return USV_ERR_HIP;
    }
    if (!pageable) return USV_ERR_INVALID_ARG;
    int device = 0;
    if (hipGetDevice(&device) != hipSuccess) return USV_ERR_HIP;
    std::lock_guard<std::mutex> lock(g_tables_mu);
    for (const HostTable* t : g_tables)
        if (t->device == device && std::memcmp(t->values, lut, sizeof(t->values)) == 0) {
            *dev_lut = t->dev;
            return USV_OK;
        }
    if (g_tables.size() >= kMaxHostTables) return USV_ERR_UNSUPPORTED;
    auto* t = new HostTable{};
    t->device = device;
    std::memcpy(t->values, lut, sizeof(t->values));
    if (hipMalloc(&t->dev, sizeof(t->values)) != hipSuccess) {
        delete t;
        return USV_ERR_HIP;
    }
    if (hipMemcpy(t->dev, t->values, sizeof(t->values), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(t->dev);
        delete t;
        return USV_ERR_HIP;
    }
    g_tables.push_back(t);
    *dev_lut = t->dev;
    return USV_OK;
}

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

// Checks a match and resolves what every launch of it uses: the distance table's device address and the
// concrete kernel (AUTO: SSD on the matrix cores where supported, else the fast kernels, else the tiled
// sliding-window kernel -- any shape, w <= 31 -- else the direct-window kernel: w > 31, or a window too large
// for the tiled ring).
usv_status prepare(usv::MatchArgs& a, int& kernel) {
    usv_status st = validate(a);
    if (st != USV_OK) return st;
    if (kernel != USV_KERNEL_AUTO && kernel != USV_KERNEL_FAST && kernel != USV_KERNEL_GENERIC &&
        kernel != USV_KERNEL_TILED && kernel != USV_KERNEL_MATRIX)
        return USV_ERR_INVALID_ARG;
    if (kernel == USV_KERNEL_FAST && !usv::fast_path_supported(a)) return USV_ERR_UNSUPPORTED;
    if (kernel == USV_KERNEL_TILED && !usv::tiled_path_supported(a)) return USV_ERR_UNSUPPORTED;
    if (kernel == USV_KERNEL_MATRIX && !usv::ssd_mfma_supported(a)) return USV_ERR_UNSUPPORTED;
    if (a.dist && (st = resolve_lut(a.lut, &a.lut)) != USV_OK) return st;
    if (kernel == USV_KERNEL_AUTO)
        kernel = usv::ssd_mfma_supported(a)      ? USV_KERNEL_MATRIX
                 : usv::fast_path_supported(a)   ? USV_KERNEL_FAST
                 : usv::tiled_path_supported(a)  ? USV_KERNEL_TILED
                                                 : USV_KERNEL_GENERIC;
    return USV_OK;
}

usv_status launch(const usv::MatchArgs& a, int kernel, hipStream_t s) {
    switch (kernel) {
        case USV_KERNEL_FAST: return to_status(usv::launch_fast(a, s));
        case USV_KERNEL_TILED: return to_status(usv::launch_tiled(a, s));
        case USV_KERNEL_GENERIC: return to_status(usv::launch_generic(a, s));
        case USV_KERNEL_MATRIX: return to_status(usv::launch_ssd_mfma(a, s));
        default: return USV_ERR_INVALID_ARG;
    }
}

usv_status dispatch(usv::MatchArgs a, int kernel, void* stream) {
    const usv_status st = prepare(a, kernel);
    return st != USV_OK ? st : launch(a, kernel, static_cast<hipStream_t>(stream));
}

}  // namespace

struct usv_match_plan {
    usv::MatchArgs a;
    int kernel;  // concrete (never AUTO)
    hipStream_t stream;
};

extern "C" {

const char* usv_version(void) { return "usv-mi355x 0.4.3 (gfx950, " USV_BUILD_KIND ")"; }

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

usv_status usv_match_plan_create(const uint8_t* L, const uint8_t* R, int batch, size_t pair_stride, int W, int H,
                                 int pitch, int D, int w, int metric, uint8_t* disp, size_t disp_stride,
                                 int disp_pitch, double* dist_cm, size_t dist_stride, int dist_pitch,
                                 const double* lut_cm, int kernel, void* stream, usv_match_plan** out) {
    if (!out) return USV_ERR_INVALID_ARG;
    *out = nullptr;
    if (batch > 1 && kernel != USV_KERNEL_AUTO) return USV_ERR_INVALID_ARG;  // as usv_sad_disparity_batch
    usv::MatchArgs a{};
    a.L = L; a.R = R; a.W = W; a.H = H; a.pitch = pitch; a.D = D; a.w = w; a.metric = metric;
    a.disp = disp; a.disp_pitch = disp_pitch; a.dist = dist_cm; a.dist_pitch = dist_pitch;
    a.lut = lut_cm; a.batch = batch; a.pair_stride = pair_stride; a.disp_stride = disp_stride;
    a.dist_stride = dist_stride;
    const usv_status st = prepare(a, kernel);
    if (st != USV_OK) return st;
    *out = new usv_match_plan{a, kernel, static_cast<hipStream_t>(stream)};
    return USV_OK;
}

usv_status usv_match_plan_launch(const usv_match_plan* p) {
    return p ? launch(p->a, p->kernel, p->stream) : USV_ERR_INVALID_ARG;
}

usv_status usv_match_plan_destroy(usv_match_plan* p) {
    if (!p) return USV_ERR_INVALID_ARG;
    delete p;
    return USV_OK;
}

usv_status usv_disparity_to_distance(const uint8_t* disp, int W, int H, int disp_pitch,
                                     const double* lut_cm, double* out, int out_pitch, void* stream) {
    if (!disp || !lut_cm || !out || W <= 0 || H <= 0 || disp_pitch < W || out_pitch < W)
        return USV_ERR_INVALID_ARG;
    usv_status st = resolve_lut(lut_cm, &lut_cm);
    if (st != USV_OK) return st;
    return to_status(usv::launch_disp_to_dist(disp, W, H, disp_pitch, lut_cm, out, out_pitch,
                                              static_cast<hipStream_t>(stream)));
}

}  // extern "C"
