// usv_stream.hip -- streaming host frames through the matcher (include/usv.h,
// usv_frame_stream_*).
//
// The reference's caller owns HOST frames: each camera thread grabs a frame,
// rectifies and pre-processes it and hands it on (P/Main.cpp:876-921,
// 1238-1242).  A per-frame blocking call (copy in, match, copy out, sync)
// serialises the PCIe transfers with the kernel.  This engine keeps `depth`
// frames in flight instead: every slot owns pinned host staging and device
// buffers; three streams carry the stages -- H2D copies, the match, D2H copies
// -- ordered per frame by events, so frame k+1's H2D, frame k's match and
// frame k-1's D2H run at once (the copy engines are separate from the CUs and
// PCIe is full duplex).  (Round 3 gave every slot its own stream and measured
// depth 3 ~20 % slower than depth 2 or 4 -- streams share the process's four
// hardware queues, so the overlap depended on how the slots' streams landed on
// them; one stream per stage makes the schedule the same at every depth.)  Results are the u8 disparity maps by default: the
// per-pixel distance is a 256-entry table lookup of the disparity
// (P/DistanceCalculator.cpp:84), expanded on the host only where a caller asks
// for it (usv_distance_expand_host), so the link carries 1 B per pixel instead
// of 9.  USV_STREAM_DEVICE_DIST keeps the f64 map on the device path as well.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <functional>
#include <vector>

#include "usv.h"
#include "usv_host_pool.hpp"
#include "usv_kernels.hpp"

struct usv_frame_stream {
    int W = 0, H = 0, D = 0, w = 0, metric = 0, depth = 0, flags = 0, device = 0;
    size_t frame = 0;  // W * H
    struct Slot {
        uint8_t *hL = nullptr, *hR = nullptr, *hDisp = nullptr;  // pinned host staging (hR = hL + frame)
        double* hDist = nullptr;                                 // pinned (USV_STREAM_DEVICE_DIST)
        uint8_t *dL = nullptr, *dR = nullptr, *dDisp = nullptr;  // device (dR = dL + frame)
        double* dDist = nullptr;
        hipEvent_t in = nullptr, matched = nullptr, done = nullptr;  // after the H2D, the match, the D2H
        long long ticket = -1;  // frame in this slot, -1 = free
        bool ready = false;     // its results were waited for
    };
    std::vector<Slot> slot;
    hipStream_t s_in = nullptr, s_match = nullptr, s_out = nullptr;  // H2D copies, matcher, D2H copies
    long long next = 0;      // ticket of the next submit
    double* lut = nullptr;   // device distance table (USV_STREAM_DEVICE_DIST)
};

namespace {

// the expansion's workers (usv_host_pool.hpp); never destroyed, so no worker is joined during static destruction.
// One pool per process: a forked child finds its parent's pool (whose threads it does not have) and installs a
// fresh one; the parent's copy is left untouched (a HostPool never locks or joins in a process it was not made in).
usv::HostPool& host_pool() {
    static std::atomic<usv::HostPool*> pool{nullptr};
    usv::HostPool* p = pool.load(std::memory_order_acquire);
    if (p && p->owner() == getpid()) return *p;
    auto* fresh = new usv::HostPool;
    if (pool.compare_exchange_strong(p, fresh, std::memory_order_acq_rel)) return *fresh;
    delete fresh;  // another thread of this process installed one first (p now holds it); fresh has no workers
    return *p;
}

void free_slot(usv_frame_stream::Slot& s) {
    (void)hipHostFree(s.hL);  // hR = hL + frame
    (void)hipHostFree(s.hDisp);
    (void)hipHostFree(s.hDist);
    (void)hipFree(s.dL);  // dR = dL + frame
    (void)hipFree(s.dDisp);
    (void)hipFree(s.dDist);
    if (s.in) (void)hipEventDestroy(s.in);
    if (s.matched) (void)hipEventDestroy(s.matched);
    if (s.done) (void)hipEventDestroy(s.done);
}

void release(usv_frame_stream* e) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(e->device);
    for (hipStream_t st : {e->s_in, e->s_match, e->s_out})
        if (st) (void)hipStreamSynchronize(st);
    for (auto& s : e->slot) free_slot(s);
    for (hipStream_t st : {e->s_in, e->s_match, e->s_out})
        if (st) (void)hipStreamDestroy(st);
    (void)hipFree(e->lut);
    (void)hipSetDevice(cur);
    delete e;
}

usv_frame_stream::Slot* find(usv_frame_stream* e, long long ticket) {
    if (ticket < 0) return nullptr;
    auto& s = e->slot[(size_t)(ticket % e->depth)];
    return s.ticket == ticket ? &s : nullptr;
}

// Restores the caller's current device on every exit path.
struct DeviceGuard {
    int prev = 0;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        ok = hipGetDevice(&prev) == hipSuccess && hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() { (void)hipSetDevice(prev); }
};

}  // namespace

extern "C" {

usv_status usv_frame_stream_create(int W, int H, int D, int w, int metric, int depth, int flags,
                                   usv_frame_stream** out) {
    if (!out) return USV_ERR_INVALID_ARG;
    *out = nullptr;
    if (W <= 0 || H <= 0 || depth < 2 || depth > 8 || (flags & ~USV_STREAM_DEVICE_DIST)) return USV_ERR_INVALID_ARG;
    if (D < 1 || D > 256 || w < 1 || w > 63 || (w & 1) == 0) return USV_ERR_UNSUPPORTED;
    if (metric != USV_METRIC_SAD && metric != USV_METRIC_SSD) return USV_ERR_UNSUPPORTED;
    auto* e = new usv_frame_stream;
    if (hipGetDevice(&e->device) != hipSuccess) {
        delete e;
        return USV_ERR_NO_DEVICE;
    }
    e->W = W; e->H = H; e->D = D; e->w = w; e->metric = metric; e->depth = depth; e->flags = flags;
    e->frame = (size_t)W * H;
    e->slot.resize((size_t)depth);
    const bool dd = flags & USV_STREAM_DEVICE_DIST;
    for (auto& s : e->slot) {
        // L and R back to back in one pinned and one device allocation: the pair crosses the link as ONE copy
        // (round 5: depth 3 0.106 -> 0.097 ms per 1080p frame, profiles/probes_r05/ab_stream_contig_r05.txt)
        if (hipHostMalloc(&s.hL, 2 * e->frame, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc(&s.hDisp, e->frame, hipHostMallocDefault) != hipSuccess ||
            hipMalloc(&s.dL, 2 * e->frame) != hipSuccess || hipMalloc(&s.dDisp, e->frame) != hipSuccess ||
            (dd && (hipHostMalloc(&s.hDist, e->frame * sizeof(double), hipHostMallocDefault) != hipSuccess ||
                    hipMalloc(&s.dDist, e->frame * sizeof(double)) != hipSuccess)) ||
            hipEventCreateWithFlags(&s.in, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&s.matched, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess) {
            release(e);
            return USV_ERR_HIP;
        }
        s.hR = s.hL + e->frame;
        s.dR = s.dL + e->frame;
    }
    if (hipStreamCreateWithFlags(&e->s_in, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&e->s_match, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&e->s_out, hipStreamNonBlocking) != hipSuccess) {
        release(e);
        return USV_ERR_HIP;
    }
    if (dd) {
        double lut[256];
        usv_distance_lut_cm(USV_DIST_MOVING_OBJECT, lut);
        if (hipMalloc(&e->lut, sizeof(lut)) != hipSuccess ||
            hipMemcpy(e->lut, lut, sizeof(lut), hipMemcpyHostToDevice) != hipSuccess) {
            release(e);
            return USV_ERR_HIP;
        }
    }
    *out = e;
    return USV_OK;
}

usv_status usv_frame_stream_destroy(usv_frame_stream* e) {
    if (!e) return USV_ERR_INVALID_ARG;
    release(e);
    return USV_OK;
}

usv_status usv_frame_stream_next_inputs(usv_frame_stream* e, uint8_t** L, uint8_t** R) {
    if (!e || !L || !R) return USV_ERR_INVALID_ARG;
    auto& s = e->slot[(size_t)(e->next % e->depth)];
    if (s.ticket >= 0) return USV_ERR_INVALID_ARG;  // the slot's previous frame was not collected yet
    *L = s.hL;
    *R = s.hR;
    return USV_OK;
}

usv_status usv_frame_stream_submit(usv_frame_stream* e, const uint8_t* L, const uint8_t* R, int pitch,
                                   long long* ticket) {
    if (!e || !L || !R || !ticket || pitch < e->W) return USV_ERR_INVALID_ARG;
    auto& s = e->slot[(size_t)(e->next % e->depth)];
    if ((L == s.hL || R == s.hR) && pitch != e->W) return USV_ERR_INVALID_ARG;  // the staging is dense
    if (s.ticket >= 0) return USV_ERR_INVALID_ARG;  // depth frames in flight: collect the oldest first
    DeviceGuard g(e->device);
    if (!g.ok) return USV_ERR_HIP;
    const size_t W = (size_t)e->W, H = (size_t)e->H;
    // Inputs: the slot's own pinned staging (zero-copy, usv_frame_stream_next_inputs) go straight to
    // the copy engine; any other host buffer is packed into the staging first (a host memcpy).
    auto stage = [&](const uint8_t* src, uint8_t* pinned) {
        if (src == pinned) return;
        for (size_t y = 0; y < H; ++y) std::memcpy(pinned + y * W, src + y * (size_t)pitch, W);
    };
    stage(L, s.hL);
    stage(R, s.hR);
    // every error path drains the three streams: nothing of this frame may still read the staging
    auto drain = [&](usv_status st) {
        for (hipStream_t q : {e->s_in, e->s_match, e->s_out}) (void)hipStreamSynchronize(q);
        return st;
    };
    if (hipMemcpyAsync(s.dL, s.hL, 2 * e->frame, hipMemcpyHostToDevice, e->s_in) != hipSuccess ||
        hipEventRecord(s.in, e->s_in) != hipSuccess || hipStreamWaitEvent(e->s_match, s.in, 0) != hipSuccess)
        return drain(USV_ERR_HIP);
    const bool dd = e->flags & USV_STREAM_DEVICE_DIST;
    usv_status st = usv_sad_disparity_ex(s.dL, s.dR, e->W, e->H, e->W, e->D, e->w, e->metric, s.dDisp, e->W,
                                         dd ? s.dDist : nullptr, e->W, dd ? e->lut : nullptr, USV_KERNEL_AUTO,
                                         e->s_match);
    if (st != USV_OK) return drain(st);
    if (hipEventRecord(s.matched, e->s_match) != hipSuccess || hipStreamWaitEvent(e->s_out, s.matched, 0) != hipSuccess ||
        hipMemcpyAsync(s.hDisp, s.dDisp, e->frame, hipMemcpyDeviceToHost, e->s_out) != hipSuccess ||
        (dd && hipMemcpyAsync(s.hDist, s.dDist, e->frame * sizeof(double), hipMemcpyDeviceToHost, e->s_out) !=
                   hipSuccess) ||
        hipEventRecord(s.done, e->s_out) != hipSuccess)
        return drain(USV_ERR_HIP);
    s.ticket = e->next++;
    s.ready = false;
    *ticket = s.ticket;
    return USV_OK;
}

usv_status usv_frame_stream_wait(usv_frame_stream* e, long long ticket, const uint8_t** disp, const double** dist_cm) {
    if (!e || !disp) return USV_ERR_INVALID_ARG;
    auto* s = find(e, ticket);
    if (!s) return USV_ERR_INVALID_ARG;
    if (dist_cm && !(e->flags & USV_STREAM_DEVICE_DIST)) return USV_ERR_INVALID_ARG;
    if (!s->ready) {
        if (hipEventSynchronize(s->done) != hipSuccess) return USV_ERR_HIP;
        s->ready = true;
    }
    *disp = s->hDisp;
    if (dist_cm) *dist_cm = s->hDist;
    return USV_OK;
}

usv_status usv_frame_stream_release(usv_frame_stream* e, long long ticket) {
    if (!e) return USV_ERR_INVALID_ARG;
    auto* s = find(e, ticket);
    if (!s) return USV_ERR_INVALID_ARG;
    if (!s->ready && hipEventSynchronize(s->done) != hipSuccess) return USV_ERR_HIP;
    s->ticket = -1;
    s->ready = false;
    return USV_OK;
}

usv_status usv_distance_expand_host(const uint8_t* disp, int W, int H, int disp_pitch, const double* lut,
                                    double* out, int out_pitch, int n_threads) {
    if (!disp || !lut || !out || W <= 0 || H <= 0 || disp_pitch < W || out_pitch < W || n_threads < 0)
        return USV_ERR_INVALID_ARG;
    const int nt = std::max(1, std::min(n_threads == 0 ? 1 : n_threads, H));
    const std::function<void(int)> rows = [&](int part) {
        const int y0 = (int)((long long)H * part / nt), y1 = (int)((long long)H * (part + 1) / nt);
        for (int y = y0; y < y1; ++y) {
            const uint8_t* __restrict__ d = disp + (size_t)y * disp_pitch;
            double* __restrict__ o = out + (size_t)y * out_pitch;
            for (int x = 0; x < W; ++x) o[x] = lut[d[x]];
        }
    };
    if (nt == 1) rows(0);
    else host_pool().run(nt, rows);
    return USV_OK;
}

}  // extern "C"
