// usv_sharded.hip -- one process driving several MI355X GPUs (include/usv.h,
// usv_sharded_*, usv_batch_sharded).
//
// The reference's caller is one C++ process with camera threads
// (P/Main.cpp:1407-1420), so the multi-GPU entry is a C-ABI engine object,
// not a launcher: one device, HIP stream and RCCL communicator per GPU
// (ncclCommInitAll), a batch of independent frame pairs split into contiguous
// shards (pair i -> GPU i at batch = n), each GPU block-matching its shard with
// the batched kernel and no data-path exchange, then ONE collective: an
// ncclGather of the u8 disparity maps to devices[0] (rccl.h:745).  Root's own
// shard is computed in place into slot 0 of the gather buffer (RCCL's in-place
// gather), so it never moves.  Distance maps are a 256-entry table lookup of
// the disparity and are expanded on devices[0] after the gather instead of
// crossing xGMI (8x the bytes).
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "usv.h"
#include "usv_kernels.hpp"

struct usv_sharded_engine {
    int n = 0;
    std::vector<int> dev;
    std::vector<hipStream_t> stream;
    std::vector<ncclComm_t> comm;
    int W = 0, H = 0, D = 0, w = 0, metric = 0, max_pairs = 0, per = 0;
    size_t frame = 0;                   // W * H bytes: inputs and outputs are dense (pitch W)
    std::vector<uint8_t*> L, R;         // per device: per * frame bytes each
    std::vector<uint8_t*> disp;         // per device: its send buffer (root: gathered + 0)
    uint8_t* gathered = nullptr;        // devices[0]: n * per * frame bytes
    double* dist = nullptr;             // devices[0]: max_pairs * frame doubles (lazy)
};

namespace {

usv_status nccl_st(ncclResult_t r) { return r == ncclSuccess ? USV_OK : USV_ERR_COMM; }

void shard(int batch, int n, int k, int* first, int* count) {
    const int base = batch / n, extra = batch % n;
    *first = k * base + std::min(k, extra);
    *count = base + (k < extra ? 1 : 0);
}

usv_status run_batch(usv_sharded_engine* e, const uint8_t* L, const uint8_t* R, int batch, size_t pair_stride,
                     int pitch, uint8_t* disp, double* dist_cm, const double* lut_cm, bool want_dist);

void release(usv_sharded_engine* e) {
    for (int k = 0; k < (int)e->dev.size(); ++k) {
        (void)hipSetDevice(e->dev[k]);
        if (k < (int)e->comm.size() && e->comm[k]) ncclCommDestroy(e->comm[k]);
        if (k < (int)e->L.size()) (void)hipFree(e->L[k]);
        if (k < (int)e->R.size()) (void)hipFree(e->R[k]);
        if (k > 0 && k < (int)e->disp.size()) (void)hipFree(e->disp[k]);
        if (k == 0) {
            (void)hipFree(e->gathered);
            (void)hipFree(e->dist);
        }
        if (k < (int)e->stream.size() && e->stream[k]) (void)hipStreamDestroy(e->stream[k]);
    }
    delete e;
}

}  // namespace

extern "C" {

usv_status usv_shard_range(int batch, int n_devices, int k, int* first, int* count) {
    if (!first || !count || batch < 0 || n_devices < 1 || k < 0 || k >= n_devices) return USV_ERR_INVALID_ARG;
    shard(batch, n_devices, k, first, count);
    return USV_OK;
}

usv_status usv_sharded_create(const int* devices, int n_devices, int max_pairs, int W, int H, int D, int w,
                              int metric, usv_sharded_engine** out) {
    if (!out) return USV_ERR_INVALID_ARG;
    *out = nullptr;
    if (!devices || n_devices < 1 || max_pairs < 1 || W <= 0 || H <= 0) return USV_ERR_INVALID_ARG;
    if (D < 1 || D > 256 || w < 1 || w > 63 || (w & 1) == 0) return USV_ERR_UNSUPPORTED;
    if (metric != USV_METRIC_SAD && metric != USV_METRIC_SSD) return USV_ERR_UNSUPPORTED;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return USV_ERR_NO_DEVICE;
    for (int k = 0; k < n_devices; ++k) {
        if (devices[k] < 0 || devices[k] >= count) return USV_ERR_INVALID_ARG;
        for (int j = 0; j < k; ++j)
            if (devices[j] == devices[k]) return USV_ERR_INVALID_ARG;  // one rank per GPU (RCCL)
    }
    auto* e = new usv_sharded_engine;
    e->n = n_devices;
    e->dev.assign(devices, devices + n_devices);
    e->W = W; e->H = H; e->D = D; e->w = w; e->metric = metric; e->max_pairs = max_pairs;
    e->per = (max_pairs + n_devices - 1) / n_devices;
    e->frame = (size_t)W * H;
    const size_t shard_bytes = (size_t)e->per * e->frame;
    e->stream.assign(n_devices, nullptr);
    e->L.assign(n_devices, nullptr);
    e->R.assign(n_devices, nullptr);
    e->disp.assign(n_devices, nullptr);
    for (int k = 0; k < n_devices; ++k) {
        if (hipSetDevice(devices[k]) != hipSuccess ||
            hipStreamCreateWithFlags(&e->stream[k], hipStreamNonBlocking) != hipSuccess ||
            hipMalloc(&e->L[k], shard_bytes) != hipSuccess || hipMalloc(&e->R[k], shard_bytes) != hipSuccess) {
            release(e);
            return USV_ERR_HIP;
        }
        if (k == 0) {
            if (hipMalloc(&e->gathered, shard_bytes * n_devices) != hipSuccess) {
                release(e);
                return USV_ERR_HIP;
            }
            e->disp[0] = e->gathered;  // in-place gather: root's slot 0
        } else if (hipMalloc(&e->disp[k], shard_bytes) != hipSuccess) {
            release(e);
            return USV_ERR_HIP;
        }
    }
    e->comm.assign(n_devices, nullptr);
    if (ncclCommInitAll(e->comm.data(), n_devices, devices) != ncclSuccess) {
        e->comm.assign(n_devices, nullptr);
        release(e);
        return USV_ERR_COMM;
    }
    *out = e;
    return USV_OK;
}

usv_status usv_sharded_destroy(usv_sharded_engine* e) {
    if (!e) return USV_ERR_INVALID_ARG;
    for (int k = 0; k < e->n; ++k) {
        (void)hipSetDevice(e->dev[k]);
        (void)hipStreamSynchronize(e->stream[k]);
    }
    release(e);
    return USV_OK;
}

usv_status usv_sharded_input_buffers(usv_sharded_engine* e, int k, uint8_t** L, uint8_t** R) {
    if (!e || k < 0 || k >= e->n || !L || !R) return USV_ERR_INVALID_ARG;
    *L = e->L[k];
    *R = e->R[k];
    return USV_OK;
}

usv_status usv_sharded_outputs(usv_sharded_engine* e, const uint8_t** disp, const double** dist_cm) {
    if (!e || !disp) return USV_ERR_INVALID_ARG;
    *disp = e->gathered;
    if (dist_cm) *dist_cm = e->dist;
    return USV_OK;
}

usv_status usv_batch_sharded(usv_sharded_engine* e, const uint8_t* L, const uint8_t* R, int batch,
                             size_t pair_stride, int pitch, uint8_t* disp, double* dist_cm,
                             const double* lut_cm, int with_distance) {
    if (!e || batch < 1 || batch > e->max_pairs) return USV_ERR_INVALID_ARG;
    const bool host_in = L || R;
    if (host_in && (!L || !R || pitch < e->W || (batch > 1 && pair_stride < (size_t)pitch * e->H)))
        return USV_ERR_INVALID_ARG;
    if ((with_distance || dist_cm) && !lut_cm) return USV_ERR_INVALID_ARG;
    int caller_dev = 0;
    if (hipGetDevice(&caller_dev) != hipSuccess) return USV_ERR_HIP;
    usv_status rc = run_batch(e, L, R, batch, pair_stride, pitch, disp, dist_cm, lut_cm, with_distance || dist_cm);
    (void)hipSetDevice(caller_dev);  // the caller's current device is left as it was
    return rc;
}

}  // extern "C"

namespace {

usv_status run_batch(usv_sharded_engine* e, const uint8_t* L, const uint8_t* R, int batch, size_t pair_stride,
                     int pitch, uint8_t* disp, double* dist_cm, const double* lut_cm, bool want_dist) {
    const bool host_in = L || R;
    const size_t frame = e->frame;
    const size_t shard_bytes = (size_t)e->per * frame;

    // 1. per GPU: inputs in (host batch -> its shard, or already resident), then one batched launch.
    //    One host thread per GPU so the pageable-host H2D copies of different GPUs overlap.
    std::vector<usv_status> st(e->n, USV_OK);
    auto work = [&](int k) {
        int first = 0, count = 0;
        shard(batch, e->n, k, &first, &count);
        if (hipSetDevice(e->dev[k]) != hipSuccess) { st[k] = USV_ERR_HIP; return; }
        hipStream_t s = e->stream[k];
        if (count == 0) return;
        if (host_in) {
            for (int b = 0; b < count; ++b) {
                const size_t src = (size_t)(first + b) * pair_stride;
                if (hipMemcpy2DAsync(e->L[k] + b * frame, e->W, L + src, pitch, e->W, e->H, hipMemcpyHostToDevice,
                                     s) != hipSuccess ||
                    hipMemcpy2DAsync(e->R[k] + b * frame, e->W, R + src, pitch, e->W, e->H, hipMemcpyHostToDevice,
                                     s) != hipSuccess) {
                    st[k] = USV_ERR_HIP;
                    return;
                }
            }
        }
        st[k] = usv_sad_disparity_batch(e->L[k], e->R[k], count, frame, e->W, e->H, e->W, e->D, e->w, e->metric,
                                        e->disp[k], frame, e->W, nullptr, 0, 0, nullptr, s);
    };
    if (e->n == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int k = 0; k < e->n; ++k) th.emplace_back(work, k);
        for (auto& t : th) t.join();
    }
    for (usv_status s : st)
        if (s != USV_OK) return s;

    // 2. the one collective: every GPU's shard (padded to `per` pairs) -> devices[0], slot k at k * per.
    usv_status cst = nccl_st(ncclGroupStart());
    if (cst != USV_OK) return cst;
    for (int k = 0; k < e->n; ++k) {
        ncclResult_t r = ncclGather(e->disp[k], k == 0 ? e->gathered : nullptr, shard_bytes, ncclUint8, 0, e->comm[k],
                                    e->stream[k]);
        if (r != ncclSuccess) {
            (void)ncclGroupEnd();
            return USV_ERR_COMM;
        }
    }
    if ((cst = nccl_st(ncclGroupEnd())) != USV_OK) return cst;

    // 3. root: distance expansion and copies out, in batch order (slot k holds pairs first_k ..).
    if (hipSetDevice(e->dev[0]) != hipSuccess) return USV_ERR_HIP;
    hipStream_t s0 = e->stream[0];
    if (want_dist && !e->dist && hipMalloc(&e->dist, (size_t)e->max_pairs * frame * sizeof(double)) != hipSuccess)
        return USV_ERR_HIP;
    for (int k = 0; k < e->n; ++k) {
        int first = 0, count = 0;
        shard(batch, e->n, k, &first, &count);
        if (count == 0) continue;
        const uint8_t* slot = e->gathered + (size_t)k * shard_bytes;
        if (want_dist) {
            usv_status d = usv_disparity_to_distance(slot, e->W, e->H * count, e->W, lut_cm,
                                                     e->dist + (size_t)first * frame, e->W, s0);
            if (d != USV_OK) return d;
            if (dist_cm && hipMemcpyAsync(dist_cm + (size_t)first * frame, e->dist + (size_t)first * frame,
                                          (size_t)count * frame * sizeof(double), hipMemcpyDeviceToHost,
                                          s0) != hipSuccess)
                return USV_ERR_HIP;
        }
        if (disp && hipMemcpyAsync(disp + (size_t)first * frame, slot, (size_t)count * frame, hipMemcpyDeviceToHost,
                                   s0) != hipSuccess)
            return USV_ERR_HIP;
    }
    for (int k = 0; k < e->n; ++k) {
        if (hipSetDevice(e->dev[k]) != hipSuccess || hipStreamSynchronize(e->stream[k]) != hipSuccess)
            return USV_ERR_HIP;
    }
    return USV_OK;
}

}  // namespace
