// usv_sharded.hip -- one process driving several MI355X GPUs (include/usv.h,
// usv_sharded_*, usv_batch_sharded*).
//
// The reference's caller is one C++ process with camera threads
// (P/Main.cpp:1407-1420), so the multi-GPU entry is a C-ABI engine object,
// not a launcher: one device and RCCL communicator per GPU (ncclCommInitAll),
// a batch of independent frame pairs split into contiguous shards (pair i ->
// GPU i at batch = n), each GPU block-matching its shard with the batched
// kernel and no data-path exchange, then ONE collective: an ncclGather of the
// u8 disparity maps to devices[0] (rccl.h:745).  Root's own shard is computed
// in place into slot 0 of the gather buffer (RCCL's in-place gather), so it
// never moves.  Distance maps are a 256-entry table lookup of the disparity and
// are expanded on devices[0] after the gather instead of crossing xGMI (8x the
// bytes).
//
// Two slots of buffers and streams per GPU: usv_batch_sharded_submit enqueues a
// batch on one slot and returns, so batch k+1's H2D copies and kernels run
// while batch k's gather, distance expansion and D2H are still in flight on the
// other slot; usv_batch_sharded_wait completes a batch (results copied to the
// caller's host buffers in batch order).  usv_batch_sharded = submit + wait.
// The n > 1 path (per-GPU worker threads, the multi-rank gather, slot -> batch
// order) is exercised on hardware only with one GPU so far; usv_shard_slot is
// the slot mapping, unit-tested for n = 1..8 on the CPU.
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "usv.h"
#include "usv_host_pool.hpp"
#include "usv_kernels.hpp"

namespace {
constexpr int kSlots = 2;
}

struct usv_sharded_engine {
    int n = 0;
    std::vector<int> dev;
    std::vector<ncclComm_t> comm;
    int W = 0, H = 0, D = 0, w = 0, metric = 0, max_pairs = 0, per = 0;
    size_t frame = 0;  // W * H bytes: inputs and outputs are dense (pitch W)
    struct Slot {
        std::vector<hipStream_t> stream;  // per device
        std::vector<uint8_t*> L, R;       // per device: per * frame bytes each
        std::vector<uint8_t*> disp;       // per device: its send buffer (root: gathered + 0)
        uint8_t* gathered = nullptr;      // devices[0]: n * per * frame bytes
        double* dist = nullptr;           // devices[0]: max_pairs * frame doubles (lazy)
        uint8_t* hdisp = nullptr;         // pinned host copy of `gathered` (lazy)
        hipEvent_t done = nullptr;        // on devices[0]'s stream after the last step
        std::vector<hipEvent_t> h2d;      // per device: after its host-input copies (pageable sources)
        long long ticket = -1;            // batch in flight here, -1 = free
        int batch = 0;
        uint8_t* out_disp = nullptr;      // the caller's host outputs of that batch
        double* out_dist = nullptr;
        bool want_dist = false;
    };
    Slot slot[kSlots];
    long long next = 0;   // ticket of the next submit
    int last_done = -1;   // slot of the last completed batch (usv_sharded_outputs)
    // Batches completed implicitly (a submit or usv_sharded_input_buffers needed their slot) and not
    // waited for yet: usv_batch_sharded_wait(ticket) reports each one's own completion status.
    struct Retired {
        long long ticket;
        usv_status status;
    };
    std::vector<Retired> retired;
    // workers for the per-GPU input copies of host batches (n > 1), started on the first such batch and joined
    // by usv_sharded_destroy (usv_host_pool.hpp: per-call threads cost ~25-30 us each)
    usv::HostPool pool;
};

namespace {

usv_status nccl_st(ncclResult_t r) { return r == ncclSuccess ? USV_OK : USV_ERR_COMM; }

void shard(int batch, int n, int k, int* first, int* count) {
    const int base = batch / n, extra = batch % n;
    *first = k * base + std::min(k, extra);
    *count = base + (k < extra ? 1 : 0);
}

void release(usv_sharded_engine* e) {
    for (auto& s : e->slot)
        for (int k = 0; k < (int)s.stream.size(); ++k) {
            (void)hipSetDevice(e->dev[k]);
            if (s.stream[k]) (void)hipStreamSynchronize(s.stream[k]);
        }
    for (int k = 0; k < (int)e->dev.size(); ++k) {
        (void)hipSetDevice(e->dev[k]);
        if (k < (int)e->comm.size() && e->comm[k]) ncclCommDestroy(e->comm[k]);
        for (auto& s : e->slot) {
            if (k < (int)s.L.size()) (void)hipFree(s.L[k]);
            if (k < (int)s.R.size()) (void)hipFree(s.R[k]);
            if (k > 0 && k < (int)s.disp.size()) (void)hipFree(s.disp[k]);
            if (k < (int)s.h2d.size() && s.h2d[k]) (void)hipEventDestroy(s.h2d[k]);
            if (k == 0) {
                (void)hipFree(s.gathered);
                (void)hipFree(s.dist);
                (void)hipHostFree(s.hdisp);
                if (s.done) (void)hipEventDestroy(s.done);
            }
            if (k < (int)s.stream.size() && s.stream[k]) (void)hipStreamDestroy(s.stream[k]);
        }
    }
    delete e;
}

// Every stream of slot s drained (before reporting an error, or before the slot is reused): no
// copy or kernel of that batch may still read the caller's buffers or write the slot's.
usv_status drain(usv_sharded_engine* e, usv_sharded_engine::Slot& s) {
    usv_status st = USV_OK;
    for (int k = 0; k < e->n; ++k)
        if (hipSetDevice(e->dev[k]) != hipSuccess || hipStreamSynchronize(s.stream[k]) != hipSuccess) st = USV_ERR_HIP;
    return st;
}

usv_status complete(usv_sharded_engine* e, int si);

// Complete slot si's batch because its slot is needed again; its status is kept for the wait on its
// ticket (so a caller can tell a delivered batch from a failed one) instead of being reported by the
// call that needed the slot.  The record is unbounded (16 bytes per batch not waited for yet): dropping
// entries would turn a failed implicit completion into "never submitted"; a wait erases its entry.
void complete_implicit(usv_sharded_engine* e, int si) {
    const long long t = e->slot[si].ticket;
    const usv_status st = complete(e, si);
    e->retired.push_back({t, st});
}

usv_status submit(usv_sharded_engine* e, const uint8_t* L, const uint8_t* R, int batch, size_t pair_stride, int pitch,
                  uint8_t* disp, double* dist_cm, const double* lut_cm, bool want_dist, long long* ticket) {
    const int si = (int)(e->next % kSlots);
    usv_sharded_engine::Slot& s = e->slot[si];
    if (s.ticket >= 0) complete_implicit(e, si);  // both slots busy: finish the older batch first
    const bool host_in = L || R;
    const size_t frame = e->frame;
    const size_t shard_bytes = (size_t)e->per * frame;

    // 1. per GPU: inputs in (host batch -> its shard, or already resident), then one batched launch.
    //    Host batches: one persistent worker per GPU, so the pageable-host H2D copies of different GPUs overlap;
    //    resident inputs: launches only, issued in turn from this thread (no copy to overlap).
    std::vector<usv_status> st(e->n, USV_OK);
    auto work = [&](int k) {
        int first = 0, count = 0;
        shard(batch, e->n, k, &first, &count);
        if (hipSetDevice(e->dev[k]) != hipSuccess) { st[k] = USV_ERR_HIP; return; }
        hipStream_t hs = s.stream[k];
        if (count == 0) return;
        if (host_in) {
            if ((size_t)pitch == (size_t)e->W && pair_stride == frame) {
                // a dense batch: the shard's frames are one run per camera, one copy each
                const size_t src = (size_t)first * frame, n = (size_t)count * frame;
                if (hipMemcpyAsync(s.L[k], L + src, n, hipMemcpyHostToDevice, hs) != hipSuccess ||
                    hipMemcpyAsync(s.R[k], R + src, n, hipMemcpyHostToDevice, hs) != hipSuccess) {
                    st[k] = USV_ERR_HIP;
                    return;
                }
            } else {
                for (int b = 0; b < count; ++b) {
                    const size_t src = (size_t)(first + b) * pair_stride;
                    if (hipMemcpy2DAsync(s.L[k] + b * frame, e->W, L + src, pitch, e->W, e->H,
                                         hipMemcpyHostToDevice, hs) != hipSuccess ||
                        hipMemcpy2DAsync(s.R[k] + b * frame, e->W, R + src, pitch, e->W, e->H,
                                         hipMemcpyHostToDevice, hs) != hipSuccess) {
                        st[k] = USV_ERR_HIP;
                        return;
                    }
                }
            }
            if (hipEventRecord(s.h2d[k], hs) != hipSuccess) {
                st[k] = USV_ERR_HIP;
                return;
            }
        }
        st[k] = usv_sad_disparity_batch(s.L[k], s.R[k], count, frame, e->W, e->H, e->W, e->D, e->w, e->metric,
                                        s.disp[k], frame, e->W, nullptr, 0, 0, nullptr, hs);
        // The host inputs may be pageable, where an async copy need not have read its source when the
        // call returns: wait for the copies (not the kernel) so the caller may reuse L / R at once.
        if (host_in && hipEventSynchronize(s.h2d[k]) != hipSuccess && st[k] == USV_OK) st[k] = USV_ERR_HIP;
    };
    if (e->n == 1 || !host_in) {
        for (int k = 0; k < e->n; ++k) work(k);
    } else {
        e->pool.run(e->n, work);
    }
    for (usv_status x : st)
        if (x != USV_OK) {
            (void)drain(e, s);
            return x;
        }

    // 2. the one collective: every GPU's shard (padded to `per` pairs) -> devices[0], slot k at k * per.
    usv_status cst = nccl_st(ncclGroupStart());
    if (cst != USV_OK) {
        (void)drain(e, s);
        return cst;
    }
    for (int k = 0; k < e->n; ++k) {
        ncclResult_t r = ncclGather(s.disp[k], k == 0 ? s.gathered : nullptr, shard_bytes, ncclUint8, 0, e->comm[k],
                                    s.stream[k]);
        if (r != ncclSuccess) {
            (void)ncclGroupEnd();
            (void)drain(e, s);
            return USV_ERR_COMM;
        }
    }
    if ((cst = nccl_st(ncclGroupEnd())) != USV_OK) {
        (void)drain(e, s);
        return cst;
    }

    // 3. root: distance expansion in batch order (slot k holds pairs first_k ..), the gathered maps
    //    to pinned host memory; both asynchronous on root's stream of this slot.
    auto fail = [&](usv_status x) {
        (void)drain(e, s);
        return x;
    };
    if (hipSetDevice(e->dev[0]) != hipSuccess) return fail(USV_ERR_HIP);
    hipStream_t s0 = s.stream[0];
    if (want_dist && !s.dist && hipMalloc(&s.dist, (size_t)e->max_pairs * frame * sizeof(double)) != hipSuccess)
        return fail(USV_ERR_HIP);
    if (disp && !s.hdisp && hipHostMalloc(&s.hdisp, shard_bytes * e->n, hipHostMallocDefault) != hipSuccess)
        return fail(USV_ERR_HIP);
    for (int k = 0; k < e->n; ++k) {
        int first = 0, count = 0;
        shard(batch, e->n, k, &first, &count);
        if (count == 0 || !want_dist) continue;
        const usv_status d = usv_disparity_to_distance(s.gathered + (size_t)k * shard_bytes, e->W, e->H * count, e->W,
                                                       lut_cm, s.dist + (size_t)first * frame, e->W, s0);
        if (d != USV_OK) return fail(d);
    }
    if (disp && hipMemcpyAsync(s.hdisp, s.gathered, shard_bytes * e->n, hipMemcpyDeviceToHost, s0) != hipSuccess)
        return fail(USV_ERR_HIP);
    if (hipEventRecord(s.done, s0) != hipSuccess) return fail(USV_ERR_HIP);
    s.ticket = e->next++;
    s.batch = batch;
    s.out_disp = disp;
    s.out_dist = dist_cm;
    s.want_dist = want_dist;
    *ticket = s.ticket;
    return USV_OK;
}

// Finish slot si's batch: wait for it, copy its results to the caller's host buffers in batch order.
usv_status complete(usv_sharded_engine* e, int si) {
    usv_sharded_engine::Slot& s = e->slot[si];
    usv_status st = USV_OK;
    if (hipSetDevice(e->dev[0]) != hipSuccess || hipEventSynchronize(s.done) != hipSuccess) st = USV_ERR_HIP;
    if (drain(e, s) != USV_OK) st = USV_ERR_HIP;
    if (st == USV_OK) {
        const size_t frame = e->frame, shard_bytes = (size_t)e->per * frame;
        for (int k = 0; k < e->n && s.out_disp; ++k) {
            int first = 0, count = 0;
            shard(s.batch, e->n, k, &first, &count);
            std::memcpy(s.out_disp + (size_t)first * frame, s.hdisp + (size_t)k * shard_bytes, (size_t)count * frame);
        }
        if (s.out_dist && (hipSetDevice(e->dev[0]) != hipSuccess ||
                           hipMemcpy(s.out_dist, s.dist, (size_t)s.batch * frame * sizeof(double),
                                     hipMemcpyDeviceToHost) != hipSuccess))
            st = USV_ERR_HIP;
    }
    s.ticket = -1;
    e->last_done = si;
    return st;
}

// The caller's current device is restored on every exit path.
struct DeviceRestore {
    int prev = 0;
    bool ok = false;
    DeviceRestore() { ok = hipGetDevice(&prev) == hipSuccess; }
    ~DeviceRestore() {
        if (ok) (void)hipSetDevice(prev);
    }
};

}  // namespace

extern "C" {

usv_status usv_shard_range(int batch, int n_devices, int k, int* first, int* count) {
    if (!first || !count || batch < 0 || n_devices < 1 || k < 0 || k >= n_devices) return USV_ERR_INVALID_ARG;
    shard(batch, n_devices, k, first, count);
    return USV_OK;
}

usv_status usv_shard_slot(int batch, int n_devices, int per, int pair, long long* slot) {
    if (!slot || batch < 1 || n_devices < 1 || pair < 0 || pair >= batch || per < (batch + n_devices - 1) / n_devices)
        return USV_ERR_INVALID_ARG;
    for (int k = 0; k < n_devices; ++k) {
        int first = 0, count = 0;
        shard(batch, n_devices, k, &first, &count);
        if (pair >= first && pair < first + count) {
            *slot = (long long)k * per + (pair - first);
            return USV_OK;
        }
    }
    return USV_ERR_INVALID_ARG;
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
    DeviceRestore restore;
    auto* e = new usv_sharded_engine;
    e->n = n_devices;
    e->dev.assign(devices, devices + n_devices);
    e->W = W; e->H = H; e->D = D; e->w = w; e->metric = metric; e->max_pairs = max_pairs;
    e->per = (max_pairs + n_devices - 1) / n_devices;
    e->frame = (size_t)W * H;
    const size_t shard_bytes = (size_t)e->per * e->frame;
    for (auto& s : e->slot) {
        s.stream.assign(n_devices, nullptr);
        s.L.assign(n_devices, nullptr);
        s.R.assign(n_devices, nullptr);
        s.disp.assign(n_devices, nullptr);
        s.h2d.assign(n_devices, nullptr);
    }
    for (int k = 0; k < n_devices; ++k) {
        if (hipSetDevice(devices[k]) != hipSuccess) {
            release(e);
            return USV_ERR_HIP;
        }
        for (auto& s : e->slot) {
            if (hipStreamCreateWithFlags(&s.stream[k], hipStreamNonBlocking) != hipSuccess ||
                hipEventCreateWithFlags(&s.h2d[k], hipEventDisableTiming) != hipSuccess ||
                hipMalloc(&s.L[k], shard_bytes) != hipSuccess || hipMalloc(&s.R[k], shard_bytes) != hipSuccess) {
                release(e);
                return USV_ERR_HIP;
            }
            if (k == 0) {
                if (hipMalloc(&s.gathered, shard_bytes * n_devices) != hipSuccess ||
                    hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess) {
                    release(e);
                    return USV_ERR_HIP;
                }
                s.disp[0] = s.gathered;  // in-place gather: root's slot 0
            } else if (hipMalloc(&s.disp[k], shard_bytes) != hipSuccess) {
                release(e);
                return USV_ERR_HIP;
            }
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
    DeviceRestore restore;
    release(e);
    return USV_OK;
}

usv_status usv_sharded_input_buffers(usv_sharded_engine* e, int k, uint8_t** L, uint8_t** R) {
    if (!e || k < 0 || k >= e->n || !L || !R) return USV_ERR_INVALID_ARG;
    const int si = (int)(e->next % kSlots);  // the slot the next submit uses
    if (e->slot[si].ticket >= 0) {
        // that slot's batch may still be reading these buffers: complete it first (its status stays
        // with its ticket), so filling them cannot race with the running batch
        DeviceRestore restore;
        complete_implicit(e, si);
    }
    const auto& s = e->slot[si];
    *L = s.L[k];
    *R = s.R[k];
    return USV_OK;
}

usv_status usv_sharded_outputs(usv_sharded_engine* e, const uint8_t** disp, const double** dist_cm) {
    if (!e || !disp) return USV_ERR_INVALID_ARG;
    const auto& s = e->slot[e->last_done >= 0 ? e->last_done : 0];
    *disp = s.gathered;
    if (dist_cm) *dist_cm = s.dist;
    return USV_OK;
}

usv_status usv_batch_sharded_submit(usv_sharded_engine* e, const uint8_t* L, const uint8_t* R, int batch,
                                    size_t pair_stride, int pitch, uint8_t* disp, double* dist_cm,
                                    const double* lut_cm, int with_distance, long long* ticket) {
    if (!e || !ticket || batch < 1 || batch > e->max_pairs) return USV_ERR_INVALID_ARG;
    const bool host_in = L || R;
    if (host_in && (!L || !R || pitch < e->W || (batch > 1 && pair_stride < (size_t)pitch * e->H)))
        return USV_ERR_INVALID_ARG;
    if ((with_distance || dist_cm) && !lut_cm) return USV_ERR_INVALID_ARG;
    DeviceRestore restore;
    if (!restore.ok) return USV_ERR_HIP;
    return submit(e, L, R, batch, pair_stride, pitch, disp, dist_cm, lut_cm, with_distance || dist_cm, ticket);
}

usv_status usv_batch_sharded_wait(usv_sharded_engine* e, long long ticket) {
    if (!e || ticket < 0) return USV_ERR_INVALID_ARG;
    const int si = (int)(ticket % kSlots);
    if (e->slot[si].ticket != ticket) {
        // completed implicitly when its slot was needed: report that completion's status once
        for (auto it = e->retired.begin(); it != e->retired.end(); ++it)
            if (it->ticket == ticket) {
                const usv_status st = it->status;
                e->retired.erase(it);
                return st;
            }
        return USV_ERR_INVALID_ARG;
    }
    DeviceRestore restore;
    return complete(e, si);
}

usv_status usv_batch_sharded(usv_sharded_engine* e, const uint8_t* L, const uint8_t* R, int batch,
                             size_t pair_stride, int pitch, uint8_t* disp, double* dist_cm,
                             const double* lut_cm, int with_distance) {
    long long t = -1;
    const usv_status st = usv_batch_sharded_submit(e, L, R, batch, pair_stride, pitch, disp, dist_cm, lut_cm,
                                                   with_distance, &t);
    if (st != USV_OK) return st;
    return usv_batch_sharded_wait(e, t);
}

}  // extern "C"
