// usv_tiles.hpp -- the block-match launches' work map (workgroup -> x-tile, pair, output rows) and its
// per-geometry device table; shared by usv_sad_pair.hip and usv_sad_group.hip.  Internal to libusv.so.
#pragma once
#include <hip/hip_runtime.h>

#include <array>
#include <map>
#include <mutex>
#include <vector>

#include "usv_band.hpp"
#include "usv_kernels.hpp"

namespace usv {
namespace {

// Work map of one launch (the sad_fast_kernel map: XCD-contiguous tile runs, generation-weighted
// bands): workgroup `lin` of `total` -> its x-tile, pair and output rows.  Host and device run the
// same function: the launcher tabulates it once per launch geometry (tile_table), so a workgroup
// normally reads its span with one scalar load instead of ~500 SALU of divisions and band sums.
struct TileSpan {
    unsigned xt, pair;
    int y_begin, y_end;
};
__host__ __device__ __forceinline__ TileSpan tile_span(unsigned lin, unsigned total, int n_xt, int m, int extra,
                                                      int gen_g, unsigned weights, int H) {
    const unsigned xcd = lin & 7u, base = total >> 3, rem = total & 7u;
    const unsigned tile = xcd * base + (xcd < rem ? xcd : rem) + (lin >> 3);
    const unsigned nxt = (unsigned)n_xt, per_pair = nxt * (unsigned)m;
    const bool past = tile >= per_pair && extra > 0;
    const unsigned col_xt = past ? tile - per_pair : tile % nxt;
    const unsigned s = past ? (unsigned)m : (tile / nxt) % (unsigned)m;
    const unsigned pair = past ? 0u : tile / per_pair;
    const unsigned m_col = (unsigned)m + (col_xt < (unsigned)extra ? 1u : 0u);
    const unsigned long_run = base + 1u, split = rem * long_run;
    const BandSpan bs = band_span(pair, per_pair, nxt, col_xt, s, m_col, base, long_run, split,
                                  (unsigned)gen_g, weights);
    return TileSpan{col_xt, pair, (int)((unsigned long long)H * bs.pre / bs.tot),
                    (int)((unsigned long long)H * (bs.pre + bs.own) / bs.tot)};
}

// The work map of a launch geometry as a device table (one uint2 per workgroup), built on the host
// from tile_span and uploaded once per geometry and device; immutable afterwards.  The upload is
// enqueued on the launch's own stream (a synchronous hipMemcpy would go through the legacy stream, which
// another thread's global-mode stream capture forbids) and ordered by an event: the launch behind it on
// the same stream needs nothing more, a launch on another stream waits on the event until it has
// completed -- no host stall, and the cache lock is never held across a HIP call that can block.
// nullptr (the kernel computes its span itself) while the stream is being captured into a graph and the
// table is not resident yet, or when a field does not fit 16 bits.  Tables live for the process (a few
// KB per geometry).
struct TileTableEntry {
    uint2* d = nullptr;
    hipEvent_t ready_ev = nullptr;
    hipStream_t upload_stream = nullptr;
    bool ready = false;
    std::vector<uint2> host;  // the upload's source, kept until the process ends
};

inline const uint2* tile_table(int kind, int variant, const MatchArgs& a, int n_xt, int m, int extra, int gen_g,
                               unsigned weights, unsigned total, hipStream_t s) {
    if (a.H > 0xFFFF || n_xt > 0xFFFF || a.batch > 0xFFFF) return nullptr;
    // the launch's device is the stream's (the caller's current device may be another one)
    int dev = 0, cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return nullptr;
    dev = cur;
    if (s != nullptr && hipStreamGetDevice(s, &dev) != hipSuccess) return nullptr;
    const std::array<long long, 11> key{dev, kind, variant, a.W, a.H, a.batch, n_xt, m, extra,
                                        ((long long)gen_g << 32) | weights, total};
    static std::mutex mu;
    static std::map<std::array<long long, 11>, TileTableEntry*> cache;
    TileTableEntry* hit = nullptr;
    {
        std::lock_guard<std::mutex> lock(mu);
        auto it = cache.find(key);
        if (it != cache.end()) {
            hit = it->second;
            if (!hit->ready && hipEventQuery(hit->ready_ev) == hipSuccess) hit->ready = true;
            if (hit->ready || hit->upload_stream == s) return hit->d;  // the steady state: no HIP call
        }
    }
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    // a table whose upload (on another stream) may still be in flight: order this stream behind it
    if (hit) return hipStreamWaitEvent(s, hit->ready_ev, 0) == hipSuccess ? hit->d : nullptr;
    auto* e = new TileTableEntry;
    e->host.resize(total);
    for (unsigned lin = 0; lin < total; ++lin) {
        const TileSpan sp = tile_span(lin, total, n_xt, m, extra, gen_g, weights, a.H);
        e->host[lin] = make_uint2(sp.xt | (sp.pair << 16), (unsigned)sp.y_begin | ((unsigned)sp.y_end << 16));
    }
    e->upload_stream = s;
    if (dev != cur && hipSetDevice(dev) != hipSuccess) {
        delete e;
        return nullptr;
    }
    bool ok = hipMalloc(&e->d, total * sizeof(uint2)) == hipSuccess &&
              hipEventCreateWithFlags(&e->ready_ev, hipEventDisableTiming) == hipSuccess &&
              hipMemcpyAsync(e->d, e->host.data(), total * sizeof(uint2), hipMemcpyHostToDevice, s) == hipSuccess &&
              hipEventRecord(e->ready_ev, s) == hipSuccess;
    if (!ok) {
        // nothing may still read the host copy or write the table when they are freed
        (void)hipStreamSynchronize(s);
        if (e->ready_ev) (void)hipEventDestroy(e->ready_ev);
        if (e->d) (void)hipFree(e->d);
        delete e;
        if (dev != cur) (void)hipSetDevice(cur);
        return nullptr;
    }
    if (dev != cur) (void)hipSetDevice(cur);
    std::lock_guard<std::mutex> lock(mu);
    // (another thread may have uploaded the same geometry meanwhile: then ours is not cached but stays
    // alive -- its copy may still be in flight; a few KB, once per race -- and this launch, ordered
    // behind our upload on this stream, uses it)
    cache.emplace(key, e);
    return e->d;
}

}  // namespace
}  // namespace usv
