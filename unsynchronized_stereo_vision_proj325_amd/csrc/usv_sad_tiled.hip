// usv_sad_tiled.hip -- sliding-window SAD / SSD block match for every shape the
// fast kernels do not take: SSD, any width (W % 4 != 0, W < 48), any pitch or
// base alignment, windows up to 31 x 31.  Same spec, border rule and tie rule
// as oracle/sad_oracle.c; integer arithmetic only, so it
// is bit-exact with the oracle by construction.
//
// Mapping:
//   * lane = disparity: wave v of a workgroup owns d = 64 v + l, the L operand
//     is the same for the whole wave (broadcast LDS reads), R is gathered per
//     lane.  Lanes past D - 1 replay the last valid disparity.
//   * one workgroup = one x-tile of K = 32 output columns x one band of rows.
//     Vertical-first running sums: per input column c of the tile (+ halo) a
//     lane keeps V[c] = sum over the w window rows of cost(L, R), updated per
//     output row by the entering row and MINUS the leaving row, which is
//     recomputed from the staged rows instead of being stored (no w-deep
//     register ring, so any w <= 31 fits and the u32 SSD sums need no packing).
//     The row-window sum then slides across the tile: H(x+1) = H(x) + V(x+w) - V(x).
//   * rows arrive by LDS-DMA (global_load_lds_ubyte: one zero-extended byte per
//     dword) into a per-wave ring of w + 1 + PD row slots; each slot holds the
//     wave's R span twice (shifted by one entry, so every lane's reads start
//     8-byte aligned: ds_read_b64) and the L span once.  Byte DMAs take any
//     pitch and base alignment.
//   * argmin: keys (cost << 6) | lane, transposed through LDS 16 pixels at a
//     time (lane 4p + q reduces 16 keys of pixel p), two quad DPP rounds; the
//     waves' minima meet in LDS every CH rows, where the smallest (cost, d)
//     wins (ties -> smallest d).
#include <utility>

#include "usv_kernels.hpp"

namespace usv {
namespace {

constexpr int kTK = 32;        // output columns per x-tile
constexpr int kTPD = 2;        // rows in flight ahead of the newest row computed
constexpr int kTCH = 8;        // output rows per cross-wave combine
constexpr int kTSpan = 128;    // R entries per copy (K + 2r + 63 <= 125 for r <= 15)
constexpr int kTSlot = 2 * kTSpan + 64;  // u32 entries per ring slot: R copy A, R copy B, L

__device__ __forceinline__ void tdma(const uint8_t* row, uint32_t voff, uint32_t m0) {
    // one byte per lane -> LDS dword at M0 + 4 * lane (GFX9: one wait state after the M0 write)
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_ubyte %0, %1"
                 :: "v"(voff), "s"(row), "s"(m0) : "memory", "m0");
}
template <int N>
__device__ __forceinline__ void t_wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ uint32_t t_lds_addr(const uint32_t* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t*)p;
}
template <int CTRL>
__device__ __forceinline__ uint32_t tdpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)0, (int)v, CTRL, 0xF, 0xF, false);
}

// per-element cost, as an update of V: + cost(new) - cost(old)
template <int METRIC>
__device__ __forceinline__ uint32_t cost_update(uint32_t v, uint32_t ln, uint32_t rn, uint32_t lo, uint32_t ro) {
    if constexpr (METRIC == 0) {
        return __builtin_amdgcn_sad_u8(ln, rn, v) - __builtin_amdgcn_sad_u8(lo, ro, 0u);
    } else {
        const int dn = (int)ln - (int)rn, dold = (int)lo - (int)ro;
        return (uint32_t)((int)v + __mul24(dn, dn) - __mul24(dold, dold));
    }
}
template <int METRIC>
__device__ __forceinline__ uint32_t cost_add(uint32_t v, uint32_t ln, uint32_t rn) {
    if constexpr (METRIC == 0) {
        return __builtin_amdgcn_sad_u8(ln, rn, v);
    } else {
        const int dn = (int)ln - (int)rn;
        return (uint32_t)((int)v + __mul24(dn, dn));
    }
}

struct TiledPlan {
    int n_xt;  // x-tiles per pair
    int m;     // bands per column
    int nb;    // ring slots per wave (w + 1 + kTPD)
};

template <int METRIC, int RAD>
__global__ __launch_bounds__(256) void sad_tiled_kernel(MatchArgs a, TiledPlan P) {
    constexpr int K = kTK, WIN = 2 * RAD + 1, NPOS = K + 2 * RAD;
    constexpr int NPV = (NPOS + 3) / 4 * 4;  // columns rounded up to whole uint4 L reads
    static_assert(K + 2 * RAD + 63 <= kTSpan, "R span fits one copy");
    static_assert(NPOS <= 64, "L span is one DMA");
    extern __shared__ __attribute__((aligned(16))) uint32_t tsm[];
    const int NW = (int)(blockDim.x >> 6);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int NB = P.nb;
    // LDS carve: per-wave ring, per-wave transpose buffer (16 x 64), combine (2 x CH x NW x K)
    uint32_t* ring = tsm + wave * NB * kTSlot;
    uint32_t* tb = tsm + NW * NB * kTSlot + wave * 16 * 64;
    uint32_t* comb = tsm + NW * NB * kTSlot + NW * 16 * 64;
    double* lut_s = reinterpret_cast<double*>(comb + 2 * kTCH * NW * K);
    if (a.dist)
        for (int i = threadIdx.x; i < 256; i += NW * 64) lut_s[i] = a.lut[i];
    __syncthreads();

    // work map: tile = (pair, band, x-tile), x fastest; XCD k takes the k-th contiguous run
    const unsigned total = gridDim.x, lin = blockIdx.x;
    const unsigned xcd = lin & 7u, base = total >> 3, rem = total & 7u;
    const unsigned tile = xcd * base + min(xcd, rem) + (lin >> 3);
    const int xt = (int)(tile % (unsigned)P.n_xt);
    const int band = (int)((tile / (unsigned)P.n_xt) % (unsigned)P.m);
    const size_t pair = tile / ((unsigned)P.n_xt * (unsigned)P.m);
    const int x0 = a.W >= K ? min(xt * K, a.W - K) : 0;
    const int y_begin = (int)((long)a.H * band / P.m), y_end = (int)((long)a.H * (band + 1) / P.m);
    const uint8_t* L = a.L + pair * a.pair_stride;
    const uint8_t* R = a.R + pair * a.pair_stride;
    uint8_t* disp = a.disp + pair * a.disp_stride;
    double* dist = a.dist ? a.dist + pair * a.dist_stride : nullptr;
    if (y_end <= y_begin) return;  // uniform over the workgroup

    // lane l of wave v: d = 64 v + l, lanes past D - 1 replay the last valid one
    const int lmax = min(63, a.D - 1 - 64 * wave);
    const int l_eff = min(lane, lmax);
    const int Wm1 = a.W - 1, Hm1 = a.H - 1;
    const int cbase = x0 - RAD - (64 * wave + 63);  // column of R copy-A entry 0 of this wave
    uint32_t offA[2], offB[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        offA[q] = (uint32_t)min(max(cbase + 64 * q + lane, 0), Wm1);
        offB[q] = (uint32_t)min(max(cbase + 64 * q + lane + 1, 0), Wm1);
    }
    const uint32_t offL = (uint32_t)min(max(x0 - RAD + lane, 0), Wm1);
    const uint32_t rbase = t_lds_addr(ring);
    const int y0 = y_begin - RAD;  // input row t = 0
    auto issue_row = [&](int t, int slot) {
        const int y = min(max(y0 + t, 0), Hm1);
        const uint8_t* rr = R + (size_t)y * a.pitch;
        const uint8_t* lr = L + (size_t)y * a.pitch;
        const uint32_t sb = rbase + 4u * (uint32_t)(slot * kTSlot);
        tdma(rr, offA[0], sb);
        tdma(rr, offA[1], sb + 4u * 64);
        tdma(rr, offB[0], sb + 4u * kTSpan);
        tdma(rr, offB[1], sb + 4u * (kTSpan + 64));
        tdma(lr, offL, sb + 4u * 2 * kTSpan);
    };
    constexpr int NDMA = 5;
    // this lane's first R entry: 63 - l_eff, read from the copy where it is even
    const int e0 = 63 - l_eff;
    const int roff = (e0 & 1) ? kTSpan + e0 - 1 : e0;

    // transposed reads: lane m = 4p + q reads words 64 p + 16 q .. + 15 in the rotated order (j + p) & 3
    uint32_t rd[4];
    {
        const int p = lane >> 2, q = lane & 3;
#pragma unroll
        for (int j = 0; j < 4; ++j) rd[j] = (uint32_t)(16 * p + 4 * q + ((j + p) & 3));
    }

    uint32_t V[NPOS];
#pragma unroll
    for (int j = 0; j < NPOS; ++j) V[j] = 0;

    // one row step: V += cost(row tn) [- cost(row to)], then keys of the K outputs -> comb slot
    auto load_L = [&](const uint32_t* slot, uint32_t (&Lv)[NPV]) {
        const uint4* lp = reinterpret_cast<const uint4*>(slot + 2 * kTSpan);
#pragma unroll
        for (int k = 0; k < NPV / 4; ++k) {
            const uint4 v = lp[k];
            Lv[4 * k] = v.x; Lv[4 * k + 1] = v.y; Lv[4 * k + 2] = v.z; Lv[4 * k + 3] = v.w;
        }
    };
    auto load_R = [&](const uint32_t* slot, uint32_t (&Rv)[NPV]) {
        const uint2* rp = reinterpret_cast<const uint2*>(slot + roff);
#pragma unroll
        for (int k = 0; k < NPV / 2; ++k) {
            const uint2 v = rp[k];
            Rv[2 * k] = v.x; Rv[2 * k + 1] = v.y;
        }
    };

    int cb = 0, y_chunk = y_begin, filled = 0;
    auto flush = [&](int rows) {
        if (NW > 1) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const uint32_t* cs = comb + cb * kTCH * NW * K;
        for (int i = threadIdx.x; i < rows * K; i += NW * 64) {
            const int row = i / K, p = i - row * K;
            uint64_t best = ~0ull;
            for (int v = 0; v < NW; ++v) {
                const uint32_t key = cs[(row * NW + v) * K + p];
                const uint64_t c = ((uint64_t)(key >> 6) << 8) | (uint64_t)(64 * v + (key & 63u));
                best = c < best ? c : best;
            }
            const int x = x0 + p;
            if (x < a.W) {
                const uint32_t dv = (uint32_t)(best & 0xFFu);
                const size_t y = (size_t)(y_chunk + row);
                disp[y * a.disp_pitch + x] = (uint8_t)dv;
                if (dist) dist[y * a.dist_pitch + x] = lut_s[dv];
            }
        }
        y_chunk += rows;
        cb ^= 1;
    };
    auto emit = [&]() {
        uint32_t* cs = comb + cb * kTCH * NW * K + (filled * NW + wave) * K;
        // the horizontal window slides over V; keys in two halves of 16 pixels
        uint32_t h = 0;
#pragma unroll
        for (int j = 0; j < WIN; ++j) h += V[j];
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            uint32_t key[16];
#pragma unroll
            for (int p = 0; p < 16; ++p) {
                const int x = 16 * half + p;
                key[p] = (h << 6) | (uint32_t)l_eff;
                if (x + 1 < K) h = h + V[x + WIN] - V[x];
            }
#pragma unroll
            for (int p = 0; p < 16; ++p) tb[64 * p + lane] = key[p];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            uint32_t v[16];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint4 q = reinterpret_cast<const uint4*>(tb)[rd[j]];
                v[4 * j] = q.x; v[4 * j + 1] = q.y; v[4 * j + 2] = q.z; v[4 * j + 3] = q.w;
            }
            uint32_t m0 = min(min(v[0], v[1]), v[2]), m1 = min(min(v[3], v[4]), v[5]);
            uint32_t m2 = min(min(v[6], v[7]), v[8]), m3 = min(min(v[9], v[10]), v[11]);
            uint32_t m4 = min(min(v[12], v[13]), v[14]);
            m0 = min(min(m0, m1), m2);
            m3 = min(min(m3, m4), v[15]);
            uint32_t m = min(m0, m3);
            m = min(m, tdpp<0x4E>(m));  // quad_perm [2,3,0,1]
            m = min(m, tdpp<0xB1>(m));  // quad_perm [1,0,3,2]
            // the next half's stores must not pass this half's reads (in-order LDS queue)
            if ((lane & 3) == 0) cs[16 * half + (lane >> 2)] = m;
        }
        if (++filled == kTCH) {
            flush(kTCH);
            filled = 0;
        }
    };

    // prologue: rows 0 .. PD-1 in flight.  Ring slot of input row t = t mod NB, kept as counters.
#pragma unroll
    for (int t = 0; t < kTPD; ++t) issue_row(t, t);
    auto wrap = [&](int i) { return i + 1 == NB ? 0 : i + 1; };
    int s_new = 0, s_old = 0, s_pf = kTPD;  // slots of rows tn, k - 1 and tn + PD
    const int nout = y_end - y_begin;
    // warm-up: V = sum of rows 0 .. w-1
    for (int t = 0; t < WIN; ++t) {
        t_wait_vmcnt<(kTPD - 1) * NDMA>();
        issue_row(t + kTPD, s_pf);
        s_pf = wrap(s_pf);
        const uint32_t* sn = ring + s_new * kTSlot;
        uint32_t Lv[NPV], Rv[NPV];
        load_L(sn, Lv);
        load_R(sn, Rv);
#pragma unroll
        for (int j = 0; j < NPOS; ++j) V[j] = cost_add<METRIC>(V[j], Lv[j], Rv[j]);
        if (t + 1 < WIN) s_new = wrap(s_new);
    }
    emit();
    // steady state: output row k adds input row k + w - 1 and drops row k - 1
    for (int k = 1; k < nout; ++k) {
        const int tn = k + WIN - 1;
        s_new = wrap(s_new);
        t_wait_vmcnt<(kTPD - 1) * NDMA>();
        issue_row(tn + kTPD, s_pf);
        s_pf = wrap(s_pf);
        const uint32_t* sn = ring + s_new * kTSlot;
        const uint32_t* so = ring + s_old * kTSlot;
        s_old = wrap(s_old);
        uint32_t Ln[NPV], Rn[NPV], Lo[NPV], Ro[NPV];
        load_L(sn, Ln);
        load_R(sn, Rn);
        load_L(so, Lo);
        load_R(so, Ro);
#pragma unroll
        for (int j = 0; j < NPOS; ++j) V[j] = cost_update<METRIC>(V[j], Ln[j], Rn[j], Lo[j], Ro[j]);
        emit();
    }
    if (filled) flush(filled);
    t_wait_vmcnt<0>();  // drain the look-ahead DMAs before the wave retires
}

template <int METRIC, int RAD>
hipError_t launch_tiled_r(const MatchArgs& a, hipStream_t s) {
    TiledPlan P{};
    const int NW = (a.D + 63) / 64;
    const int w = 2 * RAD + 1;
    P.nb = w + 1 + kTPD;
    const size_t smem = 4u * ((size_t)NW * P.nb * kTSlot + (size_t)NW * 16 * 64 + 2u * kTCH * NW * kTK + 512u);
    if (smem > 160u * 1024u) return hipErrorInvalidValue;
    // more than 64 KB of dynamic LDS needs the attribute (set once per process)
    static const bool big_ok =
        hipFuncSetAttribute(reinterpret_cast<const void*>(sad_tiled_kernel<METRIC, RAD>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    if (smem > 64u * 1024u && !big_ok) return hipErrorInvalidValue;
    P.n_xt = (a.W + kTK - 1) / kTK;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    const int per_cu = (int)((160u * 1024u) / smem) < 4 ? (int)((160u * 1024u) / smem) : 4;
    const long slots = (long)cus * (per_cu > 0 ? per_cu : 1);
    const long cols = (long)P.n_xt * a.batch;
    long m = (slots + cols - 1) / cols;
    const long m_max = a.H / (3 * w) > 0 ? a.H / (3 * w) : 1;  // bands of >= 3 windows (warm-up cost)
    if (m > m_max) m = m_max;
    if (m < 1) m = 1;
    P.m = (int)m;
    const long total = cols * m;
    if (total > 0x7FFFFFFFL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((sad_tiled_kernel<METRIC, RAD>), dim3((unsigned)total), dim3(NW * 64), smem, s, a, P);
    return hipGetLastError();
}

template <int METRIC, int... RS>
hipError_t launch_tiled_m(const MatchArgs& a, hipStream_t s, std::integer_sequence<int, RS...>) {
    hipError_t e = hipErrorInvalidValue;
    const int rad = (a.w - 1) / 2;
    ((rad == RS ? (e = launch_tiled_r<METRIC, RS>(a, s), 0) : 0), ...);
    return e;
}

}  // namespace

bool tiled_path_supported(const MatchArgs& a) {
    if (a.w < 1 || a.w > 31 || !(a.w & 1) || a.D < 1 || a.D > 256 || a.W < 1 || a.H < 1) return false;
    const int NW = (a.D + 63) / 64, nb = a.w + 1 + kTPD;
    const size_t smem = 4u * ((size_t)NW * nb * kTSlot + (size_t)NW * 16 * 64 + 2u * kTCH * NW * kTK + 512u);
    return smem <= 160u * 1024u;
}

hipError_t launch_tiled(const MatchArgs& a, hipStream_t s) {
    if (!tiled_path_supported(a)) return hipErrorInvalidValue;
    return a.metric == 0 ? launch_tiled_m<0>(a, s, std::make_integer_sequence<int, 16>{})
                         : launch_tiled_m<1>(a, s, std::make_integer_sequence<int, 16>{});
}

}  // namespace usv
