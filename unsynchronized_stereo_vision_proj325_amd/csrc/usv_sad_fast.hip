// usv_sad_fast.hip -- the hot path: fused SAD block match + argmin on gfx950.
//
// Spec: SURVEY.md §8(a) A1 (restated in oracle/sad_oracle.c).  The reference
// has no block matcher; its nearest primitive is the u8
// absdiff motion mask at P/Main.cpp:304.
//
// Mapping (DESIGN.md §3 has the derivation):
//   * lane = disparity.  A workgroup is NW waves; lane l of wave w owns
//     d = NW*l + w, so the L operand is uniform across the wave (SGPRs) and
//     only R is gathered per lane.  Lanes with d >= D replay the wave's last
//     valid disparity (same data, same key), which cannot change the argmin.
//   * one workgroup = one x-tile of K outputs x one band of rows, walking down
//     the band.  Per input row each lane runs a horizontal prefix chain over
//     K + 2r columns with v_sad_u8 (one instruction per |L-R| + accumulate),
//     giving the row-window sums H[x] = B[x+w] - B[x].
//   * the vertical window is a running sum S += H(new row) - H(row w back);
//     the w rows of H history live in a packed-u16 register ring (H <= 57375
//     for w <= 15), rotated statically by unrolling the row loop w times.
//   * S is kept as a key (cost << 8) | d, so the argmin over disparities is a
//     plain unsigned min and the smallest d wins ties by construction.
//   * the min over the 64 lanes of K pixels is a transpose-reduction
//     (permlane32_swap, permlane16_swap, then DPP mirror rounds): ~2.2 VALU
//     instructions per pixel-disparity instead of 6 for per-pixel reductions.
//   * per-wave R rows are staged to LDS as one u32 per column (lane-linear
//     b64/b128 reads need no per-lane alignment fix-up with the d = NW*l + w
//     interleave); loads for row t+2 are in flight while row t computes.
//   * the NW waves' partial minima are combined through LDS every kRB rows.
// Integer arithmetic only: bit-exact with the oracle by construction.
#include <type_traits>
#include <utility>

#include "usv_kernels.hpp"

namespace usv {
namespace {

constexpr int kRB = 8;  // output rows buffered between cross-wave combines
#ifndef USV_FAST_K
#define USV_FAST_K 16  // outputs per x-tile (16 or 32)
#endif

template <int RAD, int NW, int K>
struct Cfg {
    static constexpr int WIN = 2 * RAD + 1;
    static constexpr int NPOS = K + 2 * RAD;             // chain positions per input row
    static constexpr int NR = NPOS + NW * 63;            // R columns a wave stages per row
    static constexpr int VEC = NW >= 4 ? 4 : (NW == 2 ? 2 : 1);  // LDS read width (dwords)
    static constexpr int NPOS_V = (NPOS + VEC - 1) / VEC * VEC;
    static constexpr int NRP = (NW * 63 + NPOS_V + 3) / 4 * 4;  // padded entries per buffer
    static constexpr int NQ = (NRP + 63) / 64;                  // staging loads per lane
    static constexpr int NPOSP = (NPOS + 3) / 4 * 4;            // L entries (edge tiles)
    static constexpr int LOFF = (4 - (RAD & 3)) & 3;            // (x0 - RAD) mod 4, x0 % 4 == 0
    static constexpr int NLW = (LOFF + NPOS + 3) / 4;           // L dwords (interior tiles)
    // LDS carve (u32 words, every region 16-byte aligned)
    static constexpr int RBUF_OFF = 0;
    static constexpr int LBUF_OFF = RBUF_OFF + NW * 2 * NRP;
    static constexpr int COMB_OFF = LBUF_OFF + NW * 2 * NPOSP;
    static constexpr int LUT_OFF = COMB_OFF + 2 * kRB * NW * 64;
    static constexpr int SMEM_WORDS = LUT_OFF + 2 * 256;
    static_assert(K == 16 || K == 32, "transpose-reduction is written for K = 16 or 32");
    static_assert(RAD >= 1 && RAD <= 7, "packed-u16 ring needs w <= 15");
};

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)0, (int)v, CTRL, 0xF, 0xF, false);
}
constexpr int kRowMirror = 0x140;
constexpr int kRowHalfMirror = 0x141;
constexpr int kQuadSwap2 = 0x4E;  // quad_perm [2,3,0,1]
constexpr int kQuadSwap1 = 0xB1;  // quad_perm [1,0,3,2]

// One transposing round at in-row distance S: result lane l holds, for the
// S-half it sits in, the min over itself and its mirror partner.
template <int S, int CTRL>
__device__ __forceinline__ uint32_t tr_round(uint32_t a, uint32_t b, bool hi) {
    const uint32_t u = hi ? b : a;
    const uint32_t v = hi ? a : b;
    return min(u, dpp<CTRL>(v));
}

// Reduce K keys (each a 64-lane vector over disparities) to one register:
// afterwards lane l holds the minimum key of pixel l / (64 / K).
template <int K>
__device__ __forceinline__ uint32_t reduce_keys(const uint32_t (&k)[K], int lane) {
    const bool h8 = lane & 8, h4 = lane & 4, h2 = lane & 2;
    if constexpr (K == 32) {
        uint32_t r1[16], r2[8], r3[4], r4[2];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            auto p = __builtin_amdgcn_permlane32_swap(k[i], k[i + 16], false, false);
            r1[i] = min((uint32_t)p[0], (uint32_t)p[1]);  // lanes 0-31: pixel i, 32-63: pixel i+16
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            auto p = __builtin_amdgcn_permlane16_swap(r1[i], r1[i + 8], false, false);
            r2[i] = min((uint32_t)p[0], (uint32_t)p[1]);  // 16-lane row q: pixel i + 8q
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) r3[i] = tr_round<8, kRowMirror>(r2[i], r2[i + 4], h8);
#pragma unroll
        for (int i = 0; i < 2; ++i) r4[i] = tr_round<4, kRowHalfMirror>(r3[i], r3[i + 2], h4);
        const uint32_t r5 = tr_round<2, kQuadSwap2>(r4[0], r4[1], h2);
        return min(r5, dpp<kQuadSwap1>(r5));  // lane l: pixel l >> 1
    } else {
        uint32_t r1[8], r2[4], r3[2];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            auto p = __builtin_amdgcn_permlane32_swap(k[i], k[i + 8], false, false);
            r1[i] = min((uint32_t)p[0], (uint32_t)p[1]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            auto p = __builtin_amdgcn_permlane16_swap(r1[i], r1[i + 4], false, false);
            r2[i] = min((uint32_t)p[0], (uint32_t)p[1]);  // row q: pixel i + 4q
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) r3[i] = tr_round<8, kRowMirror>(r2[i], r2[i + 2], h8);
        uint32_t r4 = tr_round<4, kRowHalfMirror>(r3[0], r3[1], h4);
        r4 = min(r4, dpp<kQuadSwap2>(r4));
        return min(r4, dpp<kQuadSwap1>(r4));  // lane l: pixel l >> 2
    }
}

template <int VEC> struct VecT;
template <> struct VecT<1> { using T = uint32_t; };
template <> struct VecT<2> { using T = uint2; };
template <> struct VecT<4> { using T = uint4; };

template <int VEC>
__device__ __forceinline__ uint32_t vget(const typename VecT<VEC>::T& v, int e) {
    if constexpr (VEC == 1) return v;
    else if constexpr (VEC == 2) return e == 0 ? v.x : v.y;
    else return e == 0 ? v.x : (e == 1 ? v.y : (e == 2 ? v.z : v.w));
}

__device__ __forceinline__ void wave_lds_fence() {
    // Same-wave LDS ops execute in order; this only stops the compiler from
    // moving another lane's reads above this lane's writes.
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

template <int RAD, int NW, int K, bool INTERIOR>
__device__ __forceinline__ void band_loop(const uint8_t* __restrict__ L,
                                          const uint8_t* __restrict__ R,
                                          uint8_t* __restrict__ disp, double* __restrict__ dist,
                                          const MatchArgs& a, uint32_t* smem, int lane,
                                          int wave, int x0, int y_begin, int y_end) {
    using C = Cfg<RAD, NW, K>;
    constexpr int WIN = C::WIN;
    // Lanes past D-1 replay the last valid lane of this wave (same R column
    // alignment, same key), so they can never change the argmin.
    const int l_eff = min(lane, (a.D - 1 - wave) / NW);
    const int d_eff = NW * l_eff + wave;
    const int cbase = x0 - RAD - (NW * 63 + wave);  // first R column this wave stages
    uint32_t* rbuf = smem + C::RBUF_OFF + wave * 2 * C::NRP;
    uint32_t* comb = smem + C::COMB_OFF;
    const double* lut_s = reinterpret_cast<const double*>(smem + C::LUT_OFF);
    const int s_l = NW * (63 - l_eff);  // this lane's first chain entry in rbuf
    const int nout = y_end - y_begin;
    const int T = nout + 2 * RAD;  // input rows walked
    const int Hm1 = a.H - 1, Wm1 = a.W - 1;

    auto row_ptr = [&](const uint8_t* img, int t) {
        const int y = min(max(y_begin - RAD + t, 0), Hm1);
        return img + (size_t)y * a.pitch;
    };

    // ---- staging: global -> registers (issue) -> LDS (commit) ----
    // Edge tiles (border clamping on the L side) build the same dword words as
    // the interior SGPR path: lane i < NLW packs 4 clamped L bytes, and the row
    // is moved to SGPRs with v_readlane.
    uint32_t q[C::NQ];
    uint32_t ql = 0;
    auto issue_row = [&](int t) {
        const uint8_t* rr = row_ptr(R, t);
#pragma unroll
        for (int i = 0; i < C::NQ; ++i) q[i] = rr[min(max(cbase + lane + 64 * i, 0), Wm1)];
        if constexpr (!INTERIOR) {
            const uint8_t* lr = row_ptr(L, t);
            const int c0 = x0 - RAD - C::LOFF + 4 * lane;
            ql = 0;
            if (lane < C::NLW) {
#pragma unroll
                for (int k = 0; k < 4; ++k) ql |= (uint32_t)lr[min(max(c0 + k, 0), Wm1)] << (8 * k);
            }
        }
    };
    auto commit_row = [&](int t) {
        uint32_t* dst = rbuf + (t & 1) * C::NRP;
#pragma unroll
        for (int i = 0; i < C::NQ; ++i)
            if (C::NRP % 64 == 0 || lane + 64 * i < C::NRP) dst[lane + 64 * i] = q[i];
    };

    // One input row t: chain over the K + 2r columns, and as soon as a
    // row-window sum H[x] = B[x+w] - B[x] exists fold it into the key S[x] and
    // the ring slot.  WARM: first w rows (no subtraction).  Consuming H on the
    // fly keeps the live set at ring + S + a (w+1)-deep chain window.
    uint32_t lw_next[C::NLW];
    auto load_lw = [&](int t) {
        if constexpr (INTERIOR) {
            const uint32_t* p =
                reinterpret_cast<const uint32_t*>(row_ptr(L, t) + (x0 - RAD - C::LOFF));
#pragma unroll
            for (int i = 0; i < C::NLW; ++i) lw_next[i] = p[i];
        } else {
#pragma unroll
            for (int i = 0; i < C::NLW; ++i) lw_next[i] = __builtin_amdgcn_readlane(ql, i);
        }
    };
    auto do_row = [&](int t, auto warm_tag, auto slot_tag, uint32_t(&S)[K],
                      uint32_t(&ring)[WIN][K / 2]) {
        constexpr bool WARM = decltype(warm_tag)::value;
        constexpr int SL = decltype(slot_tag)::value;
        // L operand of this row (uniform, SGPRs): bytes of the dword-aligned segment.
        uint32_t Lv[C::NPOS];
        uint32_t lw[C::NLW];
#pragma unroll
        for (int i = 0; i < C::NLW; ++i) lw[i] = lw_next[i];
#pragma unroll
        for (int j = 0; j < C::NPOS; ++j) {
            const int bidx = C::LOFF + j;
            Lv[j] = (lw[bidx >> 2] >> (8 * (bidx & 3))) & 0xFFu;
        }
        // stage row t+1 (loaded a row ago) and put row t+2 in flight
        if constexpr (!INTERIOR) load_lw(t + 1);  // ql holds row t+1 (issued a row ago)
        commit_row(t + 1);
        wave_lds_fence();
        issue_row(t + 2);
        if constexpr (INTERIOR) load_lw(t + 1);

        using VT = typename VecT<C::VEC>::T;
        const VT* rb = reinterpret_cast<const VT*>(rbuf + (t & 1) * C::NRP + s_l);
        uint32_t B[C::NPOS + 1];
        uint32_t Hlo = 0;
        B[0] = 0;
#pragma unroll
        for (int jv = 0; jv < C::NPOS_V / C::VEC; ++jv) {
            const VT v = rb[jv];
#pragma unroll
            for (int e = 0; e < C::VEC; ++e) {
                const int j = jv * C::VEC + e;
                if (j < C::NPOS) {
                    B[j + 1] = __builtin_amdgcn_sad_u8(Lv[j], vget<C::VEC>(v, e), B[j]);
                    const int x = j + 1 - WIN;  // H[x] complete
                    if (x >= 0) {
                        const uint32_t h = B[x + WIN] - B[x];
                        if constexpr (WARM) {
                            S[x] += h << 8;
                        } else {
                            const uint32_t old = (x & 1) ? (ring[SL][x >> 1] >> 16)
                                                         : (ring[SL][x >> 1] & 0xFFFFu);
                            S[x] += (h - old) << 8;
                        }
                        if (x & 1) ring[SL][x >> 1] = Hlo | (h << 16);
                        else Hlo = h;
                    }
                }
            }
        }
    };

    // ---- output: per-row keys -> LDS, cross-wave min every kRB rows ----
    int slot = 0, cb = 0, y_chunk = y_begin;
    auto flush = [&]() {
        __syncthreads();
        const int items = slot * K;
        for (int i = threadIdx.x; i < items; i += NW * 64) {
            const int row = i / K, p = i - row * K;
            uint32_t key = 0xFFFFFFFFu;
#pragma unroll
            for (int w2 = 0; w2 < NW; ++w2)
                key = min(key, comb[((cb * kRB + row) * NW + w2) * 64 + p * (64 / K)]);
            const int x = x0 + p;
            if (x < a.W) {
                const uint32_t dv = key & 0xFFu;
                const size_t y = (size_t)(y_chunk + row);
                disp[y * a.disp_pitch + x] = (uint8_t)dv;
                if (dist) dist[y * a.dist_pitch + x] = lut_s[dv];
            }
        }
        y_chunk += slot;
        slot = 0;
        cb ^= 1;
    };
    auto emit = [&](const uint32_t(&S)[K], bool last) {
        const uint32_t m = reduce_keys<K>(S, lane);
        comb[((cb * kRB + slot) * NW + wave) * 64 + lane] = m;
        ++slot;
        if (slot == kRB || last) flush();
    };

    uint32_t S[K];
#pragma unroll
    for (int x = 0; x < K; ++x) S[x] = (uint32_t)d_eff;
    uint32_t ring[WIN][K / 2];

    // prologue: row 0 staged, row 1 in flight
    issue_row(0);
    load_lw(0);
    commit_row(0);
    wave_lds_fence();
    issue_row(1);

    using WarmT = std::integral_constant<bool, true>;
    using SteadyT = std::integral_constant<bool, false>;
    // ---- warm-up: the first WIN input rows fill the ring ----
    [&]<int... I>(std::integer_sequence<int, I...>) {
        (do_row(I, WarmT{}, std::integral_constant<int, I>{}, S, ring), ...);
    }(std::make_integer_sequence<int, WIN>{});
    emit(S, nout == 1);

    // ---- steady state: one output row per input row ----
    for (int t0 = WIN; t0 < T; t0 += WIN) {
        bool done = false;
        [&]<int... I>(std::integer_sequence<int, I...>) {
            ((done = done || (t0 + I >= T),
              done ? void() : (do_row(t0 + I, SteadyT{}, std::integral_constant<int, I>{}, S, ring),
                               emit(S, t0 + I == T - 1))),
             ...);
        }(std::make_integer_sequence<int, WIN>{});
    }
}

template <int RAD, int NW, int K>
__global__ __launch_bounds__(NW * 64, 2) void sad_fast_kernel(const uint8_t* __restrict__ L,
                                                              const uint8_t* __restrict__ R,
                                                              uint8_t* __restrict__ disp,
                                                              double* __restrict__ dist,
                                                              MatchArgs a, int band_rows) {
    using C = Cfg<RAD, NW, K>;
    __shared__ __attribute__((aligned(16))) uint32_t smem[C::SMEM_WORDS];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int x0 = blockIdx.x * K;
    const int y_begin = blockIdx.y * band_rows;
    const int y_end = min(a.H, y_begin + band_rows);
    const size_t b = blockIdx.z;
    L += b * a.pair_stride;
    R += b * a.pair_stride;
    disp += b * a.disp_stride;
    if (dist) {
        dist += b * a.dist_stride;
        double* lut_s = reinterpret_cast<double*>(smem + C::LUT_OFF);
        for (int i = threadIdx.x; i < 256; i += NW * 64) lut_s[i] = a.lut[i];
    }
    __syncthreads();
    const bool interior = (x0 - RAD >= 0) && (x0 + K - 1 + RAD <= a.W - 1);
    if (interior)
        band_loop<RAD, NW, K, true>(L, R, disp, dist, a, smem, lane, wave, x0, y_begin, y_end);
    else
        band_loop<RAD, NW, K, false>(L, R, disp, dist, a, smem, lane, wave, x0, y_begin, y_end);
}

template <int RAD>
constexpr int k_for_rad() { return USV_FAST_K; }

template <int RAD, int NW>
hipError_t launch_rn(const MatchArgs& a, hipStream_t s) {
    constexpr int K = k_for_rad<RAD>();
    const int n_xt = (a.W + K - 1) / K;
    // ~2 resident waves per SIMD: 8 waves per CU on 256 CUs.
    const int target_blocks = 256 * 8 / NW;
    int n_bands = (target_blocks + n_xt * a.batch - 1) / (n_xt * a.batch);
    const int min_rows = 4 * (2 * RAD + 1);
    int band_rows = (a.H + n_bands - 1) / n_bands;
    if (band_rows < min_rows) band_rows = min_rows;
    n_bands = (a.H + band_rows - 1) / band_rows;
    dim3 grid(n_xt, n_bands, a.batch), block(NW * 64);
    hipLaunchKernelGGL((sad_fast_kernel<RAD, NW, K>), grid, block, 0, s, a.L, a.R, a.disp, a.dist,
                       a, band_rows);
    return hipGetLastError();
}

template <int RAD>
hipError_t launch_r(const MatchArgs& a, hipStream_t s) {
    if (a.D <= 64) return launch_rn<RAD, 1>(a, s);
    if (a.D <= 128) return launch_rn<RAD, 2>(a, s);
    return launch_rn<RAD, 4>(a, s);
}

}  // namespace

bool fast_path_supported(const MatchArgs& a) {
    return a.metric == 0 && a.w >= 3 && a.w <= 15 && (a.w & 1) && a.D >= 1 && a.D <= 256 &&
           (a.pitch % 4) == 0 && (reinterpret_cast<uintptr_t>(a.L) % 4) == 0 &&
           (reinterpret_cast<uintptr_t>(a.R) % 4) == 0 && (a.batch <= 1 || a.pair_stride % 4 == 0);
}

hipError_t launch_fast(const MatchArgs& a, hipStream_t s) {
    if (!fast_path_supported(a)) return hipErrorInvalidValue;
#ifdef USV_DEV_ONLY_RAD  // development: build a single instantiation for ISA inspection
    return launch_rn<USV_DEV_ONLY_RAD, USV_DEV_ONLY_NW>(a, s);
#else
    switch ((a.w - 1) / 2) {
        case 1: return launch_r<1>(a, s);
        case 2: return launch_r<2>(a, s);
        case 3: return launch_r<3>(a, s);
        case 4: return launch_r<4>(a, s);
        case 5: return launch_r<5>(a, s);
        case 6: return launch_r<6>(a, s);
        case 7: return launch_r<7>(a, s);
        default: return hipErrorInvalidValue;
    }
#endif
}

}  // namespace usv
