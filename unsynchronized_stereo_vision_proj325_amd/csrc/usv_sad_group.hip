// usv_sad_group.hip -- the paired-disparity SAD kernel for SMALL disparity ranges (configs A, B).
//
// Spec: SURVEY.md §8(a) A1 (restated in oracle/sad_oracle.c), as the kernels in usv_sad_fast.hip.
//
// The paired kernel (usv_sad_fast.hip) gives a lane two adjacent disparities (d in the low half of its
// packed-u16 sums, d + 1 in the high half), so one wave covers 128 disparities.  With D <= 64 only D / 2
// lanes of such a wave would have work.  Here a wave holds G = 2 or 4 column GROUPS of 8 output columns
// side by side, PP = 64 / G lanes (= disparity pairs) per group:
//   lane l: group g = l / PP, pair p = l % PP (d = 2p, 2p + 1), columns x0 + 8g .. x0 + 8g + 7,
//   G = 2 for 32 < D <= 64 (16 columns per wave), G = 4 for 16 < D <= 32 (32 columns per wave).
// The L byte of a chain step now differs between groups, so L is no longer a wave-uniform scalar: the
// L row segment is staged in LDS by the same LDS-DMA that stages the R row (its columns clamped: the
// replicate border comes for free, no edge-tile variants) and every lane reads its group's entries as
// VGPRs (ds_read_b128).  No scalar byte extraction is left on the per-row path.
// Per input row and lane (r = (w - 1) / 2, NPOS = 8 + 2r):
//   P[j + 1] = v_sad_hi_u8(L_j, R_j, v_sad_u8(L_j, R_{j+1}, P[j]))    (R_j: column of disparity d + 1)
//   H[x] = P[x + w] - P[x] (packed, no borrow), S[x] += H[x] - ring[row - w][x]  (8 columns)
// Argmin per output row: lane l writes its 8 packed words to LDS; lane m = LPP * P + q (LPP = 8 / G lanes
// per pixel, 8G pixels) reads word P % 8 of the 8 source lanes PP (P / 8) + 8q .. + 7 (two ds_read_b128),
// builds 16 keys (cost << 8) | d with v_perm, a v_min3 tree, log2(LPP) DPP rounds.  Ties -> smallest d.
// Work map, band heights and output flush follow sad_pair_kernel (XCD-contiguous tiles, one band per
// one-wave workgroup).  Integer arithmetic only: bit-exact with the oracle by construction.
#include <utility>

#include "usv_band.hpp"
#include "usv_kernels.hpp"
#include "usv_tiles.hpp"

namespace usv {
namespace {

template <int N>
__device__ __forceinline__ void g_wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ uint32_t g_lds_addr(const uint32_t* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t*)p;
}
template <int CTRL>
__device__ __forceinline__ uint32_t g_dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)0, (int)v, CTRL, 0xF, 0xF, false);
}
constexpr int kGQuadSwap2 = 0x4E;  // quad_perm [2,3,0,1]
constexpr int kGQuadSwap1 = 0xB1;  // quad_perm [1,0,3,2]

using gsu4 = uint32_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ gsu4 raw_buffer(const uint8_t* base) {
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    gsu4 r;
    r[0] = (uint32_t)b;
    r[1] = (uint32_t)(b >> 32);  // stride 0: raw buffer
    r[2] = 0xFFFFFFFFu;          // no range limit (offsets stay inside the image)
    r[3] = 0x00020000u;          // gfx9 raw-buffer word 3
    return r;
}

// One input row's LDS-DMAs under ONE M0 write: NQ R DMAs (LDS entries 64 q .. 64 q + 63 of the slot)
// and the L DMA (entries 64 NQ ..).  The immediate offset moves the LDS destination and the global
// address alike, so every per-lane offset is pre-biased by -256 q (DMA q) and both bases carry -kGBias.
// GFX9 needs one wait state between the M0 write and an LDS-DMA that reads it: s_nop 0.
constexpr uint32_t kGBias = 1024;
template <int NQ>
__device__ __forceinline__ void dma_row_lr(gsu4 rsrcR, gsu4 rsrcL, uint32_t soff, const uint32_t (&vo)[NQ + 1],
                                           uint32_t m0) {
    static_assert(NQ == 1 || NQ == 2, "one or two R DMAs per row");
    if constexpr (NQ == 1)
        asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_ubyte %0, %3, %5 offen lds\n\t"
                     "buffer_load_ubyte %1, %4, %5 offen offset:256 lds"
                     :: "v"(vo[0]), "v"(vo[1]), "s"(m0), "s"(rsrcR), "s"(rsrcL), "s"(soff) : "memory", "m0");
    else
        asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_ubyte %0, %4, %6 offen lds\n\t"
                     "buffer_load_ubyte %1, %4, %6 offen offset:256 lds\n\t"
                     "buffer_load_ubyte %2, %5, %6 offen offset:512 lds"
                     :: "v"(vo[0]), "v"(vo[1]), "v"(vo[2]), "s"(m0), "s"(rsrcR), "s"(rsrcL), "s"(soff)
                     : "memory", "m0");
}

// LDS-cycle forms (MI355X_MICROARCH.md LDS table), as in sad_pair_kernel: staged-entry reads as single
// ds_read_b64 / ds_read_b128 issued by inline asm in order of first use, each retired by a counted lgkmcnt
// wait before the chain step that first needs it (the compiler pairs plain 8-byte reads into ds_read2_b64,
// 8 cycles per pair against 2 per single read), and the argmin transpose stores as ds_write_addtid_b32.
// (these forms: rocprof A/B B 10.62 -> 10.34 us, A 5.78 -> 5.70 us, round 4)
typedef uint32_t gu2 __attribute__((ext_vector_type(2)));
template <uint32_t OFF>
__device__ __forceinline__ void g_ds_read_b64(gu2& v, uint32_t addr) {
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
}
template <uint32_t OFF>
__device__ __forceinline__ void g_ds_read_b128(gsu4& v, uint32_t addr) {
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
}

template <int RAD, int G>
struct GCfg {
    static constexpr int K = 8;                          // columns per group
    static constexpr int PP = 64 / G;                    // disparity pairs (lanes) per group
    static constexpr int LPP = 8 / G;                    // argmin lanes per pixel
    static constexpr int KW = K * G;                     // output columns per wave
    static constexpr int WIN = 2 * RAD + 1;
    static constexpr int NPOS = K + 2 * RAD;             // chain steps
    static constexpr int NE = NPOS + 1;                  // R entries a lane reads per row
    static constexpr int NE_V = (NE + 1) / 2 * 2;        // read as b64 pairs
    static constexpr int NL_V = (NPOS + 3) / 4 * 4;      // L entries read as b128 quads
    static constexpr int NR = KW + 2 * RAD + 2 * PP - 1; // R columns staged per row
    static constexpr int NQ = (NR + 63) / 64;
    static constexpr int NL = KW + 2 * RAD;              // L columns staged per row
    static constexpr int SLOT = (NQ + 1) * 64;           // entries per ring slot: R, then L
    static constexpr int NB = 8;
    static constexpr int PD = NB - 1;
    static constexpr int NDMA = NQ + 1;
    static constexpr int KRB = WIN;                      // output rows per flush
    static constexpr int RBUF_OFF = 0;
    static constexpr int TB_OFF = RBUF_OFF + NB * SLOT;
    static constexpr int COMB_OFF = TB_OFF + K * 64;
    static constexpr int LUT_OFF = (COMB_OFF + 2 * KRB * KW + 3) / 4 * 4;  // 16-byte aligned (LDS-DMA x4)
    static constexpr int SMEM_WORDS = LUT_OFF + 2 * 256;
    static_assert(G == 2 || G == 4, "two or four column groups");
    static_assert(RAD >= 1 && RAD <= 7, "packed-u16 costs: w <= 15");
    static_assert(NQ <= 2 && NL <= 64, "one L DMA, at most two R DMAs per row");
    static_assert(NE_V + 2 * (PP - 1) + K * (G - 1) <= NQ * 64, "a lane's entries stay inside the R part");
    static_assert(NL_V + K * (G - 1) <= 64, "a lane's L entries stay inside the L part");
    static_assert(PD * NDMA < 64, "look-ahead DMAs fit the 6-bit vmcnt");
    // asm read schedule: NEP b64 R pairs (pair k first used by chain step k ? 2k - 1 : 0),
    // NLQ b128 L quads (quad m first used by step 4m), issued in order of first use (L first on ties)
    static constexpr int NEP = NE_V / 2, NLQ = NL_V / 4, NRD = NEP + NLQ;
    static constexpr int first_use(int code) { return code >= 64 ? 4 * (code - 64) : (code == 0 ? 0 : 2 * code - 1); }
    struct Order { int code[NRD]; };
    static constexpr Order order() {
        Order o{};
        int n = 0, k = 0, m = 0;
        while (n < NRD) {
            const bool takeL = m < NLQ && (k >= NEP || first_use(64 + m) <= first_use(k));
            o.code[n++] = takeL ? 64 + m++ : k++;
        }
        return o;
    }
    // reads whose first use is at or before step j
    static constexpr int needed(int j) {
        int c = 0;
        for (int n = 0; n < NRD; ++n) c += first_use(order().code[n]) <= j;
        return c;
    }
};

template <int RAD, int G>
__device__ __forceinline__ void group_band_loop(const uint8_t* __restrict__ L, const uint8_t* __restrict__ R,
                                                uint8_t* __restrict__ disp, double* __restrict__ dist,
                                                const MatchArgs& a, uint32_t* smem, int lane, int x0, int y_begin,
                                                int y_end) {
    using C = GCfg<RAD, G>;
    constexpr int WIN = C::WIN, K = C::K, NB = C::NB, PD = C::PD, KRB = C::KRB, NPOS = C::NPOS, PP = C::PP;
    constexpr int LPP = C::LPP, KW = C::KW;
    const int lmax = a.D / 2 - 1;                 // last pair with work (D even, D / 2 <= PP)
    const int grp = lane / PP, p_eff = min(lane % PP, lmax);
    uint32_t* tb = smem + C::TB_OFF;
    uint32_t* comb = smem + C::COMB_OFF;
    const double* lut_s = reinterpret_cast<const double*>(smem + C::LUT_OFF);
    // argmin read side: lane m = LPP * P + q reads word P % 8 of source lanes PP (P / 8) + 8q .. + 7
    uint32_t rdw[2], dlo[2], dhi[2];
    {
        const int P = lane / LPP, q = lane % LPP, i = P & 7, gs = P >> 3;
        const int s0 = PP * gs + 8 * q;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            rdw[j] = (uint32_t)((64 * i + s0 + 4 * j) / 4);  // uint4 index
            uint32_t lo = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) lo |= (uint32_t)(2 * min(8 * q + 4 * j + e, lmax)) << (8 * e);
            dlo[j] = lo;
            dhi[j] = lo + 0x01010101u;  // d even: + 1 per byte, no carry (d + 1 <= 63)
        }
    }
    const int s_r = 8 * grp + 2 * (PP - 1 - p_eff);  // this lane's first R entry
    const int s_lv = C::NQ * 64 + 8 * grp;            // this lane's first L entry
    const int nout = y_end - y_begin;
    const int T = nout + 2 * RAD;
    const int Hm1 = a.H - 1, Wm1 = a.W - 1;
    const int y0 = y_begin - RAD;
    const int last_off = Hm1 * a.pitch;
    // per-lane DMA offsets: R columns cR0 + lane + 64 q, L columns x0 - r + lane, clamped (replicate)
    const int cR0 = x0 - RAD - (2 * PP - 1);
    uint32_t vo[C::NQ + 1];
#pragma unroll
    for (int q = 0; q < C::NQ; ++q)
        vo[q] = (uint32_t)min(max(cR0 + lane + 64 * q, 0), Wm1) + kGBias - 256u * (uint32_t)q;
    vo[C::NQ] = (uint32_t)min(max(x0 - RAD + lane, 0), Wm1) + kGBias - 256u * (uint32_t)C::NQ;
    const gsu4 rsrcR = raw_buffer(R - kGBias), rsrcL = raw_buffer(L - kGBias);
    const uint32_t rbase = g_lds_addr(smem + C::RBUF_OFF);
    auto row_off = [&](int t) -> uint32_t { return (uint32_t)(min(max(y0 + t, 0), Hm1) * a.pitch); };
    auto issue_dma = [&](int t, uint32_t soff) {
        dma_row_lr<C::NQ>(rsrcR, rsrcL, soff, vo, rbase + 4u * (uint32_t)((t & (NB - 1)) * C::SLOT));
    };
    int raw = (y0 + PD) * a.pitch;  // unclamped offset of the next row to stage (rows y0 + PD, ...)

    auto do_row = [&](int t_in, auto warm_tag, auto i_tag, uint32_t(&S)[K], uint32_t(&ring)[WIN][K]) {
        constexpr bool WARM = decltype(warm_tag)::value;
        constexpr int I = decltype(i_tag)::value;
        int t = t_in;
        asm volatile("" : "+s"(t));
        g_wait_vmcnt<(PD - 1) * C::NDMA>();  // row t has landed
        __builtin_amdgcn_wave_barrier();
        {
            int rr = raw;
            asm volatile("" : "+s"(rr));
            issue_dma(t + PD, (uint32_t)min(max(rr, 0), last_off));
            raw = rr + a.pitch;
        }
        // the ring row leaving the window is subtracted first: its registers are then free for this row's
        // H (no copies at the ring write below)
        if constexpr (!WARM) {
#pragma unroll
            for (int x = 0; x < K; ++x) S[x] -= ring[I][x];
        }
        int boff = (t & (NB - 1)) * C::SLOT;
        asm volatile("" : "+s"(boff));
        const uint32_t* slot = smem + C::RBUF_OFF + boff;
        uint32_t Lv[C::NL_V], E[C::NE_V];
        gu2 ev[C::NEP];
        gsu4 lv[C::NLQ];
        {
            const uint32_t sa = g_lds_addr(slot);
            const uint32_t ra = sa + 4u * (uint32_t)s_r, la = sa + 4u * (uint32_t)s_lv;
            [&]<int... N>(std::integer_sequence<int, N...>) {
                auto one = [&](auto nt) {
                    constexpr int code = C::order().code[decltype(nt)::value];
                    if constexpr (code >= 64) g_ds_read_b128<16u * (code - 64)>(lv[code - 64], la);
                    else g_ds_read_b64<8u * code>(ev[code], ra);
                };
                (one(std::integral_constant<int, N>{}), ...);
            }(std::make_integer_sequence<int, C::NRD>{});
        }
        uint32_t A[NPOS + 1];
        A[0] = 0;
        {
            auto step_j = [&](auto jt) {
                constexpr int j = decltype(jt)::value;
                constexpr int have = j == 0 ? 0 : C::needed(j - 1), need = C::needed(j);
                if constexpr (need > have) {
                    __builtin_amdgcn_sched_barrier(0);
                    __builtin_amdgcn_s_waitcnt(0xC07F | ((C::NRD - need) << 8));
                    // the newly retired registers: stay allocated up to here, then unpacked
                    [&]<int... N>(std::integer_sequence<int, N...>) {
                        auto take = [&](auto nt) {
                            constexpr int code = C::order().code[have + decltype(nt)::value];
                            if constexpr (code >= 64) {
                                asm volatile("" ::"v"(lv[code - 64]));
                                Lv[4 * (code - 64)] = lv[code - 64].x; Lv[4 * (code - 64) + 1] = lv[code - 64].y;
                                Lv[4 * (code - 64) + 2] = lv[code - 64].z; Lv[4 * (code - 64) + 3] = lv[code - 64].w;
                            } else {
                                asm volatile("" ::"v"(ev[code]));
                                E[2 * code] = ev[code].x;
                                E[2 * code + 1] = ev[code].y;
                            }
                        };
                        (take(std::integral_constant<int, N>{}), ...);
                    }(std::make_integer_sequence<int, need - have>{});
                    __builtin_amdgcn_sched_barrier(0);
                }
                A[j + 1] = __builtin_amdgcn_sad_hi_u8(Lv[j], E[j], __builtin_amdgcn_sad_u8(Lv[j], E[j + 1], A[j]));
            };
            [&]<int... J>(std::integer_sequence<int, J...>) {
                (step_j(std::integral_constant<int, J>{}), ...);
            }(std::make_integer_sequence<int, NPOS>{});
            static_assert(C::needed(NPOS - 1) == C::NRD, "every read retired by the last step");
        }
#pragma unroll
        for (int x = 0; x < K; ++x) {
            const uint32_t h = A[x + WIN] - A[x];  // both halves in [0, 65535], no borrow
            S[x] = S[x] + h;  // (S - ring is a (w - 1)-row sum: no half leaves [0, 65535])
            ring[I][x] = h;
        }
        __builtin_amdgcn_sched_barrier(0);
    };

    int cb = 0, y_chunk = y_begin;
    const bool wide = ((reinterpret_cast<uintptr_t>(disp + x0) | (uintptr_t)a.disp_pitch) & 3u) == 0 &&
                      (!dist || ((reinterpret_cast<uintptr_t>(dist + x0) | ((uintptr_t)a.dist_pitch * 8)) & 15u) == 0);
    auto flush = [&](int rows) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: its LDS ops run in order
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const uint32_t* crow = comb + cb * KRB * KW;
        if (wide) {
            // disparity: 4 pixels (one dword) per item; distance: 2 pixels (16 bytes) per item
            for (int i = tid; i < rows * (KW / 4); i += 64) {
                const int row = i / (KW / 4), c = i - row * (KW / 4);
                const uint4 k = reinterpret_cast<const uint4*>(crow + row * KW)[c];
                const uint32_t v = (k.x & 0xFFu) | ((k.y & 0xFFu) << 8) | ((k.z & 0xFFu) << 16) | ((k.w & 0xFFu) << 24);
                *reinterpret_cast<uint32_t*>(disp + (size_t)(y_chunk + row) * a.disp_pitch + x0 + 4 * c) = v;
            }
            if (dist) {
                struct __attribute__((aligned(16))) D2 { double a, b; };
                for (int i = tid; i < rows * (KW / 2); i += 64) {
                    const int row = i / (KW / 2), c = i - row * (KW / 2);
                    const uint2 k = reinterpret_cast<const uint2*>(crow + row * KW)[c];
                    *reinterpret_cast<D2*>(dist + (size_t)(y_chunk + row) * a.dist_pitch + x0 + 2 * c) =
                        D2{lut_s[k.x & 0xFFu], lut_s[k.y & 0xFFu]};
                }
            }
        } else {
            for (int i = tid; i < rows * KW; i += 64) {
                const int row = i / KW, p = i - row * KW;
                const uint32_t dv = crow[row * KW + p] & 0xFFu;
                const size_t y = (size_t)(y_chunk + row);
                disp[y * a.disp_pitch + x0 + p] = (uint8_t)dv;
                if (dist) dist[y * a.dist_pitch + x0 + p] = lut_s[dv];
            }
        }
        y_chunk += rows;
        cb ^= 1;
    };
    const uint32_t tb_lds = g_lds_addr(tb);
    auto emit = [&](const uint32_t(&S)[K], int slot_row) {
        {
            static_assert(K == 8, "eight transpose stores");
            asm volatile("s_mov_b32 m0, %8\n\ts_nop 0\n\t"
                         "ds_write_addtid_b32 %0\n\tds_write_addtid_b32 %1 offset:256\n\t"
                         "ds_write_addtid_b32 %2 offset:512\n\tds_write_addtid_b32 %3 offset:768\n\t"
                         "ds_write_addtid_b32 %4 offset:1024\n\tds_write_addtid_b32 %5 offset:1280\n\t"
                         "ds_write_addtid_b32 %6 offset:1536\n\tds_write_addtid_b32 %7 offset:1792"
                         :: "v"(S[0]), "v"(S[1]), "v"(S[2]), "v"(S[3]), "v"(S[4]), "v"(S[5]), "v"(S[6]), "v"(S[7]),
                            "s"(tb_lds) : "memory", "m0");
        }
        asm volatile("" ::: "memory");
        uint4 w2[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) w2[j] = reinterpret_cast<const uint4*>(tb)[rdw[j]];
        asm volatile("" ::: "memory");
        uint32_t fv[16];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t w = e == 0 ? w2[j].x : e == 1 ? w2[j].y : e == 2 ? w2[j].z : w2[j].w;
                fv[8 * j + 2 * e] = __builtin_amdgcn_perm(w, dlo[j], 0x0c050400u + (uint32_t)e);      // (lo << 8) | d
                fv[8 * j + 2 * e + 1] = __builtin_amdgcn_perm(w, dhi[j], 0x0c070600u + (uint32_t)e);  // (hi << 8) | d+1
            }
        }
        uint32_t b0 = min(min(fv[0], fv[1]), fv[2]), b1 = min(min(fv[3], fv[4]), fv[5]);
        uint32_t b2 = min(min(fv[6], fv[7]), fv[8]), b3 = min(min(fv[9], fv[10]), fv[11]);
        uint32_t b4 = min(min(fv[12], fv[13]), fv[14]);
        b0 = min(min(b0, b1), b2);
        b3 = min(min(b3, b4), fv[15]);
        uint32_t m = min(b0, b3);
        m = min(m, g_dpp<kGQuadSwap1>(m));
        if constexpr (LPP == 4) m = min(m, g_dpp<kGQuadSwap2>(m));
        comb[(cb * KRB + slot_row) * KW + lane / LPP] = m;  // the LPP lanes of a pixel write the same key
        __builtin_amdgcn_sched_barrier(0);
    };

    uint32_t S[K];
#pragma unroll
    for (int i = 0; i < K; ++i) S[i] = 0;
    uint32_t ring[WIN][K];
    // The 2 KB distance table goes to LDS by two 16-byte-per-lane LDS-DMAs issued ahead of the row
    // prologue: vector-memory ops retire in order, so the first row's counted wait also retires them and
    // nothing waits for the table's round trip on its own (a register load + ds_write would wait vmcnt(0)).
    if (dist)
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %2\n\t"
                     "global_load_lds_dwordx4 %0, %2 offset:1024"
                     :: "v"((uint32_t)lane * 16u), "s"(g_lds_addr(smem + C::LUT_OFF)), "s"(a.lut) : "memory", "m0");
    // prologue: PD rows in flight
#pragma unroll
    for (int t = 0; t < PD; ++t) issue_dma(t, row_off(t));
    using WarmT = std::integral_constant<bool, true>;
    using SteadyT = std::integral_constant<bool, false>;
    [&]<int... I>(std::integer_sequence<int, I...>) {
        (do_row(I, WarmT{}, std::integral_constant<int, I>{}, S, ring), ...);
    }(std::make_integer_sequence<int, WIN>{});
    emit(S, 0);
    auto step = [&](int t0, auto i_tag) {
        constexpr int I = decltype(i_tag)::value;
        do_row(t0 + I, SteadyT{}, i_tag, S, ring);
        emit(S, (I + 1) % WIN);
        if constexpr ((I + 1) % WIN == KRB - 1) flush(KRB);
    };
    for (int t0 = WIN; t0 < T; t0 += WIN) {
        [&]<int... I>(std::integer_sequence<int, I...>) {
            bool go = true;
            ((go = go && (t0 + I < T), go ? step(t0, std::integral_constant<int, I>{}) : void()), ...);
        }(std::make_integer_sequence<int, WIN>{});
    }
    const int rest = nout % KRB;
    if (rest) flush(rest);
    g_wait_vmcnt<0>();  // drain the look-ahead DMAs before the wave retires
}

struct GroupPlan {
    int n_xt, m, gen_g;
    unsigned weights;
    int extra;
};

#ifndef USV_GROUP_OCC
#define USV_GROUP_OCC 3  // waves per SIMD the group kernel is compiled for
#endif
template <int RAD, int G>
__global__ __launch_bounds__(64, USV_GROUP_OCC) void sad_group_kernel(const uint8_t* __restrict__ L,
                                                                     const uint8_t* __restrict__ R,
                                                                     uint8_t* __restrict__ disp,
                                                                     double* __restrict__ dist, MatchArgs a,
                                                                     GroupPlan P, const uint2* __restrict__ tiles) {
    using C = GCfg<RAD, G>;
    __shared__ __attribute__((aligned(16))) uint32_t smem[C::SMEM_WORDS];
    const int lane = threadIdx.x & 63;
    // work map of sad_pair_kernel (usv_tiles.hpp): XCD k owns the k-th contiguous run of tiles (x-tile
    // fastest, then band, then pair); normally one scalar load from the launcher's table
    unsigned xtu, pair;
    int y_begin, y_end;
    if (tiles) {
        const uint2 t = tiles[blockIdx.x];
        xtu = t.x & 0xFFFFu;
        pair = t.x >> 16;
        y_begin = (int)(t.y & 0xFFFFu);
        y_end = (int)(t.y >> 16);
    } else {
        const TileSpan sp = tile_span(blockIdx.x, gridDim.x, P.n_xt, P.m, P.extra, P.gen_g, P.weights, a.H);
        xtu = sp.xt;
        pair = sp.pair;
        y_begin = sp.y_begin;
        y_end = sp.y_end;
    }
    const int xt = (int)xtu;
    // the last tile is aligned to the right border (it may overlap its neighbour; both write the same values)
    const int x0 = xt == P.n_xt - 1 ? a.W - C::KW : xt * C::KW;
    L += (size_t)pair * a.pair_stride;
    R += (size_t)pair * a.pair_stride;
    disp += (size_t)pair * a.disp_stride;
    if (dist) dist += (size_t)pair * a.dist_stride;  // (its table is staged inside the band loop)
    if (y_end <= y_begin) return;
    group_band_loop<RAD, G>(L, R, disp, dist, a, smem, lane, x0, y_begin, y_end);
}

template <int RAD, int G>
int resident_group_blocks_per_cu() {
    static const int n = [] {
        int v = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, sad_group_kernel<RAD, G>, 64, 0) != hipSuccess || v <= 0)
            v = 1;
        return v;
    }();
    return n;
}
int group_cu_count() {
    static const int n = [] {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
            v = 256;
        return v;
    }();
    return n;
}

#ifndef USV_GROUP_MIN_BAND_WINS
#define USV_GROUP_MIN_BAND_WINS 1  // shortest band, in windows (the ring warm-up costs w rows per band)
#endif
#ifndef USV_GROUP_MIN_BAND_ROWS
#define USV_GROUP_MIN_BAND_ROWS 0  // experiment: shortest band in rows (0: USV_GROUP_MIN_BAND_WINS windows)
#endif
#ifndef USV_GROUP_WEIGHTS
#define USV_GROUP_WEIGHTS 0x01010101u  // band heights by dispatch generation (uniform until fitted)
#endif
template <int RAD, int G>
hipError_t launch_group_rg(const MatchArgs& a, hipStream_t s) {
    constexpr int KW = GCfg<RAD, G>::KW, WIN = 2 * RAD + 1;
    GroupPlan P{};
    P.n_xt = (a.W + KW - 1) / KW;
    const int per_cu = resident_group_blocks_per_cu<RAD, G>();
    const long slots = (long)group_cu_count() * per_cu;
    const long NC = (long)P.n_xt * a.batch;
    long m = slots / NC;
    if (m < 1) m = 1;
    // One-window bands are the optimum while they still give every CU ~8 waves (config B: 10.6).  Below that
    // the frame is too small to fill the chip with them (config A: 480 one-window bands = 1.9 waves per CU)
    // and bands down to 2 rows run faster despite the extra warm-up rows each (interleaved A/Bs: A 4.54 ->
    // 4.29 us and 4.57 -> 4.33 us; B with 2-row bands 9.27 -> 9.39 us, so B keeps one-window bands;
    // profiles/probes_r05/ab_group_rows_*_r05.txt, ab_group_pipe_*_r05.txt).
    const bool underfilled = NC * (long)std::max(1, a.H / (USV_GROUP_MIN_BAND_WINS * WIN)) < 8L * group_cu_count();
    const long min_rows = USV_GROUP_MIN_BAND_ROWS > 0 ? USV_GROUP_MIN_BAND_ROWS
                                                      : (underfilled ? 2 : USV_GROUP_MIN_BAND_WINS * WIN);
    const long m_max = a.H / min_rows > 0 ? a.H / min_rows : 1;
    if (m > m_max) m = m_max;
    P.m = (int)m;
    const long ex = slots - NC * m;
    P.extra = (a.batch == 1 && ex > 0 && ex < P.n_xt && a.H / (m + 1) >= min_rows) ? (int)ex : 0;
    const long total = NC * m + P.extra;
    if (total > 0x7FFFFFFFL) return hipErrorInvalidValue;
    P.gen_g = (int)(4L * (group_cu_count() / 8));
    if (P.gen_g < 1) P.gen_g = 1;
    P.weights = per_cu == 12 && total > 2L * 8 * P.gen_g ? USV_GROUP_WEIGHTS : 0x01010101u;
    const uint2* tiles = tile_table(2, RAD * 16 + G, a, P.n_xt, P.m, P.extra, P.gen_g, P.weights, (unsigned)total, s);
    hipLaunchKernelGGL((sad_group_kernel<RAD, G>), dim3((unsigned)total), dim3(64), 0, s, a.L, a.R, a.disp, a.dist,
                       a, P, tiles);
    return hipGetLastError();
}

template <int G>
hipError_t launch_group_g(const MatchArgs& a, hipStream_t s) {
    switch ((a.w - 1) / 2) {
        case 2: return launch_group_rg<2, G>(a, s);
        case 3: return launch_group_rg<3, G>(a, s);
        case 4: return launch_group_rg<4, G>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

// the grouped paired kernel: even 16 < D <= 64, 5 <= w <= 9
bool group_path_supported(const MatchArgs& a) {
    // (fast_path_supported holds: W % 4 == 0, W >= 48, 4-byte aligned bases and pitch, pitch * H < 2^31)
    return a.metric == 0 && (a.D % 2) == 0 && a.D > 16 && a.D <= 64 && a.w >= 5 && a.w <= 9 &&
           a.W >= 32;
}

hipError_t launch_group(const MatchArgs& a, hipStream_t s) {
    if (!group_path_supported(a)) return hipErrorInvalidValue;
    return a.D > 32 ? launch_group_g<2>(a, s) : launch_group_g<4>(a, s);
}

}  // namespace usv
