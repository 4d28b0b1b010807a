// usv_sad_ssd.hip -- the SSD block-match kernel on gfx950 (ssd_fast_kernel; 11 <= w <= 15).
//
// Spec: SURVEY.md §8(a) A1, SSD variant (restated in oracle/sad_oracle.c).  Integer arithmetic only:
// bit-exact with the oracle by construction.
#include "usv_sad_common.hpp"

namespace usv {
namespace {

// ===================================================================================
// SSD kernel (metric 1, 11 <= w <= 15): lane = one disparity, K = 8 output columns, u32 costs.
//
// The squared-difference window cost of a 15 x 15 window reaches 225 x 255^2 = 14.6 M: no packed u16
// halves, so a lane carries ONE disparity (d = NW l + w as in the column kernel above, NW = ceil(D /
// 64) waves per workgroup) and 8 u32 column sums.  Per input row:
//   * prefix chain over the K + 2r staged entries: P[j + 1] = P[j] + (L_j - R_j)^2, one v_sub and one
//     24-bit multiply-add per step (L_j a wave-uniform SGPR byte, R_j the staged u32 entry);
//   * H[x] = P[x + w] - P[x], S[x] += H[x] - ring[row - w][x] (register ring of w rows x 8 columns);
//   * argmin: the LDS transpose of the paired kernel (lane 8p + q reads the 8 costs of pixel p from
//     lanes 8q .. 8q + 7), keys (cost << 8) | d by one v_perm (cost < 2^24), a v_min3 tree, three DPP
//     rounds across the 8 lanes of the pixel; each wave's minimum goes to the combine buffer and the
//     flush takes the min over the NW waves.  The 14 argmin pieces of row k ride on row k + 1's chain
//     steps.  Ties -> smallest d, as in the SAD kernels.
// Integer arithmetic only: bit-exact with oracle/sad_oracle.c's SSD by construction.
// ===================================================================================
// LDS-cycle forms of the paired kernel (usv_sad_pair.hip; config C SSD 108.0 -> 102.3 us): the staged
// entries as single ds_read_b64 issued by inline asm with a counted wait before the first chain step that needs
// each pair (the compiler pairs plain reads into ds_read2_b64), the transpose stores as ds_write_addtid_b32.
typedef uint32_t ssd_u2 __attribute__((ext_vector_type(2)));
typedef uint32_t ssd_u4 __attribute__((ext_vector_type(4)));
template <uint32_t OFF>
__device__ __forceinline__ void ssd_ds_read_b64(ssd_u2& v, uint32_t addr) {
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
}

template <int RAD, int NW>
struct SCfg {
    static constexpr int K = 8;
    static constexpr int WIN = 2 * RAD + 1;
    static constexpr int NPOS = K + 2 * RAD;            // chain steps = staged entries a lane reads
    static constexpr int VEC = NW >= 4 ? 4 : NW;        // lane offsets are NW entries apart
    static constexpr int NPOS_V = (NPOS + VEC - 1) / VEC * VEC;
    static constexpr int NR = NW * 63 + NPOS_V;         // entries a wave stages per row
    static constexpr int NQ = (NR + 63) / 64;
    static constexpr int NRS = NQ * 64;
    static constexpr int NB = NW <= 2 ? 8 : 4;
    static constexpr int PD = NB - 1;
    static constexpr int KRB = WIN;
    static constexpr int NPC = 14;                      // argmin pieces per row
    static constexpr int RBUF_OFF = 0;
    static constexpr int TB_OFF = RBUF_OFF + NW * NB * NRS;
    static constexpr int TB_WORDS = K * 64;
    static constexpr int COMB_OFF = TB_OFF + NW * TB_WORDS;
    static constexpr int LUT_OFF = COMB_OFF + 2 * KRB * NW * K;
    static constexpr int SMEM_WORDS = LUT_OFF + 2 * 256;
    static_assert(RAD >= 5 && RAD <= 7, "SSD kernel: 11 <= w <= 15 (the 8-column L segments)");
    static_assert(PD * NQ < 64, "look-ahead DMAs must fit the 6-bit vmcnt");
    static_assert(NQ <= 5, "dma_row_buf issues at most 5 DMAs");
    static_assert(NPOS >= NPC, "the argmin pieces ride on the chain steps");
    static_assert(NW * 63 + NW - 1 <= 255, "key disparities are one byte");
};

template <int RAD, int NW, int EDGE>
__device__ __forceinline__ void ssd_band_loop(const uint8_t* __restrict__ L, const uint8_t* __restrict__ R,
                                              uint8_t* __restrict__ disp, double* __restrict__ dist,
                                              const MatchArgs& a, uint32_t* smem, int lane, int wave, int x0,
                                              int y_begin, int y_end) {
    using C = SCfg<RAD, NW>;
    using LS = LSeg<RAD, EDGE, C::K>;
    using LWords = typename SWords<LS::NLD>::T;
    constexpr int WIN = C::WIN, K = C::K, NB = C::NB, PD = C::PD, KRB = C::KRB, NPOS = C::NPOS;
    constexpr int NDMA = C::NQ;
    // lane l owns d = NW l + wave; lanes past D - 1 replay the wave's last valid disparity's data
    const int lmax = (a.D - 1 - wave) / NW;
    const int l_eff = min(lane, lmax);
    const int cbase = x0 - RAD - (NW * 63 + wave);  // first R column this wave stages
    uint32_t* rbuf = smem + C::RBUF_OFF + wave * NB * C::NRS;
    uint32_t* comb = smem + C::COMB_OFF;
    uint32_t* tb = smem + C::TB_OFF + wave * C::TB_WORDS;
    // transposed reads (the paired kernel's conflict-free window order): lane m = 8p + q takes words
    // 64 p + 8 q .. + 7; key d bytes of the source lanes 8 q + 4 win + e.  Replaying lanes keep their
    // own (larger) d: same cost as lane lmax, so they never win; NW 63 + wave <= 255.
    uint32_t rdw[2], dtab[2];
    {
        const int p = lane >> 3, q = lane & 7, rot = ((q >> 2) ^ (p >> 1)) & 1;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int win = j ^ rot;
            rdw[j] = (uint32_t)(16 * p + 2 * q + win);
            uint32_t w = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) w |= (uint32_t)(NW * (8 * q + 4 * win + e) + wave) << (8 * e);
            dtab[j] = w;
        }
    }
    const double* lut_s = reinterpret_cast<const double*>(smem + C::LUT_OFF);
    const int s_l = NW * (63 - l_eff);  // this lane's first staged entry (a multiple of VEC)
    const int nout = y_end - y_begin;
    const int T = nout + 2 * RAD;
    const int Hm1 = a.H - 1, Wm1 = a.W - 1;
    auto row_off = [&](int t) -> uint32_t {
        const int y = min(max(y_begin - RAD + t, 0), Hm1);
        return (uint32_t)(y * a.pitch);
    };
    const uint8_t* const Lseg = L + LS::base(x0);
    const uint8_t* const Rdma = R - kDmaBias;
    const int y0 = y_begin - RAD;
    const int last_off = Hm1 * a.pitch;
    int rawL = (y0 + WIN + 1) * a.pitch, rawR = (y0 + WIN + PD) * a.pitch;
    const su4 rsrc = [&] {
        const uint64_t base = reinterpret_cast<uint64_t>(Rdma);
        su4 r;
        r[0] = (uint32_t)base;
        r[1] = (uint32_t)(base >> 32);
        r[2] = 0xFFFFFFFFu;
        r[3] = 0x00020000u;
        return r;
    }();
    uint32_t colRb[C::NQ];
#pragma unroll
    for (int i = 0; i < C::NQ; ++i)
        colRb[i] = (uint32_t)min(max(cbase + lane + 64 * i, 0), Wm1) + kDmaBias - 256u * (uint32_t)i;
    const uint32_t rbase = lds_addr(rbuf);
    auto issue_dma = [&](int t) {
        const int buf = t & (NB - 1);
        dma_row<C::NQ>(Rdma + row_off(t), colRb, rbase + 4u * (uint32_t)(buf * C::NRS));
    };
    LWords lw_next;
    auto load_lw = [&](int t) { lw_next = s_load_words_pin<LS::NLD>(Lseg, row_off(t)); };
    using VT = typename VecT<C::VEC>::T;
    ssd_u4 trq[2];  // the pipelined argmin's transposed words
    const uint32_t ra0 = lds_addr(rbuf + s_l);

    auto do_row = [&](int t_in, auto warm_tag, auto i_tag, uint32_t(&S)[K], uint32_t(&ring)[WIN][K], auto&& pre) {
        constexpr bool WARM = decltype(warm_tag)::value;
        constexpr int I = decltype(i_tag)::value;
        int t = t_in;
        asm volatile("" : "+s"(t));
        wait_vmcnt<(PD - 1) * NDMA>();  // row t has landed in LDS
        __builtin_amdgcn_wave_barrier();
        if constexpr (WARM) {
            issue_dma(t + PD);
        } else {
            int rr = rawR;
            asm volatile("" : "+s"(rr));
            const int buf = (t + PD) & (NB - 1);
            dma_row_buf<C::NQ>(rsrc, (uint32_t)min(rr, last_off), colRb, rbase + 4u * (uint32_t)(buf * C::NRS));
            rawR = rr + a.pitch;
        }
        if constexpr (!WARM) {
#pragma unroll
            for (int x = 0; x < K; ++x) S[x] -= ring[I][x];
        }
        uint32_t Lv[NPOS];
        {
            wait_lgkm0_pin<LS::NLD>(lw_next);
            LWords cur = lw_next;
            uint32_t lw[8];
            unpack_words<LS::NLD>(cur, lw);
#pragma unroll
            for (int j = 0; j < NPOS; ++j) {
                const int bidx = LS::byte(j);
                Lv[j] = (lw[bidx >> 2] >> (8 * (bidx & 3))) & 0xFFu;
            }
        }
        int boff = (t & (NB - 1)) * C::NRS;
        asm volatile("" : "+s"(boff));
        const VT* rb = reinterpret_cast<const VT*>(rbuf + boff + s_l);
        uint32_t E[C::NPOS_V];
        constexpr bool LDSR = C::VEC == 2;
        constexpr int NV = C::NPOS_V / 2;
        ssd_u2 ev[NV];
        if constexpr (LDSR) {
            // the previous row's transposed words retired first (see usv_sad_pair.hip)
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(trq[0]), "+v"(trq[1]) : : "memory");
            const uint32_t ra = ra0 + 4u * (uint32_t)boff;
            [&]<int... Kk>(std::integer_sequence<int, Kk...>) {
                (ssd_ds_read_b64<8u * Kk>(ev[Kk], ra), ...);
            }(std::make_integer_sequence<int, NV>{});
        } else {
#pragma unroll
            for (int k = 0; k < C::NPOS_V / C::VEC; ++k) {
                const VT v = rb[k];
#pragma unroll
                for (int e = 0; e < C::VEC; ++e) E[k * C::VEC + e] = vget<C::VEC>(v, e);
            }
        }
        // P[j + 1] = P[j] + (L_j - R_j)^2; H[x] is formed as soon as P[x + w] exists
        uint32_t A[NPOS + 1];
        A[0] = 0;
        auto chain_step = [&](auto jt) {
            constexpr int j = decltype(jt)::value;
            if constexpr (LDSR && (j & 1) == 0) {  // step j = 2k first needs pair k
                constexpr int k = j / 2;
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_waitcnt(0xC07F | ((NV - 1 - k) << 8));
                asm volatile("" ::"v"(ev[k]));
                __builtin_amdgcn_sched_barrier(0);
                E[2 * k] = ev[k].x;
                E[2 * k + 1] = ev[k].y;
            }
            const int diff = (int)Lv[j] - (int)E[j];
            A[j + 1] = (uint32_t)((int)A[j] + __mul24(diff, diff));
            if constexpr (j + 1 >= WIN) {
                constexpr int x = j + 1 - WIN;
                const uint32_t h = A[x + WIN] - A[x];
                S[x] += h;
                ring[I][x] = h;
            }
            pre(jt);
            if constexpr (!WARM) __builtin_amdgcn_sched_barrier(0);
        };
        [&]<int... J>(std::integer_sequence<int, J...>) {
            (chain_step(std::integral_constant<int, J>{}), ...);
        }(std::make_integer_sequence<int, NPOS>{});
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (WARM) {
            load_lw(t + 1);
        } else {
            int rl = rawL;
            asm volatile("" : "+s"(rl));
            lw_next = s_load_words_pin<LS::NLD>(Lseg, (uint32_t)min(rl, last_off));
            rawL = rl + a.pitch;
        }
        __builtin_amdgcn_sched_barrier(0);
    };

    int cb = 0, y_chunk = y_begin;
    // the paired kernel's wide flush: one 8-byte disparity store per row, 16-byte distance stores
    const bool wide = ((reinterpret_cast<uintptr_t>(disp + x0) | (uintptr_t)a.disp_pitch) & 3u) == 0;
    auto flush = [&](int rows) {
        if constexpr (NW > 1) lds_barrier();
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const uint32_t* crow = comb + (cb * KRB) * NW * K;
        if (wide) {
            if (tid < rows) {
                uint4 k0 = reinterpret_cast<const uint4*>(crow + tid * NW * K)[0];
                uint4 k1 = reinterpret_cast<const uint4*>(crow + tid * NW * K)[1];
#pragma unroll
                for (int w2 = 1; w2 < NW; ++w2) {
                    const uint4 m0 = reinterpret_cast<const uint4*>(crow + (tid * NW + w2) * K)[0];
                    const uint4 m1 = reinterpret_cast<const uint4*>(crow + (tid * NW + w2) * K)[1];
                    k0 = make_uint4(min(k0.x, m0.x), min(k0.y, m0.y), min(k0.z, m0.z), min(k0.w, m0.w));
                    k1 = make_uint4(min(k1.x, m1.x), min(k1.y, m1.y), min(k1.z, m1.z), min(k1.w, m1.w));
                }
                const uint32_t lo = __builtin_amdgcn_perm(k0.y, k0.x, 0x0c0c0400u) | __builtin_amdgcn_perm(k0.w, k0.z, 0x04000c0cu);
                const uint32_t hi = __builtin_amdgcn_perm(k1.y, k1.x, 0x0c0c0400u) | __builtin_amdgcn_perm(k1.w, k1.z, 0x04000c0cu);
                const size_t y = (size_t)(y_chunk + tid);
                *reinterpret_cast<uint2*>(disp + y * a.disp_pitch + x0) = make_uint2(lo, hi);
            }
            if (dist && tid < 4 * rows) {
                struct __attribute__((aligned(8))) D2 { double a, b; };
                const int r = tid >> 2, q = tid & 3;
                uint2 kk = reinterpret_cast<const uint2*>(crow + r * NW * K)[q];
#pragma unroll
                for (int w2 = 1; w2 < NW; ++w2) {
                    const uint2 m = reinterpret_cast<const uint2*>(crow + (r * NW + w2) * K)[q];
                    kk = make_uint2(min(kk.x, m.x), min(kk.y, m.y));
                }
                const size_t y = (size_t)(y_chunk + r);
                *reinterpret_cast<D2*>(dist + y * a.dist_pitch + x0 + 2 * q) = D2{lut_s[kk.x & 0xFFu], lut_s[kk.y & 0xFFu]};
            }
        } else {
            for (int i = tid; i < rows * K; i += NW * 64) {
                const int row = i / K, p = i - row * K;
                uint32_t key = 0xFFFFFFFFu;
#pragma unroll
                for (int w2 = 0; w2 < NW; ++w2) key = min(key, crow[(row * NW + w2) * K + p]);
                const uint32_t dv = key & 0xFFu;
                const size_t y = (size_t)(y_chunk + row);
                disp[y * a.disp_pitch + x0 + p] = (uint8_t)dv;
                if (dist) dist[y * a.dist_pitch + x0 + p] = lut_s[dv];
            }
        }
        y_chunk += rows;
        cb ^= 1;
    };
    const uint32_t tb_lds = lds_addr(tb);
    auto tr_issue = [&](const uint32_t(&S)[K]) {
        if constexpr (C::VEC == 2) {  // (NW = 1, 4: more VGPRs, a spill at r = 5, NW = 4)
            static_assert(K == 8, "eight transpose stores");
            asm volatile("s_mov_b32 m0, %8\n\ts_nop 0\n\t"
                         "ds_write_addtid_b32 %0\n\tds_write_addtid_b32 %1 offset:256\n\t"
                         "ds_write_addtid_b32 %2 offset:512\n\tds_write_addtid_b32 %3 offset:768\n\t"
                         "ds_write_addtid_b32 %4 offset:1024\n\tds_write_addtid_b32 %5 offset:1280\n\t"
                         "ds_write_addtid_b32 %6 offset:1536\n\tds_write_addtid_b32 %7 offset:1792"
                         :: "v"(S[0]), "v"(S[1]), "v"(S[2]), "v"(S[3]), "v"(S[4]), "v"(S[5]), "v"(S[6]), "v"(S[7]),
                            "s"(tb_lds) : "memory", "m0");
        } else {
#pragma unroll
            for (int i = 0; i < K; ++i) tb[64 * i + lane] = S[i];
        }
        asm volatile("" ::: "memory");
#pragma unroll
        for (int j = 0; j < 2; ++j) trq[j] = reinterpret_cast<const ssd_u4*>(tb)[rdw[j]];
        asm volatile("" ::: "memory");
    };
    uint32_t fv[8], fb, fm;
    auto tr_piece = [&](auto jt, int slot) {
        constexpr int J = decltype(jt)::value;
        if constexpr (J < 8) {
            constexpr int j = J >> 2, e = J & 3;
            const uint32_t w = e == 0 ? trq[j].x : e == 1 ? trq[j].y : e == 2 ? trq[j].z : trq[j].w;
            fv[J] = __builtin_amdgcn_perm(w, dtab[j], 0x06050400u + (uint32_t)e);  // (cost << 8) | d
        } else if constexpr (J == 8) {
            fb = min(min(fv[0], fv[1]), fv[2]);
            fm = min(min(fv[3], fv[4]), fv[5]);
        } else if constexpr (J == 9) {
            fm = min(min(fv[6], fv[7]), min(fm, fb));
        } else if constexpr (J == 10) {
            fm = min(fm, dpp<kQuadSwap1>(fm));
        } else if constexpr (J == 11) {
            fm = min(fm, dpp<kQuadSwap2>(fm));
        } else if constexpr (J == 12) {
            fm = min(fm, dpp<kRowHalfMirror>(fm));
        } else if constexpr (J == 13) {
            comb[((cb * KRB + slot) * NW + wave) * K + (lane >> 3)] = fm;
        }
    };
    auto tr_finish = [&](int slot) {
        [&]<int... J>(std::integer_sequence<int, J...>) {
            (tr_piece(std::integral_constant<int, J>{}, slot), ...);
        }(std::make_integer_sequence<int, C::NPC>{});
    };
    auto no_pre = [](auto) {};

    uint32_t S[K];
#pragma unroll
    for (int i = 0; i < K; ++i) S[i] = 0;
    uint32_t ring[WIN][K];
    static_assert(C::LUT_OFF % 4 == 0, "16-byte aligned table");
    if (dist) lut_dma(a.lut, smem + C::LUT_OFF, lane);
    [&]<int... P>(std::integer_sequence<int, P...>) { (issue_dma(P), ...); }(std::make_integer_sequence<int, PD>{});
    load_lw(0);
    using WarmT = std::integral_constant<bool, true>;
    using SteadyT = std::integral_constant<bool, false>;
    [&]<int... I>(std::integer_sequence<int, I...>) {
        (do_row(I, WarmT{}, std::integral_constant<int, I>{}, S, ring, no_pre), ...);
    }(std::make_integer_sequence<int, WIN>{});
    // pipelined argmin: output row k is slot k % KRB, issued after its chain and finished during the
    // next row's chain; slot I is pending when the I-th row of a WIN-row group starts
    static_assert(KRB == WIN, "pending slot = row index in the unrolled group");
    tr_issue(S);
    __builtin_amdgcn_sched_barrier(0);
    auto step = [&](int t0, auto i_tag) {
        constexpr int I = decltype(i_tag)::value;
        do_row(t0 + I, SteadyT{}, i_tag, S, ring, [&](auto jt) {
            if constexpr (decltype(jt)::value < C::NPC) tr_piece(jt, I);
        });
        if constexpr (I == KRB - 1) flush(KRB);
        tr_issue(S);
        __builtin_amdgcn_sched_barrier(0);
    };
    for (int t0 = WIN; t0 < T; t0 += WIN) {
        [&]<int... I>(std::integer_sequence<int, I...>) {
            bool go = true;
            ((go = go && (t0 + I < T), go ? step(t0, std::integral_constant<int, I>{}) : void()), ...);
        }(std::make_integer_sequence<int, WIN>{});
    }
    wait_lgkm0_pin<LS::NLD>(lw_next);  // retire the unused last L load before its SGPRs are reused
    const int last = (nout - 1) % KRB;
    tr_finish(last);
    if (last == KRB - 1) flush(KRB);
    const int rest = nout % KRB;
    if (rest) flush(rest);
    wait_vmcnt<0>();
}

// Per-tile work of the band plan (the map of sad_fast_kernel: XCD-contiguous tile runs,
// generation-weighted band heights).
struct TileWork {
    int xt, x0, y_begin, y_end;
    unsigned pair;
};
__device__ __forceinline__ TileWork tile_work(const BandPlan& P, const MatchArgs& a, int K) {
    const unsigned total = gridDim.x, lin = blockIdx.x;
    const unsigned xcd = lin & 7u, base = total >> 3, rem = total & 7u;
    const unsigned tile = xcd * base + min(xcd, rem) + (lin >> 3);
    const unsigned nxt = (unsigned)P.n_xt, per_pair = nxt * (unsigned)P.m;
    const bool past = tile >= per_pair && P.extra > 0;
    const unsigned col_xt = past ? tile - per_pair : tile % nxt;
    const unsigned s = past ? (unsigned)P.m : (tile / nxt) % (unsigned)P.m;
    const unsigned pair = past ? 0u : tile / per_pair;
    const unsigned m_col = (unsigned)P.m + (col_xt < (unsigned)P.extra ? 1u : 0u);
    const unsigned long_run = base + 1u, split = rem * long_run;
    const BandSpan bs = band_span(pair, per_pair, nxt, col_xt, s, m_col, base, long_run, split,
                                  (unsigned)P.gen_g, P.weights);
    const unsigned pre = bs.pre, tot = bs.tot;
    TileWork tw;
    tw.xt = (int)col_xt;
    tw.x0 = tw.xt * K;
    if (tw.xt == P.n_xt - 1) tw.x0 = a.W - K;
    else if (tw.xt == P.n_xt - 2) tw.x0 = min(tw.x0, a.W - 2 * K);
    tw.y_begin = (int)((unsigned long long)a.H * pre / tot);
    tw.y_end = (int)((unsigned long long)a.H * (pre + bs.own) / tot);
    tw.pair = pair;
    return tw;
}

// r = 5 holds its 11-row ring at three waves per SIMD; r = 6, 7 (13 / 15 rows) at two.
constexpr int ssd_occ(int rad) { return rad == 5 ? 3 : 2; }

template <int RAD, int NW>
__global__ __launch_bounds__(NW * 64, ssd_occ(RAD)) void ssd_fast_kernel(const uint8_t* __restrict__ L,
                                                                        const uint8_t* __restrict__ R,
                                                                        uint8_t* __restrict__ disp,
                                                                        double* __restrict__ dist, MatchArgs a,
                                                                        BandPlan P) {
    using C = SCfg<RAD, NW>;
    __shared__ __attribute__((aligned(16))) uint32_t smem[C::SMEM_WORDS];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const TileWork tw = tile_work(P, a, C::K);
    L += (size_t)tw.pair * a.pair_stride;
    R += (size_t)tw.pair * a.pair_stride;
    disp += (size_t)tw.pair * a.disp_stride;
    if (dist) dist += (size_t)tw.pair * a.dist_stride;  // (the table is staged inside the band loop)
    if (tw.y_end <= tw.y_begin) return;
    if (tw.xt == 0)
        ssd_band_loop<RAD, NW, kLeft>(L, R, disp, dist, a, smem, lane, wave, tw.x0, tw.y_begin, tw.y_end);
    else if (tw.xt == P.n_xt - 1)
        ssd_band_loop<RAD, NW, kRight>(L, R, disp, dist, a, smem, lane, wave, tw.x0, tw.y_begin, tw.y_end);
    else
        ssd_band_loop<RAD, NW, kInterior>(L, R, disp, dist, a, smem, lane, wave, tw.x0, tw.y_begin, tw.y_end);
}

template <int RAD, int NW>
int resident_ssd_blocks_per_cu() {
    static const int n = [] {
        int v = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, ssd_fast_kernel<RAD, NW>, NW * 64, 0) != hipSuccess ||
            v <= 0)
            v = 1;
        return v;
    }();
    return n;
}

#ifndef USV_SSD_GEN_WEIGHTS
#define USV_SSD_GEN_WEIGHTS 0x46465A64u  // 100, 90, 70, 70: rocprof A/B at config C SSD 102.4 -> 97.7 us (100:75:50 118.0, 100:95:85 98.4)
#endif
template <int RAD, int NW>
hipError_t launch_ssd_rn(const MatchArgs& a, hipStream_t s) {
    constexpr int K = SCfg<RAD, NW>::K, WIN = 2 * RAD + 1;
    BandPlan P{};
    P.n_xt = (a.W + K - 1) / K;
    const int per_cu = resident_ssd_blocks_per_cu<RAD, NW>();
    const long slots = (long)cu_count() * per_cu;
    const long NC = (long)P.n_xt * a.batch;
    long m = slots / NC;
    if (m < 1) m = 1;
    const long m_max = a.H / (kMinBandWins * WIN) > 0 ? a.H / (kMinBandWins * WIN) : 1;
    if (m > m_max) m = m_max;
    P.m = (int)m;
    const long ex = slots - NC * m;
    P.extra = (a.batch == 1 && ex > 0 && ex < P.n_xt &&
               a.H / (m + 1) >= kMinBandWins * WIN) ? (int)ex : 0;
    const long total = NC * m + P.extra;
    if (total > 0x7FFFFFFFL) return hipErrorInvalidValue;
    P.gen_g = (int)((4L * (cu_count() / 8)) / NW);
    if (P.gen_g < 1) P.gen_g = 1;
    const bool three = per_cu * NW == 12 && total > 2L * 8 * P.gen_g;
    P.weights = three ? USV_SSD_GEN_WEIGHTS : 0x01010101u;
    hipLaunchKernelGGL((ssd_fast_kernel<RAD, NW>), dim3((unsigned)total), dim3(NW * 64), 0, s, a.L, a.R, a.disp,
                       a.dist, a, P);
    return hipGetLastError();
}
template <int RAD>
hipError_t launch_ssd_r(const MatchArgs& a, hipStream_t s) {
    if (a.D <= 64) return launch_ssd_rn<RAD, 1>(a, s);
    if (a.D <= 128) return launch_ssd_rn<RAD, 2>(a, s);
    return launch_ssd_rn<RAD, 4>(a, s);
}

}  // namespace

hipError_t launch_ssd(const MatchArgs& a, hipStream_t s) {
    switch ((a.w - 1) / 2) {
        case 5: return launch_ssd_r<5>(a, s);
        case 6: return launch_ssd_r<6>(a, s);
        case 7: return launch_ssd_r<7>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace usv
