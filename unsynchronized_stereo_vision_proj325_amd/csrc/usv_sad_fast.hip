// usv_sad_fast.hip -- the hot path: fused SAD block match + argmin on gfx950.
//
// Spec: SURVEY.md §8(a) A1 (restated in oracle/sad_oracle.c).  The reference
// has no block matcher; its nearest primitive is the u8
// absdiff motion mask at P/Main.cpp:304.
//
// Mapping (DESIGN.md §3 has the derivation and the instruction budget):
//   * lane = disparity.  A workgroup is NW waves; lane l of wave w owns
//     d = NW*l + w, so the L operand is uniform across the wave (SGPRs) and
//     only R is gathered per lane.  Lanes with d >= D replay the wave's last
//     valid disparity (same data, same key), which cannot change the argmin.
//   * one workgroup = one x-tile of K = 16 outputs x one band of rows, walking
//     down the band.  Per input row each lane runs a horizontal prefix chain
//     packed two-per-register: the low half accumulates columns x, the high
//     half columns x + K/2 (v_sad_u8 / v_sad_hi_u8: one |L-R| + accumulate
//     each), so the row-window sums of two outputs come from one packed
//     subtraction H = P[x+w] - P[x].
//   * the vertical window is a running sum S += H(new row) - H(row w back) in
//     packed u16 (the cost of a 15x15 SAD window is <= 57375); the w rows of H
//     history live in a register ring rotated statically by unrolling the row
//     loop w times.
//   * argmin: keys (cost << 8) | d are assembled with one v_perm per pixel,
//     then the min over the 64 lanes of the 16 pixels is a transpose-reduction
//     (permlane32_swap, permlane16_swap, DPP mirror rounds); the smallest d
//     wins ties by construction.
//   * R rows are staged by LDS-DMA (global_load_lds_ubyte writes one u32 per
//     column) into a per-wave ring of NB row buffers, PD rows ahead, so input
//     latency is hidden without registers; L rows come through the scalar
//     cache one row ahead, border replication as compile-time byte maps.
//   * the NW waves' partial minima are combined through LDS every WIN rows.
// Integer arithmetic only: bit-exact with the oracle by construction.
#include "usv_sad_common.hpp"

namespace usv {
namespace {

#if USV_STAMPS
// phases: 0 DMA wait, 1 L-word wait, 2 chain+H+S, 3 keys+reduce, 4 flush, 5 rows, 6 waves, 7 total
__device__ unsigned long long g_usv_stamps[8];
struct Stamps {
    uint64_t acc[5] = {0, 0, 0, 0, 0}, last = 0, t_begin = 0, rows = 0;
    __device__ static uint64_t now() {
        uint64_t t;
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
        __builtin_amdgcn_sched_barrier(0);
        return t;
    }
    __device__ void mark(int phase) { const uint64_t t = now(); acc[phase] += t - last; last = t; }
    __device__ void skip() { last = now(); }
};
#define USV_STAMP(p) st.mark(p)
#define USV_STAMP_SKIP() st.skip()
#else
#define USV_STAMP(p) ((void)0)
#define USV_STAMP_SKIP() ((void)0)
#endif

#if USV_WGTIME
// per workgroup: {start, end} (100 MHz realtime), HW_ID, XCC_ID, x-tile, band
__device__ unsigned long long g_usv_wgtime[4096 * 8];
#endif

template <int RAD, int NW, int EDGE>
__device__ __forceinline__ void band_loop(const uint8_t* __restrict__ L,
                                          const uint8_t* __restrict__ R,
                                          uint8_t* __restrict__ disp, double* __restrict__ dist,
                                          const MatchArgs& a, uint32_t* smem, int lane,
                                          int wave, int x0, int y_begin, int y_end) {
    using C = Cfg<RAD, NW>;
    using LS = LSeg<RAD, EDGE>;
    using LWords = typename SWords<LS::NLD>::T;
    constexpr int WIN = C::WIN, K = C::K, HALF = C::HALF, NB = C::NB, PD = C::PD, KRB = C::KRB;
    constexpr int NDMA = C::NQ;  // VMEM ops issued per input row
    // lane l owns d = NW*l + wave; lanes past D-1 replay the wave's last valid
    // disparity (same data, same key: they cannot change the argmin)
    const int lmax = (a.D - 1 - wave) / NW;
    const int l_eff = min(lane, lmax);
    const uint32_t d_eff = (uint32_t)(NW * l_eff + wave);
    const int cbase = x0 - RAD - (NW * 63 + wave);  // first R column this wave stages
    uint32_t* rbuf = smem + C::RBUF_OFF + wave * NB * C::NRS;
    uint32_t* comb = smem + C::COMB_OFF;
    uint32_t* tb = smem + C::TB_OFF + wave * C::TB_WORDS;
    // transposed-read windows (uint4 index): lane m = 4p + q, window j visited as (j + p) & 3
    uint32_t rd[4];
    {
        const int p = lane >> 2, q = lane & 3;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            rd[j] = (uint32_t)(16 * (C::RED_PACKED ? (p & 7) : p) + 4 * q + ((j + p) & 3));
    }
    // packed transpose: source disparities of each read (bytes) and the v_perm selectors
    uint32_t dpk[4], psel[4];
    {
        const int p = lane >> 2, q = lane & 3;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint32_t w = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int src = 16 * q + 4 * ((j + p) & 3) + e;
                w |= (uint32_t)(NW * min(src, lmax) + wave) << (8 * e);
            }
            dpk[j] = w;
        }
        const uint32_t half = p >= 8 ? 0x00020200u : 0u;  // cost bytes 6,7 (high half) or 4,5 (low)
#pragma unroll
        for (int e = 0; e < 4; ++e) psel[e] = (0x0c050400u | half) + (uint32_t)e;
    }
    const double* lut_s = reinterpret_cast<const double*>(smem + C::LUT_OFF);
    const int s_l = NW * (63 - l_eff);  // this lane's first chain entry in a row buffer
    const int nout = y_end - y_begin;
    const int T = nout + 2 * RAD;  // input rows walked
    const int Hm1 = a.H - 1, Wm1 = a.W - 1;

    // Row t's byte offset (clamped row; 32-bit: the host keeps pitch * H < 2^31)
    // against per-band bases that already carry the constant parts (L's segment
    // start, R's DMA bias): one multiply and one 64-bit add per pointer per row.
    auto row_off = [&](int t) -> uint32_t {
        const int y = min(max(y_begin - RAD + t, 0), Hm1);
        return (uint32_t)(y * a.pitch);
    };
    const uint8_t* const Lseg = L + LS::base(x0);
    const uint8_t* const Rdma = R - kDmaBias;  // (dma_row: one M0 per row, lane offsets biased by kDmaBias)
    // raw (unclamped) byte offsets of the rows the next steady row loads: L row t + 1, R row t + PD
    const int y0 = y_begin - RAD;
    const int last_off = Hm1 * a.pitch;
    int rawL = (y0 + WIN + 1) * a.pitch, rawR = (y0 + WIN + PD) * a.pitch;
    const su4 rsrc = [&] {
        const uint64_t base = reinterpret_cast<uint64_t>(Rdma);
        su4 r;
        r[0] = (uint32_t)base;
        r[1] = (uint32_t)(base >> 32);  // stride 0: raw buffer
        r[2] = 0xFFFFFFFFu;             // num_records: no range limit (offsets stay inside R)
        r[3] = 0x00020000u;             // gfx9 raw-buffer word 3 (CK_BUFFER_RESOURCE_3RD_DWORD)
        return r;
    }();

    // ---- R rows: LDS-DMA into the ring, PD rows ahead ----
    // Rows past the band are clamped to real rows: harmless extra loads.
    // Clamped source columns do not depend on the row: 32-bit lane offsets
    // against a scalar row base (the saddr form of the DMA, no 64-bit VGPRs).
    uint32_t colR[C::NQ];
#pragma unroll
    for (int i = 0; i < C::NQ; ++i) colR[i] = (uint32_t)min(max(cbase + lane + 64 * i, 0), Wm1);
    uint32_t colRb[C::NQ];  // dma_row: + kDmaBias - 256 q (the row pointer carries -kDmaBias)
#pragma unroll
    for (int i = 0; i < C::NQ; ++i) colRb[i] = colR[i] + kDmaBias - 256u * (uint32_t)i;
    const uint32_t rbase = lds_addr(rbuf);
    // row t into ring slot t & (NB - 1)
    auto issue_dma = [&](int t) {
        const int buf = t & (NB - 1);
        dma_row<C::NQ>(Rdma + row_off(t), colRb, rbase + 4u * (uint32_t)(buf * C::NRS));
    };

    // ---- L bytes: the row segment through the scalar cache, one row ahead.
    // Issued as inline asm: the compiler would otherwise turn it into a
    // vector load (the LDS-DMA intrinsic defeats its no-clobber proof) and
    // drain the DMA look-ahead with vmcnt(0).
    LWords lw_next;
    auto load_lw = [&](int t) { lw_next = s_load_words<LS::NLD>(Lseg + row_off(t)); };

#if USV_STAMPS
    Stamps st;
    st.t_begin = st.last = Stamps::now();
#endif
    // One input row t = t0 + I (t0 a multiple of WIN): packed chain, H pairs,
    // S / ring update.  I selects the H ring slot at compile time.
    auto do_row = [&](int t_in, auto warm_tag, auto i_tag, uint32_t(&S)[HALF], uint32_t(&ring)[WIN][HALF]) {
        constexpr bool WARM = decltype(warm_tag)::value;
        constexpr int I = decltype(i_tag)::value;
        // opaque row index: keeps the compiler from computing every unrolled
        // row's pointers up front (SGPR pressure that ends in VGPR spills)
        int t = t_in;
        asm volatile("" : "+s"(t));
        wait_vmcnt<(PD - 1) * NDMA>();  // row t has landed in LDS
        __builtin_amdgcn_wave_barrier();
        if constexpr (!WARM) {
            int rr = rawR;
            asm volatile("" : "+s"(rr));  // opaque: one row's offset at a time
            const int buf = (t + PD) & (NB - 1);
            dma_row_buf<C::NQ>(rsrc, (uint32_t)min(rr, last_off), colRb, rbase + 4u * (uint32_t)(buf * C::NRS));
            rawR = rr + a.pitch;
        } else {
            issue_dma(t + PD);
        }
        USV_STAMP(0);

        uint32_t Lv[C::NPOS];
        {
            LWords cur = lw_next;
            wait_lgkm0<LS::NLD>(cur);  // row t's words have arrived
            USV_STAMP(1);
            uint32_t lw[8];
            unpack_words<LS::NLD>(cur, lw);
#pragma unroll
            for (int j = 0; j < C::NPOS; ++j) {
                const int bidx = LS::byte(j);
                if (kLWholeWord<RAD, EDGE> && (bidx & 3) == 0) Lv[j] = lw[bidx >> 2];
                else Lv[j] = (lw[bidx >> 2] >> (8 * (bidx & 3))) & 0xFFu;
            }
        }

        using VT = typename VecT<C::VEC>::T;
        // Row-buffer offset as an opaque scalar: one v_add per row, instead
        // of the compiler keeping a VGPR base per static ring slot (the
        // ds_read2 offset field only spans 2 KB) live through the loop.
        int boff = (t & (NB - 1)) * C::NRS;
        asm volatile("" : "+s"(boff));
        const VT* rb = reinterpret_cast<const VT*>(rbuf + boff + s_l);
        uint32_t Rv[C::NPOS_V];
        // issue the reads in the chain's order of use (step j needs columns j
        // and j + HALF) so the first steps only wait for the first reads
#pragma unroll
        for (int k = 0; k < C::NPOS_V / C::VEC; ++k) {
            constexpr int NV = C::NPOS_V / C::VEC, HV = HALF / C::VEC;
            const int jv = read_order<NV, HV>(k);
            const VT v = rb[jv];
#pragma unroll
            for (int e = 0; e < C::VEC; ++e) Rv[jv * C::VEC + e] = vget<C::VEC>(v, e);
        }
        // Packed prefix P[j] = [sum_{i<j} e(i), sum_{i<j} e(i + HALF)] (one chain: two independent
        // half-chains for ILP measured no faster, round 1)
        uint32_t A[C::NSTEP + 1];
        A[0] = 0;
#pragma unroll
        for (int j = 0; j < C::NSTEP; ++j)
            A[j + 1] = __builtin_amdgcn_sad_hi_u8(Lv[j + HALF], Rv[j + HALF], __builtin_amdgcn_sad_u8(Lv[j], Rv[j], A[j]));
#pragma unroll
        for (int x = 0; x < HALF; ++x) {
            // H pair (x, x + HALF) = P[x + WIN] - P[x].  Packed pairs, but
            // every intermediate half stays in [0, 65535] (prefixes are
            // monotone, S - ring is a w-1 row sum), so plain 32-bit add/sub
            // give the packed result exactly: v_add/v_sub_u32 issue at full
            // rate, v_pk_*_u16 at half rate (scripts/probes/valu_rate.hip).
            const uint32_t h = A[x + WIN] - A[x];
            if constexpr (WARM) S[x] = S[x] + h;
            else S[x] = (S[x] - ring[I][x]) + h;
            ring[I][x] = h;
        }
        // The row's LDS reads are all consumed: request row t+1's L words now,
        // so the lgkmcnt waits of this row's LDS reads never retire (and wait
        // for) that scalar load; it has the rest of this row to land.
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        USV_STAMP(2);
#if USV_STAMPS
        st.rows++;
#endif
        if constexpr (!WARM) {
            int rl = rawL;
            asm volatile("" : "+s"(rl));
            lw_next = s_load_words_off<LS::NLD>(Lseg, (uint32_t)min(rl, last_off));
            rawL = rl + a.pitch;
        } else {
            load_lw(t + 1);
        }
        // Keep rows apart: interleaving the unrolled rows only raises
        // register pressure (spills whose reloads would drain the DMA queue).
        __builtin_amdgcn_sched_barrier(0);
    };

    // ---- output: per-row keys -> LDS, cross-wave min every KRB rows ----
    // Output row o goes to combine slot o % KRB; with KRB = WIN the flush
    // points sit at fixed positions of the WIN-unrolled row loop.
    int cb = 0, y_chunk = y_begin;
    auto flush = [&](int rows) {
        lds_barrier();
        // opaque thread id: the flush's per-lane addresses must not be hoisted
        // out of the row loop (they would stay live through it and spill)
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const int items = rows * K;
        for (int i = tid; i < items; i += NW * 64) {
            const int row = i / K, p = i - row * K;
            uint32_t key = 0xFFFFFFFFu;
#pragma unroll
            for (int w2 = 0; w2 < NW; ++w2) key = min(key, comb[((cb * KRB + row) * NW + w2) * K + p]);
            const uint32_t dv = key & 0xFFu;
            const size_t y = (size_t)(y_chunk + row);
            disp[y * a.disp_pitch + x0 + p] = (uint8_t)dv;
            if (dist) dist[y * a.dist_pitch + x0 + p] = lut_s[dv];
        }
        y_chunk += rows;
        cb ^= 1;
    };
    auto emit = [&](const uint32_t(&S)[HALF], int slot) {
        uint32_t m;
        if constexpr (C::RED_PACKED) {
            m = reduce16_lds_packed(S, tb, lane, rd, dpk, psel);
            comb[((cb * KRB + slot) * NW + wave) * K + (lane >> 2)] = m;
            USV_STAMP(3);
            __builtin_amdgcn_sched_barrier(0);
            return;
        }
        uint32_t keys[K];
#pragma unroll
        for (int i = 0; i < HALF; ++i) {
            keys[i] = __builtin_amdgcn_perm(S[i], d_eff, 0x0c050400u);         // (S.lo << 8) | d
            keys[i + HALF] = __builtin_amdgcn_perm(S[i], d_eff, 0x0c070600u);  // (S.hi << 8) | d
        }
        if constexpr (C::RED_LDS) {
            m = reduce16_lds(keys, tb, lane, rd);
        } else {
            m = reduce16(keys);
        }
        // the 4 lanes of a quad hold the same key: same value, same address
        comb[((cb * KRB + slot) * NW + wave) * K + (lane >> 2)] = m;
        USV_STAMP(3);
        // the next row's loads must not be hoisted into the reduction (the
        // rows are one basic block now: keys + R values + ring would spill)
        __builtin_amdgcn_sched_barrier(0);
    };

    uint32_t S[HALF];
#pragma unroll
    for (int i = 0; i < HALF; ++i) S[i] = 0;
    uint32_t ring[WIN][HALF];

    // prologue: PD rows in flight, L words of row 0 requested
    [&]<int... P>(std::integer_sequence<int, P...>) {
        (issue_dma(P), ...);
    }(std::make_integer_sequence<int, PD>{});
    load_lw(0);

    using WarmT = std::integral_constant<bool, true>;
    using SteadyT = std::integral_constant<bool, false>;
    // ---- warm-up: the first WIN input rows fill the ring; output row 0 ----
    [&]<int... I>(std::integer_sequence<int, I...>) {
        (do_row(I, WarmT{}, std::integral_constant<int, I>{}, S, ring), ...);
    }(std::make_integer_sequence<int, WIN>{});
    emit(S, 0);

    // ---- steady state: input row t0 + I -> output row t0 + I - 2r, slot (I + 1) % WIN
    auto step = [&](int t0, auto i_tag) {
        constexpr int I = decltype(i_tag)::value;
        do_row(t0 + I, SteadyT{}, i_tag, S, ring);
        emit(S, (I + 1) % WIN);
        if constexpr ((I + 1) % WIN == KRB - 1) {
            flush(KRB);
            USV_STAMP(4);
        }
    };
    // (the per-row guard also splits the group into basic blocks: one
    // 2000-instruction block makes the register allocator spill the ring)
    for (int t0 = WIN; t0 < T; t0 += WIN) {
        [&]<int... I>(std::integer_sequence<int, I...>) {
            bool go = true;
            ((go = go && (t0 + I < T), go ? step(t0, std::integral_constant<int, I>{}) : void()), ...);
        }(std::make_integer_sequence<int, WIN>{});
    }
    // The last row requested row T's L words, which nothing reads.  Retire that
    // scalar load before its destination SGPRs can be reused: it writes them
    // whenever its data returns (a late return clobbered the flush's row count
    // and pointers -- an illegal address on the GPU; tests/test_isa_lint.py).
    wait_lgkm0<LS::NLD>(lw_next);
    // rows emitted since the last flush: outputs o with o % WIN in [0, rest)
    const int rest = nout % KRB;
    if (rest) flush(rest);
    wait_vmcnt<0>();  // drain the look-ahead DMAs before the wave retires
#if USV_STAMPS
    if (lane == 0) {
        for (int i = 0; i < 5; ++i) atomicAdd(&g_usv_stamps[i], (unsigned long long)st.acc[i]);
        atomicAdd(&g_usv_stamps[5], (unsigned long long)st.rows);
        atomicAdd(&g_usv_stamps[6], 1ull);
        atomicAdd(&g_usv_stamps[7], (unsigned long long)(Stamps::now() - st.t_begin));
    }
#endif
}

// r = 7 (15-row ring) and r = 6 with four waves need more than 168 VGPRs:
// two waves per SIMD instead of spilling (tests/test_isa_lint.py checks).
constexpr int fast_occ(int rad, int nw) { return (rad >= 7 || (rad == 6 && nw == 4)) ? 2 : kFastOcc; }

template <int RAD, int NW>
__global__ __launch_bounds__(NW * 64, fast_occ(RAD, NW)) void sad_fast_kernel(const uint8_t* __restrict__ L,
                                                              const uint8_t* __restrict__ R,
                                                              uint8_t* __restrict__ disp,
                                                              double* __restrict__ dist,
                                                              MatchArgs a, BandPlan P) {
    using C = Cfg<RAD, NW>;
    __shared__ __attribute__((aligned(16))) uint32_t smem[C::SMEM_WORDS];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#if USV_WGTIME
    const unsigned long long wg_t0 = __builtin_amdgcn_s_memrealtime();
#endif
    // Work map.  Workgroups are dispatched round-robin over the 8 XCDs
    // (linear id mod 8), each with its own L2: XCD k owns the k-th contiguous
    // run of tiles (x-tile fastest, then band, then pair), so the tiles of one
    // band share an L2 and every L/R row is fetched about once.
    // Band heights are weighted by dispatch generation: the SIMD arbitrates
    // VALU issue by age, so with three resident waves per SIMD the first-
    // dispatched generation of workgroups runs ~1.4x faster than the last
    // (scripts/wgtime.py); equal bands end in a one- and two-wave tail.
    // Generation of a tile = (its index in its XCD's run) / P.gen_g, weight =
    // byte g of P.weights; a column's bands get heights proportional to the
    // weights of the tiles that carry them.  Any placement keeps the map a
    // bijection; only speed depends on the dispatch model.
    const unsigned total = gridDim.x, lin = blockIdx.x;
    const unsigned xcd = lin & 7u, base = total >> 3, rem = total & 7u;
    const unsigned tile = xcd * base + min(xcd, rem) + (lin >> 3);
    const unsigned nxt = (unsigned)P.n_xt, per_pair = nxt * (unsigned)P.m;
    // tiles past nxt * m (P.extra > 0, one pair) are band m of x-tiles 0..extra-1
    const bool past = tile >= per_pair && P.extra > 0;
    const unsigned col_xt = past ? tile - per_pair : tile % nxt;
    const unsigned s = past ? (unsigned)P.m : (tile / nxt) % (unsigned)P.m;
    const unsigned pair = past ? 0u : tile / per_pair;
    const unsigned m_col = (unsigned)P.m + (col_xt < (unsigned)P.extra ? 1u : 0u);
    const unsigned long_run = base + 1u, split = rem * long_run;
    // weight sums of the column's bands (usv_band.hpp: one band per lane, three wave sums)
    const BandSpan bs = band_span(pair, per_pair, nxt, col_xt, s, m_col, base, long_run, split,
                                  (unsigned)P.gen_g, P.weights);
    const unsigned pre = bs.pre, tot = bs.tot;
    const unsigned col = pair * nxt + col_xt;
    const int xt = (int)(col % (unsigned)P.n_xt);
    const int band = (int)s;
    const size_t b = col / (unsigned)P.n_xt;
    // x-tile origin: the last tile is aligned to the right border and the one
    // before it pulled left if needed, so only tiles 0 and n-1 clamp L.
    int x0 = xt * C::K;
    const int n_xt = P.n_xt;
    if (xt == n_xt - 1) x0 = a.W - C::K;
    else if (xt == n_xt - 2) x0 = min(x0, a.W - 2 * C::K);
    const int y_begin = (int)((unsigned long long)a.H * pre / tot);
    const int y_end = (int)((unsigned long long)a.H * (pre + bs.own) / tot);
    L += b * a.pair_stride;
    R += b * a.pair_stride;
    disp += b * a.disp_stride;
    if (dist) {
        dist += b * a.dist_stride;
        double* lut_s = reinterpret_cast<double*>(smem + C::LUT_OFF);
        for (int i = threadIdx.x; i < 256; i += NW * 64) lut_s[i] = a.lut[i];
    }
    __syncthreads();
    if (y_end <= y_begin) return;  // (uniform) an empty band: nothing to emit
    if (xt == 0)
        band_loop<RAD, NW, kLeft>(L, R, disp, dist, a, smem, lane, wave, x0, y_begin, y_end);
    else if (xt == n_xt - 1)
        band_loop<RAD, NW, kRight>(L, R, disp, dist, a, smem, lane, wave, x0, y_begin, y_end);
    else
        band_loop<RAD, NW, kInterior>(L, R, disp, dist, a, smem, lane, wave, x0, y_begin, y_end);
#if USV_WGTIME
    __syncthreads();
    if (lane == 0 && blockIdx.x < 4096) {
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        unsigned long long* o = g_usv_wgtime + 8 * blockIdx.x + 4 * (wave & 1);
        o[0] = wg_t0;
        o[1] = __builtin_amdgcn_s_memrealtime();
        o[2] = hw | ((unsigned long long)xcc << 32);
        o[3] = (unsigned long long)xt | ((unsigned long long)band << 32);
    }
#endif
}

// Blocks resident per CU for this instantiation (queried once).
template <int RAD, int NW>
int resident_blocks_per_cu() {
    static const int n = [] {
        int v = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, sad_fast_kernel<RAD, NW>, NW * 64, 0) !=
                hipSuccess || v <= 0)
            v = 1;
        return v;
    }();
    return n;
}

// Relative band heights by dispatch generation, three resident waves per SIMD
// (config C, profiles/probes/wgtime_*.txt: equal bands took 61.5 / 70.0 /
// 84.0 us by generation; one refinement step of heights ~ 1/time gave
// 100 : 85 : 63).  Since every SIMD holds three waves (P.extra), flatter
// heights won: interleaved A/B 100:80:58 / 85:63 / 90:70 / 94:78 / 97:85 =
// 80.5 / 79.1 / 76.8 / 77.9 / 78.7 us (profiles/probes/ab_extra_weights_r01.txt).
#ifndef USV_GEN_WEIGHTS
#define USV_GEN_WEIGHTS 0x46465A64u  // 100, 90, 70, 70
#endif

template <int RAD, int NW>
hipError_t launch_rn(const MatchArgs& a, hipStream_t s) {
    constexpr int K = kK, WIN = 2 * RAD + 1;
    BandPlan P{};
    P.n_xt = (a.W + K - 1) / K;
    // One round of resident workgroups: bands = slots / (x-tiles * pairs),
    // keeping bands at least 2w rows so the ring warm-up stays amortised.
    const int per_cu = resident_blocks_per_cu<RAD, NW>();
    const long slots = (long)cu_count() * per_cu;
    const long NC = (long)P.n_xt * a.batch;
    long m = slots / NC;
    if (m < 1) m = 1;
    const long m_max = a.H / (kMinBandWins * WIN) > 0 ? a.H / (kMinBandWins * WIN) : 1;
    if (m > m_max) m = m_max;
    P.m = (int)m;
    // e.g. 1080p, D = 128: 1536 slots over 120 x-tiles = 12 bands + 96 x-tiles with a 13th
    const long ex = slots - NC * m;
    P.extra = (a.batch == 1 && ex > 0 && ex < P.n_xt &&
               a.H / (m + 1) >= kMinBandWins * WIN) ? (int)ex : 0;
    const long total = NC * m + P.extra;
    if (total > 0x7FFFFFFFL) return hipErrorInvalidValue;
    P.gen_g = (int)((4L * (cu_count() / 8)) / NW);
    if (P.gen_g < 1) P.gen_g = 1;
    // weighted only when every SIMD holds three waves of one round
    const bool three = per_cu * NW == 12 && total > 2L * 8 * P.gen_g;
    P.weights = three ? USV_GEN_WEIGHTS : 0x01010101u;
    dim3 grid((unsigned)total), block(NW * 64);
    hipLaunchKernelGGL((sad_fast_kernel<RAD, NW>), grid, block, 0, s, a.L, a.R, a.disp, a.dist, a, P);
    return hipGetLastError();
}

template <int RAD>
hipError_t launch_r(const MatchArgs& a, hipStream_t s) {
    if (a.D <= 64) return launch_rn<RAD, 1>(a, s);
    if (a.D <= 128) return launch_rn<RAD, 2>(a, s);
    return launch_rn<RAD, 4>(a, s);
}

}  // namespace

#if USV_STAMPS
extern "C" __attribute__((visibility("default"))) int usv_debug_stamps(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_usv_stamps), sizeof(g_usv_stamps)) != hipSuccess) return 1;
    if (reset) {
        static const unsigned long long z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_usv_stamps), z, sizeof(z)) != hipSuccess) return 1;
    }
    return 0;
}
#endif

#if USV_WGTIME
extern "C" __attribute__((visibility("default"))) int usv_debug_wgtime(unsigned long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_usv_wgtime), sizeof(unsigned long long) * 4 * n) != hipSuccess;
}
#endif

bool fast_path_supported(const MatchArgs& a) {
    // W % 4 == 0 and W >= 3 tiles: the border tiles' L maps are compile-time.  SSD (metric 1): the
    // SSD kernel's 8-column L segments exist for 11 <= w <= 15.
    const bool metric_ok = a.metric == 0 || (a.metric == 1 && a.w >= 11);
    return metric_ok && a.w >= 3 && a.w <= 15 && (a.w & 1) && a.D >= 1 && a.D <= 256 &&
           (a.W % 4) == 0 && a.W >= 3 * kK && (a.pitch % 4) == 0 && (long long)a.pitch * a.H < (1LL << 31) &&
           (reinterpret_cast<uintptr_t>(a.L) % 4) == 0 &&
           (reinterpret_cast<uintptr_t>(a.R) % 4) == 0 && (a.batch <= 1 || a.pair_stride % 4 == 0);
}

hipError_t launch_fast(const MatchArgs& a, hipStream_t s) {
    if (!fast_path_supported(a)) return hipErrorInvalidValue;
    if (a.metric == 1) return launch_ssd(a, s);                 // usv_sad_ssd.hip: 11 <= w <= 15
    if (group_path_supported(a)) return launch_group(a, s);   // usv_sad_group.hip: D <= 64, w <= 9
    if (pair_path_supported(a)) return launch_pair(a, s);     // usv_sad_pair.hip: even D > 64, w >= 11
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
}

}  // namespace usv
