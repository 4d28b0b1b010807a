// usv_sad_pair.hip -- the headline block-match kernel on gfx950: SAD with lane = two adjacent
// disparities (sad_pair_kernel; even D > 64, 11 <= w <= 15: configs C, D, E).
//
// Spec: SURVEY.md §8(a) A1 (restated in oracle/sad_oracle.c); DESIGN.md §3 has the derivation.  The
// reference has no block matcher; its nearest primitive is the u8 absdiff motion mask
// at P/Main.cpp:304.  Integer arithmetic only: bit-exact with the oracle by construction.
#include "usv_sad_common.hpp"
#include "usv_tiles.hpp"

namespace usv {
namespace {

// ===================================================================================
// Paired-disparity kernel (D > 64, even D, 5 <= r <= 7): lane = two ADJACENT disparities.
//
// Lane l of wave w owns d = 2 (64 w + l) in the low half of its packed-u16 sums and
// d + 1 in the high half, for K = 8 output columns (wave w: disparities [128 w, 128 w + 128)).  The two share the L byte of each
// chain step (one SGPR for both v_sad_u8 and v_sad_hi_u8) and their R bytes are adjacent
// columns of the staged row: step j reads entries j (d + 1) and j + 1 (d), so a lane reads
// K + 2r + 1 staged entries for 2 x K (column, disparity) pairs per step instead of
// K + 2r for K, and a whole 128-disparity search is ONE wave: per (pixel, disparity) half
// the L-byte extraction, row addressing and LDS-DMA instructions of the column-paired
// kernel above, ~30 % less LDS traffic, and no cross-wave combine barrier at D <= 128.
// Keys: lo = (cost << 8) | d, hi = (cost << 8) | (d + 1); the transpose gives lane
// 8p + q the 8 packed words of pixel p from lanes 8q .. 8q + 7 (16 keys), then three DPP
// rounds across the 8 lanes of the pixel.  Ties -> smallest d as before.
// ===================================================================================
// Argmin transpose of row t finished during row t + 1 (latency hidden by the chain): r = 5 only (at
// r = 6, 7 the held transpose words spill).
template <int RAD>
constexpr bool kPairPipe = RAD == 5;
template <int RAD, int NW>
struct PCfg {
    static constexpr int K = 8;
    static constexpr int WIN = 2 * RAD + 1;
    static constexpr int NPOS = K + 2 * RAD;            // chain steps
    static constexpr int NE = NPOS + 1;                 // staged entries a lane reads per row
    static constexpr int VEC = 2;                       // lane offsets are 2 entries apart
    static constexpr int NE_V = (NE + VEC - 1) / VEC * VEC;
    static constexpr int NR = 2 * 63 + NE_V;            // entries a wave stages per row
    static constexpr int NQ = (NR + 63) / 64;           // DMA instructions per row
    static constexpr int NRS = NQ * 64;
    // Ring slots per wave.  r = 5 with one wave: WIN slots (a static ring -- row t sits in slot t mod WIN,
    // so in the WIN-unrolled row loop every slot, LDS offset and M0 value is a compile-time constant;
    // 12 waves x 13.0 KB fit the CU's 160 KB).  Otherwise 8 slots indexed t & 7 (r = 6, 7 or two waves
    // per workgroup would not fit WIN slots at three waves per SIMD).
#ifndef USV_PAIR_RDASM
#define USV_PAIR_RDASM 1  // staged-entry reads as single ds_read_b64 (inline asm, explicit lgkmcnt waits): C 51.70 -> 49.32 us
#endif
#ifndef USV_PAIR_LEARLY
#define USV_PAIR_LEARLY 5  // the next row's L segment is loaded before the row's chain (not after it) at r <= this
#endif
#ifndef USV_PAIR_M0REUSE
#define USV_PAIR_M0REUSE 1  // static ring: transpose stores off the row DMA's M0; row clamp in the DMA's wait state (SALU -2.9 per row)
#endif
    // (transpose stores as ds_write_addtid_b32: C 52.33 -> 51.77 us, E 511.9 -> 508.0 us, round 4)
    static constexpr bool STATIC = RAD == 5 && NW == 1;
    static constexpr int NB = STATIC ? WIN : 8;
    static constexpr int SPLIT = RAD >= 7 ? 2 : 1;  // r = 7 reads the row's entries in two batches
    // Chain jump: the row sums H[x] = A[x + WIN] - A[x] (x < K) read the prefix A only at 0..K-1 and
    // WIN..WIN+K-1, so the WIN - K + 1 increments j = K-1 .. WIN-1 between them are folded into quads:
    // one 4-byte v_sad_u8 (+ v_sad_hi_u8) per 4 columns, the R bytes packed from the staged entries
    // (r = 5: 18 -> 15 chain steps, r = 7: 22 -> 16).
    static constexpr int JA = K - 1;                                  // first increment in a quad
    static constexpr int JN = (WIN - K + 1) / 4;                      // quads
    static constexpr int JE = JA + 4 * JN;                            // singles resume here
    static constexpr int PD = NB - 1;  // rows of DMA look-ahead
    static constexpr int KRB = WIN;
    static constexpr int RBUF_OFF = 0;
    static constexpr int TB_OFF = RBUF_OFF + NW * NB * NRS;
    static constexpr int TB_WORDS = K * 64;
    static constexpr int COMB_OFF = TB_OFF + NW * TB_WORDS;
    // one wave: its LDS ops run in order, so the flush's reads of a chunk precede the next chunk's
    // writes and one combine buffer suffices (slot addresses are then compile-time); two or more waves
    // alternate two buffers so a flush needs one barrier
    static constexpr int NCB = NW == 1 ? 1 : 2;
    // comb row stride (words): NW x K, padded to 24 at two waves.  The flush reads a row per lane (16-byte reads,
    // 16-lane groups) and a row's quarter per lane (8-byte reads, 32-lane groups); at a 16-word stride both put
    // rows r and r + 4 on the same banks, at 24 every row of a group lands on its own banks.
    static constexpr int CSTR = NW == 1 ? K : NW * K + 8;
    static constexpr int LUT_OFF = COMB_OFF + NCB * KRB * CSTR;
    // distance table in LDS: one wave means D <= 128, so every output disparity is < 128 and half the
    // table suffices (1 KB less: the static ring's 12 workgroups per CU fit only below ~12.5 KB each,
    // profiles/probes_r04/lds_residency_r04.txt)
    static constexpr int LUTN = NW == 1 ? 128 : 256;
    static constexpr int SMEM_WORDS = LUT_OFF + 2 * LUTN;
    static_assert(RAD >= 2 && RAD <= 7, "paired kernel: 5 <= w <= 15");
    static_assert(PD * NQ < 64, "look-ahead DMAs must fit the 6-bit vmcnt");
    static_assert(NQ <= 5, "dma_row_buf issues at most 5 DMAs");
};

typedef uint32_t u2x __attribute__((ext_vector_type(2)));
typedef uint32_t u4x __attribute__((ext_vector_type(4)));
// one ds_read_b64 the compiler cannot pair or count (USV_PAIR_RDASM): the caller waits for it explicitly
template <uint32_t OFF>
__device__ __forceinline__ void ds_read_b64_at(u2x& v, uint32_t addr) {
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
}

template <int RAD, int NW, int EDGE>
__device__ __forceinline__ void pair_band_loop(const uint8_t* __restrict__ L, const uint8_t* __restrict__ R,
                                               uint8_t* __restrict__ disp, double* __restrict__ dist,
                                               const MatchArgs& a, uint32_t* smem, int lane, int wave, int x0,
                                               int y_begin, int y_end) {
    using C = PCfg<RAD, NW>;
    using LS = LSeg<RAD, EDGE, C::K>;
    using LWords = typename SWords<LS::NLD>::T;
    constexpr int WIN = C::WIN, K = C::K, NB = C::NB, PD = C::PD, KRB = C::KRB, NPOS = C::NPOS;
    constexpr int NDMA = C::NQ;
    // lane l owns (d, d + 1), d = 2 (64 wave + l); lanes past the last full pair replay it
    const int lmax = min(63, a.D / 2 - 1 - 64 * wave);
    const int l_eff = min(lane, lmax);
    const int dwave = 128 * wave;
    const int cbase = x0 - RAD - (dwave + 2 * 63 + 1);  // first R column this wave stages
    uint32_t* rbuf = smem + C::RBUF_OFF + wave * NB * C::NRS;
    uint32_t* comb = smem + C::COMB_OFF;
    uint32_t* tb = smem + C::TB_OFF + wave * C::TB_WORDS;
    // transposed reads: lane m = 8p + q takes words 64 p + 8 q .. + 7 as two 16-B windows.  A
    // ds_read_b128 is serviced in four 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32)
    // over 64 banks, and window w of lane (p, q) sits on banks 8 q + 4 w: visiting the windows in
    // the order w = j ^ ((q >> 2) ^ (p >> 1)) gives the 16 lanes of every group 16 distinct
    // 4-bank slots (no conflict; without the p term two lanes of each group collide).
    uint32_t rdw[2], dlo[2], dhi[2];
    {
        const int p = lane >> 3, q = lane & 7, rot = ((q >> 2) ^ (p >> 1)) & 1;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int win = j ^ rot;
            rdw[j] = (uint32_t)(16 * p + 2 * q + win);  // uint4 index: (64 p + 8 q + 4 win) / 4
            // source lanes past lmax replay lane lmax's data: the same cost with a larger d, so
            // their keys never win and their d bytes need no clamp (max 2 (64 + 63) + 1 = 255)
            uint32_t lo = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int src = 8 * q + 4 * win + e;
                lo |= (uint32_t)(dwave + 2 * src) << (8 * e);
            }
            dlo[j] = lo;
            dhi[j] = lo + 0x01010101u;  // d even: + 1 per byte, no carry
        }
    }
    const double* lut_s = reinterpret_cast<const double*>(smem + C::LUT_OFF);
    const int s_l = 2 * (63 - l_eff);  // this lane's first staged entry
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
    // ring slot of input row t (static ring: t mod WIN, known at compile time wherever it is used)
    auto slot_of = [&](int t) { return C::STATIC ? t % NB : (t & (NB - 1)); };
    auto issue_dma = [&](int t, int buf) {
        dma_row<C::NQ>(Rdma + row_off(t), colRb, rbase + 4u * (uint32_t)(buf * C::NRS));
    };
    LWords lw_next;
    auto load_lw = [&](int t) { lw_next = s_load_words_pin<LS::NLD>(Lseg, row_off(t)); };

    u4x trq[2];  // the pipelined argmin's transposed words (tr_issue -> tr_piece)
    const uint32_t ra0 = lds_addr(rbuf + s_l);  // this lane's first staged entry in slot 0
    // the staged-entry pairs of a row (single ds_read_b64 each, do_row).  (Reading the first 2 / 4 / 6 pairs of row
    // t + 1 right after row t's transpose ties: 43.42 / 43.35 / 43.49 vs 43.39 us per step,
    // profiles/probes_r06/ab_k16_r06.txt -- three waves per SIMD already cover that latency.)
    u2x ev[C::NE_V / C::VEC];
    auto do_row = [&](int t_in, auto warm_tag, auto i_tag, uint32_t(&S)[K], uint32_t(&ring)[WIN][K], auto&& pre) {
        constexpr bool WARM = decltype(warm_tag)::value;
        constexpr int I = decltype(i_tag)::value;
        int t = t_in;
        asm volatile("" : "+s"(t));
        wait_vmcnt<(PD - 1) * NDMA>();
        __builtin_amdgcn_wave_barrier();
        // static ring: rows of an unrolled group sit at t = (multiple of WIN) + I, so row t + PD's slot is
        // (I + PD) mod WIN
        constexpr int SLOT_NEXT = C::STATIC ? (I + PD) % NB : -1;
        if constexpr (WARM) {
            issue_dma(t + PD, C::STATIC ? SLOT_NEXT : slot_of(t + PD));
        } else {
            int rr = rawR;
            asm volatile("" : "+s"(rr));
            if constexpr (C::STATIC && USV_PAIR_M0REUSE && C::NQ == 3) {
                dma_row3_at_min<4u * SLOT_NEXT * C::NRS>(rsrc, rr, last_off, colRb, rbase);
            } else if constexpr (C::STATIC) {
                dma_row_buf_at<C::NQ, 4u * SLOT_NEXT * C::NRS>(rsrc, (uint32_t)min(rr, last_off), colRb, rbase);
            } else {
                const int buf = slot_of(t + PD);
                dma_row_buf<C::NQ>(rsrc, (uint32_t)min(rr, last_off), colRb, rbase + 4u * (uint32_t)(buf * C::NRS));
            }
            rawR = rr + a.pitch;
        }
        // (pipelined argmin: the ring row leaving the window is subtracted first, so its registers
        // are free for this row's staged entries -- no copies)
        constexpr bool EARLY_SUB = !WARM && kPairPipe<RAD>;
        if constexpr (EARLY_SUB) {
#pragma unroll
            for (int x = 0; x < K; ++x) S[x] -= ring[I][x];
        }
        uint32_t Lv[NPOS];
        uint32_t Lw[8];
        {
            wait_lgkm0_pin<LS::NLD>(lw_next);
            LWords cur = lw_next;
            unpack_words<LS::NLD>(cur, Lw);
#pragma unroll
            for (int j = 0; j < NPOS; ++j) {
                const int bidx = LS::byte(j);
                if (kLWholeWord<RAD, EDGE> && (bidx & 3) == 0) Lv[j] = Lw[bidx >> 2];
                else Lv[j] = (Lw[bidx >> 2] >> (8 * (bidx & 3))) & 0xFFu;
            }
        }
        // the next row's L segment: issued before the chain (r <= USV_PAIR_LEARLY: the whole chain covers its latency;
        // an SMEM op in flight only makes the chain's counted LDS waits stricter) or after it.  Interleaved A/B
        // (profiles/probes_r06/ab_k16_r06.txt): config C (r = 5) 43.90 -> 43.29 us per two-stream step, the one-launch
        // kernel 48.27 -> 48.48 us; config E (r = 7) 495 -> 519 us, so r = 7 keeps the late load
        constexpr bool LEARLY = RAD <= USV_PAIR_LEARLY;
        auto next_lw = [&] {
            if constexpr (WARM) {
                load_lw(t + 1);
            } else {
                int rl = rawL;
                asm volatile("" : "+s"(rl));
                lw_next = s_load_words_pin<LS::NLD>(Lseg, (uint32_t)min(rl, last_off));
                rawL = rl + a.pitch;
            }
        };
        auto lbyte = [&](int j) -> uint32_t { return Lv[j]; };
        // the 4 L bytes of quad increments j .. j + 3 as one dword (one funnel shift of two segment words when
        // the bytes are consecutive, i.e. interior tiles; the border tiles' replicated bytes are or-ed)
        auto lquad = [&](auto jt) -> uint32_t {
            constexpr int j = decltype(jt)::value;
            constexpr int b0 = LS::byte(j);
            constexpr bool consec = LS::byte(j + 1) == b0 + 1 && LS::byte(j + 2) == b0 + 2 && LS::byte(j + 3) == b0 + 3;
            if constexpr (consec && (b0 & 3) == 0) {
                return Lw[b0 >> 2];
            } else if constexpr (consec) {
                return (uint32_t)((((uint64_t)Lw[(b0 >> 2) + 1] << 32) | Lw[b0 >> 2]) >> (8 * (b0 & 3)));
            } else {
                uint32_t v = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int b = LS::byte(j + i);
                    v |= ((Lw[b >> 2] >> (8 * (b & 3))) & 0xFFu) << (8 * i);
                }
                return v;
            }
        };
        using VT = typename VecT<C::VEC>::T;
        int boff = C::STATIC ? I * C::NRS : slot_of(t) * C::NRS;
        if constexpr (!C::STATIC) asm volatile("" : "+s"(boff));
        const VT* rb = reinterpret_cast<const VT*>(rbuf + boff + s_l);
        // The staged entries come in C::SPLIT batches of vector reads, each consumed by the chain
        // steps it completes before the next batch is read (r = 7: fewer live VGPRs, so three
        // waves fit per SIMD; the second batch's latency is covered by the other waves).
        uint32_t E[C::NE_V];
        constexpr int NV = C::NE_V / C::VEC, NV1 = C::SPLIT > 1 ? (NV + 1) / 2 : NV;
        constexpr int J1 = C::SPLIT > 1 ? NV1 * C::VEC - 1 : NPOS;  // steps the first batch completes
        // USV_PAIR_RDASM: the entries as NV single ds_read_b64 (2 LDS cycles each; the compiler pairs plain
        // 8-byte reads into ds_read2_b64 at 8 cycles per pair, MI355X_MICROARCH.md LDS table).  They are
        // invisible to the compiler's wait counting, so the first chain step that needs pair k is preceded
        // by an explicit counted lgkmcnt wait between two scheduling barriers (in-order LDS returns;
        // nothing else is outstanding in lgkm but the compiler's own later LDS ops, which only make a wait
        // stricter).  The previous row's transposed words are retired first (an asm that redefines them),
        // so the compiler has no pending read left to drain with a lgkmcnt(0) of its own.
        // (1: single-batch rows, r <= 6; 2: also r = 7's two batches, which spill 24 B at two waves)
        constexpr bool RDASM = C::VEC == 2 && (USV_PAIR_RDASM == 2 || (USV_PAIR_RDASM == 1 && C::SPLIT == 1));
        constexpr uint32_t BOFF = C::STATIC ? 4u * (uint32_t)(I * C::NRS) : 0u;
        uint32_t ra = ra0;
        if constexpr (RDASM && !C::STATIC) ra += 4u * (uint32_t)boff;
        auto issue_reads = [&](auto k0t, auto k1t) {
            constexpr int k0 = decltype(k0t)::value, k1 = decltype(k1t)::value;
            [&]<int... Kk>(std::integer_sequence<int, Kk...>) {
                (ds_read_b64_at<BOFF + 8u * (k0 + Kk)>(ev[k0 + Kk], ra), ...);
            }(std::make_integer_sequence<int, k1 - k0>{});
        };
        if constexpr (RDASM) {
            // (pipelined argmin only: otherwise the words are consumed within their own row, and keeping
            // them live into the next row costs r = 7 its last free registers)
            if constexpr (kPairPipe<RAD>) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(trq[0]), "+v"(trq[1]) : : "memory");
            issue_reads(std::integral_constant<int, 0>{}, std::integral_constant<int, NV1>{});
        } else {
#pragma unroll
            for (int k = 0; k < NV1; ++k) {
                const VT v = rb[k];
#pragma unroll
                for (int e = 0; e < C::VEC; ++e) E[k * C::VEC + e] = vget<C::VEC>(v, e);
            }
        }
        // (after the pending transposed words' lgkmcnt(0) above, which would otherwise wait for it)
        if constexpr (LEARLY) next_lw();
        // P[j + 1] = P[j] + (|L_j - R(d)| low half, |L_j - R(d + 1)| high half).  With the argmin
        // pipelined, piece j of the previous row's argmin follows chain step j and the pair is
        // fenced: the two independent dependency chains interleave instruction by instruction.
        uint32_t A[NPOS + 1];
        A[0] = 0;
        // op at increment j: a single step (A[j + 1]), the first increment of a quad (A[j + 4]), or an
        // increment folded into the quad before it (no op; its argmin piece still follows here)
        constexpr auto is_quad = [](int j) { return j >= C::JA && j < C::JE && (j - C::JA) % 4 == 0; };
        constexpr auto is_op = [](int j) { return j < C::JA || j >= C::JE || (j - C::JA) % 4 == 0; };
        // highest staged entry the ops up to increment j read (single j: j + 1; quad at j: j + 4)
        constexpr auto need = [is_quad, is_op](int j) {
            int n = 0;
            for (int i = 0; i <= j; ++i)
                if (is_op(i)) n = is_quad(i) ? i + 4 : i + 1;
            return n;
        };
        auto chain_step = [&](auto jt) {
            constexpr int j = decltype(jt)::value;
            // the pairs this op needs that no earlier op waited for, retired by one counted wait
            // (a group never spans the two read batches of r = 7)
            constexpr int GRP = 1;
            constexpr int kp = j == 0 ? -1 : need(j - 1) / 2;  // pairs [0, kp] already retired
            constexpr int kn = need(j) / 2;                    // pairs [0, kn] needed now
            if constexpr (RDASM && is_op(j) && kn > kp) {
                constexpr int k0 = kp + 1;
                constexpr int bstart = k0 < NV1 ? 0 : NV1, bend = k0 < NV1 ? NV1 : NV;
                constexpr int kg = ((kn - bstart) / GRP + 1) * GRP + bstart;  // whole groups up to kn
                constexpr int k1 = kg < bend ? kg : bend;                      // pairs [k0, k1)
                constexpr int later = bend - k1;                               // reads of its batch issued after them
                static_assert(kn < bend, "an op's pairs lie in one read batch");
                // lgkmcnt(later), vmcnt / expcnt left at their maxima; the scheduling barriers keep the
                // pairs' uses below the wait (the compiler believes the asm outputs ready at once)
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_waitcnt(0xC07F | (later << 8));
                // both registers of a pair stay allocated until here even when one is never read (the last
                // pair's second entry): a register the compiler thought free would be overwritten by the load
#pragma unroll
                for (int k = k0; k < k1; ++k) asm volatile("" ::"v"(ev[k]));
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int k = k0; k < k1; ++k) {
                    E[2 * k] = ev[k].x;
                    E[2 * k + 1] = ev[k].y;
                }
            }
            if constexpr (is_quad(j)) {
                // four increments in one step: lo (d) |L_{j+i} - E[j+i+1]|, hi (d + 1) |L_{j+i} - E[j+i]|,
                // i = 0..3; the entries are zero-extended bytes, packed here by four v_perm (m = bytes of
                // E[j+1..j+3], then E[j] below it for hi and E[j+4] above it for lo)
                const uint32_t t = __builtin_amdgcn_perm(E[j + 2], E[j + 1], 0x0c0c0400u);
                const uint32_t m = __builtin_amdgcn_perm(E[j + 3], t, 0x0c040100u);
                const uint32_t r_hi = __builtin_amdgcn_perm(m, E[j], 0x06050400u);
                const uint32_t r_lo = __builtin_amdgcn_perm(E[j + 4], m, 0x04020100u);
                const uint32_t l4 = lquad(jt);
                A[j + 4] = __builtin_amdgcn_sad_hi_u8(l4, r_hi, __builtin_amdgcn_sad_u8(l4, r_lo, A[j]));
            } else if constexpr (is_op(j)) {
                const uint32_t l = lbyte(j);
                A[j + 1] = __builtin_amdgcn_sad_hi_u8(l, E[j], __builtin_amdgcn_sad_u8(l, E[j + 1], A[j]));
            }
            pre(jt);
            if constexpr (EARLY_SUB) __builtin_amdgcn_sched_barrier(0);
        };
        [&]<int... J>(std::integer_sequence<int, J...>) {
            (chain_step(std::integral_constant<int, J>{}), ...);
        }(std::make_integer_sequence<int, J1>{});
        if constexpr (C::SPLIT > 1 && RDASM) {
            static_assert(!kPairPipe<RAD>, "the second batch's chain steps carry no argmin pieces");
            __builtin_amdgcn_sched_barrier(0);
            issue_reads(std::integral_constant<int, NV1>{}, std::integral_constant<int, NV>{});
            [&]<int... J>(std::integer_sequence<int, J...>) {
                (chain_step(std::integral_constant<int, J1 + J>{}), ...);
            }(std::make_integer_sequence<int, NPOS - J1>{});
        } else if constexpr (C::SPLIT > 1) {
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = NV1; k < NV; ++k) {
                const VT v = rb[k];
#pragma unroll
                for (int e = 0; e < C::VEC; ++e) E[k * C::VEC + e] = vget<C::VEC>(v, e);
            }
            [&]<int... J>(std::integer_sequence<int, J...>) {
                (chain_step(std::integral_constant<int, J1 + J>{}), ...);
            }(std::make_integer_sequence<int, NPOS - J1>{});
        }
#pragma unroll
        for (int x = 0; x < K; ++x) {
            const uint32_t h = A[x + WIN] - A[x];  // both halves in [0, 65535], no borrow
            if constexpr (WARM || EARLY_SUB) S[x] = S[x] + h;
            else S[x] = (S[x] - ring[I][x]) + h;
            ring[I][x] = h;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (!LEARLY) next_lw();
        __builtin_amdgcn_sched_barrier(0);
    };

    int cb = 0, y_chunk = y_begin;
    // Wide flush: a chunk's outputs leave in two store instructions -- lane r
    // writes row r's 8 disparity bytes as one 8-byte store, lane 4r + q row r's distances 2q, 2q+1
    // as one 16-byte store -- instead of a byte + a double per lane and item (4 per 11-row chunk).
    // Global stores count in vmcnt on gfx9 with the LDS-DMA look-ahead, so fewer, wider stores also
    // hold up fewer of the next rows' counted DMA waits.  Needs 4-byte aligned disparity rows.
    const bool wide = ((reinterpret_cast<uintptr_t>(disp + x0) | (uintptr_t)a.disp_pitch) & 3u) == 0;
    auto flush = [&](int rows) {
        if constexpr (NW > 1) lds_barrier();
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: its LDS ops run in order
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        if (wide) {
            static_assert(K == 8, "one 8-byte disparity store per row");
            const uint32_t* crow = comb + (C::NCB > 1 ? cb * KRB * C::CSTR : 0);
            if (tid < rows) {
                uint4 k0 = reinterpret_cast<const uint4*>(crow + tid * C::CSTR)[0];
                uint4 k1 = reinterpret_cast<const uint4*>(crow + tid * C::CSTR)[1];
#pragma unroll
                for (int w2 = 1; w2 < NW; ++w2) {
                    const uint4 m0 = reinterpret_cast<const uint4*>(crow + tid * C::CSTR + w2 * K)[0];
                    const uint4 m1 = reinterpret_cast<const uint4*>(crow + tid * C::CSTR + w2 * K)[1];
                    k0 = make_uint4(min(k0.x, m0.x), min(k0.y, m0.y), min(k0.z, m0.z), min(k0.w, m0.w));
                    k1 = make_uint4(min(k1.x, m1.x), min(k1.y, m1.y), min(k1.z, m1.z), min(k1.w, m1.w));
                }
                // byte 0 of each key is its disparity
                const uint32_t lo = __builtin_amdgcn_perm(k0.y, k0.x, 0x0c0c0400u) | __builtin_amdgcn_perm(k0.w, k0.z, 0x04000c0cu);
                const uint32_t hi = __builtin_amdgcn_perm(k1.y, k1.x, 0x0c0c0400u) | __builtin_amdgcn_perm(k1.w, k1.z, 0x04000c0cu);
                const size_t y = (size_t)(y_chunk + tid);
                *reinterpret_cast<uint2*>(disp + y * a.disp_pitch + x0) = make_uint2(lo, hi);
            }
            if (dist && tid < 4 * rows) {
                struct __attribute__((aligned(8))) D2 { double a, b; };
                const int r = tid >> 2, q = tid & 3;
                uint2 kk = reinterpret_cast<const uint2*>(crow + r * C::CSTR)[q];
#pragma unroll
                for (int w2 = 1; w2 < NW; ++w2) {
                    const uint2 m = reinterpret_cast<const uint2*>(crow + r * C::CSTR + w2 * K)[q];
                    kk = make_uint2(min(kk.x, m.x), min(kk.y, m.y));
                }
                const size_t y = (size_t)(y_chunk + r);
                *reinterpret_cast<D2*>(dist + y * a.dist_pitch + x0 + 2 * q) = D2{lut_s[kk.x & 0xFFu], lut_s[kk.y & 0xFFu]};
            }
            y_chunk += rows;
            if constexpr (C::NCB > 1) cb ^= 1;
            return;
        }
        const int items = rows * K;
        for (int i = tid; i < items; i += NW * 64) {
            const int row = i / K, p = i - row * K;
            uint32_t key = 0xFFFFFFFFu;
#pragma unroll
            for (int w2 = 0; w2 < NW; ++w2) key = min(key, comb[((C::NCB > 1 ? cb : 0) * KRB + row) * C::CSTR + w2 * K + p]);
            const uint32_t dv = key & 0xFFu;
            const size_t y = (size_t)(y_chunk + row);
            disp[y * a.disp_pitch + x0 + p] = (uint8_t)dv;
            if (dist) dist[y * a.dist_pitch + x0 + p] = lut_s[dv];
        }
        y_chunk += rows;
        if constexpr (C::NCB > 1) cb ^= 1;
    };
    // Argmin of one row, in two halves so that the LDS round trip of the transpose and the
    // dependent min / DPP tail overlap the next row's chain (USV_PAIR_PIPE):
    //   tr_issue:  lane l stores its 8 packed words, lane 8p + q reads the 8 words of pixel p from
    //              lanes 8q .. 8q + 7 (two ds_read_b128) -- nothing waits on them here;
    //   tr_finish: 16 keys (cost << 8) | d by v_perm, a v_min3 tree, three DPP rounds across the 8
    //              lanes of the pixel, one comb word per pixel.
    const uint32_t tb_lds = lds_addr(tb);
    // (USV_PAIR_M0REUSE, static ring + pipelined argmin: called right after row I's do_row, whose DMA left
    // M0 = rbase + 4 ((I + PD) mod NB) NRS -- nothing in between writes M0 -- so the stores address tb from it)
    auto tr_issue = [&](const uint32_t(&S)[K], auto i_tag) {
        constexpr int I = decltype(i_tag)::value;
        constexpr bool REUSE = USV_PAIR_M0REUSE && C::STATIC && kPairPipe<RAD> && NW == 1;
        if constexpr (REUSE) {
            static_assert(K == 8 && C::TB_OFF >= NB * C::NRS, "eight transpose stores above the ring");
            constexpr uint32_t D0 = 4u * (uint32_t)(C::TB_OFF - ((I + PD) % NB) * C::NRS);
            static_assert(D0 + 1792u < 65536u, "16-bit DS offsets");
            asm volatile("ds_write_addtid_b32 %0 offset:%8\n\tds_write_addtid_b32 %1 offset:%9\n\t"
                         "ds_write_addtid_b32 %2 offset:%10\n\tds_write_addtid_b32 %3 offset:%11\n\t"
                         "ds_write_addtid_b32 %4 offset:%12\n\tds_write_addtid_b32 %5 offset:%13\n\t"
                         "ds_write_addtid_b32 %6 offset:%14\n\tds_write_addtid_b32 %7 offset:%15"
                         :: "v"(S[0]), "v"(S[1]), "v"(S[2]), "v"(S[3]), "v"(S[4]), "v"(S[5]), "v"(S[6]), "v"(S[7]),
                            "n"(D0), "n"(D0 + 256u), "n"(D0 + 512u), "n"(D0 + 768u), "n"(D0 + 1024u), "n"(D0 + 1280u),
                            "n"(D0 + 1536u), "n"(D0 + 1792u) : "memory");
        } else {
            // ds_write_addtid_b32: address = M0 + offset + 4 lane, no address VGPR; 2 LDS cycles per store
            // against 6 for each ds_write2st64_b32 pair (MI355X_MICROARCH.md LDS table)
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
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            // (r = 7: the second window's index is rebuilt per row as well)
            const uint32_t ri = (C::SPLIT > 1 && j == 1) ? (rdw[0] ^ 1u) : rdw[j];
            trq[j] = reinterpret_cast<const u4x*>(tb)[ri];
        }
        asm volatile("" ::: "memory");
    };
    // tr_finish in 16 pieces (piece J after chain step J of the next row when pipelined)
    uint32_t fv[16], fb[5], fm;
    auto tr_piece = [&](auto jt, int slot) {
        constexpr int J = decltype(jt)::value;
        if constexpr (J < 8) {
            constexpr int j = J >> 2, e = J & 3;
            const uint32_t w = e == 0 ? trq[j].x : e == 1 ? trq[j].y : e == 2 ? trq[j].z : trq[j].w;
            // (r = 7: the second window's d table and both d + 1 tables are rebuilt per row from
            // dlo[0], three VGPRs fewer across the loop: bit 3 of every d byte is the window)
            uint32_t dl = dlo[j], dh = dhi[j];
            if constexpr (C::SPLIT > 1) {
                dl = j == 0 ? dlo[0] : (dlo[0] ^ 0x08080808u);
                dh = dl + 0x01010101u;
            }
            fv[8 * j + 2 * e] = __builtin_amdgcn_perm(w, dl, 0x0c050400u + (uint32_t)e);
            fv[8 * j + 2 * e + 1] = __builtin_amdgcn_perm(w, dh, 0x0c070600u + (uint32_t)e);
        } else if constexpr (J == 8) {
            fb[0] = min(min(fv[0], fv[1]), fv[2]);
            fb[1] = min(min(fv[3], fv[4]), fv[5]);
        } else if constexpr (J == 9) {
            fb[2] = min(min(fv[6], fv[7]), fv[8]);
            fb[3] = min(min(fv[9], fv[10]), fv[11]);
        } else if constexpr (J == 10) {
            fb[4] = min(min(fv[12], fv[13]), fv[14]);
            fb[0] = min(min(fb[0], fb[1]), fb[2]);
        } else if constexpr (J == 11) {
            fb[3] = min(min(fb[3], fb[4]), fv[15]);
            fm = min(fb[0], fb[3]);
        } else if constexpr (J == 12) {
            fm = min(fm, dpp<kQuadSwap1>(fm));
        } else if constexpr (J == 13) {
            fm = min(fm, dpp<kQuadSwap2>(fm));
        } else if constexpr (J == 14) {
            fm = min(fm, dpp<kRowHalfMirror>(fm));
        } else if constexpr (J == 15) {
            int px = lane >> 3;
            if constexpr (C::SPLIT > 1) {  // r = 7: rebuilt, not kept live through the row loop
                px = threadIdx.x;
                asm volatile("" : "+v"(px));
                px = (px & 63) >> 3;
            }
            comb[((C::NCB > 1 ? cb : 0) * KRB + slot) * C::CSTR + wave * K + px] = fm;
        }
    };
    auto tr_finish = [&](int slot) {
        [&]<int... J>(std::integer_sequence<int, J...>) {
            (tr_piece(std::integral_constant<int, J>{}, slot), ...);
        }(std::make_integer_sequence<int, 16>{});
    };
    auto emit = [&](const uint32_t(&S)[K], int slot) {
        tr_issue(S, std::integral_constant<int, -1>{});
        tr_finish(slot);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto no_pre = [](auto) {};

    uint32_t S[K];
#pragma unroll
    for (int i = 0; i < K; ++i) S[i] = 0;
    uint32_t ring[WIN][K];
    static_assert(C::LUT_OFF % 4 == 0, "16-byte aligned table");
    if (dist) lut_dma<C::LUTN / 128>(a.lut, smem + C::LUT_OFF, lane);
    [&]<int... P>(std::integer_sequence<int, P...>) { (issue_dma(P, P % NB), ...); }(std::make_integer_sequence<int, PD>{});
    load_lw(0);
    using WarmT = std::integral_constant<bool, true>;
    using SteadyT = std::integral_constant<bool, false>;
    [&]<int... I>(std::integer_sequence<int, I...>) {
        (do_row(I, WarmT{}, std::integral_constant<int, I>{}, S, ring, no_pre), ...);
    }(std::make_integer_sequence<int, WIN>{});
    // Pipelined argmin (PIPE): output row k is slot k % KRB.  Row k's transpose is issued after its
    // chain and finished inside the next row's do_row (after that row's staged reads are issued), so
    // slot I is pending when the I-th row of a WIN-row group starts; the chunk is flushed once slot
    // KRB - 1 is finished.  (r = 6, 7 keep the unpipelined order: the held transpose words spill.)
    constexpr bool PIPE = kPairPipe<RAD>;
    static_assert(KRB == WIN, "pending slot = row index in the unrolled group");
    static_assert(!PIPE || NPOS >= 16, "16 argmin pieces ride on the chain steps");
    if constexpr (PIPE) {
        tr_issue(S, std::integral_constant<int, WIN - 1>{});  // after the last warm-up row
        __builtin_amdgcn_sched_barrier(0);
    } else {
        emit(S, 0);
    }
    auto step = [&](int t0, auto i_tag) {
        constexpr int I = decltype(i_tag)::value;
        if constexpr (PIPE) {
            do_row(t0 + I, SteadyT{}, i_tag, S, ring, [&](auto jt) {
                if constexpr (decltype(jt)::value < 16) tr_piece(jt, I);
            });
            if constexpr (I == KRB - 1) flush(KRB);
            tr_issue(S, i_tag);
            __builtin_amdgcn_sched_barrier(0);
        } else {
            do_row(t0 + I, SteadyT{}, i_tag, S, ring, no_pre);
            emit(S, (I + 1) % WIN);
            if constexpr ((I + 1) % WIN == KRB - 1) flush(KRB);
        }
    };
    int t0 = WIN;
    if constexpr (EDGE == kInterior && C::STATIC) {
        // whole groups without a bound check per row (r = 5 interior tiles: the edge tiles keep one copy
        // of the row code; at r = 6, 7 the unchecked copy spills)
        for (; t0 + WIN <= T; t0 += WIN) {
            [&]<int... I>(std::integer_sequence<int, I...>) {
                (step(t0, std::integral_constant<int, I>{}), ...);
            }(std::make_integer_sequence<int, WIN>{});
        }
    }
    for (; t0 < T; t0 += WIN) {
        [&]<int... I>(std::integer_sequence<int, I...>) {
            bool go = true;
            ((go = go && (t0 + I < T), go ? step(t0, std::integral_constant<int, I>{}) : void()), ...);
        }(std::make_integer_sequence<int, WIN>{});
    }
    wait_lgkm0_pin<LS::NLD>(lw_next);  // retire the unused last L load before its SGPRs are reused
    if constexpr (PIPE) {
        const int last = (nout - 1) % KRB;  // the pending slot: the band's last output row
        tr_finish(last);
        if (last == KRB - 1) flush(KRB);
    }
    const int rest = nout % KRB;
    if (rest) flush(rest);
    wait_vmcnt<0>();
}

// ===================================================================================
// K = 16 form of the paired kernel (r = 5, D <= 128: config C), two waves per SIMD.
//
// Same lane mapping as above (lane = disparities d, d + 1 of one 128-disparity wave), 16 output columns per
// x-tile instead of 8.  Per 16 columns and row: the prefix chain has 26 steps (52 v_sad; all 27 prefix positions
// are read, since K > w leaves no run to jump), the row sums, running sums and ring 3 x 16, the argmin
// 32 keys per lane.  Against two K = 8 tiles: 52 instead of 2 x 34 chain VALU, 14 instead of 2 x 10 entry
// reads, 3 instead of 2 x 3 row DMAs and 26 instead of 2 x 18 L-byte extractions for the same outputs; the
// argmin and the H / S work per column are unchanged.  The price is the ring: 11 rows x 16 columns of
// (d, d + 1) pairs = 176 VGPRs, so the kernel is compiled for two waves per SIMD (256 VGPRs) instead of three,
// and a band covers 1 / 8 instead of 1 / 12 of a CU's rows (more warm-up rows per output row).
// ===================================================================================
#ifndef USV_PAIR_K16
#define USV_PAIR_K16 0  // 1: config C's shape (r = 5, D <= 128) takes sad_pair16_kernel (variant builds only)
#endif
#if USV_PAIR_K16
#ifndef USV_PAIR16_LEARLY
#define USV_PAIR16_LEARLY 0  // 1: the next row's L segment is loaded before the row's chain
#endif
#ifndef USV_PAIR16_RA
#define USV_PAIR16_RA 0  // > 0: this many entry pairs of row t + 1 are read before row t's argmin
#endif
#ifndef USV_PAIR16_GEN_WEIGHTS
#define USV_PAIR16_GEN_WEIGHTS 0x3C3C3C64u  // band heights by dispatch generation: 100 : 60 (two generations)
#endif
#ifndef USV_PAIR16_MIDT
#define USV_PAIR16_MIDT 0  // > 0: row t - 1's transposed words are read at chain step MIDT of row t, its argmin after the chain
#endif

// the four transposed reads of one argmin (inline asm: retired by the caller's explicit waits)
__device__ __forceinline__ void ds_read_b128_x4(u4x (&q)[4], uint32_t addr) {
    asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\t"
                 "ds_read_b128 %2, %4 offset:32\n\tds_read_b128 %3, %4 offset:48"
                 : "=&v"(q[0]), "=&v"(q[1]), "=&v"(q[2]), "=&v"(q[3]) : "v"(addr) : "memory");
}

struct P16 {
    static constexpr int RAD = 5, K = 16, WIN = 2 * RAD + 1;
    static constexpr int NPOS = K + 2 * RAD;         // 26 chain steps
    static constexpr int NV = (NPOS + 2) / 2;         // 14 ds_read_b64: entries 0 .. 26 (+ one unused)
    static constexpr int NR = 2 * 63 + 2 * NV;        // entries a wave stages per row
    static constexpr int NQ = (NR + 63) / 64;         // DMA instructions per row
    static constexpr int NRS = NQ * 64;
    static constexpr int NB = WIN, PD = NB - 1;       // static ring: row t in slot t mod WIN
    static constexpr int KRB = WIN;                   // output rows per flush
    // transpose buffer: pixel x's 64 words at 68 x (see pair16_band_loop); 16 pixels
    static constexpr int TSTR = 68;
    static constexpr int TB_OFF = NB * NRS;
    static constexpr int COMB_OFF = TB_OFF + K * TSTR;  // per-row minima, KRB rows x 16 pixels
    static constexpr int LUT_OFF = COMB_OFF + KRB * K;
    static constexpr int LUTN = 128;                  // one wave: every disparity < 128
    static constexpr int SMEM_WORDS = LUT_OFF + 2 * LUTN;
    static constexpr int RA = USV_PAIR16_RA;
    static constexpr int MIDT = USV_PAIR16_MIDT;
    static_assert(MIDT == 0 || (MIDT >= 2 * 4 && MIDT < NPOS && 2 * RA <= MIDT),
                  "mid-chain transpose: the counted waits after step MIDT hold 4 more reads");
    static_assert(NQ == 3 && PD * NQ < 64, "three DMAs per row; look-ahead fits the 6-bit vmcnt");
    static_assert(TB_OFF % 4 == 0 && COMB_OFF % 4 == 0 && LUT_OFF % 4 == 0, "16-byte aligned regions");
    static_assert(NV <= 15 && RA >= 0 && RA < NV, "counted lgkmcnt waits hold at most 15 reads");
};

template <int EDGE>
__device__ __forceinline__ void pair16_band_loop(const uint8_t* __restrict__ L, const uint8_t* __restrict__ R,
                                                 uint8_t* __restrict__ disp, double* __restrict__ dist,
                                                 const MatchArgs& a, uint32_t* smem, int lane, int x0, int y_begin,
                                                 int y_end) {
    using C = P16;
    constexpr int RAD = C::RAD, WIN = C::WIN, K = C::K, NB = C::NB, PD = C::PD, NPOS = C::NPOS, NV = C::NV;
    constexpr int KRB = C::KRB, RA = C::RA, MIDT = C::MIDT;
    using LS = LSeg<RAD, EDGE, K>;
    using LWords = typename SWords<LS::NLD>::T;
    const int lmax = min(63, a.D / 2 - 1);
    const int l_eff = min(lane, lmax);
    const int cbase = x0 - RAD - (2 * 63 + 1);  // first R column the wave stages
    uint32_t* rbuf = smem;
    uint32_t* comb = smem + C::COMB_OFF;
    uint32_t* tb = smem + C::TB_OFF;
    // Transpose: lane l stores word x (pixel x's (d, d + 1) costs) at tb[68 x + l]; lane m = 4p + q reads pixel p's
    // words of source lanes 16 q .. 16 q + 15 as four 16-byte windows j = 0..3 at 68 p + 16 q + 4 j.  Window j of
    // lane (p, q) starts on bank slot (p + 4 q + j) mod 16 (4-bank slots), and each 16-lane read group of a
    // ds_read_b128 is four q times four values of p mod 4, so every group reads 16 distinct slots: conflict-free
    // with the windows in fixed order -- one address VGPR, the window in the instruction's offset.
    // dlo[j]: the four source lanes' d = 2 (16 q + 4 j + e) as bytes (lanes past lmax replay lane lmax's costs with a
    // larger d, so their keys never win).
    const int p_lane = lane >> 2, q_lane = lane & 3;
    const uint32_t tr_addr = lds_addr(tb) + 4u * (uint32_t)(C::TSTR * p_lane + 16 * q_lane);
    uint32_t dlo[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) dlo[j] = (uint32_t)(32 * q_lane + 8 * j) * 0x01010101u + 0x06040200u;
    const double* lut_s = reinterpret_cast<const double*>(smem + C::LUT_OFF);
    const int s_l = 2 * (63 - l_eff);  // this lane's first staged entry
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
    auto issue_dma = [&](int t, int buf) {
        dma_row<C::NQ>(Rdma + row_off(t), colRb, rbase + 4u * (uint32_t)(buf * C::NRS));
    };
    LWords lw_next;
    auto load_lw = [&](int t) { lw_next = s_load_words_pin<LS::NLD>(Lseg, row_off(t)); };
    const uint32_t ra0 = lds_addr(rbuf + s_l);
    // the entries as single ds_read_b64 (inline asm: the compiler would pair them into ds_read2_b64), pairs [k0, k1)
    // of ring slot I, each retired by a counted lgkmcnt wait before the first chain step that needs it (in-order LDS
    // returns)
    u2x ev[NV];
    u4x trq[4];  // MIDT: the pending output row's transposed words, in flight from chain step MIDT to the row's end
    auto issue_reads = [&](auto i_tag, auto k0t, auto k1t) {
        constexpr int I = decltype(i_tag)::value, k0 = decltype(k0t)::value, k1 = decltype(k1t)::value;
        constexpr uint32_t BOFF = 4u * (uint32_t)(I * C::NRS);
        [&]<int... Kk>(std::integer_sequence<int, Kk...>) {
            (ds_read_b64_at<BOFF + 8u * (k0 + Kk)>(ev[k0 + Kk], ra0), ...);
        }(std::make_integer_sequence<int, k1 - k0>{});
    };

    // One input row t (ring slot I = t mod WIN): R DMA of row t + PD, the entry reads (pairs [RA, NV) when the first RA
    // were read ahead: those are retired by the L words' lgkmcnt(0)), the 26-step chain with the row sums
    // H[x] = A[x + WIN] - A[x] folded into the running sums as soon as A[x + WIN] exists.
    auto do_row = [&](int t_in, auto warm_tag, auto i_tag, uint32_t(&S)[K], uint32_t(&ring)[WIN][K]) {
        constexpr bool WARM = decltype(warm_tag)::value;
        constexpr int I = decltype(i_tag)::value;
        constexpr int K0 = WARM ? 0 : RA;  // pairs read ahead
        constexpr bool PEND = MIDT > 0 && !WARM;  // row t - 1's argmin is pending (its words are in the buffer)
        int t = t_in;
        asm volatile("" : "+s"(t));
        wait_vmcnt<(PD - 1) * C::NQ>();
        __builtin_amdgcn_wave_barrier();
        constexpr int SLOT_NEXT = (I + PD) % NB;
        if constexpr (WARM) {
            issue_dma(t + PD, SLOT_NEXT);
        } else {
            int rr = rawR;
            asm volatile("" : "+s"(rr));
            dma_row3_at_min<4u * SLOT_NEXT * C::NRS>(rsrc, rr, last_off, colRb, rbase);
            rawR = rr + a.pitch;
        }
        // the ring row leaving the window first: its registers are free for this row's entries
        if constexpr (!WARM) {
#pragma unroll
            for (int x = 0; x < K; ++x) S[x] -= ring[I][x];
        }
        uint32_t Lv[NPOS];
        {
            uint32_t Lw[8];
            wait_lgkm0_pin<LS::NLD>(lw_next);
            LWords cur = lw_next;
            unpack_words<LS::NLD>(cur, Lw);
#pragma unroll
            for (int j = 0; j < NPOS; ++j) {
                const int bidx = LS::byte(j);
                if (kLWholeWord<RAD, EDGE> && (bidx & 3) == 0) Lv[j] = Lw[bidx >> 2];
                else Lv[j] = (Lw[bidx >> 2] >> (8 * (bidx & 3))) & 0xFFu;
            }
        }
        issue_reads(i_tag, std::integral_constant<int, K0>{}, std::integral_constant<int, NV>{});
        auto next_lw = [&] {
            if constexpr (WARM) {
                load_lw(t + 1);
            } else {
                int rl = rawL;
                asm volatile("" : "+s"(rl));
                lw_next = s_load_words_pin<LS::NLD>(Lseg, (uint32_t)min(rl, last_off));
                rawL = rl + a.pitch;
            }
        };
        if constexpr (USV_PAIR16_LEARLY) next_lw();  // (as in pair_band_loop: a loss here, 44.2 -> 44.8 us per step)
        uint32_t E[2 * NV];
        uint32_t A[NPOS + 1];
        A[0] = 0;
        auto chain_step = [&](auto jt) {
            constexpr int j = decltype(jt)::value;
            constexpr int kp = j == 0 ? -1 : j / 2;  // pairs [0, kp] retired by earlier steps
            constexpr int kn = (j + 1) / 2;          // step j reads E[j], E[j + 1]
            constexpr bool TQ = PEND && j >= MIDT;   // the four transposed reads are the newest LDS operations
            if constexpr (PEND && j == MIDT) {
                // the entry registers of pairs < MIDT / 2 are dead: the transposed words take their place
                __builtin_amdgcn_sched_barrier(0);
                ds_read_b128_x4(trq, tr_addr);
                __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (kn > kp) {
                if constexpr (kn >= K0) {
                    constexpr int later = NV - 1 - kn + (TQ ? 4 : 0);
                    static_assert(later <= 15, "lgkmcnt holds 4 bits");
                    __builtin_amdgcn_sched_barrier(0);
                    __builtin_amdgcn_s_waitcnt(0xC07F | (later << 8));
                    // both registers of a pair stay allocated up to the wait (the last pair's second entry is never
                    // read)
#pragma unroll
                    for (int k = kp + 1; k <= kn; ++k) asm volatile("" ::"v"(ev[k]));
                    __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
                for (int k = kp + 1; k <= kn; ++k) {
                    E[2 * k] = ev[k].x;
                    E[2 * k + 1] = ev[k].y;
                }
            }
            const uint32_t l = Lv[j];
            A[j + 1] = __builtin_amdgcn_sad_hi_u8(l, E[j], __builtin_amdgcn_sad_u8(l, E[j + 1], A[j]));
            if constexpr (j + 1 >= WIN) {
                constexpr int x = j + 1 - WIN;
                const uint32_t h = A[j + 1] - A[x];  // both halves in [0, 65535], no borrow
                S[x] = S[x] + h;
                ring[I][x] = h;
            }
        };
        [&]<int... J>(std::integer_sequence<int, J...>) {
            (chain_step(std::integral_constant<int, J>{}), ...);
        }(std::make_integer_sequence<int, NPOS>{});
        if constexpr (PEND)
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(trq[0]), "+v"(trq[1]), "+v"(trq[2]), "+v"(trq[3]) : : "memory");
        else
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (!USV_PAIR16_LEARLY) next_lw();
        __builtin_amdgcn_sched_barrier(0);
    };

    int y_chunk = y_begin;
    const bool wide = ((reinterpret_cast<uintptr_t>(disp + x0) | (uintptr_t)a.disp_pitch) & 3u) == 0;
    // a chunk's outputs: lane r stores row r's 16 disparity bytes (one 16-byte store), lane 4r + q the row's
    // distances 4q .. 4q + 3 (two 16-byte stores)
    auto flush = [&](int rows) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: its LDS ops run in order
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        if (wide) {
            if (tid < rows) {
                const uint4* c4 = reinterpret_cast<const uint4*>(comb + tid * K);
                uint32_t o[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint4 k = c4[i];  // byte 0 of each key is its disparity
                    o[i] = __builtin_amdgcn_perm(k.y, k.x, 0x0c0c0400u) | __builtin_amdgcn_perm(k.w, k.z, 0x04000c0cu);
                }
                const size_t y = (size_t)(y_chunk + tid);
                *reinterpret_cast<uint4*>(disp + y * a.disp_pitch + x0) = make_uint4(o[0], o[1], o[2], o[3]);
            }
            if (dist && tid < 4 * rows) {
                struct __attribute__((aligned(8))) D2 { double a, b; };
                const int r = tid >> 2, q = tid & 3;
                const uint4 k = reinterpret_cast<const uint4*>(comb + r * K)[q];
                double* o = dist + (size_t)(y_chunk + r) * a.dist_pitch + x0 + 4 * q;
                *reinterpret_cast<D2*>(o) = D2{lut_s[k.x & 0xFFu], lut_s[k.y & 0xFFu]};
                *reinterpret_cast<D2*>(o + 2) = D2{lut_s[k.z & 0xFFu], lut_s[k.w & 0xFFu]};
            }
            y_chunk += rows;
            return;
        }
        const int items = rows * K;
        for (int i = tid; i < items; i += 64) {
            const int row = i / K, p = i - row * K;
            const uint32_t dv = comb[row * K + p] & 0xFFu;
            const size_t y = (size_t)(y_chunk + row);
            disp[y * a.disp_pitch + x0 + p] = (uint8_t)dv;
            if (dist) dist[y * a.dist_pitch + x0 + p] = lut_s[dv];
        }
        y_chunk += rows;
    };
    // Argmin of one row, whose window sums S are final: the 16 transpose stores (ds_write_addtid_b32: address
    // M0 + offset + 4 lane) and the four transposed reads (inline asm, so the compiler has no load of its own to drain);
    // with read-ahead, the first RA entry pairs of the next row (ring slot I_NEXT) are issued behind them and only
    // the transpose is waited for (lgkmcnt(RA)); then per transposed word two keys (cost << 8) | d by v_perm folded
    // into a v_min3 tree, two quad DPP rounds and the pixel's comb word.
    const uint32_t tb_m0 = lds_addr(tb);
    auto store_t = [&](const uint32_t(&S)[K]) {
        asm volatile("s_mov_b32 m0, %16\n\ts_nop 0\n\t"
                     "ds_write_addtid_b32 %0\n\tds_write_addtid_b32 %1 offset:272\n\t"
                     "ds_write_addtid_b32 %2 offset:544\n\tds_write_addtid_b32 %3 offset:816\n\t"
                     "ds_write_addtid_b32 %4 offset:1088\n\tds_write_addtid_b32 %5 offset:1360\n\t"
                     "ds_write_addtid_b32 %6 offset:1632\n\tds_write_addtid_b32 %7 offset:1904\n\t"
                     "ds_write_addtid_b32 %8 offset:2176\n\tds_write_addtid_b32 %9 offset:2448\n\t"
                     "ds_write_addtid_b32 %10 offset:2720\n\tds_write_addtid_b32 %11 offset:2992\n\t"
                     "ds_write_addtid_b32 %12 offset:3264\n\tds_write_addtid_b32 %13 offset:3536\n\t"
                     "ds_write_addtid_b32 %14 offset:3808\n\tds_write_addtid_b32 %15 offset:4080"
                     :: "v"(S[0]), "v"(S[1]), "v"(S[2]), "v"(S[3]), "v"(S[4]), "v"(S[5]), "v"(S[6]), "v"(S[7]),
                        "v"(S[8]), "v"(S[9]), "v"(S[10]), "v"(S[11]), "v"(S[12]), "v"(S[13]), "v"(S[14]), "v"(S[15]),
                        "s"(tb_m0) : "memory", "m0");
        static_assert(4 * C::TSTR == 272, "the store offsets above are 4 x TSTR apart");
    };
    auto argmin = [&](const u4x(&trq)[4], int slot) {
        uint32_t fv[32];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t dl = dlo[j], dh = dlo[j] + 0x01010101u;  // d even: + 1 per byte, no carry
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t w = trq[j][e];
                fv[8 * j + 2 * e] = __builtin_amdgcn_perm(w, dl, 0x0c050400u + (uint32_t)e);
                fv[8 * j + 2 * e + 1] = __builtin_amdgcn_perm(w, dh, 0x0c070600u + (uint32_t)e);
            }
        }
        uint32_t m[12];
#pragma unroll
        for (int i = 0; i < 10; ++i) m[i] = min(min(fv[3 * i], fv[3 * i + 1]), fv[3 * i + 2]);
        m[10] = fv[30];
        m[11] = fv[31];
        const uint32_t n0 = min(min(m[0], m[1]), m[2]), n1 = min(min(m[3], m[4]), m[5]);
        const uint32_t n2 = min(min(m[6], m[7]), m[8]), n3 = min(min(m[9], m[10]), m[11]);
        uint32_t fm = min(min(n0, n1), min(n2, n3));
        fm = min(fm, dpp<kQuadSwap1>(fm));
        fm = min(fm, dpp<kQuadSwap2>(fm));
        comb[slot * K + p_lane] = fm;
    };
    auto emit = [&](const uint32_t(&S)[K], int slot, auto inext_tag) {
        constexpr int I_NEXT = decltype(inext_tag)::value;
        store_t(S);
        u4x trq[4];
        asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\t"
                     "ds_read_b128 %2, %4 offset:32\n\tds_read_b128 %3, %4 offset:48"
                     : "=&v"(trq[0]), "=&v"(trq[1]), "=&v"(trq[2]), "=&v"(trq[3]) : "v"(tr_addr) : "memory");
        if constexpr (RA > 0 && I_NEXT >= 0) {
            wait_vmcnt<(PD - 1) * C::NQ>();  // the next row's DMA has landed (issued PD - 1 rows ago)
            issue_reads(std::integral_constant<int, I_NEXT>{}, std::integral_constant<int, 0>{},
                        std::integral_constant<int, RA>{});
            asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(trq[0]), "+v"(trq[1]), "+v"(trq[2]), "+v"(trq[3])
                         : "n"(RA) : "memory");
        } else {
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(trq[0]), "+v"(trq[1]), "+v"(trq[2]), "+v"(trq[3]) : : "memory");
        }
        argmin(trq, slot);
        __builtin_amdgcn_sched_barrier(0);
    };

    uint32_t S[K];
#pragma unroll
    for (int i = 0; i < K; ++i) S[i] = 0;
    uint32_t ring[WIN][K];
    if (dist) lut_dma<C::LUTN / 128>(a.lut, smem + C::LUT_OFF, lane);
    [&]<int... P>(std::integer_sequence<int, P...>) { (issue_dma(P, P % NB), ...); }(std::make_integer_sequence<int, PD>{});
    load_lw(0);
    using WarmT = std::integral_constant<bool, true>;
    using SteadyT = std::integral_constant<bool, false>;
    [&]<int... I>(std::integer_sequence<int, I...>) {
        (do_row(I, WarmT{}, std::integral_constant<int, I>{}, S, ring), ...);
    }(std::make_integer_sequence<int, WIN>{});
    // output row 0; the first steady row (t = WIN) is in slot 0
    if constexpr (MIDT > 0) {
        store_t(S);
        if constexpr (RA > 0) {
            wait_vmcnt<(PD - 1) * C::NQ>();
            issue_reads(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, std::integral_constant<int, RA>{});
        }
    } else {
        emit(S, 0, std::integral_constant<int, 0>{});
    }
    // output row k = t - 2r sits in comb slot k mod KRB; the chunk leaves once slot KRB - 1 is written
    auto step = [&](int t0, auto i_tag) {
        constexpr int I = decltype(i_tag)::value;
        do_row(t0 + I, SteadyT{}, i_tag, S, ring);
        if constexpr (MIDT > 0) {
            // row t - 1's output k = t - 1 - 2r: slot I (its words are in registers: row t's may overwrite the buffer)
            store_t(S);
            if constexpr (RA > 0) {  // the next row's first RA entry pairs, covered by the argmin
                wait_vmcnt<(PD - 1) * C::NQ>();
                issue_reads(std::integral_constant<int, (I + 1) % NB>{}, std::integral_constant<int, 0>{},
                            std::integral_constant<int, RA>{});
            }
            argmin(trq, I);
            if constexpr (I == KRB - 1) flush(KRB);
            __builtin_amdgcn_sched_barrier(0);
        } else {
            // (the band's last row reads ahead into a slot nobody uses: harmless, retired by the final lgkmcnt(0))
            emit(S, (I + 1) % WIN, std::integral_constant<int, (I + 1) % NB>{});
            if constexpr ((I + 1) % WIN == KRB - 1) flush(KRB);
        }
    };
    int t0 = WIN;
    if constexpr (EDGE == kInterior) {
        for (; t0 + WIN <= T; t0 += WIN) {
            [&]<int... I>(std::integer_sequence<int, I...>) {
                (step(t0, std::integral_constant<int, I>{}), ...);
            }(std::make_integer_sequence<int, WIN>{});
        }
    }
    for (; t0 < T; t0 += WIN) {
        [&]<int... I>(std::integer_sequence<int, I...>) {
            bool go = true;
            ((go = go && (t0 + I < T), go ? step(t0, std::integral_constant<int, I>{}) : void()), ...);
        }(std::make_integer_sequence<int, WIN>{});
    }
    wait_lgkm0_pin<LS::NLD>(lw_next);  // retire the unused last L load (and any read-ahead) before the SGPRs are reused
    if constexpr (MIDT > 0) {  // the last output row's argmin
        ds_read_b128_x4(trq, tr_addr);
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(trq[0]), "+v"(trq[1]), "+v"(trq[2]), "+v"(trq[3]) : : "memory");
        argmin(trq, (nout - 1) % KRB);
        const int rest = nout - (y_chunk - y_begin);
        if (rest) flush(rest);
    } else {
        const int rest = nout % KRB;
        if (rest) flush(rest);
    }
    wait_vmcnt<0>();
}

__global__ __launch_bounds__(64, 2) void sad_pair16_kernel(const uint8_t* __restrict__ L, const uint8_t* __restrict__ R,
                                                          uint8_t* __restrict__ disp, double* __restrict__ dist,
                                                          MatchArgs a, BandPlan P, const uint2* __restrict__ tiles) {
    __shared__ __attribute__((aligned(16))) uint32_t smem[P16::SMEM_WORDS];
    const int lane = threadIdx.x & 63;
    unsigned xtu, pair;
    int y_begin, y_end;
    if (tiles) {  // the launcher's table: x-tile | pair << 16, y_begin | y_end << 16
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
    constexpr int K = P16::K;
    const int xt = (int)xtu;
    const int n_xt = P.n_xt;
    // interior tiles read L columns x0 - 8 .. x0 + 23: the one before the last stops at W - 2K
    int x0 = xt * K;
    if (xt == n_xt - 1) x0 = a.W - K;
    else if (xt == n_xt - 2) x0 = min(x0, a.W - 2 * K);
    L += (size_t)pair * a.pair_stride;
    R += (size_t)pair * a.pair_stride;
    disp += (size_t)pair * a.disp_stride;
    if (dist) dist += (size_t)pair * a.dist_stride;
    if (y_end <= y_begin) return;
    if (xt == 0)
        pair16_band_loop<kLeft>(L, R, disp, dist, a, smem, lane, x0, y_begin, y_end);
    else if (xt == n_xt - 1)
        pair16_band_loop<kRight>(L, R, disp, dist, a, smem, lane, x0, y_begin, y_end);
    else
        pair16_band_loop<kInterior>(L, R, disp, dist, a, smem, lane, x0, y_begin, y_end);
}

hipError_t launch_pair16(const MatchArgs& a, hipStream_t s) {
    constexpr int K = P16::K, WIN = P16::WIN;
    static const int per_cu = [] {
        int v = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, sad_pair16_kernel, 64, 0) != hipSuccess || v <= 0) v = 1;
        return v;
    }();
    BandPlan P{};
    P.n_xt = (a.W + K - 1) / K;
    const long slots = (long)cu_count() * per_cu;
    const long NC = (long)P.n_xt * a.batch;
    long m = slots / NC;
    if (m < 1) m = 1;
    const long m_max = a.H / (kMinBandWins * WIN) > 0 ? a.H / (kMinBandWins * WIN) : 1;
    if (m > m_max) m = m_max;
    P.m = (int)m;
    const long ex = slots - NC * m;
    P.extra = (a.batch == 1 && ex > 0 && ex < P.n_xt && a.H / (m + 1) >= kMinBandWins * WIN) ? (int)ex : 0;
    const long total = NC * m + P.extra;
    if (total > 0x7FFFFFFFL) return hipErrorInvalidValue;
    P.gen_g = (int)(4L * (cu_count() / 8));  // one generation = one workgroup per SIMD-wave slot
    if (P.gen_g < 1) P.gen_g = 1;
    const bool two = per_cu == 8 && total > 8L * P.gen_g;
    P.weights = two ? USV_PAIR16_GEN_WEIGHTS : 0x01010101u;
    const uint2* tiles = tile_table(1, 0x100 + 5 * 16 + 1, a, P.n_xt, P.m, P.extra, P.gen_g, P.weights, (unsigned)total, s);
    hipLaunchKernelGGL(sad_pair16_kernel, dim3((unsigned)total), dim3(64), 0, s, a.L, a.R, a.disp, a.dist, a, P, tiles);
    return hipGetLastError();
}
#endif  // USV_PAIR_K16

#ifndef USV_PAIR_OCC7
#define USV_PAIR_OCC7 3  // waves per SIMD the r = 7 paired kernel is compiled for
#endif
#ifndef USV_PAIR_OCC5
#define USV_PAIR_OCC5 3  // waves per SIMD the r <= 6 paired kernel is compiled for
#endif
constexpr int pair_occ(int rad, int) { return rad >= 7 ? USV_PAIR_OCC7 : USV_PAIR_OCC5; }

template <int RAD, int NW>
__global__ __launch_bounds__(NW * 64, pair_occ(RAD, NW)) void sad_pair_kernel(const uint8_t* __restrict__ L,
                                                              const uint8_t* __restrict__ R,
                                                              uint8_t* __restrict__ disp,
                                                              double* __restrict__ dist, MatchArgs a, BandPlan P,
                                                              const uint2* __restrict__ tiles) {
    using C = PCfg<RAD, NW>;
    __shared__ __attribute__((aligned(16))) uint32_t smem[C::SMEM_WORDS];
    const int lane = threadIdx.x & 63;
    const int wave = NW == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    unsigned xtu, pair;
    int y_begin, y_end;
    if (tiles) {  // the launcher's table: x-tile | pair << 16, y_begin | y_end << 16
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
    const int n_xt = P.n_xt;
    int x0 = xt * C::K;
    if (xt == n_xt - 1) x0 = a.W - C::K;
    else if (xt == n_xt - 2) x0 = min(x0, a.W - 2 * C::K);
    L += (size_t)pair * a.pair_stride;
    R += (size_t)pair * a.pair_stride;
    disp += (size_t)pair * a.disp_stride;
    if (dist) dist += (size_t)pair * a.dist_stride;  // (the table is staged inside the band loop)
    if (y_end <= y_begin) return;
    if (xt == 0)
        pair_band_loop<RAD, NW, kLeft>(L, R, disp, dist, a, smem, lane, wave, x0, y_begin, y_end);
    else if (xt == n_xt - 1)
        pair_band_loop<RAD, NW, kRight>(L, R, disp, dist, a, smem, lane, wave, x0, y_begin, y_end);
    else
        pair_band_loop<RAD, NW, kInterior>(L, R, disp, dist, a, smem, lane, wave, x0, y_begin, y_end);
}

template <int RAD, int NW>
int resident_pair_blocks_per_cu() {
    static const int n = [] {
        int v = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, sad_pair_kernel<RAD, NW>, NW * 64, 0) != hipSuccess ||
            v <= 0)
            v = 1;
        return v;
    }();
    return n;
}

// Generation weights of the paired kernel (one-wave workgroups, three generations per SIMD):
// interleaved A/B on config C, 100:90:70 / 100:80:58 / 100:85:55 / 100:80:50 / 100:75:50 /
// 100:70:45 = 69.75 / 68.61 / 67.63 / 67.42 / 67.27 / 68.25 us (profiles/probes_r02/ab_pair_weights_*).
// Re-fitted after the argmin was pipelined into the next row's chain (two A/B runs on two boxes, 4 rounds
// each): 100:75:50 65.3 / 65.0, 100:70:45 64.4 / 64.7, 100:70:40 64.6, 100:65:40 66.3, 100:60:35 68.5,
// 100:80:55 66.2, 100:85:60 66.6 us (profiles/probes_r02/ab_pair_weights_3_r02.txt).
// Config E (r = 7, argmin not pipelined) keeps 100:75:50: 617.0 vs 639.9 us with 100:70:45 (same A/B run).
#ifndef USV_PAIR_GEN_WEIGHTS
#define USV_PAIR_GEN_WEIGHTS 0x2D2D4664u  // 100, 70, 45, 45: pipelined argmin (r = 5)
#endif
#ifndef USV_PAIR_GEN_WEIGHTS_UNPIPED
#define USV_PAIR_GEN_WEIGHTS_UNPIPED 0x32324B64u  // 100, 75, 50, 50: r = 6, 7 with one-wave workgroups
#endif
// Two-wave workgroups (D > 128: config E) want flatter heights (three interleaved A/B runs of 3 rounds on
// config E): 100:75:50 620-625, 100:65:40 684, 100:80:60 570, 100:85:60 568, 100:85:65 553-555,
// 100:85:70 555, 100:90:70 557, 100:90:80 565, 100:95:85 570, uniform 573 us
// (profiles/probes_r02/ab_pair_weights_E_r02.txt).
#ifndef USV_PAIR_GEN_WEIGHTS_NW2
#define USV_PAIR_GEN_WEIGHTS_NW2 0x41415564u  // 100, 85, 65, 65
#endif

template <int RAD, int NW>
hipError_t launch_pair_rn(const MatchArgs& a, hipStream_t s) {
    constexpr int K = PCfg<RAD, NW>::K, WIN = 2 * RAD + 1;
    BandPlan P{};
    P.n_xt = (a.W + K - 1) / K;
    const int per_cu = resident_pair_blocks_per_cu<RAD, NW>();
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
    P.gen_g = (int)((4L * (cu_count() / 8)) / NW);  // one generation = one workgroup per SIMD-wave slot
    if (P.gen_g < 1) P.gen_g = 1;
    const bool three = per_cu * NW == 12 && total > 2L * 8 * P.gen_g;
    P.weights = !three ? 0x01010101u
              : NW > 1 ? USV_PAIR_GEN_WEIGHTS_NW2
              : kPairPipe<RAD> ? USV_PAIR_GEN_WEIGHTS : USV_PAIR_GEN_WEIGHTS_UNPIPED;
    dim3 grid((unsigned)total), block(NW * 64);
    const uint2* tiles = tile_table(1, RAD * 16 + NW, a, P.n_xt, P.m, P.extra, P.gen_g, P.weights, (unsigned)total, s);
    hipLaunchKernelGGL((sad_pair_kernel<RAD, NW>), grid, block, 0, s, a.L, a.R, a.disp, a.dist, a, P, tiles);
    return hipGetLastError();
}

// the paired-disparity kernel: even D > 64, 11 <= w <= 15 (smaller D take the grouped kernel, usv_sad_group.hip)
bool pair_supported(const MatchArgs& a) { return a.D > 64 && (a.D % 2) == 0 && a.w >= 11 && a.w <= 15; }
template <int RAD>
hipError_t launch_pair_r(const MatchArgs& a, hipStream_t s) {
#if USV_PAIR_K16
    if constexpr (RAD == 5)
        if (a.D <= 128) return launch_pair16(a, s);
#endif
    return a.D <= 128 ? launch_pair_rn<RAD, 1>(a, s) : launch_pair_rn<RAD, 2>(a, s);
}

}  // namespace

bool pair_path_supported(const MatchArgs& a) { return pair_supported(a); }

hipError_t launch_pair(const MatchArgs& a, hipStream_t s) {
    if (!pair_supported(a)) return hipErrorInvalidValue;
    switch ((a.w - 1) / 2) {
        case 5: return launch_pair_r<5>(a, s);
        case 6: return launch_pair_r<6>(a, s);
        case 7: return launch_pair_r<7>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace usv
