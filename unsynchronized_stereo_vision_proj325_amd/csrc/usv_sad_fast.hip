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
#include <type_traits>
#include <utility>

#include "usv_band.hpp"
#include "usv_kernels.hpp"

namespace usv {
namespace {

constexpr int kK = 16;  // outputs per x-tile
#ifndef USV_STAMPS
#define USV_STAMPS 0  // diagnostic build: per-phase s_memtime totals (scripts/stamps.py)
#endif
#ifndef USV_PRIO
// Wave-priority rotation.  The SIMD arbitrates VALU issue by priority, then
// age: with equal priorities the oldest of the three resident waves runs
// nearly unimpeded and the youngest finishes ~27 us later on config C
// (scripts/wgtime.py), so the launch ends in a one- and two-wave tail.
// 1: rotate s_setprio by the wave's slot on its SIMD every flush; 2: by the
// workgroup index (both waves of a workgroup share a phase); 3: by slot,
// every input row; 0: off.
#define USV_PRIO 0
#endif
#ifndef USV_WGTIME
#define USV_WGTIME 0  // diagnostic build: per-workgroup start/end s_memrealtime + hardware id (scripts/wgtime.py)
#endif
#ifndef USV_SPLIT_CHAIN
#define USV_SPLIT_CHAIN 0  // 1: two independent prefix chains per row (ILP); 0: one chain
#endif
#ifndef USV_STATIC_RING
#define USV_STATIC_RING 0  // 1: WIN-slot R ring with compile-time slots (more LDS); 0: 8-slot dynamic ring
#endif
#ifndef USV_RED_LDS
#define USV_RED_LDS 1  // argmin transpose through LDS (1) or permlane/DPP rounds (0)
#endif
#ifndef USV_RED_PACKED
// 1: the LDS transpose stores the 8 packed (cost_x, cost_x+8) words instead of
// 16 keys (half the ds_write), the reader builds the keys with v_perm from the
// source lane's disparity (per-lane byte tables); 0: keys stored.
#define USV_RED_PACKED 1
#endif
#ifndef USV_FAST_OCC
#define USV_FAST_OCC 3  // target waves per SIMD (__launch_bounds__) for r <= 6: 3 -> <= 168 VGPRs
#endif

template <int RAD, int NW>
struct Cfg {
    static constexpr int K = kK;
    static constexpr int HALF = K / 2;
    static constexpr int WIN = 2 * RAD + 1;
    static constexpr int NPOS = K + 2 * RAD;    // columns of one input row the tile needs
    static constexpr int NSTEP = HALF + 2 * RAD;  // packed chain steps
    static constexpr int VEC = NW >= 4 ? 4 : (NW == 2 ? 2 : 1);  // LDS read width (dwords)
    static constexpr int NPOS_V = (NPOS + VEC - 1) / VEC * VEC;
    static constexpr int NR = NW * 63 + NPOS_V;  // R entries a wave reads per row
    static constexpr int NQ = (NR + 63) / 64;    // DMA instructions per R row
    static constexpr int NRS = NQ * 64;          // row-buffer stride (entries)
    // Row buffers per wave.  With one or two waves the ring holds WIN rows, so
    // in the row loop (unrolled WIN times) every buffer index, LDS offset and
    // M0 value is a compile-time constant; four waves keep a 4-row ring.
    static constexpr bool STATIC_RING = USV_STATIC_RING && NW <= 2;
    static constexpr int NB = STATIC_RING ? WIN : (NW <= 2 ? 8 : 4);
    static constexpr int PD = NB - 1;            // rows in flight ahead of the one computed
    static constexpr int KRB = WIN;              // output rows per cross-wave combine
    static constexpr int LOFF = (4 - (RAD & 3)) & 3;  // (x0 - RAD) mod 4, x0 % 4 == 0
    // LDS carve (u32 words, every region 16-byte aligned)
    static constexpr int RBUF_OFF = 0;
    // per-wave argmin transpose buffer: 16 pixels x 64 keys (USV_RED_LDS)
    static constexpr int TB_OFF = RBUF_OFF + NW * NB * NRS;
    // (r = 6 with two waves sits at the 168-VGPR limit: the DPP rounds need fewer registers)
    static constexpr bool RED_LDS = USV_RED_LDS && !(RAD == 6 && NW == 2);
    // packed transpose (USV_RED_PACKED): +8 VGPRs of per-lane tables; r = 6 with one wave would spill
    static constexpr bool RED_PACKED = USV_RED_PACKED && RED_LDS && !(RAD == 6 && NW == 1);
    static constexpr int TB_WORDS = RED_LDS ? K * 64 : 0;
    static constexpr int COMB_OFF = TB_OFF + NW * TB_WORDS;
    static constexpr int LUT_OFF = COMB_OFF + 2 * KRB * NW * K;
    static constexpr int SMEM_WORDS = LUT_OFF + 2 * 256;
    static_assert(RAD >= 1 && RAD <= 7, "packed-u16 cost needs w <= 15");
    static_assert(PD * NQ < 64, "look-ahead DMAs must fit the 6-bit vmcnt");
};

// Where a tile's L row segment comes from.  Every tile reads its L bytes from
// one exact-size scalar load; the border replication of the two edge tiles is
// a compile-time byte map:
//   kInterior  columns x0-r .. x0+K-1+r, all in range;
//   kLeft      x0 = 0: load from column 0, positions j < r replicate column 0;
//   kRight     x0 = W-K (the last tile is aligned to the right border, so it
//              may overlap its neighbour; both write identical values):
//              load up to column W-1, the last r positions replicate it.
enum : int { kInterior = 0, kLeft = 1, kRight = 2 };
//   (an edge segment shorter than 4 dwords -- K = 8 with r <= 4 -- is loaded as 4: the left one reads
//   on past its last byte, the right one starts PAD dwords earlier, so neither leaves the row)
template <int RAD, int EDGE, int KK = kK>
struct LSeg {
    static constexpr int K = KK, NPOS = K + 2 * RAD;
    static constexpr int LOFF = (4 - (RAD & 3)) & 3;  // (x0 - r) mod 4 for x0 % 4 == 0
    static constexpr int NLD0 = EDGE == kInterior ? (LOFF + NPOS + 3) / 4
                              : EDGE == kLeft     ? (K + RAD + 3) / 4
                                                  : (LOFF + K + RAD) / 4;
    static constexpr int PAD = NLD0 < 4 ? 4 - NLD0 : 0;
    static constexpr int NLD = NLD0 + PAD;
    static constexpr int SHIFT = EDGE == kRight ? 4 * PAD : 0;  // bytes the right segment starts early
    __device__ static constexpr int base(int x0) { return EDGE == kLeft ? 0 : x0 - RAD - LOFF - SHIFT; }
    __device__ static constexpr int byte(int j) {
        return EDGE == kInterior ? LOFF + j
             : EDGE == kLeft     ? (j < RAD ? 0 : j - RAD)
                                 : SHIFT + (LOFF + j < LOFF + K + RAD - 1 ? LOFF + j : LOFF + K + RAD - 1);
    }
    static_assert(EDGE != kRight || (LOFF + K + RAD) % 4 == 0, "right segment ends on a dword");
    static_assert(NLD >= 4 && NLD <= 8 && (NLD != 7 || K == 12), "scalar segment is 4, 5, 6 or 8 dwords (7: K = 12, loaded as 8)");
};

// An L byte that sits at byte 0 of its dword is used as the whole dword: the
// R operand's bytes 1-3 are zero (LDS-DMA zero-extends), so v_sad_u8 adds
// L's other three bytes to every lane's sum -- the same amount for every
// disparity of an output pixel, so the argmin (and the smallest-d tie rule) is
// unchanged and one SALU per such byte is saved.  The extra cost must not
// overflow the packed u16 sums: interior tiles only (a window of w consecutive
// positions holds at most ceil(w/4) such bytes), r <= 5: 11 rows x (11 x 255 +
// 3 x 765) = 56 100 < 65 536.  Edge tiles replicate byte 0 and keep the mask.
#ifndef USV_L_WHOLE_WORD
#define USV_L_WHOLE_WORD 1
#endif
template <int RAD, int EDGE>
constexpr bool kLWholeWord = USV_L_WHOLE_WORD && EDGE == 0 /* kInterior */ && RAD <= 5;

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)0, (int)v, CTRL, 0xF, 0xF, false);
}
constexpr int kRowMirror = 0x140;
constexpr int kRowHalfMirror = 0x141;
constexpr int kQuadSwap2 = 0x4E;  // quad_perm [2,3,0,1]
constexpr int kQuadSwap1 = 0xB1;  // quad_perm [1,0,3,2]

// v_cndmask with an explicit SGPR-pair lane mask (a VCC-sourced select issues
// several times slower on gfx950: scripts/probes/valu_rate.hip).
__device__ __forceinline__ uint32_t sel_mask(uint32_t if0, uint32_t if1, uint64_t mask) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if0), "v"(if1), "s"(mask));
    return r;
}

// 16 keys (cost << 8 | d, 64-lane vectors over disparities) -> lane l holds
// the min key of pixel l >> 2 (ties -> smaller d):
//  1. lanes l, l^32: permlane32 swap + min: lanes < 32 keep pixels 0-7;
//  2. lanes l, l^16: permlane16 swap + min: 16-lane row q keeps 4q .. 4q+3;
//  3. inside rows two transposing DPP rounds (mirror, half-mirror) and two
//     quad rounds.
template <int CTRL>
__device__ __forceinline__ uint32_t tr_round(uint32_t a, uint32_t b, uint64_t hi_mask) {
    // lanes in hi_mask keep b's pixel, the others a's; min with the DPP partner
    return min(sel_mask(a, b, hi_mask), dpp<CTRL>(sel_mask(b, a, hi_mask)));
}
__device__ __forceinline__ uint32_t reduce16(const uint32_t (&k)[16]) {
    uint32_t r1[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        auto p = __builtin_amdgcn_permlane32_swap(k[i], k[i + 8], false, false);
        r1[i] = min((uint32_t)p[0], (uint32_t)p[1]);  // lanes 0-31: pixel i, 32-63: pixel i+8
    }
    uint32_t r2[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        auto p = __builtin_amdgcn_permlane16_swap(r1[i], r1[i + 4], false, false);
        r2[i] = min((uint32_t)p[0], (uint32_t)p[1]);  // 16-lane row q: pixel i + 4q
    }
    constexpr uint64_t kBit3 = 0xFF00FF00FF00FF00ull, kBit2 = 0xF0F0F0F0F0F0F0F0ull;
    uint32_t r3[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) r3[i] = tr_round<kRowMirror>(r2[i], r2[i + 2], kBit3);
    uint32_t r4 = tr_round<kRowHalfMirror>(r3[0], r3[1], kBit2);
    r4 = min(r4, dpp<kQuadSwap2>(r4));
    return min(r4, dpp<kQuadSwap1>(r4));
}

// The same reduction through LDS (no permlane / DPP rounds but the last two):
// lane l stores key p at tb[64 p + l] (pixel-major: eight ds_write2st64), then
// lane m = 4p + q reads the 16 keys of pixel p from lanes 16q .. 16q+15 as
// four 16-byte windows, visiting them in the rotated order (k + p) & 3 so that
// the 16 lanes of each read phase touch 16 distinct bank quads; a v_min3 tree
// and two quad DPP rounds finish.  The wave's own LDS ops run in order, so the
// next row's stores cannot overtake this row's reads.
__device__ __forceinline__ uint32_t reduce16_lds(const uint32_t (&k)[16], uint32_t* tb, int lane,
                                                 const uint32_t (&rd)[4]) {
#pragma unroll
    for (int p = 0; p < 16; ++p) tb[64 * p + lane] = k[p];
    asm volatile("" ::: "memory");
    uint32_t v[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint4 q = reinterpret_cast<const uint4*>(tb)[rd[j]];
        v[4 * j] = q.x; v[4 * j + 1] = q.y; v[4 * j + 2] = q.z; v[4 * j + 3] = q.w;
    }
    asm volatile("" ::: "memory");
    uint32_t a = min(min(v[0], v[1]), v[2]), b = min(min(v[3], v[4]), v[5]);
    uint32_t c = min(min(v[6], v[7]), v[8]), d = min(min(v[9], v[10]), v[11]);
    uint32_t e = min(min(v[12], v[13]), v[14]);
    a = min(min(a, b), c);
    d = min(min(d, e), v[15]);
    uint32_t r = min(a, d);
    r = min(r, dpp<kQuadSwap2>(r));
    return min(r, dpp<kQuadSwap1>(r));
}

// Packed variant: lane l stores S[i] (costs of pixels i and i + 8 in the low /
// high halves) at tb[64 i + l]; lane m = 4p + q reads S[p % 8] of source lanes
// 16q .. 16q+15 and forms key = (half << 8) | d_src with one v_perm per value:
// dpk[j] holds the four source disparities of read j as bytes, sel[e] picks
// byte e of dpk and the low (p < 8) or high (p >= 8) half of the cost.
__device__ __forceinline__ uint32_t reduce16_lds_packed(const uint32_t (&S)[8], uint32_t* tb, int lane,
                                                        const uint32_t (&rd)[4], const uint32_t (&dpk)[4],
                                                        const uint32_t (&sel)[4]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) tb[64 * i + lane] = S[i];
    asm volatile("" ::: "memory");
    uint32_t v[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint4 q = reinterpret_cast<const uint4*>(tb)[rd[j]];
        v[4 * j] = __builtin_amdgcn_perm(q.x, dpk[j], sel[0]);
        v[4 * j + 1] = __builtin_amdgcn_perm(q.y, dpk[j], sel[1]);
        v[4 * j + 2] = __builtin_amdgcn_perm(q.z, dpk[j], sel[2]);
        v[4 * j + 3] = __builtin_amdgcn_perm(q.w, dpk[j], sel[3]);
    }
    asm volatile("" ::: "memory");
    uint32_t a = min(min(v[0], v[1]), v[2]), b = min(min(v[3], v[4]), v[5]);
    uint32_t c = min(min(v[6], v[7]), v[8]), d = min(min(v[9], v[10]), v[11]);
    uint32_t e = min(min(v[12], v[13]), v[14]);
    a = min(min(a, b), c);
    d = min(min(d, e), v[15]);
    uint32_t r = min(a, d);
    r = min(r, dpp<kQuadSwap2>(r));
    return min(r, dpp<kQuadSwap1>(r));
}

// k-th vector read of a row in order of first use by the packed chain:
// interleave the low-half columns [0, HALF) with the high-half ones.
template <int NV, int HV>
__device__ __forceinline__ constexpr int read_order(int k) {
    // first 2*HV reads alternate lo / hi, the rest are the remaining hi columns
    return k < 2 * HV ? ((k & 1) ? HV + (k >> 1) : (k >> 1)) : k;
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

// Wait until at most N vector-memory operations of this wave are outstanding
// (they retire in issue order, so every older LDS-DMA row has landed).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS-DMA of one byte per lane (zero-extended to a dword at M0 + 4*lane),
// saddr form: scalar row base + 32-bit lane offset.  GFX9 needs one wait
// state between an SALU write of M0 and an LDS-DMA that reads it (the
// compiler's hazard recognizer does not look inside inline asm): s_nop 0.  Inline asm so the
// compiler cannot precompute 64-bit per-lane addresses for the look-ahead
// rows (it hoisted and spilled them); the vmcnt waits are all explicit.
__device__ __forceinline__ uint32_t lds_addr(const uint32_t* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t*)p;
}
__device__ __forceinline__ void dma_u8(const uint8_t* row, uint32_t voff, uint32_t m0) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_ubyte %0, %1"
                 :: "v"(voff), "s"(row), "s"(m0) : "memory", "m0");
}
template <uint32_t OFF>
__device__ __forceinline__ void dma_u8_at(const uint8_t* row, uint32_t voff, uint32_t lds_base) {
    asm volatile("s_add_u32 m0, %2, %3\n\ts_nop 0\n\tglobal_load_lds_ubyte %0, %1"
                 :: "v"(voff), "s"(row), "s"(lds_base), "n"(OFF) : "memory", "m0", "scc");
}


// A whole row's R DMAs under ONE M0 write: the immediate offset of an LDS-DMA
// moves the LDS destination and the global address alike
// (scripts/probes/glds_offset_probe.hip), so DMA q uses offset:256 q and a
// per-lane offset pre-biased by -256 q; the row pointer carries a -kDmaBias
// bias so that every per-lane offset stays non-negative (the 32-bit VGPR
// offset is zero-extended).  Saves the M0 write + wait state of every DMA but
// the first.
#ifndef USV_DMA_ONE_M0
#define USV_DMA_ONE_M0 1
#endif
constexpr uint32_t kDmaBias = 1024;  // >= 256 (NQ - 1), NQ <= 5
template <int NQ>
__device__ __forceinline__ void dma_row(const uint8_t* rr_biased, const uint32_t (&vo)[NQ], uint32_t m0) {
    static_assert(NQ >= 1 && NQ <= 5, "1..5 DMAs per row");
    if constexpr (NQ == 1)
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_ubyte %0, %2"
                     :: "v"(vo[0]), "s"(m0), "s"(rr_biased) : "memory", "m0");
    else if constexpr (NQ == 2)
        asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_ubyte %0, %3\n\t"
                     "global_load_lds_ubyte %1, %3 offset:256"
                     :: "v"(vo[0]), "v"(vo[1]), "s"(m0), "s"(rr_biased) : "memory", "m0");
    else if constexpr (NQ == 3)
        asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_ubyte %0, %4\n\t"
                     "global_load_lds_ubyte %1, %4 offset:256\n\tglobal_load_lds_ubyte %2, %4 offset:512"
                     :: "v"(vo[0]), "v"(vo[1]), "v"(vo[2]), "s"(m0), "s"(rr_biased) : "memory", "m0");
    else if constexpr (NQ == 4)
        asm volatile("s_mov_b32 m0, %4\n\ts_nop 0\n\tglobal_load_lds_ubyte %0, %5\n\t"
                     "global_load_lds_ubyte %1, %5 offset:256\n\tglobal_load_lds_ubyte %2, %5 offset:512\n\t"
                     "global_load_lds_ubyte %3, %5 offset:768"
                     :: "v"(vo[0]), "v"(vo[1]), "v"(vo[2]), "v"(vo[3]), "s"(m0), "s"(rr_biased)
                     : "memory", "m0");
    else
        asm volatile("s_mov_b32 m0, %5\n\ts_nop 0\n\tglobal_load_lds_ubyte %0, %6\n\t"
                     "global_load_lds_ubyte %1, %6 offset:256\n\tglobal_load_lds_ubyte %2, %6 offset:512\n\t"
                     "global_load_lds_ubyte %3, %6 offset:768\n\tglobal_load_lds_ubyte %4, %6 offset:1024"
                     :: "v"(vo[0]), "v"(vo[1]), "v"(vo[2]), "v"(vo[3]), "v"(vo[4]), "s"(m0), "s"(rr_biased)
                     : "memory", "m0");
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() would also wait
// vmcnt(0), draining the LDS-DMA look-ahead; the comb buffers are plain LDS
// stores, so lgkmcnt(0) before the barrier is all the hand-off needs.
__device__ __forceinline__ void set_prio(int p) {
    if (p == 0) __builtin_amdgcn_s_setprio(0);
    else if (p == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(2);
}
// The wave's slot on its SIMD (HW_ID.WAVE_ID), wave-uniform.
__device__ __forceinline__ int wave_slot() {
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    return (int)(hw & 0xFu);
}

__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// The 2 KB distance table into LDS by two 16-byte-per-lane LDS-DMAs, issued ahead of a band loop's row
// prologue: vector-memory ops retire in order, so the first row's counted DMA wait also retires them, and
// nothing waits on the table's own round trip (a register load + ds_write + barrier waited vmcnt(0)).
// Every wave of a workgroup stages the whole table (identical bytes): no barrier before its first use.
__device__ __forceinline__ void lut_dma(const double* lut, uint32_t* lds, int lane) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %2\n\t"
                 "global_load_lds_dwordx4 %0, %2 offset:1024"
                 :: "v"((uint32_t)lane * 16u), "s"(lds_addr(lds)), "s"(lut) : "memory", "m0");
}

// Scalar-load an exact number of dwords (5, 6 or 8: never past the row) into SGPRs.
// Two-instruction forms use early-clobber outputs: the first load's
// destination must not overlap the base the second one reads.
using su4 = uint32_t __attribute__((ext_vector_type(4)));
using su2 = uint32_t __attribute__((ext_vector_type(2)));
using su8 = uint32_t __attribute__((ext_vector_type(8)));
template <int N> struct SWords;
template <> struct SWords<4> { using T = su4; };
template <> struct SWords<5> { struct T { su4 a; uint32_t b; }; };
template <> struct SWords<6> { struct T { su4 a; su2 b; }; };
template <> struct SWords<8> { using T = su8; };
template <int N>
__device__ __forceinline__ typename SWords<N>::T s_load_words(const uint8_t* p) {
    typename SWords<N>::T w;
    if constexpr (N == 8) {
        asm volatile("s_load_dwordx8 %0, %1, 0x0" : "=s"(w) : "s"(p) : "memory");
    } else if constexpr (N == 4) {
        asm volatile("s_load_dwordx4 %0, %1, 0x0" : "=s"(w) : "s"(p) : "memory");
    } else if constexpr (N == 6) {
        asm volatile("s_load_dwordx4 %0, %2, 0x0\n\ts_load_dwordx2 %1, %2, 0x10"
                     : "=&s"(w.a), "=&s"(w.b) : "s"(p) : "memory");
    } else {
        asm volatile("s_load_dwordx4 %0, %2, 0x0\n\ts_load_dword %1, %2, 0x10"
                     : "=&s"(w.a), "=&s"(w.b) : "s"(p) : "memory");
    }
    return w;
}
// Scalar loads return out of order: only lgkmcnt(0) retires one.  The words
// are in/out operands so nothing that reads them can be scheduled above.
template <int N>
__device__ __forceinline__ void wait_lgkm0(typename SWords<N>::T& w) {
    if constexpr (N == 8 || N == 4) asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(w) : : "memory");
    else asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(w.a), "+s"(w.b) : : "memory");
}
template <int N>
__device__ __forceinline__ void unpack_words(const typename SWords<N>::T& w, uint32_t (&o)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = 0;
    if constexpr (N == 8) {
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = w[i];
    } else if constexpr (N == 4) {
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = w[i];
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = w.a[i];
        if constexpr (N == 6) { o[4] = w.b[0]; o[5] = w.b[1]; }
        else o[4] = w.b;
    }
}

// Steady-state row addressing without 64-bit pointer arithmetic: the R row's LDS-DMAs
// are MUBUF loads whose soffset carries the row offset (buffer over R - kDmaBias,
// no range limit), the L row segment an s_load with an SGPR offset; both offsets are
// running sums clamped at the last image row (two SALU per pointer and row instead of
// clamp, multiply and a 64-bit add).  Warm-up rows keep the clamped per-row form.
#ifndef USV_RUN_ADDR
#define USV_RUN_ADDR 1
#endif
template <int NQ>
__device__ __forceinline__ void dma_row_buf(su4 rsrc, uint32_t soff, const uint32_t (&vo)[NQ], uint32_t m0) {
    static_assert(NQ >= 1 && NQ <= 5, "1..5 DMAs per row");
    if constexpr (NQ == 1)
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_ubyte %0, %2, %3 offen lds"
                     :: "v"(vo[0]), "s"(m0), "s"(rsrc), "s"(soff) : "memory", "m0");
    else if constexpr (NQ == 2)
        asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_ubyte %0, %3, %4 offen lds\n\t"
                     "buffer_load_ubyte %1, %3, %4 offen offset:256 lds"
                     :: "v"(vo[0]), "v"(vo[1]), "s"(m0), "s"(rsrc), "s"(soff) : "memory", "m0");
    else if constexpr (NQ == 3)
        asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_ubyte %0, %4, %5 offen lds\n\t"
                     "buffer_load_ubyte %1, %4, %5 offen offset:256 lds\n\t"
                     "buffer_load_ubyte %2, %4, %5 offen offset:512 lds"
                     :: "v"(vo[0]), "v"(vo[1]), "v"(vo[2]), "s"(m0), "s"(rsrc), "s"(soff) : "memory", "m0");
    else if constexpr (NQ == 4)
        asm volatile("s_mov_b32 m0, %4\n\ts_nop 0\n\tbuffer_load_ubyte %0, %5, %6 offen lds\n\t"
                     "buffer_load_ubyte %1, %5, %6 offen offset:256 lds\n\t"
                     "buffer_load_ubyte %2, %5, %6 offen offset:512 lds\n\t"
                     "buffer_load_ubyte %3, %5, %6 offen offset:768 lds"
                     :: "v"(vo[0]), "v"(vo[1]), "v"(vo[2]), "v"(vo[3]), "s"(m0), "s"(rsrc), "s"(soff)
                     : "memory", "m0");
    else
        asm volatile("s_mov_b32 m0, %5\n\ts_nop 0\n\tbuffer_load_ubyte %0, %6, %7 offen lds\n\t"
                     "buffer_load_ubyte %1, %6, %7 offen offset:256 lds\n\t"
                     "buffer_load_ubyte %2, %6, %7 offen offset:512 lds\n\t"
                     "buffer_load_ubyte %3, %6, %7 offen offset:768 lds\n\t"
                     "buffer_load_ubyte %4, %6, %7 offen offset:1024 lds"
                     :: "v"(vo[0]), "v"(vo[1]), "v"(vo[2]), "v"(vo[3]), "v"(vo[4]), "s"(m0), "s"(rsrc), "s"(soff)
                     : "memory", "m0");
}
template <int N>
__device__ __forceinline__ typename SWords<N>::T s_load_words_off(const uint8_t* p, uint32_t off) {
    typename SWords<N>::T w;
    if constexpr (N == 8) {
        asm volatile("s_load_dwordx8 %0, %1, %2" : "=s"(w) : "s"(p), "s"(off) : "memory");
    } else if constexpr (N == 4) {
        asm volatile("s_load_dwordx4 %0, %1, %2" : "=s"(w) : "s"(p), "s"(off) : "memory");
    } else if constexpr (N == 6) {
        asm volatile("s_load_dwordx4 %0, %2, %3\n\ts_load_dwordx2 %1, %2, %3 offset:0x10"
                     : "=&s"(w.a), "=&s"(w.b) : "s"(p), "s"(off) : "memory");
    } else {
        asm volatile("s_load_dwordx4 %0, %2, %3\n\ts_load_dword %1, %2, %3 offset:0x10"
                     : "=&s"(w.a), "=&s"(w.b) : "s"(p), "s"(off) : "memory");
    }
    return w;
}

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
    const int prio_slot = USV_PRIO == 3 ? wave_slot() : 0;
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
    const uint8_t* const Rdma = (USV_DMA_ONE_M0 && !C::STATIC_RING) ? R - kDmaBias : R;
    constexpr bool RUN = USV_RUN_ADDR && USV_DMA_ONE_M0 && !C::STATIC_RING;
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
    // BUF >= 0: compile-time ring slot (static ring); BUF < 0: slot t & (NB-1)
    auto issue_dma = [&](int t, auto buf_tag) {
        constexpr int BUF = decltype(buf_tag)::value;
        const uint8_t* rr = Rdma + row_off(t);
        if constexpr (BUF >= 0) {
            [&]<int... Q>(std::integer_sequence<int, Q...>) {
                (dma_u8_at<4u * (BUF * C::NRS + 64 * Q)>(rr, colR[Q], rbase), ...);
            }(std::make_integer_sequence<int, C::NQ>{});
        } else if constexpr (USV_DMA_ONE_M0 && !C::STATIC_RING) {
            const int buf = t & (NB - 1);
            dma_row<C::NQ>(rr, colRb, rbase + 4u * (uint32_t)(buf * C::NRS));
        } else {
            const int buf = t & (NB - 1);
#pragma unroll
            for (int i = 0; i < C::NQ; ++i)
                dma_u8(rr, colR[i], rbase + 4u * (buf * C::NRS + 64 * i));
        }
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
    // S / ring update.  I selects the ring slot (and, with the static ring,
    // the row buffers) at compile time.
    auto do_row = [&](int t_in, auto warm_tag, auto i_tag, uint32_t(&S)[HALF], uint32_t(&ring)[WIN][HALF]) {
        constexpr bool WARM = decltype(warm_tag)::value;
        constexpr int I = decltype(i_tag)::value;
        // opaque row index: keeps the compiler from computing every unrolled
        // row's pointers up front (SGPR pressure that ends in VGPR spills)
        int t = t_in;
        asm volatile("" : "+s"(t));
        wait_vmcnt<(PD - 1) * NDMA>();  // row t has landed in LDS
        __builtin_amdgcn_wave_barrier();
        if constexpr (USV_PRIO == 3) set_prio((prio_slot + t) % 3);
        if constexpr (C::STATIC_RING) {
            issue_dma(t + PD, std::integral_constant<int, (I + PD) % NB>{});
        } else if constexpr (RUN && !WARM) {
            int rr = rawR;
            asm volatile("" : "+s"(rr));  // opaque: one row's offset at a time
            const int buf = (t + PD) & (NB - 1);
            dma_row_buf<C::NQ>(rsrc, (uint32_t)min(rr, last_off), colRb, rbase + 4u * (uint32_t)(buf * C::NRS));
            rawR = rr + a.pitch;
        } else {
            issue_dma(t + PD, std::integral_constant<int, -1>{});
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
        int boff = (C::STATIC_RING ? I % NB : (t & (NB - 1))) * C::NRS;
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
        // Packed prefix P[j] = [sum_{i<j} e(i), sum_{i<j} e(i + HALF)]; with
        // USV_SPLIT_CHAIN two independent chains: A covers steps [0, SP), B
        // steps [SP, NSTEP) from zero, so P[j] = A[SP] + B[j - SP] for j > SP.
        constexpr int SP = USV_SPLIT_CHAIN ? HALF : C::NSTEP;
        constexpr int NB_STEPS = C::NSTEP - SP;
        uint32_t A[SP + 1], Bc[NB_STEPS + 1];
        A[0] = 0;
        Bc[0] = 0;
#pragma unroll
        for (int j = 0; j < (SP > NB_STEPS ? SP : NB_STEPS); ++j) {
            if (j < SP)
                A[j + 1] = __builtin_amdgcn_sad_hi_u8(Lv[j + HALF], Rv[j + HALF],
                                                      __builtin_amdgcn_sad_u8(Lv[j], Rv[j], A[j]));
            if (j < NB_STEPS) {
                const int jj = j + SP;
                Bc[j + 1] = __builtin_amdgcn_sad_hi_u8(Lv[jj + HALF], Rv[jj + HALF],
                                                       __builtin_amdgcn_sad_u8(Lv[jj], Rv[jj], Bc[j]));
            }
        }
#pragma unroll
        for (int x = 0; x < HALF; ++x) {
            // H pair (x, x + HALF) = P[x + WIN] - P[x].  Packed pairs, but
            // every intermediate half stays in [0, 65535] (prefixes are
            // monotone, S - ring is a w-1 row sum), so plain 32-bit add/sub
            // give the packed result exactly: v_add/v_sub_u32 issue at full
            // rate, v_pk_*_u16 at half rate (scripts/probes/valu_rate.hip).
            uint32_t h;
            if (x + WIN <= SP) h = A[x + WIN] - A[x];
            else h = Bc[x + WIN - SP] + (A[SP] - A[x]);
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
        if constexpr (RUN && !WARM) {
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
    int prio_phase = USV_PRIO == 2 ? (int)blockIdx.x : (USV_PRIO == 1 || USV_PRIO == 3 ? wave_slot() : 0);
    if (USV_PRIO) set_prio(prio_phase % 3);
    auto flush = [&](int rows) {
        if (USV_PRIO == 1 || USV_PRIO == 2) set_prio(++prio_phase % 3);
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
        (issue_dma(P, std::integral_constant<int, C::STATIC_RING ? P : -1>{}), ...);
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

// Band decomposition of one launch (launch_rn): m bands per column, their
// heights weighted by dispatch generation (see sad_fast_kernel).
struct BandPlan {
    int n_xt;      // x-tiles per pair
    int m;         // bands per column (pair, x-tile)
    int gen_g;     // workgroups per dispatch generation per XCD (4 SIMDs x CUs per XCD / waves per WG)
    unsigned weights;  // byte g: relative band height of generation g (g >= 3 use byte 3)
    int extra;     // single pair only: x-tiles 0..extra-1 carry m + 1 bands (fills every resident slot)
};

// r = 7 (15-row ring) and r = 6 with four waves need more than 168 VGPRs:
// two waves per SIMD instead of spilling (tests/test_isa_lint.py checks).
constexpr int fast_occ(int rad, int nw) { return (rad >= 7 || (rad == 6 && nw == 4)) ? 2 : USV_FAST_OCC; }

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

int cu_count() {
    static const int n = [] {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
            v = 256;
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
#ifndef USV_ROUNDS
#define USV_ROUNDS 1  // workgroup rounds per launch (experiment: >1 = shorter bands, later rounds fill the tail)
#endif
#ifndef USV_MIN_BAND_WINS
// shortest band, in windows (w rows): the ring warm-up costs w rows per band.  Binds only on small frames
// (1080p, D = 128 has 12-13 bands of ~85 rows); interleaved A/B at 640x480 w7 D64: 1 / 2 / 3 / 4 windows =
// 29.5 / 22.2 / 20.5 / 22.5 us, at 320x240 w5 D32: 2 / 3 / 4 = 16.8 / 15.3 / 16.4 us
// (profiles/probes/ab_minband_small_r01.txt, ab_weights_minband_r01.txt).
#define USV_MIN_BAND_WINS 3
#endif
    long m = slots * USV_ROUNDS / NC;
    if (m < 1) m = 1;
    const long m_max = a.H / (USV_MIN_BAND_WINS * WIN) > 0 ? a.H / (USV_MIN_BAND_WINS * WIN) : 1;
    if (m > m_max) m = m_max;
    P.m = (int)m;
#ifndef USV_EXTRA_BANDS
#define USV_EXTRA_BANDS 1  // one pair: give some x-tiles an extra band so the grid fills every resident slot
#endif
    // e.g. 1080p, D = 128: 1536 slots over 120 x-tiles = 12 bands + 96 x-tiles with a 13th
    const long ex = slots * USV_ROUNDS - NC * m;
    P.extra = (USV_EXTRA_BANDS && a.batch == 1 && USV_ROUNDS == 1 && ex > 0 && ex < P.n_xt &&
               a.H / (m + 1) >= USV_MIN_BAND_WINS * WIN) ? (int)ex : 0;
    const long total = NC * m + P.extra;
    if (total > 0x7FFFFFFFL) return hipErrorInvalidValue;
    P.gen_g = (int)((4L * (cu_count() / 8)) / NW);
    if (P.gen_g < 1) P.gen_g = 1;
    // weighted only when every SIMD holds three waves of one round
    const bool three = USV_ROUNDS == 1 && per_cu * NW == 12 && total > 2L * 8 * P.gen_g;
    P.weights = three ? USV_GEN_WEIGHTS : 0x01010101u;
    dim3 grid((unsigned)total), block(NW * 64);
    hipLaunchKernelGGL((sad_fast_kernel<RAD, NW>), grid, block, 0, s, a.L, a.R, a.disp, a.dist, a, P);
    return hipGetLastError();
}

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
#ifndef USV_PAIR_PIPE
#define USV_PAIR_PIPE 1  // argmin transpose of row t finished during row t + 1 (latency hidden by the chain)
#endif
#ifndef USV_NT_DIST
#define USV_NT_DIST 0  // experiment: the paired kernel's distance map through non-temporal stores
#endif
#ifndef USV_WIDE_FLUSH
#define USV_WIDE_FLUSH 1  // paired kernel: one 8-byte disparity store and one 16-byte distance store per lane per chunk
#endif
#ifndef USV_PAIR_PIPE_R7
#define USV_PAIR_PIPE_R7 0  // experiment: pipelined argmin at r = 7 (needs USV_PAIR_OCC7=2, USV_PAIR_SPLIT_R=8)
#endif
template <int RAD>
constexpr bool kPairPipe = USV_PAIR_PIPE && (RAD == 5 || (RAD == 7 && USV_PAIR_PIPE_R7));
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
    static constexpr int NB = 8;                        // ring slots per wave
#ifndef USV_PAIR_SPLIT_R
#define USV_PAIR_SPLIT_R 7  // radius from which the row's entries are read in two batches
#endif
    static constexpr int SPLIT = RAD >= USV_PAIR_SPLIT_R ? 2 : 1;
    static constexpr int PD = NB - 1;
    static constexpr int KRB = WIN;
    static constexpr int RBUF_OFF = 0;
    static constexpr int TB_OFF = RBUF_OFF + NW * NB * NRS;
    static constexpr int TB_WORDS = K * 64;
    static constexpr int COMB_OFF = TB_OFF + NW * TB_WORDS;
    static constexpr int LUT_OFF = COMB_OFF + 2 * KRB * NW * K;
    static constexpr int SMEM_WORDS = LUT_OFF + 2 * 256;
    static_assert(RAD >= 2 && RAD <= 7, "paired kernel: 5 <= w <= 15");
    static_assert(PD * NQ < 64, "look-ahead DMAs must fit the 6-bit vmcnt");
    static_assert(NQ <= 5, "dma_row_buf issues at most 5 DMAs");
};

// The paired kernel's L row segment lives in FIXED SGPRs s[40:45] from its scalar load to the wait
// that retires it: with ordinary "s" constraints the register allocator may copy the in-flight
// destination into other SGPRs before the wait (seen at loop latches), reading stale words.
template <int N>
__device__ __forceinline__ typename SWords<N>::T s_load_words_pin(const uint8_t* p, uint32_t off) {
    static_assert(N == 4 || N == 5 || N == 6 || N == 8, "paired kernel segments are 4, 5, 6 or 8 dwords");
    typename SWords<N>::T w;
    if constexpr (N == 5)
        asm volatile("s_load_dwordx4 %0, %2, %3\n\ts_load_dword %1, %2, %3 offset:0x10"
                     : "=&{s[40:43]}"(w.a), "=&{s44}"(w.b) : "s"(p), "s"(off) : "memory");
    else if constexpr (N == 4)
        asm volatile("s_load_dwordx4 %0, %1, %2" : "=&{s[40:43]}"(w) : "s"(p), "s"(off) : "memory");
    else if constexpr (N == 8)
        asm volatile("s_load_dwordx8 %0, %1, %2" : "=&{s[40:47]}"(w) : "s"(p), "s"(off) : "memory");
    else
        asm volatile("s_load_dwordx4 %0, %2, %3\n\ts_load_dwordx2 %1, %2, %3 offset:0x10"
                     : "=&{s[40:43]}"(w.a), "=&{s[44:45]}"(w.b) : "s"(p), "s"(off) : "memory");
    return w;
}
template <int N>
__device__ __forceinline__ void wait_lgkm0_pin(typename SWords<N>::T& w) {
    if constexpr (N == 4) asm volatile("s_waitcnt lgkmcnt(0)" : "+{s[40:43]}"(w) : : "memory");
    else if constexpr (N == 5) asm volatile("s_waitcnt lgkmcnt(0)" : "+{s[40:43]}"(w.a), "+{s44}"(w.b) : : "memory");
    else if constexpr (N == 8) asm volatile("s_waitcnt lgkmcnt(0)" : "+{s[40:47]}"(w) : : "memory");
    else asm volatile("s_waitcnt lgkmcnt(0)" : "+{s[40:43]}"(w.a), "+{s[44:45]}"(w.b) : : "memory");
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
    auto issue_dma = [&](int t) {
        const int buf = t & (NB - 1);
        dma_row<C::NQ>(Rdma + row_off(t), colRb, rbase + 4u * (uint32_t)(buf * C::NRS));
    };
    LWords lw_next;
    auto load_lw = [&](int t) { lw_next = s_load_words_pin<LS::NLD>(Lseg, row_off(t)); };

    auto do_row = [&](int t_in, auto warm_tag, auto i_tag, uint32_t(&S)[K], uint32_t(&ring)[WIN][K], auto&& pre) {
        constexpr bool WARM = decltype(warm_tag)::value;
        constexpr int I = decltype(i_tag)::value;
        int t = t_in;
        asm volatile("" : "+s"(t));
        wait_vmcnt<(PD - 1) * NDMA>();
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
        // (pipelined argmin: the ring row leaving the window is subtracted first, so its registers
        // are free for this row's staged entries -- no copies)
        constexpr bool EARLY_SUB = !WARM && kPairPipe<RAD>;
        if constexpr (EARLY_SUB) {
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
                if (kLWholeWord<RAD, EDGE> && (bidx & 3) == 0) Lv[j] = lw[bidx >> 2];
                else Lv[j] = (lw[bidx >> 2] >> (8 * (bidx & 3))) & 0xFFu;
            }
        }
        auto lbyte = [&](int j) -> uint32_t { return Lv[j]; };
        using VT = typename VecT<C::VEC>::T;
        int boff = (t & (NB - 1)) * C::NRS;
        asm volatile("" : "+s"(boff));
        const VT* rb = reinterpret_cast<const VT*>(rbuf + boff + s_l);
        // The staged entries come in C::SPLIT batches of vector reads, each consumed by the chain
        // steps it completes before the next batch is read (r = 7: fewer live VGPRs, so three
        // waves fit per SIMD; the second batch's latency is covered by the other waves).
        uint32_t E[C::NE_V];
        constexpr int NV = C::NE_V / C::VEC, NV1 = C::SPLIT > 1 ? (NV + 1) / 2 : NV;
        constexpr int J1 = C::SPLIT > 1 ? NV1 * C::VEC - 1 : NPOS;  // steps the first batch completes
#pragma unroll
        for (int k = 0; k < NV1; ++k) {
            const VT v = rb[k];
#pragma unroll
            for (int e = 0; e < C::VEC; ++e) E[k * C::VEC + e] = vget<C::VEC>(v, e);
        }
        // P[j + 1] = P[j] + (|L_j - R(d)| low half, |L_j - R(d + 1)| high half).  With the argmin
        // pipelined, piece j of the previous row's argmin follows chain step j and the pair is
        // fenced: the two independent dependency chains interleave instruction by instruction.
        uint32_t A[NPOS + 1];
        A[0] = 0;
        auto chain_step = [&](auto jt) {
            constexpr int j = decltype(jt)::value;
            const uint32_t l = lbyte(j);
            A[j + 1] = __builtin_amdgcn_sad_hi_u8(l, E[j], __builtin_amdgcn_sad_u8(l, E[j + 1], A[j]));
            pre(jt);
            if constexpr (EARLY_SUB) __builtin_amdgcn_sched_barrier(0);
        };
        [&]<int... J>(std::integer_sequence<int, J...>) {
            (chain_step(std::integral_constant<int, J>{}), ...);
        }(std::make_integer_sequence<int, J1>{});
        if constexpr (C::SPLIT > 1) {
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = NV1; k < NV; ++k) {
                const VT v = rb[k];
#pragma unroll
                for (int e = 0; e < C::VEC; ++e) E[k * C::VEC + e] = vget<C::VEC>(v, e);
            }
#pragma unroll
            for (int j = J1; j < NPOS; ++j)
                A[j + 1] = __builtin_amdgcn_sad_hi_u8(lbyte(j), E[j], __builtin_amdgcn_sad_u8(lbyte(j), E[j + 1], A[j]));
        }
#pragma unroll
        for (int x = 0; x < K; ++x) {
            const uint32_t h = A[x + WIN] - A[x];  // both halves in [0, 65535], no borrow
            if constexpr (WARM || EARLY_SUB) S[x] = S[x] + h;
            else S[x] = (S[x] - ring[I][x]) + h;
            ring[I][x] = h;
        }
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
    // Wide flush (USV_WIDE_FLUSH): a chunk's outputs leave in two store instructions -- lane r
    // writes row r's 8 disparity bytes as one 8-byte store, lane 4r + q row r's distances 2q, 2q+1
    // as one 16-byte store -- instead of a byte + a double per lane and item (4 per 11-row chunk).
    // Global stores count in vmcnt on gfx9 with the LDS-DMA look-ahead, so fewer, wider stores also
    // hold up fewer of the next rows' counted DMA waits.  Needs 4-byte aligned disparity rows.
    const bool wide = USV_WIDE_FLUSH && ((reinterpret_cast<uintptr_t>(disp + x0) | (uintptr_t)a.disp_pitch) & 3u) == 0;
    auto flush = [&](int rows) {
        if constexpr (NW > 1) lds_barrier();
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: its LDS ops run in order
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        if (wide) {
            static_assert(K == 8, "one 8-byte disparity store per row");
            const uint32_t* crow = comb + (cb * KRB) * NW * K;
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
                // byte 0 of each key is its disparity
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
                if constexpr (USV_NT_DIST) {  // experiment: write-once map as non-temporal stores
                        typedef double v2d __attribute__((ext_vector_type(2)));
                        v2d v = {lut_s[kk.x & 0xFFu], lut_s[kk.y & 0xFFu]};
                        __builtin_nontemporal_store(v, reinterpret_cast<v2d*>(dist + y * a.dist_pitch + x0 + 2 * q));
                    } else {
                        *reinterpret_cast<D2*>(dist + y * a.dist_pitch + x0 + 2 * q) = D2{lut_s[kk.x & 0xFFu], lut_s[kk.y & 0xFFu]};
                    }
            }
            y_chunk += rows;
            cb ^= 1;
            return;
        }
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
    // Argmin of one row, in two halves so that the LDS round trip of the transpose and the
    // dependent min / DPP tail overlap the next row's chain (USV_PAIR_PIPE):
    //   tr_issue:  lane l stores its 8 packed words, lane 8p + q reads the 8 words of pixel p from
    //              lanes 8q .. 8q + 7 (two ds_read_b128) -- nothing waits on them here;
    //   tr_finish: 16 keys (cost << 8) | d by v_perm, a v_min3 tree, three DPP rounds across the 8
    //              lanes of the pixel, one comb word per pixel.
    uint4 trq[2];
    auto tr_issue = [&](const uint32_t(&S)[K]) {
#pragma unroll
        for (int i = 0; i < K; ++i) tb[64 * i + lane] = S[i];
        asm volatile("" ::: "memory");
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            // (r = 7: the second window's index is rebuilt per row as well)
            const uint32_t ri = (C::SPLIT > 1 && j == 1) ? (rdw[0] ^ 1u) : rdw[j];
            trq[j] = reinterpret_cast<const uint4*>(tb)[ri];
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
            comb[((cb * KRB + slot) * NW + wave) * K + px] = fm;
        }
    };
    auto tr_finish = [&](int slot) {
        [&]<int... J>(std::integer_sequence<int, J...>) {
            (tr_piece(std::integral_constant<int, J>{}, slot), ...);
        }(std::make_integer_sequence<int, 16>{});
    };
    auto emit = [&](const uint32_t(&S)[K], int slot) {
        tr_issue(S);
        tr_finish(slot);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto no_pre = [](auto) {};

    // ---- prefetched row boundary (USV_PAIR_PREF, pipelined r = 5 only) ----
    // Without it every row starts with an s_waitcnt lgkmcnt(0) (the pinned L words are a scalar
    // load, which returns out of order) that also retires the previous row's transpose reads issued
    // just before, then issues its staged-entry reads and waits for the first of them: two LDS round
    // trips per row with nothing else of this wave to issue.  Here the boundary is reordered:
    //   end of row t:  lgkmcnt(0) (everything of row t, and the L words of row t + 1 loaded a row
    //                  earlier) -> extract row t + 1's L bytes -> [flush] -> scalar-load row t + 2's
    //                  L words -> vmcnt wait for row t + 1's DMA -> the first PV vector reads of
    //                  row t + 1's staged entries -> row t's transpose WRITES;
    //   row t + 1:     DMA, ring subtraction, the remaining entry reads, THEN the transpose reads,
    //                  the chain (its first steps run on the prefetched entries) with the argmin
    //                  pieces from step PIECE_OFF on, so the transpose reads have a whole run of
    //                  chain steps to land.
#ifndef USV_PAIR_PREF
#define USV_PAIR_PREF 0  // vector reads of the next row prefetched (0 = off)
#endif
#ifndef USV_PAIR_PIECE_OFF
#define USV_PAIR_PIECE_OFF 8  // chain step of the first argmin piece (USV_PAIR_PREF)
#endif
    constexpr bool PREF = USV_PAIR_PREF > 0 && kPairPipe<RAD> && C::SPLIT == 1;
    using VTp = typename VecT<C::VEC>::T;
    constexpr int NVp = C::NE_V / C::VEC;
    constexpr int PV = PREF ? (USV_PAIR_PREF < NVp ? USV_PAIR_PREF : NVp) : 1;
    constexpr int OFFP = USV_PAIR_PIECE_OFF;
    uint32_t Epf[PV * C::VEC];
    uint32_t Lv[NPOS];  // L bytes of the row about to run
    auto extract_l = [&]() {  // after wait_lgkm0_pin(lw_next)
        LWords cur = lw_next;
        uint32_t lw[8];
        unpack_words<LS::NLD>(cur, lw);
#pragma unroll
        for (int j = 0; j < NPOS; ++j) {
            const int bidx = LS::byte(j);
            if (kLWholeWord<RAD, EDGE> && (bidx & 3) == 0) Lv[j] = lw[bidx >> 2];
            else Lv[j] = (lw[bidx >> 2] >> (8 * (bidx & 3))) & 0xFFu;
        }
    };
    auto prefetch_e = [&](int t_next) {
        wait_vmcnt<(PD - 1) * NDMA>();  // row t_next's DMA (issued PD rows ago) has landed
        __builtin_amdgcn_wave_barrier();
        int boff = (t_next & (NB - 1)) * C::NRS;
        asm volatile("" : "+s"(boff));
        const VTp* rb = reinterpret_cast<const VTp*>(rbuf + boff + s_l);
#pragma unroll
        for (int k = 0; k < PV; ++k) {
            const VTp v = rb[k];
#pragma unroll
            for (int e = 0; e < C::VEC; ++e) Epf[k * C::VEC + e] = vget<C::VEC>(v, e);
        }
    };
    auto tr_write = [&](const uint32_t(&S)[K]) {
#pragma unroll
        for (int i = 0; i < K; ++i) tb[64 * i + lane] = S[i];
        asm volatile("" ::: "memory");
    };
    auto tr_read = [&]() {
#pragma unroll
        for (int j = 0; j < 2; ++j) trq[j] = reinterpret_cast<const uint4*>(tb)[rdw[j]];
        asm volatile("" ::: "memory");
    };
    auto do_row_pref = [&](int t_in, auto i_tag, uint32_t(&S)[K], uint32_t(&ring)[WIN][K]) {
        constexpr int I = decltype(i_tag)::value;
        int t = t_in;
        asm volatile("" : "+s"(t));
        {
            int rr = rawR;
            asm volatile("" : "+s"(rr));
            const int buf = (t + PD) & (NB - 1);
            dma_row_buf<C::NQ>(rsrc, (uint32_t)min(rr, last_off), colRb, rbase + 4u * (uint32_t)(buf * C::NRS));
            rawR = rr + a.pitch;
        }
#pragma unroll
        for (int x = 0; x < K; ++x) S[x] -= ring[I][x];
        uint32_t E[C::NE_V];
#pragma unroll
        for (int e = 0; e < PV * C::VEC; ++e) E[e] = Epf[e];
        int boff = (t & (NB - 1)) * C::NRS;
        asm volatile("" : "+s"(boff));
        const VTp* rb = reinterpret_cast<const VTp*>(rbuf + boff + s_l);
#pragma unroll
        for (int k = PV; k < NVp; ++k) {
            const VTp v = rb[k];
#pragma unroll
            for (int e = 0; e < C::VEC; ++e) E[k * C::VEC + e] = vget<C::VEC>(v, e);
        }
        tr_read();
        uint32_t A[NPOS + 1];
        A[0] = 0;
        auto chain_step = [&](auto jt) {
            constexpr int j = decltype(jt)::value;
            const uint32_t l = Lv[j];
            A[j + 1] = __builtin_amdgcn_sad_hi_u8(l, E[j], __builtin_amdgcn_sad_u8(l, E[j + 1], A[j]));
            if constexpr (j >= OFFP && j - OFFP < 16) tr_piece(std::integral_constant<int, j - OFFP>{}, I);
            __builtin_amdgcn_sched_barrier(0);
        };
        [&]<int... J>(std::integer_sequence<int, J...>) {
            (chain_step(std::integral_constant<int, J>{}), ...);
        }(std::make_integer_sequence<int, NPOS>{});
        [&]<int... J>(std::integer_sequence<int, J...>) {
            ((J >= (NPOS - OFFP > 0 ? NPOS - OFFP : 0) ? tr_piece(std::integral_constant<int, J>{}, I) : void()), ...);
        }(std::make_integer_sequence<int, 16>{});
#pragma unroll
        for (int x = 0; x < K; ++x) {
            const uint32_t h = A[x + WIN] - A[x];
            S[x] = S[x] + h;
            ring[I][x] = h;
        }
    };
    auto row_tail = [&](int t, bool do_flush, const uint32_t(&S)[K]) {
        wait_lgkm0_pin<LS::NLD>(lw_next);
        extract_l();
        if (do_flush) flush(KRB);
        {
            int rl = rawL;
            asm volatile("" : "+s"(rl));
            lw_next = s_load_words_pin<LS::NLD>(Lseg, (uint32_t)min(rl, last_off));
            rawL = rl + a.pitch;
        }
        prefetch_e(t + 1);
        tr_write(S);
        __builtin_amdgcn_sched_barrier(0);
    };

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
    // Pipelined argmin (PIPE): output row k is slot k % KRB.  Row k's transpose is issued after its
    // chain and finished inside the next row's do_row (after that row's staged reads are issued), so
    // slot I is pending when the I-th row of a WIN-row group starts; the chunk is flushed once slot
    // KRB - 1 is finished.  (r = 6, 7 keep the unpipelined order: the held transpose words spill.)
    constexpr bool PIPE = kPairPipe<RAD>;
    static_assert(KRB == WIN, "pending slot = row index in the unrolled group");
    static_assert(!PIPE || NPOS >= 16, "16 argmin pieces ride on the chain steps");
    if constexpr (PREF) {
        row_tail(WIN - 1, false, S);
    } else if constexpr (PIPE) {
        tr_issue(S);
        __builtin_amdgcn_sched_barrier(0);
    } else {
        emit(S, 0);
    }
    auto step = [&](int t0, auto i_tag) {
        constexpr int I = decltype(i_tag)::value;
        if constexpr (PREF) {
            do_row_pref(t0 + I, i_tag, S, ring);
            row_tail(t0 + I, I == KRB - 1, S);
        } else if constexpr (PIPE) {
            do_row(t0 + I, SteadyT{}, i_tag, S, ring, [&](auto jt) {
                if constexpr (decltype(jt)::value < 16) tr_piece(jt, I);
            });
            if constexpr (I == KRB - 1) flush(KRB);
            tr_issue(S);
            __builtin_amdgcn_sched_barrier(0);
        } else {
            do_row(t0 + I, SteadyT{}, i_tag, S, ring, no_pre);
            emit(S, (I + 1) % WIN);
            if constexpr ((I + 1) % WIN == KRB - 1) flush(KRB);
        }
    };
    for (int t0 = WIN; t0 < T; t0 += WIN) {
        [&]<int... I>(std::integer_sequence<int, I...>) {
            bool go = true;
            ((go = go && (t0 + I < T), go ? step(t0, std::integral_constant<int, I>{}) : void()), ...);
        }(std::make_integer_sequence<int, WIN>{});
    }
    wait_lgkm0_pin<LS::NLD>(lw_next);  // retire the unused last L load before its SGPRs are reused
    if constexpr (PIPE) {
        const int last = (nout - 1) % KRB;  // the pending slot: the band's last output row
        if constexpr (PREF) tr_read();
        tr_finish(last);
        if (last == KRB - 1) flush(KRB);
    }
    const int rest = nout % KRB;
    if (rest) flush(rest);
    wait_vmcnt<0>();
}

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
                                                              double* __restrict__ dist, MatchArgs a, BandPlan P) {
    using C = PCfg<RAD, NW>;
    __shared__ __attribute__((aligned(16))) uint32_t smem[C::SMEM_WORDS];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // the work map of sad_fast_kernel (XCD-contiguous tile runs, generation-weighted bands)
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
    const int xt = (int)col_xt;
    const int n_xt = P.n_xt;
    int x0 = xt * C::K;
    if (xt == n_xt - 1) x0 = a.W - C::K;
    else if (xt == n_xt - 2) x0 = min(x0, a.W - 2 * C::K);
    const int y_begin = (int)((unsigned long long)a.H * pre / tot);
    const int y_end = (int)((unsigned long long)a.H * (pre + bs.own) / tot);
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
    const long m_max = a.H / (USV_MIN_BAND_WINS * WIN) > 0 ? a.H / (USV_MIN_BAND_WINS * WIN) : 1;
    if (m > m_max) m = m_max;
    P.m = (int)m;
    const long ex = slots - NC * m;
    P.extra = (USV_EXTRA_BANDS && a.batch == 1 && ex > 0 && ex < P.n_xt &&
               a.H / (m + 1) >= USV_MIN_BAND_WINS * WIN) ? (int)ex : 0;
    const long total = NC * m + P.extra;
    if (total > 0x7FFFFFFFL) return hipErrorInvalidValue;
#ifndef USV_PAIR_GEN_G_X4
#define USV_PAIR_GEN_G_X4 4  // experiment knob: generation size x4/4 (4 = one generation per SIMD-wave slot)
#endif
    P.gen_g = (int)((4L * (cu_count() / 8)) * USV_PAIR_GEN_G_X4 / (4 * NW));
    if (P.gen_g < 1) P.gen_g = 1;
    const bool three = per_cu * NW == 12 && total > 2L * 8 * P.gen_g;
    P.weights = !three ? 0x01010101u
              : NW > 1 ? USV_PAIR_GEN_WEIGHTS_NW2
              : kPairPipe<RAD> ? USV_PAIR_GEN_WEIGHTS : USV_PAIR_GEN_WEIGHTS_UNPIPED;
    dim3 grid((unsigned)total), block(NW * 64);
    hipLaunchKernelGGL((sad_pair_kernel<RAD, NW>), grid, block, 0, s, a.L, a.R, a.disp, a.dist, a, P);
    return hipGetLastError();
}

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
#ifndef USV_SSD_FAST
#define USV_SSD_FAST 1  // 0: SSD always takes the tiled kernel
#endif
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
#pragma unroll
        for (int k = 0; k < C::NPOS_V / C::VEC; ++k) {
            const VT v = rb[k];
#pragma unroll
            for (int e = 0; e < C::VEC; ++e) E[k * C::VEC + e] = vget<C::VEC>(v, e);
        }
        // P[j + 1] = P[j] + (L_j - R_j)^2; H[x] is formed as soon as P[x + w] exists
        uint32_t A[NPOS + 1];
        A[0] = 0;
        auto chain_step = [&](auto jt) {
            constexpr int j = decltype(jt)::value;
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
    uint4 trq[2];
    auto tr_issue = [&](const uint32_t(&S)[K]) {
#pragma unroll
        for (int i = 0; i < K; ++i) tb[64 * i + lane] = S[i];
        asm volatile("" ::: "memory");
#pragma unroll
        for (int j = 0; j < 2; ++j) trq[j] = reinterpret_cast<const uint4*>(tb)[rdw[j]];
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
#define USV_SSD_GEN_WEIGHTS 0x41415564u  // 100, 85, 65, 65 (the two-wave paired kernel's heights; not refitted)
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
    const long m_max = a.H / (USV_MIN_BAND_WINS * WIN) > 0 ? a.H / (USV_MIN_BAND_WINS * WIN) : 1;
    if (m > m_max) m = m_max;
    P.m = (int)m;
    const long ex = slots - NC * m;
    P.extra = (USV_EXTRA_BANDS && a.batch == 1 && ex > 0 && ex < P.n_xt &&
               a.H / (m + 1) >= USV_MIN_BAND_WINS * WIN) ? (int)ex : 0;
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

#ifndef USV_PAIR
#define USV_PAIR 1  // paired-disparity kernel for D > 64 (even D, 11 <= w <= 15)
#endif
#ifndef USV_PAIR_SMALL
#define USV_PAIR_SMALL 0  // experiment: the paired kernel also for even 32 < D <= 64 and 5 <= w <= 9
#endif
bool pair_path_supported(const MatchArgs& a) {
    if (USV_PAIR_SMALL && a.D > 32 && a.D <= 64 && (a.D % 2) == 0 && a.w >= 5 && a.w <= 9) return true;
    return USV_PAIR && a.D > 64 && (a.D % 2) == 0 && a.w >= 11 && a.w <= 15;
}
template <int RAD>
hipError_t launch_pair_r(const MatchArgs& a, hipStream_t s) {
    return a.D <= 128 ? launch_pair_rn<RAD, 1>(a, s) : launch_pair_rn<RAD, 2>(a, s);
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
    const bool metric_ok = a.metric == 0 || (USV_SSD_FAST && a.metric == 1 && a.w >= 11);
    return metric_ok && a.w >= 3 && a.w <= 15 && (a.w & 1) && a.D >= 1 && a.D <= 256 &&
           (a.W % 4) == 0 && a.W >= 3 * kK && (a.pitch % 4) == 0 && (long long)a.pitch * a.H < (1LL << 31) &&
           (reinterpret_cast<uintptr_t>(a.L) % 4) == 0 &&
           (reinterpret_cast<uintptr_t>(a.R) % 4) == 0 && (a.batch <= 1 || a.pair_stride % 4 == 0);
}

hipError_t launch_fast(const MatchArgs& a, hipStream_t s) {
    if (!fast_path_supported(a)) return hipErrorInvalidValue;
    if (a.metric == 1) {
        switch ((a.w - 1) / 2) {
            case 5: return launch_ssd_r<5>(a, s);
            case 6: return launch_ssd_r<6>(a, s);
            case 7: return launch_ssd_r<7>(a, s);
            default: return hipErrorInvalidValue;
        }
    }
    if (group_path_supported(a)) return launch_group(a, s);  // usv_sad_group.hip: D <= 64, w <= 9
    if (pair_path_supported(a)) {
        switch ((a.w - 1) / 2) {
#if USV_PAIR_SMALL
            case 2: return launch_pair_r<2>(a, s);
            case 3: return launch_pair_r<3>(a, s);
            case 4: return launch_pair_r<4>(a, s);
#endif
            case 5: return launch_pair_r<5>(a, s);
            case 6: return launch_pair_r<6>(a, s);
            case 7: return launch_pair_r<7>(a, s);
            default: break;
        }
    }
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
