// usv_sad_common.hpp -- device helpers shared by the block-match kernels of usv_sad_fast.hip (column-
// paired, sad_fast_kernel), usv_sad_pair.hip (paired disparities, sad_pair_kernel) and usv_sad_ssd.hip
// (ssd_fast_kernel): tile configuration, border maps of the L row segment, DPP / LDS argmin
// reductions, LDS-DMA and scalar-load helpers, the band plan.  Internal to libusv.so; every helper is
// in an anonymous namespace, so each translation unit has its own copy.
#pragma once
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
#ifndef USV_WGTIME
#define USV_WGTIME 0  // diagnostic build: per-workgroup start/end s_memrealtime + hardware id (scripts/wgtime.py)
#endif
constexpr int kFastOcc = 3;  // target waves per SIMD (__launch_bounds__) of sad_fast_kernel for r <= 6: <= 168 VGPRs

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
    // Row buffers per wave: an 8-row ring (slot t & 7), four waves a 4-row one.
    static constexpr int NB = NW <= 2 ? 8 : 4;
    static constexpr int PD = NB - 1;            // rows in flight ahead of the one computed
    static constexpr int KRB = WIN;              // output rows per cross-wave combine
    static constexpr int LOFF = (4 - (RAD & 3)) & 3;  // (x0 - RAD) mod 4, x0 % 4 == 0
    // LDS carve (u32 words, every region 16-byte aligned)
    static constexpr int RBUF_OFF = 0;
    // per-wave argmin transpose buffer: 16 pixels x 64 keys (RED_LDS)
    static constexpr int TB_OFF = RBUF_OFF + NW * NB * NRS;
    // argmin transpose through LDS (the other shape: permlane / DPP rounds); r = 6 with two waves sits at the
    // 168-VGPR limit, where the DPP rounds need fewer registers
    static constexpr bool RED_LDS = !(RAD == 6 && NW == 2);
    // packed transpose: the 8 packed (cost_x, cost_x+8) words instead of 16 keys (half the ds_write), keys
    // rebuilt by v_perm from per-lane d tables (+8 VGPRs; r = 6 with one wave would spill)
    static constexpr bool RED_PACKED = RED_LDS && !(RAD == 6 && NW == 1);
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
template <int RAD, int EDGE>
constexpr bool kLWholeWord = EDGE == 0 /* kInterior */ && RAD <= 5;

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

// LDS address of a shared-memory pointer (the M0 / DS address operand of the inline-asm LDS ops below).
__device__ __forceinline__ uint32_t lds_addr(const uint32_t* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t*)p;
}

// A whole row's R DMAs under ONE M0 write (LDS-DMA of one byte per lane, zero-extended to a dword at
// M0 + 4 lane; inline asm so the compiler cannot precompute 64-bit per-lane addresses for the look-ahead rows --
// it hoisted and spilled them -- and every vmcnt wait is explicit; GFX9 needs one wait state between an SALU
// write of M0 and an LDS-DMA that reads it, which the compiler's hazard recognizer does not see inside asm:
// s_nop 0).  The immediate offset of an LDS-DMA
// moves the LDS destination and the global address alike
// (scripts/probes/glds_offset_probe.hip), so DMA q uses offset:256 q and a
// per-lane offset pre-biased by -256 q; the row pointer carries a -kDmaBias
// bias so that every per-lane offset stays non-negative (the 32-bit VGPR
// offset is zero-extended).  Saves the M0 write + wait state of every DMA but
// the first.
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
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// The 2 KB distance table into LDS by two 16-byte-per-lane LDS-DMAs, issued ahead of a band loop's row
// prologue: vector-memory ops retire in order, so the first row's counted DMA wait also retires them, and
// nothing waits on the table's own round trip (a register load + ds_write + barrier waited vmcnt(0)).
// Every wave of a workgroup stages the whole table (identical bytes): no barrier before its first use.
// N = 1: the first 128 entries only (a kernel whose disparities are all < 128: 1 KB less LDS).
template <int N = 2>
__device__ __forceinline__ void lut_dma(const double* lut, uint32_t* lds, int lane) {
    static_assert(N == 1 || N == 2, "one or two 1 KB halves");
    if constexpr (N == 2)
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %2\n\t"
                     "global_load_lds_dwordx4 %0, %2 offset:1024"
                     :: "v"((uint32_t)lane * 16u), "s"(lds_addr(lds)), "s"(lut) : "memory", "m0");
    else
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %2"
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
// dma_row_buf with the LDS destination at a compile-time offset from an SGPR base: M0 = base + OFF in
// one s_add (the static row ring's slot offsets are constants).
template <int NQ, uint32_t OFF>
__device__ __forceinline__ void dma_row_buf_at(su4 rsrc, uint32_t soff, const uint32_t (&vo)[NQ], uint32_t base) {
    static_assert(NQ >= 1 && NQ <= 5, "1..5 DMAs per row");
    if constexpr (NQ == 1)
        asm volatile("s_add_u32 m0, %1, %4\n\ts_nop 0\n\tbuffer_load_ubyte %0, %2, %3 offen lds"
                     :: "v"(vo[0]), "s"(base), "s"(rsrc), "s"(soff), "n"(OFF) : "memory", "m0", "scc");
    else if constexpr (NQ == 2)
        asm volatile("s_add_u32 m0, %2, %5\n\ts_nop 0\n\tbuffer_load_ubyte %0, %3, %4 offen lds\n\t"
                     "buffer_load_ubyte %1, %3, %4 offen offset:256 lds"
                     :: "v"(vo[0]), "v"(vo[1]), "s"(base), "s"(rsrc), "s"(soff), "n"(OFF) : "memory", "m0", "scc");
    else if constexpr (NQ == 3)
        asm volatile("s_add_u32 m0, %3, %6\n\ts_nop 0\n\tbuffer_load_ubyte %0, %4, %5 offen lds\n\t"
                     "buffer_load_ubyte %1, %4, %5 offen offset:256 lds\n\t"
                     "buffer_load_ubyte %2, %4, %5 offen offset:512 lds"
                     :: "v"(vo[0]), "v"(vo[1]), "v"(vo[2]), "s"(base), "s"(rsrc), "s"(soff), "n"(OFF)
                     : "memory", "m0", "scc");
    else if constexpr (NQ == 4)
        asm volatile("s_add_u32 m0, %4, %7\n\ts_nop 0\n\tbuffer_load_ubyte %0, %5, %6 offen lds\n\t"
                     "buffer_load_ubyte %1, %5, %6 offen offset:256 lds\n\t"
                     "buffer_load_ubyte %2, %5, %6 offen offset:512 lds\n\t"
                     "buffer_load_ubyte %3, %5, %6 offen offset:768 lds"
                     :: "v"(vo[0]), "v"(vo[1]), "v"(vo[2]), "v"(vo[3]), "s"(base), "s"(rsrc), "s"(soff), "n"(OFF)
                     : "memory", "m0", "scc");
    else
        asm volatile("s_add_u32 m0, %5, %8\n\ts_nop 0\n\tbuffer_load_ubyte %0, %6, %7 offen lds\n\t"
                     "buffer_load_ubyte %1, %6, %7 offen offset:256 lds\n\t"
                     "buffer_load_ubyte %2, %6, %7 offen offset:512 lds\n\t"
                     "buffer_load_ubyte %3, %6, %7 offen offset:768 lds\n\t"
                     "buffer_load_ubyte %4, %6, %7 offen offset:1024 lds"
                     :: "v"(vo[0]), "v"(vo[1]), "v"(vo[2]), "v"(vo[3]), "v"(vo[4]), "s"(base), "s"(rsrc), "s"(soff),
                        "n"(OFF) : "memory", "m0", "scc");
}
// dma_row_buf_at (three DMAs) with the row offset clamp min(raw, last) computed between the M0 write and the
// first DMA: the clamp is the one wait state the M0 write needs, so no s_nop (USV_PAIR_M0REUSE).
template <uint32_t OFF>
__device__ __forceinline__ void dma_row3_at_min(su4 rsrc, int raw, int last, const uint32_t (&vo)[3], uint32_t base) {
    int soff;
    asm volatile("s_add_u32 m0, %4, %8\n\ts_min_i32 %0, %6, %7\n\tbuffer_load_ubyte %1, %5, %0 offen lds\n\t"
                 "buffer_load_ubyte %2, %5, %0 offen offset:256 lds\n\t"
                 "buffer_load_ubyte %3, %5, %0 offen offset:512 lds"
                 : "=&s"(soff)
                 : "v"(vo[0]), "v"(vo[1]), "v"(vo[2]), "s"(base), "s"(rsrc), "s"(raw), "s"(last), "n"(OFF)
                 : "memory", "m0", "scc");
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

// Band decomposition of one launch (launch_rn): m bands per column, their
// heights weighted by dispatch generation (see sad_fast_kernel).
struct BandPlan {
    int n_xt;      // x-tiles per pair
    int m;         // bands per column (pair, x-tile)
    int gen_g;     // workgroups per dispatch generation per XCD (4 SIMDs x CUs per XCD / waves per WG)
    unsigned weights;  // byte g: relative band height of generation g (g >= 3 use byte 3)
    int extra;     // single pair only: x-tiles 0..extra-1 carry m + 1 bands (fills every resident slot)
};

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

// shortest band, in windows (w rows): the ring warm-up costs w rows per band.  Binds only on small frames
// (1080p, D = 128 has 12-13 bands of ~85 rows); interleaved A/B at 640x480 w7 D64: 1 / 2 / 3 / 4 windows =
// 29.5 / 22.2 / 20.5 / 22.5 us, at 320x240 w5 D32: 2 / 3 / 4 = 16.8 / 15.3 / 16.4 us
// (profiles/probes/ab_minband_small_r01.txt, ab_weights_minband_r01.txt).  With one pair some x-tiles take an
// extra band so that the grid fills every resident slot.
constexpr int kMinBandWins = 3;

}  // namespace
}  // namespace usv
