// usv_ssd_mfma.hip -- SSD block match with the window's cross term on the gfx950 matrix cores
// (ssd_mfma_kernel: v_mfma_i32_16x16x64_i8; w <= 13, D a multiple of 32 up to 160).
//
// Spec: SURVEY.md §8(a) A1, SSD variant (restated in oracle/sad_oracle.c).  With a' = a - 128 and b' = b - 128
// (signed bytes, exact: a' = (int8)(a ^ 0x80)), for output pixel x, disparity d and R window centre m = x - d:
//   cost(x, d) = Σ (a - b)^2 = SA(x) + SB(m) - 2 C(m, x),
//   SA(x) = Σ a'^2, SB(m) = Σ b'^2 and C(m, x) = Σ a' b' over the w x w window (replicate border).
// SA is the same for every d of a pixel, so the argmin over d is the argmin of SB(m) - 2 C(m, x), and C is a
// matrix product over k = (window row, window column):
//   C[m][x] = Σ_k A[m][k] B[k][x],   A[m][k] = b'(row, m - r + dx),   B[k][x] = a'(row, x - r + dx).
//
// Operands come from COLUMN RECORDS: the LDS holds, per staged column, 16 bytes = the column's value in the 16
// slots of a row ring (row ρ in byte ρ & 15).  The L records hold exactly the current window's rows and zero
// elsewhere (a row is written when it enters the window and zeroed when it leaves).  A K-step of
// v_mfma_i32_16x16x64_i8 is four window columns (dx = 4 s + g for lane group g = lane >> 4) x the 16 ring slots:
// lane (i, g) of the A operand is the record of R column m_i - r + dx, lane (j, g) of B the record of L column
// x_j - r + dx -- one aligned ds_read_b128 each, the same byte order (ring slot) in both, so the k order inside a
// step is the same permutation of window rows for A and B, which the sum does not see
// (profiles/probes_r05/mfma_i8_layout_r05.txt: any consistent k order gives the product).  dx >= w reads a zero
// record.  Unaligned LDS reads are exact on gfx950 but serialise (255 vs 39 cycles per wave-instruction,
// profiles/probes_r05/lds_unaligned_r05.txt): records keep every read 16-byte aligned, and the ring needs no
// im2col copy per output row.
//
// A wave owns XT = 64 output columns (four 16-column sub-tiles t) and a band of rows.  Sub-tile t's R centres run
// over m-blocks b = t .. t + D/16 of the wave's NBM = 4 + D/16 blocks of 16 from m_lo = x0 - D; block b = t holds
// d = D + j - i (valid for j < i), block t + D/16 holds d = j - i (valid for j >= i), the blocks between are all
// valid (i: the block's m row, j: the sub-tile's x column).  16-row blocks make the two triangular edge blocks
// 2 of D/16 + 1 per sub-tile (of D/32 + 1 with the 32 x 32 x 32 instruction: 20 % of the products at D = 128
// computed for nothing, 11 % now), and the short chains (three MFMAs at w = 11) with a 4-register accumulator keep
// the kernel at 116 VGPRs, four waves per SIMD (round 5: 66.1 -> 55.2 us at config C SSD,
// profiles/probes_r05/ab_ssd_16x16_r05.txt).  Per output row:
//   * stage: the window's new row enters the R / L records (one byte per record), the row that left is zeroed;
//   * SB: V(c) = Σ b'^2 of R column c's record (four v_dot4_i32_i8), an exclusive wave prefix X of V, then
//     SB(m) = X(n + w) - X(n) for n = m - m_lo, and the key table -T(n), T(n) = (SB << 8) + 255 - n, in LDS;
//   * B operands for the four sub-tiles and every K-step; per m-block the A operands of its K-steps, the MFMAs of
//     the sub-tiles it serves and the epilogue: -key = 512 C - T(n) (one v_lshl_add_u32 per product, the MFMA
//     writing VGPRs: -amdgpu-mfma-vgpr-form), invalid d masked in the two edge blocks, a running max per sub-tile;
//   * key = (SB - 2C) * 256 + 255 - n: the minimum is the smallest cost, ties -> the largest m = the smallest d
//     (the SAD kernels' rule).  Range: per pixel b'^2 - 2 a'b' lies in [-128^2, 128^2 + 2 * 128 * 127 = 48896], so
//     |(SB - 2C) * 256 + 255| < 2^31 and 512 C - T(n) stays inside an i32 for w <= 13 (169 * 48896 * 256 < 2^31).
// The C/D layout is column = lane & 15 (x), row = 4 (lane >> 4) + r (m): the reduction over m runs over the
// lane's four registers, then across the four lane groups (two swaps) at the end of the row.  Integer
// arithmetic: bit-exact with the oracle.
#include <algorithm>

#include "usv_sad_common.hpp"

namespace usv {
namespace {

typedef int mi32x4 __attribute__((ext_vector_type(4)));
typedef int mi32x16 __attribute__((ext_vector_type(16)));

template <int RAD, int DB>
struct MCfg {
    static constexpr int WIN = 2 * RAD + 1;
    static constexpr int NS = 4;              // 16-column sub-tiles per wave
    static constexpr int XT = 16 * NS;        // output columns per wave
    static constexpr int DB16 = 2 * DB;       // D / 16
    static constexpr int NBM = NS + DB16;     // 16-row m-blocks
    static constexpr int NM = 16 * NBM;       // R window centres per tile
    static constexpr int NSTEP = (WIN + 3) / 4;  // K-steps: window columns 4 s .. 4 s + 3 (columns >= w read zeros)
    static constexpr int NRC = 256;           // R records (columns rs .. rs + 255)
    static constexpr int NLC = 128;           // L records
    static constexpr int R_OFF = 0;
    static constexpr int L_OFF = R_OFF + 16 * NRC;
    static constexpr int Z_OFF = L_OFF + 16 * NLC;       // one zero record
    static constexpr int X_OFF = Z_OFF + 16;             // exclusive prefix of V (256 i32)
    static constexpr int T_OFF = X_OFF + 4 * 256;        // key tables -T(n), two rows (2 x 256 i32)
    static constexpr int M_OFF = T_OFF + 8 * 256;        // window byte masks by first ring slot (16 x 16 B)
    static constexpr int SMEM = M_OFF + 16 * 16;
    static_assert(WIN <= 13, "|SB - 2C| * 256 fits an i32 key for w <= 13");
    static_assert(NM <= 256, "key low byte: 255 - n");
    static_assert(NM + 4 * NSTEP <= NRC && XT + 4 * NSTEP <= NLC && NRC == 256 && NLC == 128, "records: 4 / 2 per lane");
};

#ifndef USV_SSD_MFMA_OCC
#define USV_SSD_MFMA_OCC 4  // waves per SIMD the kernel is compiled for (w = 13: 3, its four-step B operands need
                            // 64 VGPRs and would spill at 128)
#endif
template <int RAD, int DB>
__global__ __launch_bounds__(64, RAD >= 6 ? 3 : USV_SSD_MFMA_OCC) void ssd_mfma_kernel(const uint8_t* __restrict__ Lg, const uint8_t* __restrict__ Rg,
                                                      uint8_t* __restrict__ disp, double* __restrict__ dist,
                                                      MatchArgs a, int n_xt, int bands) {
    using C = MCfg<RAD, DB>;
    constexpr int WIN = C::WIN, NS = C::NS, XT = C::XT, NBM = C::NBM, NSTEP = C::NSTEP, DB16 = C::DB16, D = 32 * DB;
    __shared__ __attribute__((aligned(16))) uint8_t smem[C::SMEM];
    const int l = threadIdx.x, j = l & 15, g = l >> 4;
    int blk = blockIdx.x;
    const int xt = blk % n_xt;
    blk /= n_xt;
    const int band = blk % bands;
    const int pair = blk / bands;
    const int x0 = min(xt * XT, a.W - XT);
    const int y_begin = (int)((long long)a.H * band / bands), y_end = (int)((long long)a.H * (band + 1) / bands);
    if (y_end <= y_begin) return;
    const uint8_t* L = Lg + (size_t)pair * a.pair_stride;
    const uint8_t* R = Rg + (size_t)pair * a.pair_stride;
    disp += (size_t)pair * a.disp_stride;
    if (dist) dist += (size_t)pair * a.dist_stride;
    const int m_lo = x0 - D;
    const int rs = m_lo - RAD, ls = x0 - RAD;  // first R / L record's column
    const __amdgpu_buffer_rsrc_t rsrcL =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(L), (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsrcR =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(R), (short)0, 0x7FFFFFFF, 0x00020000);

    // every record starts empty (zero); the zero record; the window masks (the distance table is read from
    // global memory: 2 KB less LDS per workgroup lets four one-wave workgroups per SIMD fit)
    for (int i = l; i < (C::X_OFF) / 16; i += 64) reinterpret_cast<mi32x4*>(smem)[i] = mi32x4{0, 0, 0, 0};
    {  // mask f: bytes of ring slots f .. f + w - 1 (mod 16)
        const int f = l >> 2, q = l & 3;
        uint32_t m = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (((4 * q + e - f) & 15) < WIN) m |= 0xFFu << (8 * e);
        reinterpret_cast<uint32_t*>(smem + C::M_OFF)[l] = m;
    }
    // LDS hand-offs between lanes of the one wave: its LDS operations execute in program order, and a
    // wave_barrier (no instruction) keeps the compiler from moving a read of another lane's store above it
    __builtin_amdgcn_wave_barrier();

    // a row's staged bytes, lane l: R columns rs + l + 64 q (q < 4; records l + 64 q), L columns ls + l + 64 q
    // (q < 2), clamped to the image (replicate border).  Strided records keep the byte stores of one instruction
    // on 8 banks per 32 lanes (4-way) where records 4l .. 4l+3 per lane would put them on 2.
    const int Wm1 = a.W - 1;
    auto row_base = [&](int rho) { return (uint32_t)(min(max(rho, 0), a.H - 1) * a.pitch); };
    auto load_r = [&](int rho, uint32_t (&v)[4]) {
        const uint32_t base = row_base(rho);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            v[q] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rsrcR, base + (uint32_t)min(max(rs + l + 64 * q, 0), Wm1), 0, 0);
    };
    auto load_l = [&](int rho, uint32_t (&v)[2]) {
        const uint32_t base = row_base(rho);
#pragma unroll
        for (int q = 0; q < 2; ++q)
            v[q] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rsrcL, base + (uint32_t)min(max(ls + l + 64 * q, 0), Wm1), 0, 0);
    };
    // a row's bytes (XOR 0x80: signed) into ring slot rho & 15 of the lane's records.  The L records hold exactly
    // the current window (0x80 clears the slot of a row that left): every B operand is then zero outside it.  The R
    // records may run one row ahead (the next window's new row): A meets zero B bytes there, and SB masks slots.
    auto put_r = [&](int rho, const uint32_t (&v)[4]) {
#pragma unroll
        for (int q = 0; q < 4; ++q) smem[C::R_OFF + 16 * (l + 64 * q) + (rho & 15)] = (uint8_t)(v[q] ^ 0x80u);
    };
    auto put_l = [&](int rho, const uint32_t (&v)[2]) {
#pragma unroll
        for (int q = 0; q < 2; ++q) smem[C::L_OFF + 16 * (l + 64 * q) + (rho & 15)] = (uint8_t)(v[q] ^ 0x80u);
    };
    const uint32_t kClearL[2] = {0x80u, 0x80u};
    // -T(n) of output row yy into table yy & 1: V(c) = Σ b'^2 over yy's window rows of R record c (masked dot4),
    // X = its exclusive prefix (a DPP wave scan), SB(m) = X(n + w) - X(n)
    auto make_table = [&](int yy) {
        const mi32x4 mk = reinterpret_cast<const mi32x4*>(smem + C::M_OFF)[(yy - RAD) & 15];
        const mi32x4* rec = reinterpret_cast<const mi32x4*>(smem + C::R_OFF);
        int v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const mi32x4 rc = rec[4 * l + e];
            int acc = 0;
            acc = __builtin_amdgcn_sdot4(rc.x & mk.x, rc.x, acc, false);
            acc = __builtin_amdgcn_sdot4(rc.y & mk.y, rc.y, acc, false);
            acc = __builtin_amdgcn_sdot4(rc.z & mk.z, rc.z, acc, false);
            acc = __builtin_amdgcn_sdot4(rc.w & mk.w, rc.w, acc, false);
            v[e] = acc;
        }
        const int p1 = v[0] + v[1], p2 = p1 + v[2], tot = p2 + v[3];
        // inclusive scan of the lane totals: row_shr 1, 2, 4, 8 inside each 16-lane row, then row_bcast 15 / 31
        int incl = tot;
        incl += __builtin_amdgcn_update_dpp(0, incl, 0x111, 0xF, 0xF, true);
        incl += __builtin_amdgcn_update_dpp(0, incl, 0x112, 0xF, 0xF, true);
        incl += __builtin_amdgcn_update_dpp(0, incl, 0x114, 0xF, 0xF, true);
        incl += __builtin_amdgcn_update_dpp(0, incl, 0x118, 0xF, 0xF, true);
        incl += __builtin_amdgcn_update_dpp(0, incl, 0x142, 0xA, 0xF, false);
        incl += __builtin_amdgcn_update_dpp(0, incl, 0x143, 0xC, 0xF, false);
        const int ex = incl - tot;
        reinterpret_cast<mi32x4*>(smem + C::X_OFF)[l] = mi32x4{ex, ex + v[0], ex + p1, ex + p2};
        __builtin_amdgcn_wave_barrier();  // X is read at other lanes' offsets
        const int* X = reinterpret_cast<const int*>(smem + C::X_OFF);
        int* T = reinterpret_cast<int*>(smem + C::T_OFF + 1024 * (yy & 1));
        int xa[(C::NM + 63) / 64], xb[(C::NM + 63) / 64];
#pragma unroll
        for (int q = 0; q < (C::NM + 63) / 64; ++q)
            if (l + 64 * q < C::NM) {
                xa[q] = X[l + 64 * q];
                xb[q] = X[l + 64 * q + WIN];
            }
#pragma unroll
        for (int q = 0; q < (C::NM + 63) / 64; ++q)
            if (l + 64 * q < C::NM) T[l + 64 * q] = l + 64 * q - 255 - ((xb[q] - xa[q]) << 8);  // -T(n)
    };

    // prologue: L rows y_begin - r .. y_begin + r - 1, R rows y_begin - r .. y_begin + r, the first row's table
    for (int rho = y_begin - RAD; rho <= y_begin + RAD; ++rho) {
        uint32_t vr[4];
        load_r(rho, vr);
        put_r(rho, vr);
        if (rho < y_begin + RAD) {
            uint32_t vl[2];
            load_l(rho, vl);
            put_l(rho, vl);
        }
    }
    __builtin_amdgcn_wave_barrier();
    make_table(y_begin);
    uint32_t pr[4], pl[2];  // loaded one row ahead: R row y + 1 + r, L row y + r
    load_r(y_begin + 1 + RAD, pr);
    load_l(y_begin + RAD, pl);
    const mi32x4* recR = reinterpret_cast<const mi32x4*>(smem + C::R_OFF);
    const mi32x4* recL = reinterpret_cast<const mi32x4*>(smem + C::L_OFF);

    // the edge blocks' valid-d lane masks, one per accumulator register r (C row 4 g + r against column j),
    // computed once: loop-invariant lane masks the selects below read from SGPRs
    bool below[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) below[r] = j < 4 * g + r;
    for (int y = y_begin; y < y_end; ++y) {
        // (the previous row's record and table reads stay above this row's record stores)
        __builtin_amdgcn_wave_barrier();
        // L: row y + r enters the window, row y - r - 1 left; R: row y + 1 + r for the next row's table
        if (y > y_begin) put_l(y - RAD - 1, kClearL);
        put_l(y + RAD, pl);
        const bool more = y + 1 < y_end;
        if (more) put_r(y + 1 + RAD, pr);
        __builtin_amdgcn_wave_barrier();  // the records are read at other lanes' offsets below
        if (more) {
            load_r(y + 2 + RAD, pr);
            load_l(y + 1 + RAD, pl);
            make_table(y + 1);  // independent of this row's MFMAs: the compiler interleaves the two
        }
        // B operands: sub-tile t, K-step s -> window column dx = 4 s + g of output column x0 + 16 t + j
        mi32x4 Bop[NS][NSTEP];
#pragma unroll
        for (int s = 0; s < NSTEP; ++s) {
            const int dx = 4 * s + g;
#pragma unroll
            for (int t = 0; t < NS; ++t)
                Bop[t][s] = dx < WIN ? recL[16 * t + j + dx] : *reinterpret_cast<const mi32x4*>(smem + C::Z_OFF);
        }
        int run[NS];  // running max of -key
#pragma unroll
        for (int t = 0; t < NS; ++t) run[t] = (int)0x80000000u;
        const int* Tt = reinterpret_cast<const int*>(smem + C::T_OFF + 1024 * (y & 1));
#pragma unroll
        for (int b = 0; b < NBM; ++b) {
            mi32x4 Aop[NSTEP];
#pragma unroll
            for (int s = 0; s < NSTEP; ++s) Aop[s] = recR[16 * b + j + 4 * s + g];
            const mi32x4 Tv = *reinterpret_cast<const mi32x4*>(Tt + 16 * b + 4 * g);  // rows 4 g .. 4 g + 3
#pragma unroll
            for (int t = 0; t < NS; ++t) {
                if (b < t || b > t + DB16) continue;
                mi32x4 acc = {0, 0, 0, 0};
#pragma unroll
                for (int s = 0; s < NSTEP; ++s) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(Aop[s], Bop[t][s], acc, 0, 0, 0);
                int k[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) k[r] = (acc[r] << 9) + Tv[r];
                if (b == t) {  // d = D + j - i: valid for j < i
#pragma unroll
                    for (int r = 0; r < 4; ++r) k[r] = below[r] ? k[r] : (int)0x80000000u;
                } else if (b == t + DB16) {  // d = j - i: valid for j >= i
#pragma unroll
                    for (int r = 0; r < 4; ++r) k[r] = below[r] ? (int)0x80000000u : k[r];
                }
                run[t] = max(max(run[t], k[0]), max(max(k[1], k[2]), k[3]));
            }
        }
        // a column's rows are spread over the four 16-lane groups: combine; lane (j, g) writes sub-tile g's column j
#pragma unroll
        for (int t = 0; t < NS; ++t) {
            run[t] = max(run[t], __shfl_xor(run[t], 16, 64));
            run[t] = max(run[t], __shfl_xor(run[t], 32, 64));
        }
        // (every select in this kernel is compiler-visible C++, not inline asm: the compiler pads the MFMA wait
        // states of its own instructions only -- tests/test_isa_lint.py checks)
        const int key = -(g == 0 ? run[0] : g == 1 ? run[1] : g == 2 ? run[2] : run[3]);
        const int d = 16 * g + j + D - 255 + (key & 0xFF);
        const int x = x0 + 16 * g + j;
        disp[(size_t)y * a.disp_pitch + x] = (uint8_t)d;
        if (dist) dist[(size_t)y * a.dist_pitch + x] = a.lut[d];
    }
}

template <int RAD, int DB>
hipError_t launch_mfma_rd(const MatchArgs& a, hipStream_t s) {
    using C = MCfg<RAD, DB>;
    const int n_xt = (a.W + C::XT - 1) / C::XT;
#ifndef USV_SSD_MFMA_WAVES
#define USV_SSD_MFMA_WAVES 32  // workgroups per CU the grid aims for (one-wave workgroups)
#endif
#ifndef USV_SSD_MFMA_MINROWS
#define USV_SSD_MFMA_MINROWS 8  // shortest band (output rows per workgroup)
#endif
    const long target = (long)cu_count() * USV_SSD_MFMA_WAVES;
    long bands = (target + (long)n_xt * a.batch - 1) / ((long)n_xt * a.batch);
    bands = std::max(1L, std::min(bands, (long)std::max(1, a.H / USV_SSD_MFMA_MINROWS)));
    const long total = (long)n_xt * bands * a.batch;
    if (total > 0x7FFFFFFFL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((ssd_mfma_kernel<RAD, DB>), dim3((unsigned)total), dim3(64), 0, s, a.L, a.R, a.disp, a.dist, a,
                       n_xt, (int)bands);
    return hipGetLastError();
}

template <int RAD>
hipError_t launch_mfma_r(const MatchArgs& a, hipStream_t s) {
    switch (a.D / 32) {
        case 1: return launch_mfma_rd<RAD, 1>(a, s);
        case 2: return launch_mfma_rd<RAD, 2>(a, s);
        case 3: return launch_mfma_rd<RAD, 3>(a, s);
        case 4: return launch_mfma_rd<RAD, 4>(a, s);
        case 5: return launch_mfma_rd<RAD, 5>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

bool ssd_mfma_supported(const MatchArgs& a) {
    // SSD, w = 3 .. 13, D = 32 .. 160 in steps of 32, at least one 64-column tile, 32-bit row offsets
    return a.metric == 1 && (a.w & 1) && a.w >= 3 && a.w <= 13 && a.D % 32 == 0 && a.D >= 32 && a.D <= 160 &&
           a.W >= 64 && (long long)a.pitch * a.H < (1LL << 31);
}

hipError_t launch_ssd_mfma(const MatchArgs& a, hipStream_t s) {
    if (!ssd_mfma_supported(a)) return hipErrorInvalidValue;
    switch ((a.w - 1) / 2) {
        case 1: return launch_mfma_r<1>(a, s);
        case 2: return launch_mfma_r<2>(a, s);
        case 3: return launch_mfma_r<3>(a, s);
        case 4: return launch_mfma_r<4>(a, s);
        case 5: return launch_mfma_r<5>(a, s);
        case 6: return launch_mfma_r<6>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace usv
