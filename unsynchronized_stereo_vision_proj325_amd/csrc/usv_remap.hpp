// usv_remap.hpp -- the per-quad bilinear remap shared by the rectification
// kernels (usv_rectify.hip) and the fused rectify + HSV + histogram frame stage
// (usv_preproc.hip).  OpenCV 3.0 remap INTER_LINEAR / BORDER_CONSTANT(0) with a
// CV_16SC2 + CV_16UC1 map (P/Main.cpp:353,358), restated in
// oracle/rectify_oracle.c; internal to libusv.so.
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>


namespace usv {

struct RemapJob {
    const uint8_t* src;
    int spitch;
    const int16_t* map1;
    const uint16_t* map2;
    uint8_t* dst;
    int dpitch;
    const uint32_t* pmap = nullptr;  // packed map (remap_quad<CN, true>): one word per pixel, see below
};

// Packed map (usv_remap_pack_map): the CV_16SC2 + CV_16UC1 pair (6 B per pixel) as ONE u32 per pixel,
// for source images of at most kPackMaxSrc columns and rows:
//   bits  0..9   the fraction index (map2: (v & 31) * 32 + (u & 31))
//   bits 10..20  sx + 1,   bits 21..31  sy + 1          (sx, sy = map1's integer source point)
// A pixel none of whose four taps is inside the source (sx >= sW, sx < -1, sy >= sH or sy < -1) is
// stored as sx + 1 = sy + 1 = 2047: it decodes to (2046, 2046), which is outside every source the
// packed form accepts, so it still produces OpenCV's BORDER_CONSTANT 0.  Every other pixel decodes to
// its exact (sx, sy, fraction): remap results are bit-identical to the 6-byte map's.
constexpr int kPackMaxSrc = 2046;
__host__ __device__ __forceinline__ uint32_t pack_map_word(int sx, int sy, int f, int sW, int sH) {
    const bool any = sx < sW && sx + 1 >= 0 && sy < sH && sy + 1 >= 0;
    const uint32_t ex = any ? (uint32_t)(sx + 1) : 2047u, ey = any ? (uint32_t)(sy + 1) : 2047u;
    return ((uint32_t)f & 1023u) | (ex << 10) | (ey << 21);
}

typedef unsigned short remap_us2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t remap_dot2(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_udot2(__builtin_bit_cast(remap_us2, a), __builtin_bit_cast(remap_us2, b), c, false);
}

// q / d for a quad index q and the quads per row d (both wave-uniform d): through the f32 reciprocal when
// q < 2^24 and d >= 8 -- the f32 quotient is then within one of the true one and a single correction makes
// it exact -- instead of the ~15-instruction integer division sequence; plain division otherwise.
__device__ __forceinline__ unsigned quad_row(unsigned q, unsigned d, bool fast) {
    if (!fast) return q / d;
    unsigned y = (unsigned)((float)q * __builtin_amdgcn_rcpf((float)d));
    const int r = (int)(q - y * d);
    y = r < 0 ? y - 1u : (r >= (int)d ? y + 1u : y);
    return y;
}
__host__ __device__ __forceinline__ bool quad_row_fast(unsigned total_quads, unsigned d) {
    return total_quads < (1u << 24) && d >= 8u;
}

// Block b of a launch runs on XCD b % 8; the logical block number that gives XCD k the k-th
// contiguous run of blocks (so one output band's source rows are fetched into one L2).
__device__ __forceinline__ unsigned xcd_block(unsigned lin, unsigned total) {
    const unsigned xcd = lin & 7u, base = total >> 3, rem = total & 7u;
    return xcd * base + min(xcd, rem) + (lin >> 3);
}

// The bilinear blend of a quad from its two source rows' aligned dwords (u0, u1: NWD dwords per pixel
// starting at (sx * CN) & ~3) where bit k of `good` says pixel k's dwords are the exact ones and all
// four taps lie in the source; the other pixels are redone from j.src tap by tap, 0 outside
// (BORDER_CONSTANT).  Shared by the direct remap (remap_quad) and the LDS-tiled one (usv_rectify.hip).
template <int CN>
__device__ __forceinline__ void remap_blend(const RemapJob& j, int sW, int sH, const int (&mx)[4], const int (&my)[4],
                                            const int (&mf)[4], const uint32_t (&u0)[4][CN == 1 ? 2 : 3],
                                            const uint32_t (&u1)[4][CN == 1 ? 2 : 3], uint32_t good,
                                            uint32_t (&out)[4 * CN]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t ty = (uint32_t)mf[k] >> 5, tx = (uint32_t)mf[k] & 31u;
        // row weights as u16 pairs: (32 - tx, tx) scaled by (32 - ty) for row 0, by ty for row 1
        const uint32_t wx = (32u - tx) | (tx << 16);
        const uint32_t wr0 = wx * (32u - ty), wr1 = wx * ty;  // both halves <= 1024: no carry
        const int o = (mx[k] * CN) & 3;
        const uint32_t l0 = __builtin_amdgcn_alignbyte(u0[k][1], u0[k][0], o);  // tap bytes 0..3
        const uint32_t l1 = __builtin_amdgcn_alignbyte(u1[k][1], u1[k][0], o);
        uint32_t h0 = 0, h1 = 0;
        if constexpr (CN == 3) {
            h0 = __builtin_amdgcn_alignbyte(u0[k][2], u0[k][1], o);  // tap bytes 4..7
            h1 = __builtin_amdgcn_alignbyte(u1[k][2], u1[k][1], o);
        }
#pragma unroll
        for (int c = 0; c < CN; ++c) {
            // (left tap | right tap << 16) of each row: byte c and byte CN + c of (h:l); v_perm bytes 0-3
            // are its second operand, 4-7 its first, 0x0c gives zero
            const uint32_t sel = 0x0c000c00u | (uint32_t)c | ((uint32_t)(CN + c) << 16);
            const uint32_t p0 = __builtin_amdgcn_perm(h0, l0, sel);
            const uint32_t p1 = __builtin_amdgcn_perm(h1, l1, sel);
            out[k * CN + c] = remap_dot2(p0, wr0, remap_dot2(p1, wr1, 1u << 9)) >> 10;
        }
        if (!(good >> k & 1u)) {
            // border / clamped read: per-tap reads, 0 outside (BORDER_CONSTANT), all four outside -> 0
            const int sx = mx[k], sy = my[k];
            const bool x0ok = sx >= 0, x1ok = sx + 1 < sW, y0ok = sy >= 0, y1ok = sy + 1 < sH;
            const bool any = sx < sW && sx + 1 >= 0 && sy < sH && sy + 1 >= 0;
            const uint8_t* rp0 = j.src + (ptrdiff_t)sy * j.spitch + (ptrdiff_t)sx * CN;
            const uint8_t* rp1 = rp0 + j.spitch;
            const uint32_t w0 = wr0 & 0xFFFFu, w1 = wr0 >> 16, w2 = wr1 & 0xFFFFu, w3 = wr1 >> 16;
#pragma unroll
            for (int c = 0; c < CN; ++c) {
                const uint32_t v0 = (any && x0ok && y0ok) ? rp0[c] : 0;
                const uint32_t v1 = (any && x1ok && y0ok) ? rp0[CN + c] : 0;
                const uint32_t v2 = (any && x0ok && y1ok) ? rp1[c] : 0;
                const uint32_t v3 = (any && x1ok && y1ok) ? rp1[CN + c] : 0;
                out[k * CN + c] =
                    (__umul24(v0, w0) + __umul24(v1, w1) + __umul24(v2, w2) + __umul24(v3, w3) + (1u << 9)) >> 10;
            }
        }
    }
}

// One quad: output pixels (y, x0 .. x0 + n - 1) of job j into out[4 * CN] (channel-interleaved).
//   * Loads first: the map (one 16-B and one 8-B load when the rows are 4-pixel aligned), then for
//     every pixel the two aligned source reads (2 dwords for gray, 3 for BGR per row) at an address
//     clamped into the image, so the reads are unconditional straight-line code; a pixel whose taps
//     are not all inside the image (or whose aligned read was clamped) is redone on a per-tap path
//     that reads 0 outside.
//   * Fixed point: every weight of OpenCV's bilinear table is a multiple of 32 and the four sum to
//     32768, so (S00 w0 + S01 w1 + S10 w2 + S11 w3 + 2^14) >> 15 = (S00 a0 + ... + 2^9) >> 10 with
//     a = w / 32 <= 1024: products < 2^18, sums < 2^24 and never above 255 after the shift.  The
//     two taps of a row are one u16 pair and their weights another: two v_dot2_u32_u16 per channel.
//   * Source offsets are 32-bit (sy * pitch + byte, a 24-bit multiply: pitch < 2^24, checked by the
//     launchers) from the job's base pointer.
template <int CN, bool PK = false>
__device__ __forceinline__ void remap_quad(const RemapJob& j, int sW, int sH, int W, int y, int x0, int n,
                                           int vec_map, int vec_src, uint32_t (&out)[4 * CN]) {
    constexpr int NWD = CN == 1 ? 2 : 3;
    int mx[4], my[4], mf[4];
    const size_t mrow = (size_t)y * W + x0;
    if constexpr (PK) {  // one 16-B load for the quad's four packed words
        uint32_t w4[4];
        if (vec_map && n == 4) {
            const uint4 m = *reinterpret_cast<const uint4*>(j.pmap + mrow);
            w4[0] = m.x; w4[1] = m.y; w4[2] = m.z; w4[3] = m.w;
        } else {
            for (int k = 0; k < 4; ++k) w4[k] = j.pmap[mrow + (k < n ? k : 0)];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            mf[k] = (int)(w4[k] & 1023u);
            mx[k] = (int)((w4[k] >> 10) & 2047u) - 1;
            my[k] = (int)(w4[k] >> 21) - 1;
        }
    } else if (vec_map && n == 4) {
        const int4 a = *reinterpret_cast<const int4*>(j.map1 + 2 * mrow);
        const uint2 f = *reinterpret_cast<const uint2*>(j.map2 + mrow);
        const int w4[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            mx[k] = (int)(int16_t)(w4[k] & 0xFFFF);
            my[k] = (int)(int16_t)((unsigned)w4[k] >> 16);
        }
        mf[0] = f.x & 0xFFFF;
        mf[1] = f.x >> 16;
        mf[2] = f.y & 0xFFFF;
        mf[3] = f.y >> 16;
    } else {
        for (int k = 0; k < 4; ++k) {
            const int kk = k < n ? k : 0;
            mx[k] = j.map1[2 * (mrow + kk)];
            my[k] = j.map1[2 * (mrow + kk) + 1];
            mf[k] = j.map2[mrow + kk];
        }
    }
    const int amax = (j.spitch - 4 * NWD) & ~3;
    uint32_t u0[4][NWD], u1[4][NWD];
    uint32_t good = 0;  // bit k: the clamped read is the exact one and every tap is inside
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (!vec_src) {  // (uniform) unaligned source or short rows: every pixel takes the per-tap path
#pragma unroll
            for (int i = 0; i < NWD; ++i) u0[k][i] = u1[k][i] = 0;
            continue;
        }
        const int sx = mx[k], sy = my[k];
        const int a = (sx * CN) & ~3;
        const int ac = min(max(a, 0), amax), yc = min(max(sy, 0), sH - 2 > 0 ? sH - 2 : 0);
        const bool in = sx >= 0 && sx + 1 < sW && sy >= 0 && sy + 1 < sH && a == ac;
        good |= in ? 1u << k : 0u;
        const uint32_t r0 = __umul24((uint32_t)yc, (uint32_t)j.spitch) + (uint32_t)ac;
        const uint32_t r1 = r0 + (uint32_t)(sH > 1 ? j.spitch : 0);
        // a raw buffer over the source (stride 0, no range limit: the offsets stay inside the image): each
        // read is a 32-bit VGPR offset with the dword index in the instruction's immediate offset, instead
        // of a 64-bit address built per read
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(j.src), (short)0, (int)0xFFFFFFFF, 0x00020000);
#pragma unroll
        for (int i = 0; i < NWD; ++i) {
            u0[k][i] = __builtin_amdgcn_raw_buffer_load_b32(rs, r0 + 4u * (uint32_t)i, 0, 0);
            u1[k][i] = __builtin_amdgcn_raw_buffer_load_b32(rs, r1 + 4u * (uint32_t)i, 0, 0);
        }
    }
    remap_blend<CN>(j, sW, sH, mx, my, mf, u0, u1, good, out);
}

}  // namespace usv
