// usv_band.hpp -- the band plan's per-workgroup row span, shared by the block-match kernels
// (usv_sad_fast.hip, usv_sad_group.hip); internal to libusv.so.
//
// A launch cuts every x-tile column into m (or m + 1) bands whose heights are weighted by the dispatch
// generation of the workgroup that carries them (sad_fast_kernel's comment has the model).  A
// workgroup needs the weight sum of its column's bands before its own (pre), its own weight and the
// column total.  The band-by-band form with two integer divisions per band cost m x ~80 SALU per wave
// before any row work (5 000 SALU per wave at 640 x 480 with 68 bands, issued through the CU's shared
// scalar unit).  Here the tile index and its position in the XCD run are walked incrementally (a few
// divisions once, none per band) and the generation is three compares; equal heights take a closed
// form.  The same integers as before, so the same rows.
#pragma once
#include <hip/hip_runtime.h>

namespace usv {

struct BandSpan {
    unsigned pre, own, tot;
};

// Band s of the column whose band sb is carried by tile t(sb) = t0 + sb * nxt (t0 = pair * per_pair +
// col_xt); tiles run XCD-contiguously: runs of long_run tiles up to tile `split`, then runs of `base`.
// Generation of a tile = min(position in its run / gen_g, 3), weight = byte g of weights.
__host__ __device__ __forceinline__ BandSpan band_span(unsigned pair, unsigned per_pair, unsigned nxt, unsigned col_xt,
                                              unsigned s, unsigned m_col, unsigned base, unsigned long_run,
                                              unsigned split, unsigned gen_g, unsigned weights) {
    if (weights == 0x01010101u) return BandSpan{s, 1u, m_col};  // equal heights
    unsigned t = pair * per_pair + col_xt;
    unsigned jl = t % long_run;                  // t % long_run while t < split
    const unsigned nl = nxt % long_run;
    const unsigned nb = base ? nxt % base : 0u;  // (base == 0: every tile lies before split)
    unsigned jb = 0;
    bool in_b = false;
    unsigned pre = 0, own = 0, tot = 0;
    for (unsigned sb = 0; sb < m_col; ++sb) {
        if (!in_b && t >= split) {  // first band past the long runs
            in_b = true;
            jb = (t - split) % base;
        }
        const unsigned j = in_b ? jb : jl;
        const unsigned g = (j >= gen_g ? 1u : 0u) + (j >= 2 * gen_g ? 1u : 0u) + (j >= 3 * gen_g ? 1u : 0u);
        const unsigned wgt = (weights >> (8 * g)) & 0xFFu;
        pre += sb < s ? wgt : 0u;
        own += sb == s ? wgt : 0u;
        tot += wgt;
        t += nxt;
        jl += nl;
        jl = jl >= long_run ? jl - long_run : jl;
        jb += nb;
        jb = jb >= base ? jb - base : jb;
    }
    return BandSpan{pre, own, tot};
}

}  // namespace usv
