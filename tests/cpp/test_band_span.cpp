// Host check of csrc/usv_band.hpp band_span (the band prologue of every block-match kernel) against the
// band-by-band definition it replaced: for whole launch plans (x-tiles, bands, extra bands, batches,
// generation sizes, weights) and EVERY tile of the launch, the same (pre, own, tot) integers.
// Built with hipcc by tests/test_band_span.py; runs on the host (no GPU).
#include <cstdio>

#include "usv_band.hpp"

static usv::BandSpan reference(unsigned pair, unsigned per_pair, unsigned nxt, unsigned col_xt, unsigned s,
                               unsigned m_col, unsigned base, unsigned long_run, unsigned split, unsigned gen_g,
                               unsigned weights) {
    auto w = [&](unsigned sb) {
        const unsigned t = pair * per_pair + sb * nxt + col_xt;
        const unsigned j = t < split ? t % long_run : (t - split) % base;
        unsigned g = j / gen_g;
        g = g < 3u ? g : 3u;
        return (weights >> (8 * g)) & 0xFFu;
    };
    usv::BandSpan r{0, 0, 0};
    for (unsigned sb = 0; sb < m_col; ++sb) {
        r.pre += sb < s ? w(sb) : 0u;
        r.tot += w(sb);
    }
    r.own = w(s);
    return r;
}

int main() {
    const unsigned weights[] = {0x2D2D4664u, 0x41415564u, 0x32324B64u, 0x01010101u, 0x0A141E28u};
    const unsigned gens[] = {1, 3, 8, 32, 64, 128};
    long checked = 0, bad = 0;
    for (unsigned n_xt : {1u, 5u, 40u, 80u, 120u, 240u, 241u})
        for (unsigned m : {1u, 2u, 7u, 13u, 68u})
            for (unsigned batch : {1u, 2u, 8u})
                for (unsigned extra : {0u, 1u, 3u})
                    for (unsigned gen_g : gens)
                        for (unsigned wts : weights) {
                            if (extra >= n_xt || (extra && batch != 1)) continue;
                            const unsigned per_pair = n_xt * m, total = per_pair * batch + extra;
                            const unsigned base = total >> 3, rem = total & 7u, long_run = base + 1u,
                                           split = rem * long_run;
                            for (unsigned lin = 0; lin < total; ++lin) {
                                // the kernels' work map (sad_pair_kernel / sad_group_kernel)
                                const unsigned xcd = lin & 7u;
                                const unsigned tile = xcd * base + (xcd < rem ? xcd : rem) + (lin >> 3);
                                const bool past = tile >= per_pair * batch && extra > 0;
                                const unsigned col_xt = past ? tile - per_pair : tile % n_xt;
                                const unsigned s = past ? m : (tile / n_xt) % m;
                                const unsigned pair = past ? 0u : tile / per_pair;
                                const unsigned m_col = m + (col_xt < extra ? 1u : 0u);
                                const usv::BandSpan a = usv::band_span(pair, per_pair, n_xt, col_xt, s, m_col, base,
                                                                       long_run, split, gen_g, wts);
                                const usv::BandSpan b = reference(pair, per_pair, n_xt, col_xt, s, m_col, base,
                                                                  long_run, split, gen_g, wts);
                                ++checked;
                                if (a.pre != b.pre || a.own != b.own || a.tot != b.tot) {
                                    if (bad < 5)
                                        std::printf("mismatch n_xt %u m %u batch %u extra %u gen %u w %08x lin %u: "
                                                    "(%u %u %u) vs (%u %u %u)\n", n_xt, m, batch, extra, gen_g, wts,
                                                    lin, a.pre, a.own, a.tot, b.pre, b.own, b.tot);
                                    ++bad;
                                }
                            }
                        }
    std::printf("checked %ld bad %ld\n", checked, bad);
    return bad ? 1 : 0;
}
