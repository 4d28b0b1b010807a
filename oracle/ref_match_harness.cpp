// Test harness (ours) around the reference's own compiled P/Match.cpp:4-9.
// Exposes the reference constructor and the reference class layout over a C
// ABI so tests can compare them with the product's include/Match.hpp.
// Test infrastructure only (oracle/_ref); never linked into the product.
#include "Match.hpp"  // the reference header, found via -I<reference dir>
#include <cstddef>

extern "C" {
int ref_match_sizeof() { return (int)sizeof(Match); }
int ref_match_offset_left() { return (int)offsetof(Match, LeftIndex); }
int ref_match_offset_right() { return (int)offsetof(Match, RightIndex); }
int ref_match_offset_value() { return (int)offsetof(Match, MatchValue); }
// Constructs a reference Match and copies its bytes out.
void ref_match_construct(unsigned l, unsigned r, double v, unsigned char* out) {
    Match m(l, r, v);
    const unsigned char* p = reinterpret_cast<const unsigned char*>(&m);
    for (size_t i = 0; i < sizeof(Match); ++i) out[i] = p[i];
}
}
