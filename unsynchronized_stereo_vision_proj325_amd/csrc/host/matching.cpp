// matching.cpp -- the reference's cross-frame / cross-camera contour matcher.
//
// Implements include/Match.hpp (P/Match.cpp:4-9) and include/Matching.hpp
// (P/Main.cpp:403-499).  GenerateMatchingList's shape score needs OpenCV 3.0
// matchShapes(CONTOURS_MATCH_I1) and contourArea; both are restated below from
// their published definitions (Green's-theorem polygon moments -> central ->
// normalised -> Hu invariants; shoelace area).  OpenCV is absent from the image,
// so this part is "parity unpinned" against OpenCV itself; it
// is bit-exact against oracle/shape_oracle.c, an independent C restatement of
// OpenCV 3.0's contourMoments / HuMoments / matchShapes I1 / contourArea that
// recomputes every pair as P/Main.cpp:403-426 does (tests/test_shape_oracle.py);
// tests/test_matching.py adds the method's invariances.  Unlike the reference,
// which recomputes the moments and four areas for every (i, j) pair
// (P/Main.cpp:413-414), the invariants are computed once per contour; the
// per-pair arithmetic on them is unchanged, so the scores are identical.
#include "Matching.hpp"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <vector>

#include "usv.h"

Match::Match(unsigned int LeftIndex, unsigned int RightIndex, double MatchValue)
    : LeftIndex(LeftIndex), RightIndex(RightIndex), MatchValue(MatchValue) {}

static_assert(sizeof(Match) == sizeof(usv_match), "Match must keep the usv_match layout");

namespace usv {
namespace {

struct HuInvariants {
    double h[7];
};

// Spatial moments of a closed polygon by Green's theorem, then central and
// normalised central moments, then the seven Hu invariants.
HuInvariants hu_of(const std::vector<cv::Point>& c) {
    HuInvariants out{};
    const size_t n = c.size();
    if (n == 0) return out;
    double a00 = 0, a10 = 0, a01 = 0, a20 = 0, a11 = 0, a02 = 0, a30 = 0, a21 = 0, a12 = 0, a03 = 0;
    double px = c[n - 1].x, py = c[n - 1].y;
    double px2 = px * px, py2 = py * py;
    for (size_t i = 0; i < n; ++i) {
        const double x = c[i].x, y = c[i].y;
        const double x2 = x * x, y2 = y * y;
        const double cross = px * y - x * py;
        const double sx = px + x, sy = py + y;
        a00 += cross;
        a10 += cross * sx;
        a01 += cross * sy;
        a20 += cross * (px * sx + x2);
        a11 += cross * (px * (sy + py) + x * (sy + y));
        a02 += cross * (py * sy + y2);
        a30 += cross * sx * (px2 + x2);
        a03 += cross * sy * (py2 + y2);
        a21 += cross * (px2 * (3 * py + y) + 2 * x * px * sy + x2 * (py + 3 * y));
        a12 += cross * (py2 * (3 * px + x) + 2 * y * py * sx + y2 * (px + 3 * x));
        px = x;
        py = y;
        px2 = x2;
        py2 = y2;
    }
    if (!(std::fabs(a00) > FLT_EPSILON)) return out;  // degenerate: all moments zero
    const double sgn = a00 > 0 ? 1.0 : -1.0;
    const double m00 = a00 * (sgn * 0.5), m10 = a10 * (sgn / 6), m01 = a01 * (sgn / 6);
    const double m20 = a20 * (sgn / 12), m11 = a11 * (sgn / 24), m02 = a02 * (sgn / 12);
    const double m30 = a30 * (sgn / 20), m21 = a21 * (sgn / 60), m12 = a12 * (sgn / 60);
    const double m03 = a03 * (sgn / 20);

    double cx = 0, cy = 0, inv_m00 = 0;
    if (std::fabs(m00) > DBL_EPSILON) {
        inv_m00 = 1. / m00;
        cx = m10 * inv_m00;
        cy = m01 * inv_m00;
    }
    const double mu20 = m20 - m10 * cx, mu11 = m11 - m10 * cy, mu02 = m02 - m01 * cy;
    const double mu30 = m30 - cx * (3 * mu20 + cx * m10);
    const double mu21 = m21 - cx * (2 * mu11 + cx * m01) - cy * mu20;
    const double mu12 = m12 - cy * (2 * mu11 + cy * m10) - cx * mu02;
    const double mu03 = m03 - cy * (3 * mu02 + cy * m01);
    const double s2 = inv_m00 * inv_m00, s3 = s2 * std::sqrt(std::fabs(inv_m00));
    const double n20 = mu20 * s2, n11 = mu11 * s2, n02 = mu02 * s2;
    const double n30 = mu30 * s3, n21 = mu21 * s3, n12 = mu12 * s3, n03 = mu03 * s3;

    double t0 = n30 + n12, t1 = n21 + n03;
    double q0 = t0 * t0, q1 = t1 * t1;
    const double n4 = 4 * n11, s = n20 + n02, d = n20 - n02;
    out.h[0] = s;
    out.h[1] = d * d + n4 * n11;
    out.h[3] = q0 + q1;
    out.h[5] = d * (q0 - q1) + n4 * t0 * t1;
    t0 *= q0 - 3 * q1;
    t1 *= 3 * q0 - q1;
    q0 = n30 - 3 * n12;
    q1 = 3 * n21 - n03;
    out.h[2] = q0 * q0 + q1 * q1;
    out.h[4] = q0 * t0 + q1 * t1;
    out.h[6] = q1 * t0 - q0 * t1;
    return out;
}

// CONTOURS_MATCH_I1: sum_i |1/m^A_i - 1/m^B_i|, m_i = sign(h_i) log10|h_i|,
// terms with |h| <= 1e-5 on either side skipped.
double i1_distance(const HuInvariants& a, const HuInvariants& b) {
    const double eps = 1.e-5;
    double result = 0;
    for (int i = 0; i < 7; ++i) {
        double ama = std::fabs(a.h[i]), amb = std::fabs(b.h[i]);
        const int sma = a.h[i] > 0 ? 1 : (a.h[i] < 0 ? -1 : 0);
        const int smb = b.h[i] > 0 ? 1 : (b.h[i] < 0 ? -1 : 0);
        if (ama > eps && amb > eps) {
            ama = 1. / (sma * std::log10(ama));
            amb = 1. / (smb * std::log10(amb));
            result += std::fabs(-ama + amb);
        }
    }
    return result;
}

}  // namespace

double matchShapesI1(const std::vector<cv::Point>& a, const std::vector<cv::Point>& b) {
    return i1_distance(hu_of(a), hu_of(b));
}

double contourAreaAbs(const std::vector<cv::Point>& c) {
    const size_t n = c.size();
    if (n == 0) return 0.;
    double a00 = 0;
    float px = (float)c[n - 1].x, py = (float)c[n - 1].y;
    for (size_t i = 0; i < n; ++i) {
        const float x = (float)c[i].x, y = (float)c[i].y;
        a00 += (double)px * y - (double)py * x;
        px = x;
        py = y;
    }
    return std::fabs(a00 * 0.5);
}

}  // namespace usv

void GenerateMatchingList(std::vector<std::vector<cv::Point> > UsefulContoursL,
                          std::vector<std::vector<cv::Point> > UsefulContoursR,
                          std::vector<Match>& Matcher) {
    if (UsefulContoursL.empty() || UsefulContoursR.empty()) return;  // P/Main.cpp:405
    std::vector<usv::HuInvariants> huL, huR;
    std::vector<double> areaL, areaR;
    for (const auto& c : UsefulContoursL) {
        huL.push_back(usv::hu_of(c));
        areaL.push_back(usv::contourAreaAbs(c));
    }
    for (const auto& c : UsefulContoursR) {
        huR.push_back(usv::hu_of(c));
        areaR.push_back(usv::contourAreaAbs(c));
    }
    for (unsigned i = 0; i < UsefulContoursL.size(); ++i) {
        for (unsigned j = 0; j < UsefulContoursR.size(); ++j) {
            double v = usv::i1_distance(huL[i], huR[j]);
            v += std::fabs((areaL[i] - areaR[j]) / ((areaL[i] + areaR[j]) / 2));
            if (v < 0.75) Matcher.push_back({i, j, v});  // NaN (two zero areas) is dropped
        }
    }
}

void ResolveMatchList(std::vector<Match> Matcher, std::vector<Match>& TentativeMatch) {
    // One greedy pass (the reference's outer retry loop sees an emptied input,
    // P/Main.cpp:475).  A candidate replaces every conflicting tentative entry
    // it beats; if it beats none it is appended even when a better conflicting
    // entry exists, so duplicates can appear.
    //
    // The reference scans the whole tentative list for every candidate (O(n |T|),
    // "VERy slow", P/Main.cpp:1079).  Here the entries sharing an index are found
    // through per-index position lists instead: each entry's decision depends only
    // on itself and the candidate, so visiting the sharing positions in any order
    // gives the same list.  Lists are lazy (a replaced entry stays in its old
    // index's list and is skipped there when its index no longer matches).
    TentativeMatch.clear();
    if (Matcher.empty()) return;
    unsigned maxL = 0, maxR = 0;
    for (const Match& m : Matcher) {
        maxL = std::max(maxL, m.LeftIndex);
        maxR = std::max(maxR, m.RightIndex);
    }
    if (maxL >= (1u << 24) || maxR >= (1u << 24)) {  // sparse indices: the reference's scan
        for (const Match& m : Matcher) {
            bool replaced = false;
            for (Match& t : TentativeMatch) {
                const bool shares = t.LeftIndex == m.LeftIndex || t.RightIndex == m.RightIndex;
                if (shares && t.MatchValue > m.MatchValue) {
                    t = m;
                    replaced = true;
                }
            }
            if (!replaced) TentativeMatch.push_back(m);
        }
        return;
    }
    std::vector<std::vector<unsigned>> byL(maxL + 1), byR(maxR + 1);
    std::vector<size_t> seen;  // visit stamp per position (a position may sit in both lists)
    TentativeMatch.reserve(Matcher.size());
    size_t stamp = 0;
    for (const Match& m : Matcher) {
        ++stamp;
        bool replaced = false;
        auto visit = [&](std::vector<unsigned>& list, bool left) {
            // entries appended during this visit (the candidate's own) are past `n`; index access,
            // since an append may reallocate the list
            const size_t n = list.size();
            for (size_t i = 0; i < n; ++i) {
                const unsigned p = list[i];
                if (seen[p] == stamp) continue;
                Match& t = TentativeMatch[p];
                if ((left ? t.LeftIndex : t.RightIndex) != (left ? m.LeftIndex : m.RightIndex)) continue;  // stale
                seen[p] = stamp;
                if (t.MatchValue > m.MatchValue) {
                    t = m;
                    replaced = true;
                    byL[m.LeftIndex].push_back(p);  // may duplicate: the stamp skips the second visit
                    byR[m.RightIndex].push_back(p);
                }
            }
        };
        visit(byL[m.LeftIndex], true);
        visit(byR[m.RightIndex], false);
        if (!replaced) {
            const unsigned p = (unsigned)TentativeMatch.size();
            TentativeMatch.push_back(m);
            seen.push_back(0);
            byL[m.LeftIndex].push_back(p);
            byR[m.RightIndex].push_back(p);
        }
    }
}

void IDMatcher(std::vector<Match> InterframeMatchIndexes, std::vector<Match> OldInterframeMatchIndexes,
               std::vector<cv::Point3i>& InterframeMatchIndexesComplete) {
    InterframeMatchIndexesComplete.clear();
    for (const Match& cur : InterframeMatchIndexes)
        for (const Match& old : OldInterframeMatchIndexes)
            if (cur.RightIndex == old.LeftIndex)
                // (Point3i)(cur, old.RightIndex) at P/Main.cpp:492 is a comma
                // expression: Point3i(Vec3i(old.RightIndex)) = (old.RightIndex, 0, 0).
                InterframeMatchIndexesComplete.push_back(cv::Point3i((int)old.RightIndex, 0, 0));
}

// ---- C ABI over the same C++ functions ------------------------------------

extern "C" usv_status usv_resolve_match_list(const usv_match* in, int n_in, usv_match* out, int* n_out) {
    if (!n_out || n_in < 0 || (n_in && (!in || !out))) return USV_ERR_INVALID_ARG;
    std::vector<Match> v;
    v.reserve(n_in);
    for (int i = 0; i < n_in; ++i) v.push_back({in[i].left_index, in[i].right_index, in[i].match_value});
    std::vector<Match> t;
    ResolveMatchList(v, t);
    for (size_t i = 0; i < t.size(); ++i) out[i] = {t[i].LeftIndex, t[i].RightIndex, t[i].MatchValue};
    *n_out = (int)t.size();
    return USV_OK;
}

extern "C" usv_status usv_id_matcher(const usv_match* cur, int n_cur, const usv_match* old, int n_old,
                                     int* out_xyz, int* n_out) {
    if (!n_out || n_cur < 0 || n_old < 0 || (n_cur && !cur) || (n_old && !old)) return USV_ERR_INVALID_ARG;
    std::vector<Match> a, b;
    for (int i = 0; i < n_cur; ++i) a.push_back({cur[i].left_index, cur[i].right_index, cur[i].match_value});
    for (int i = 0; i < n_old; ++i) b.push_back({old[i].left_index, old[i].right_index, old[i].match_value});
    std::vector<cv::Point3i> o;
    IDMatcher(a, b, o);
    if (!o.empty() && !out_xyz) return USV_ERR_INVALID_ARG;
    for (size_t i = 0; i < o.size(); ++i) {
        out_xyz[3 * i] = o[i].x;
        out_xyz[3 * i + 1] = o[i].y;
        out_xyz[3 * i + 2] = o[i].z;
    }
    *n_out = (int)o.size();
    return USV_OK;
}

namespace {
std::vector<std::vector<cv::Point> > contours_of(const int* pts, const int* off, int n) {
    std::vector<std::vector<cv::Point> > cs(n);
    for (int i = 0; i < n; ++i)
        for (int k = off[i]; k < off[i + 1]; ++k) cs[i].push_back(cv::Point(pts[2 * k], pts[2 * k + 1]));
    return cs;
}
}  // namespace

extern "C" usv_status usv_generate_matching_list(const int* pts_a, const int* off_a, int n_a,
                                                 const int* pts_b, const int* off_b, int n_b,
                                                 usv_match* out, int cap, int* n_out) {
    if (!n_out || n_a < 0 || n_b < 0 || (n_a && (!off_a || (off_a[n_a] && !pts_a))) ||
        (n_b && (!off_b || (off_b[n_b] && !pts_b))) || cap < 0 || (cap && !out))
        return USV_ERR_INVALID_ARG;
    std::vector<Match> m;
    GenerateMatchingList(contours_of(pts_a, off_a, n_a), contours_of(pts_b, off_b, n_b), m);
    if ((int)m.size() > cap) return USV_ERR_INVALID_ARG;
    for (size_t i = 0; i < m.size(); ++i) out[i] = {m[i].LeftIndex, m[i].RightIndex, m[i].MatchValue};
    *n_out = (int)m.size();
    return USV_OK;
}

extern "C" double usv_match_shapes_i1(const int* pts_a, int n_a, const int* pts_b, int n_b) {
    std::vector<cv::Point> a, b;
    for (int i = 0; i < n_a; ++i) a.push_back(cv::Point(pts_a[2 * i], pts_a[2 * i + 1]));
    for (int i = 0; i < n_b; ++i) b.push_back(cv::Point(pts_b[2 * i], pts_b[2 * i + 1]));
    return usv::matchShapesI1(a, b);
}

extern "C" double usv_contour_area(const int* pts, int n) {
    std::vector<cv::Point> c;
    for (int i = 0; i < n; ++i) c.push_back(cv::Point(pts[2 * i], pts[2 * i + 1]));
    return usv::contourAreaAbs(c);
}
