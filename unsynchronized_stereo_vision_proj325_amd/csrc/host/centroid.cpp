// centroid.cpp -- the reference's per-match centre point.
//
// P/Main.cpp:1120-1143 (and the Canny copy at P/Main.cpp:628-654): for every
// tentative match, minAreaRect of the matched contour, its four corners via
// RotatedRect::points, summed as Point2f and divided by 4 (float), appended to
// VectorCenter_point*.  minAreaRect is OpenCV 3.0 (convexHull by Sklansky's
// scan on the x-sorted integer points, clockwise, then rotating calipers in
// float), restated here from its published algorithm: OpenCV is absent from
// the image, so this row is "parity unpinned" (SURVEY.md §8(c)); it is
// bit-exact (every float) against oracle/shape_oracle.c's independent C
// restatement (tests/test_shape_oracle.py), and tests/test_centroid.py adds
// geometric known answers and a float64 brute-force minimum rectangle.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>

#include "Matching.hpp"
#include "usv.h"

namespace usv {
namespace {

int sign_of(int64_t v) { return (v > 0) - (v < 0); }

// One monotone chain of Sklansky's scan over x-sorted points p[start..end]
// (inclusive, either direction); stack receives indices into p.  `nsign`
// rejects steps whose dy has that sign, `sign2` is the accepted turn sign.
int sklansky(const std::vector<cv::Point>& p, int start, int end, int* stack, int nsign, int sign2) {
    const int incr = end > start ? 1 : -1;
    int pprev = start, pcur = pprev + incr, pnext = pcur + incr;
    int stacksize = 3;
    if (start == end || (p[start].x == p[end].x && p[start].y == p[end].y)) {
        stack[0] = start;
        return 1;
    }
    stack[0] = pprev;
    stack[1] = pcur;
    stack[2] = pnext;
    end += incr;  // one past the end
    while (pnext != end) {
        const int cury = p[pcur].y, nexty = p[pnext].y;
        const int by = nexty - cury;
        if (sign_of(by) != nsign) {
            const int ax = p[pcur].x - p[pprev].x;
            const int bx = p[pnext].x - p[pcur].x;
            const int ay = cury - p[pprev].y;
            const int64_t convexity = (int64_t)ay * bx - (int64_t)ax * by;  // > 0: convex turn
            if (sign_of(convexity) == sign2 && (pprev != start || pcur != end)) {
                pprev = pcur;
                pcur = pnext;
                pnext += incr;
                stack[stacksize++] = pnext;
            } else if (pprev == start) {
                pcur = pnext;
                stack[1] = pcur;
                pnext += incr;
                stack[2] = pnext;
            } else {
                stack[stacksize - 2] = pnext;
                pcur = pprev;
                pprev = stack[stacksize - 4];
                stacksize--;
            }
        } else {
            pnext += incr;
            stack[stacksize - 1] = pnext;
        }
    }
    return --stacksize;
}

}  // namespace

// convexHull(points, hull, clockwise = true, returnPoints = true) for integer points.
std::vector<cv::Point> convexHullCW(const std::vector<cv::Point>& pts) {
    std::vector<cv::Point> hull;
    const int total = (int)pts.size();
    if (total == 0) return hull;
    std::vector<cv::Point> p(pts);
    std::sort(p.begin(), p.end(),
              [](const cv::Point& a, const cv::Point& b) { return a.x < b.x || (a.x == b.x && a.y < b.y); });
    int miny = 0, maxy = 0;
    for (int i = 1; i < total; ++i) {
        if (p[miny].y > p[i].y) miny = i;
        if (p[maxy].y < p[i].y) maxy = i;
    }
    if (p[0].x == p[total - 1].x && p[0].y == p[total - 1].y) {
        hull.push_back(p[0]);
        return hull;
    }
    std::vector<int> stack(total + 2);
    // upper half (clockwise: left chain forward, right chain backward)
    int* tl = stack.data();
    const int tl_n = sklansky(p, 0, maxy, tl, -1, 1);
    int* tr = tl + tl_n;
    const int tr_n = sklansky(p, total - 1, maxy, tr, -1, -1);
    for (int i = 0; i < tl_n - 1; ++i) hull.push_back(p[tl[i]]);
    for (int i = tr_n - 1; i > 0; --i) hull.push_back(p[tr[i]]);
    const int stop = tr_n > 2 ? tr[1] : tl_n > 2 ? tl[tl_n - 2] : -1;
    // lower half; clockwise swaps the two chains
    int* bl = stack.data();
    int bl_n = sklansky(p, 0, miny, bl, 1, -1);
    int* br = bl + bl_n;
    int br_n = sklansky(p, total - 1, miny, br, 1, 1);
    std::swap(bl, br);
    std::swap(bl_n, br_n);
    if (stop >= 0) {
        const int check = bl_n > 2 ? bl[1] : bl_n + br_n > 2 ? br[2 - bl_n] : -1;
        if (check == stop || (check >= 0 && p[check].x == p[stop].x && p[check].y == p[stop].y)) {
            // all points collinear: the lower part mirrors the upper one
            bl_n = std::min(bl_n, 2);
            br_n = std::min(br_n, 2);
        }
    }
    for (int i = 0; i < bl_n - 1; ++i) hull.push_back(p[bl[i]]);
    for (int i = br_n - 1; i > 0; --i) hull.push_back(p[br[i]]);
    return hull;
}

namespace {

// Rotating calipers (minimum-area mode) over a convex polygon of n > 2 float
// points.  out = {corner, edge vector 1, edge vector 2} as 6 floats.
void rotating_calipers_min_area(const cv::Point2f* pts, int n, float* out) {
    float minarea = FLT_MAX;
    int best_left = 0, best_bottom = 0;
    float best_a = 0, best_b = 0, best_w = 0, best_h = 0;
    std::vector<float> inv_len(n);
    std::vector<cv::Point2f> vect(n);
    int left = 0, bottom = 0, right = 0, top = 0;
    cv::Point2f pt0 = pts[0];
    float left_x = pt0.x, right_x = pt0.x, top_y = pt0.y, bottom_y = pt0.y;
    for (int i = 0; i < n; ++i) {
        if (pt0.x < left_x) left_x = pt0.x, left = i;
        if (pt0.x > right_x) right_x = pt0.x, right = i;
        if (pt0.y > top_y) top_y = pt0.y, top = i;
        if (pt0.y < bottom_y) bottom_y = pt0.y, bottom = i;
        const cv::Point2f pt = pts[i + 1 < n ? i + 1 : 0];
        const double dx = pt.x - pt0.x, dy = pt.y - pt0.y;
        vect[i].x = (float)dx;
        vect[i].y = (float)dy;
        inv_len[i] = (float)(1. / std::sqrt(dx * dx + dy * dy));
        pt0 = pt;
    }
    // orientation of the hull from the first non-zero cross product
    float orientation = 0;
    {
        double ax = vect[n - 1].x, ay = vect[n - 1].y;
        for (int i = 0; i < n; ++i) {
            const double bx = vect[i].x, by = vect[i].y;
            const double convexity = ax * by - ay * bx;
            if (convexity != 0) {
                orientation = convexity > 0 ? 1.f : -1.f;
                break;
            }
            ax = bx;
            ay = by;
        }
    }
    float base_a = orientation, base_b = 0;
    int seq[4] = {bottom, right, top, left};
    for (int k = 0; k < n; ++k) {
        // cosine between each caliper side and its polygon edge; rotate by the smallest angle
        const float dp[4] = {
            +base_a * vect[seq[0]].x + base_b * vect[seq[0]].y,
            -base_b * vect[seq[1]].x + base_a * vect[seq[1]].y,
            -base_a * vect[seq[2]].x - base_b * vect[seq[2]].y,
            +base_b * vect[seq[3]].x - base_a * vect[seq[3]].y,
        };
        float maxcos = dp[0] * inv_len[seq[0]];
        int main_element = 0;
        for (int i = 1; i < 4; ++i) {
            const float cosalpha = dp[i] * inv_len[seq[i]];
            if (cosalpha > maxcos) {
                main_element = i;
                maxcos = cosalpha;
            }
        }
        const int pi = seq[main_element];
        const float lead_x = vect[pi].x * inv_len[pi], lead_y = vect[pi].y * inv_len[pi];
        switch (main_element) {
            case 0: base_a = lead_x; base_b = lead_y; break;
            case 1: base_a = lead_y; base_b = -lead_x; break;
            case 2: base_a = -lead_x; base_b = -lead_y; break;
            default: base_a = -lead_y; base_b = lead_x; break;
        }
        seq[main_element] += 1;
        if (seq[main_element] == n) seq[main_element] = 0;

        float dx = pts[seq[1]].x - pts[seq[3]].x, dy = pts[seq[1]].y - pts[seq[3]].y;
        const float width = dx * base_a + dy * base_b;
        dx = pts[seq[2]].x - pts[seq[0]].x;
        dy = pts[seq[2]].y - pts[seq[0]].y;
        const float height = -dx * base_b + dy * base_a;
        const float area = width * height;
        if (area <= minarea) {
            minarea = area;
            best_left = seq[3];
            best_a = base_a;
            best_w = width;
            best_b = base_b;
            best_h = height;
            best_bottom = seq[0];
        }
    }
    // corner = intersection of the left caliper line and the bottom one
    const float A1 = best_a, B1 = best_b, A2 = -best_b, B2 = best_a;
    const float C1 = A1 * pts[best_left].x + pts[best_left].y * B1;
    const float C2 = A2 * pts[best_bottom].x + pts[best_bottom].y * B2;
    const float idet = 1.f / (A1 * B2 - A2 * B1);
    out[0] = (C1 * B2 - C2 * B1) * idet;
    out[1] = (A1 * C2 - A2 * C1) * idet;
    out[2] = A1 * best_w;
    out[3] = B1 * best_w;
    out[4] = A2 * best_h;
    out[5] = B2 * best_h;
}

}  // namespace

cv::RotatedRect minAreaRect(const std::vector<cv::Point>& points) {
    cv::RotatedRect box;
    const std::vector<cv::Point> hi = convexHullCW(points);
    const int n = (int)hi.size();
    std::vector<cv::Point2f> h(n);
    for (int i = 0; i < n; ++i) h[i] = cv::Point2f((float)hi[i].x, (float)hi[i].y);
    if (n > 2) {
        float out[6];
        rotating_calipers_min_area(h.data(), n, out);
        box.center.x = out[0] + (out[2] + out[4]) * 0.5f;
        box.center.y = out[1] + (out[3] + out[5]) * 0.5f;
        box.size.width = (float)std::sqrt((double)out[2] * out[2] + (double)out[3] * out[3]);
        box.size.height = (float)std::sqrt((double)out[4] * out[4] + (double)out[5] * out[5]);
        box.angle = (float)std::atan2((double)out[3], (double)out[2]);
    } else if (n == 2) {
        box.center.x = (h[0].x + h[1].x) * 0.5f;
        box.center.y = (h[0].y + h[1].y) * 0.5f;
        const double dx = h[1].x - h[0].x, dy = h[1].y - h[0].y;
        box.size.width = (float)std::sqrt(dx * dx + dy * dy);
        box.size.height = 0;
        box.angle = (float)std::atan2(dy, dx);
    } else if (n == 1) {
        box.center = h[0];
    }
    box.angle = (float)(box.angle * 180 / 3.14159265358979323846);
    return box;
}

cv::Point2f rectCentre(const cv::RotatedRect& r) {
    cv::Point2f pts[4];
    r.points(pts);
    cv::Point2f c(0.f, 0.f);
    for (int j = 0; j < 4; ++j) c += pts[j];
    c /= 4;  // int divisor, float arithmetic (OpenCV Point_ /= int)
    return c;
}

}  // namespace usv

void MatchCentroids(const std::vector<std::vector<cv::Point> >& Contours, const std::vector<Match>& TentativeMatch,
                    std::vector<cv::Point2f>& VectorCenter_point) {
    for (const Match& m : TentativeMatch) {
        if (m.LeftIndex >= Contours.size()) continue;  // the Canny copy's guard (P/Main.cpp:632)
        VectorCenter_point.push_back(usv::rectCentre(usv::minAreaRect(Contours[m.LeftIndex])));
    }
}

// ---- C ABI -----------------------------------------------------------------

extern "C" usv_status usv_min_area_rect(const int* pts, int n, float* out5) {
    if (n < 0 || !out5 || (n && !pts)) return USV_ERR_INVALID_ARG;
    std::vector<cv::Point> c;
    c.reserve(n);
    for (int i = 0; i < n; ++i) c.push_back(cv::Point(pts[2 * i], pts[2 * i + 1]));
    const cv::RotatedRect r = usv::minAreaRect(c);
    out5[0] = r.center.x;
    out5[1] = r.center.y;
    out5[2] = r.size.width;
    out5[3] = r.size.height;
    out5[4] = r.angle;
    return USV_OK;
}

extern "C" usv_status usv_match_centroids(const int* pts, const int* off, int n_contours, const usv_match* matches,
                                          int n_matches, float* out_xy, int* n_out) {
    if (!n_out || n_contours < 0 || n_matches < 0 || (n_contours && (!off || (off[n_contours] && !pts))) ||
        (n_matches && (!matches || !out_xy)))
        return USV_ERR_INVALID_ARG;
    std::vector<std::vector<cv::Point> > cs(n_contours);
    for (int i = 0; i < n_contours; ++i)
        for (int k = off[i]; k < off[i + 1]; ++k) cs[i].push_back(cv::Point(pts[2 * k], pts[2 * k + 1]));
    std::vector<Match> t;
    t.reserve(n_matches);
    for (int i = 0; i < n_matches; ++i) t.push_back({matches[i].left_index, matches[i].right_index, matches[i].match_value});
    std::vector<cv::Point2f> c;
    MatchCentroids(cs, t, c);
    for (size_t i = 0; i < c.size(); ++i) {
        out_xy[2 * i] = c[i].x;
        out_xy[2 * i + 1] = c[i].y;
    }
    *n_out = (int)c.size();
    return USV_OK;
}
