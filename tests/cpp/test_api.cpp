// Drives the drop-in C++ API the way the reference's Main.cpp does
// (P/Main.cpp:418 brace-init push_back, 1058-1059, 1078-1080, 1115-1117,
// 1238-1247), against include/*.hpp and libusv.so.  Prints one JSON object per
// line; tests/test_cpp_api.py checks the values against the oracle.
#include <cmath>
#include <cstdio>
#include <vector>

#include "DistanceCalculator.hpp"
#include "Match.hpp"
#include "Matching.hpp"

// JSON number (Python's json accepts Infinity / NaN)
static void pnum(const char* sep, double v) {
    if (std::isnan(v)) printf("%sNaN", sep);
    else if (std::isinf(v)) printf("%s%sInfinity", sep, v < 0 ? "-" : "");
    else printf("%s%.17g", sep, v);
}

static void print_matches(const char* tag, const std::vector<Match>& v) {
    printf("{\"%s\": [", tag);
    for (size_t i = 0; i < v.size(); ++i)
        printf("%s[%u, %u, %.17g]", i ? ", " : "", v[i].LeftIndex, v[i].RightIndex, v[i].MatchValue);
    printf("]}\n");
}

int main() {
    // ---- ResolveMatchList / IDMatcher, reference call pattern ----
    std::vector<Match> Matcher;
    Matcher.push_back({0, 0, 0.5});
    Matcher.push_back({1, 0, 0.3});
    Matcher.push_back({0, 1, 0.2});
    Matcher.push_back({1, 1, 0.1});
    std::vector<Match> TentativeMatch;
    ResolveMatchList(Matcher, TentativeMatch);
    print_matches("resolve", TentativeMatch);

    std::vector<Match> cur = {{0, 2, 0.0}, {1, 3, 0.0}}, old = {{2, 7, 0.0}, {3, 9, 0.0}};
    std::vector<Point3i> complete;
    IDMatcher(cur, old, complete);
    printf("{\"idmatcher\": [");
    for (size_t i = 0; i < complete.size(); ++i)
        printf("%s[%d, %d, %d]", i ? ", " : "", complete[i].x, complete[i].y, complete[i].z);
    printf("]}\n");

    // ---- MovingObjectDistanceCalculator + CooridinatePositionCalculator ----
    using std::chrono::nanoseconds;
    auto at = [](long long ns) { return steady_clock::time_point(std::chrono::duration_cast<steady_clock::duration>(nanoseconds(ns))); };
    std::vector<Point2f> thisPts = {Point2f(320.5f, 200.25f), Point2f(100.f, 50.f)};
    std::vector<Point2f> curO = {Point2f(300.f, 201.f), Point2f(80.5f, 49.f)};
    std::vector<Point2f> oldO = {Point2f(298.f, 200.f), Point2f(79.f, 48.5f)};
    std::vector<Point2f> olderO = {Point2f(297.f, 199.5f), Point2f(78.f, 48.f)};
    std::vector<Point2f> interp;
    std::vector<Point3i> tri = {Point3i(0, 0, 0), Point3i(1, 1, 1), Point3i(5, 0, 0)};
    std::vector<double> dist;
    MovingObjectDistanceCalculator(LeftCam, at(1040000000LL), thisPts, curO, oldO, olderO, interp, tri,
                                   at(1033000000LL), at(1000000000LL), at(966000000LL), dist);
    printf("{\"dist\": [");
    for (size_t i = 0; i < dist.size(); ++i) pnum(i ? ", " : "", dist[i]);
    printf("]}\n");

    // a non-empty caller vector, shorter (1 < 3 triples) and longer (5 > 3) than the triple list
    // (P/DistanceCalculator.cpp:67,75-80 read element i of the grown by-value copy)
    const std::vector<std::vector<Point2f> > interps = {
        {Point2f(250.f, 190.f)},
        {Point2f(250.f, 190.f), Point2f(60.f, 40.f), Point2f(1.f, 2.f), Point2f(3.f, 4.f), Point2f(5.f, 6.f)}};
    for (size_t k = 0; k < interps.size(); ++k) {
        std::vector<double> d2;
        MovingObjectDistanceCalculator(LeftCam, at(1040000000LL), thisPts, curO, oldO, olderO, interps[k], tri,
                                       at(1033000000LL), at(1000000000LL), at(966000000LL), d2);
        printf("{\"dist_interp%zu\": [", k);
        for (size_t i = 0; i < d2.size(); ++i) pnum(i ? ", " : "", d2[i]);
        printf("]}\n");
    }

    vector<Point3d> pos;
    CooridinatePositionCalculator(LeftCam, dist, thisPts, pos);  // CoordinateDisplay false: nothing
    printf("{\"pos_off\": %zu}\n", pos.size());
    CoordinateDisplay = true;
    CooridinatePositionCalculator(RightCam, dist, thisPts, pos);
    printf("{\"pos\": [");
    for (size_t i = 0; i < pos.size(); ++i) {
        pnum(i ? ", [" : "[", pos[i].x);
        pnum(", ", pos[i].y);
        pnum(", ", pos[i].z);
        printf("]");
    }
    printf("]}\n");
    printf("{\"deg2rad\": %.17g, \"rad2deg\": %.17g}\n", deg2rad(90.0), rad2deg(1.0));

    // ---- GenerateMatchingList (P/Main.cpp:1115-1117 pattern) ----
    std::vector<std::vector<Point> > A = {{Point(0, 0), Point(20, 0), Point(20, 20), Point(0, 20)},
                                          {Point(0, 0), Point(40, 0), Point(40, 10), Point(0, 10)}};
    std::vector<std::vector<Point> > B = {{Point(5, 5), Point(45, 5), Point(45, 15), Point(5, 15)},
                                          {Point(1, 1), Point(21, 1), Point(21, 21), Point(1, 21)}};
    std::vector<Match> M;
    GenerateMatchingList(A, B, M);
    print_matches("generate", M);
    ResolveMatchList(M, TentativeMatch);
    print_matches("generate_resolved", TentativeMatch);

    // ---- centre points of the matched contours (P/Main.cpp:1120-1143 pattern) ----
    std::vector<Point2f> VectorCenter_point;
    MatchCentroids(A, TentativeMatch, VectorCenter_point);
    printf("{\"centroids\": [");
    for (size_t i = 0; i < VectorCenter_point.size(); ++i) {
        pnum(i ? ", [" : "[", VectorCenter_point[i].x);
        pnum(", ", VectorCenter_point[i].y);
        printf("]");
    }
    printf("]}\n");
    return 0;
}
