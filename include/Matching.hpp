// Matching.hpp -- the cross-frame / cross-camera contour matcher.
//
// In the reference these three functions are defined inside P/Main.cpp
// (lines 403, 432, 483) and declared in no header, so an unchanged Main.cpp
// keeps its own copies; a caller that wants ours includes
// this header instead.  Signatures are identical to the reference's.
#ifndef USV_Matching_HPP
#define USV_Matching_HPP

#include "Match.hpp"
#include "cv_compat.hpp"
#include <vector>

// P/Main.cpp:403-426: score every (i, j) contour pair with Hu-moment I1
// (OpenCV matchShapes method 1) + |area ratio|; append (i, j, v) when v < 0.75.
void GenerateMatchingList(std::vector<std::vector<cv::Point> > UsefulContoursL,
                          std::vector<std::vector<cv::Point> > UsefulContoursR,
                          std::vector<Match>& Matcher);

// P/Main.cpp:432-477: greedy one-pass conflict resolution (may emit duplicates).
void ResolveMatchList(std::vector<Match> Matcher, std::vector<Match>& TentativeMatch);

// P/Main.cpp:483-499: join current and old interframe matches into triples
// ((Point3i)(a, b) comma-operator semantics: (old.RightIndex, 0, 0)).
void IDMatcher(std::vector<Match> InterframeMatchIndexes,
               std::vector<Match> OldInterframeMatchIndexes,
               std::vector<cv::Point3i>& InterframeMatchIndexesComplete);

// P/Main.cpp:1120-1143 (Canny copy P/Main.cpp:628-654): for each tentative
// match, the centre of minAreaRect(Contours[LeftIndex]) -- the four
// RotatedRect corners summed as Point2f and divided by 4 -- appended to
// VectorCenter_point.  Not a function in the reference (inline in its thread
// body); named here so a caller can reach it.
void MatchCentroids(const std::vector<std::vector<cv::Point> >& Contours,
                    const std::vector<Match>& TentativeMatch,
                    std::vector<cv::Point2f>& VectorCenter_point);

namespace usv {
// OpenCV 3.0 convexHull(pts, hull, clockwise=true) and minAreaRect (Sklansky +
// rotating calipers), restated; parity unpinned.
std::vector<cv::Point> convexHullCW(const std::vector<cv::Point>& pts);
cv::RotatedRect minAreaRect(const std::vector<cv::Point>& points);
cv::Point2f rectCentre(const cv::RotatedRect& r);
// OpenCV 3.0 matchShapes(c1, c2, CONTOURS_MATCH_I1, 0) and contourArea(c, false),
// restated (OpenCV is not in the image; parity unpinned).
double matchShapesI1(const std::vector<cv::Point>& a, const std::vector<cv::Point>& b);
double contourAreaAbs(const std::vector<cv::Point>& c);
}  // namespace usv

#endif /* USV_Matching_HPP */
