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

namespace usv {
// OpenCV 3.0 matchShapes(c1, c2, CONTOURS_MATCH_I1, 0) and contourArea(c, false),
// restated (OpenCV is not in the image; parity unpinned).
double matchShapesI1(const std::vector<cv::Point>& a, const std::vector<cv::Point>& b);
double contourAreaAbs(const std::vector<cv::Point>& c);
}  // namespace usv

#endif /* USV_Matching_HPP */
