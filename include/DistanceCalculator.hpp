// DistanceCalculator.hpp -- drop-in for the reference's P/DistanceCalculator.hpp:1-50.
//
// Same declarations, macro values and namespace leaks (using namespace cv /
// std / std::chrono, P/DistanceCalculator.hpp:12-14), so the reference's
// Main.cpp compiles against it unchanged.  The implementation lives in
// libusv.so (csrc/host/distance_calculator.cpp), built with -ffp-contract=off.
#ifndef DistanceCalculator_HPP
#define DistanceCalculator_HPP

#include "cv_compat.hpp"
#include <chrono>
#include <math.h>
#include <stdio.h>
#include <vector>

using namespace cv;
using namespace std;
using namespace std::chrono;

#define LeftCam true
#define RightCam false

#define XYFOVangle 70
#define ZYFOVangle 70
#define XPixelDimensions 640
#define YPixelDimensions 480
#define CameraDistcm 20.16
#define PI 3.14159265

// Global control variable (P/DistanceCalculator.hpp:30): gates
// CooridinatePositionCalculator.  Defined in libusv.so.
extern bool CoordinateDisplay;

double deg2rad(double deg);
double rad2deg(double rad);

void MovingObjectDistanceCalculator(
    bool CameraSide, std::chrono::steady_clock::time_point ImgTimeStampThisCamera,
    std::vector<Point2f> VectorCenter_pointThisCamera,
    std::vector<Point2f> VectorCenter_pointOtherCamera,
    std::vector<Point2f> OldVectorCenter_pointOtherCamera,
    std::vector<Point2f> OlderVectorCenter_pointOtherCamera,
    std::vector<Point2f> InterpolatedVectorCenter_pointOtherCamera,
    std::vector<Point3i> InterframeMatchIndexesCompleteOtherCamera,
    std::chrono::steady_clock::time_point ImgTimeStampOtherCamera,
    std::chrono::steady_clock::time_point OldImgTimeStampOtherCamera,
    std::chrono::steady_clock::time_point OlderImgTimeStampOtherCamera,
    std::vector<double>& dist);

void CooridinatePositionCalculator(bool CameraSide, std::vector<double> dist,
                                   std::vector<Point2f> VectorCenter_pointThisCamera,
                                   vector<Point3d>& PoscmFromReferencePointVector);

#endif /* DistanceCalculator_HPP */
