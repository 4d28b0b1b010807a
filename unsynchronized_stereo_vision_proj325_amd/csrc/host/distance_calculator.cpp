// distance_calculator.cpp -- the reference's DistanceCalculator API, restated.
//
// Implements include/DistanceCalculator.hpp (drop-in for
// P/DistanceCalculator.hpp:30-48) plus the per-disparity distance table used
// by the GPU path.  MUST be compiled with -ffp-contract=off: the extrapolated
// centroid feeds an (int) truncation, and an FMA-contracted build changes it
// (SURVEY.md §0.7).  Parity: tests/test_capi.py and tests/test_cpp_api.py (vs
// oracle/distance_oracle.c) and tests/test_oracle.py (the SURVEY.md §8(c) golden values).
#include "DistanceCalculator.hpp"

#include <cmath>

#include "usv.h"

bool CoordinateDisplay = false;  // P/DistanceCalculator.cpp:6

double deg2rad(double deg) { return deg * PI / 180.0; }  // P/DistanceCalculator.cpp:8-10
double rad2deg(double rad) { return rad * 180 / PI; }    // P/DistanceCalculator.cpp:11-13

namespace usv {

// P/DistanceCalculator.cpp:84 with an int disparity (0 -> +inf, kept, not clamped).
double distance_cm(int disp) { return pow((10760 * pow(disp, -0.877)) / 3.0752, 1 / 0.7791); }

// P/Main.cpp:694 (Canny path).
double canny_distance_cm(int disp) { return ((201.6 * 4) / (disp * 0.000043)) / 1000; }

namespace {
// P/DistanceCalculator.cpp:57-59: float(ticks) * num / den, float arithmetic.
float seconds_f(steady_clock::duration d) {
    return float(d.count()) * steady_clock::period::num / steady_clock::period::den;
}
Point2f pick(const std::vector<Point2f>& v, int idx) {
    // (unsigned) comparison as at lines 34, 40, 46: negative indices are out of range.
    return v.size() > (unsigned)idx ? v[idx] : Point2f(0, 0);
}
}  // namespace
}  // namespace usv

namespace usv {
void moving_object_distance(bool CameraSide, steady_clock::time_point ImgTimeStampThisCamera,
                            const std::vector<Point2f>& VectorCenter_pointThisCamera,
                            const std::vector<Point2f>& VectorCenter_pointOtherCamera,
                            const std::vector<Point2f>& OldVectorCenter_pointOtherCamera,
                            const std::vector<Point2f>& OlderVectorCenter_pointOtherCamera,
                            std::vector<Point2f>& InterpolatedVectorCenter_pointOtherCamera,
                            const std::vector<Point3i>& InterframeMatchIndexesCompleteOtherCamera,
                            steady_clock::time_point ImgTimeStampOtherCamera,
                            steady_clock::time_point OldImgTimeStampOtherCamera,
                            steady_clock::time_point OlderImgTimeStampOtherCamera,
                            std::vector<double>& dist);
}  // namespace usv

void MovingObjectDistanceCalculator(bool CameraSide, steady_clock::time_point ImgTimeStampThisCamera,
                                    std::vector<Point2f> VectorCenter_pointThisCamera,
                                    std::vector<Point2f> VectorCenter_pointOtherCamera,
                                    std::vector<Point2f> OldVectorCenter_pointOtherCamera,
                                    std::vector<Point2f> OlderVectorCenter_pointOtherCamera,
                                    std::vector<Point2f> InterpolatedVectorCenter_pointOtherCamera,
                                    std::vector<Point3i> InterframeMatchIndexesCompleteOtherCamera,
                                    steady_clock::time_point ImgTimeStampOtherCamera,
                                    steady_clock::time_point OldImgTimeStampOtherCamera,
                                    steady_clock::time_point OlderImgTimeStampOtherCamera,
                                    std::vector<double>& dist) {
    // All vectors by value, as in the reference; the extrapolated points land
    // in this call's copy and are discarded.
    usv::moving_object_distance(CameraSide, ImgTimeStampThisCamera, VectorCenter_pointThisCamera,
                                VectorCenter_pointOtherCamera, OldVectorCenter_pointOtherCamera,
                                OlderVectorCenter_pointOtherCamera,
                                InterpolatedVectorCenter_pointOtherCamera,
                                InterframeMatchIndexesCompleteOtherCamera, ImgTimeStampOtherCamera,
                                OldImgTimeStampOtherCamera, OlderImgTimeStampOtherCamera, dist);
}

void usv::moving_object_distance(bool CameraSide, steady_clock::time_point ImgTimeStampThisCamera,
                                 const std::vector<Point2f>& VectorCenter_pointThisCamera,
                                 const std::vector<Point2f>& VectorCenter_pointOtherCamera,
                                 const std::vector<Point2f>& OldVectorCenter_pointOtherCamera,
                                 const std::vector<Point2f>& OlderVectorCenter_pointOtherCamera,
                                 std::vector<Point2f>& InterpolatedVectorCenter_pointOtherCamera,
                                 const std::vector<Point3i>& InterframeMatchIndexesCompleteOtherCamera,
                                    steady_clock::time_point ImgTimeStampOtherCamera,
                                    steady_clock::time_point OldImgTimeStampOtherCamera,
                                    steady_clock::time_point OlderImgTimeStampOtherCamera,
                                    std::vector<double>& dist) {
    auto& thisPts = VectorCenter_pointThisCamera;
    auto& interp = InterpolatedVectorCenter_pointOtherCamera;
    const auto& triples = InterframeMatchIndexesCompleteOtherCamera;
    if (VectorCenter_pointOtherCamera.empty() || OldVectorCenter_pointOtherCamera.empty() ||
        OlderVectorCenter_pointOtherCamera.empty())
        return;  // line 28
    // The three deltas do not depend on the object; computing them once gives
    // the same floats the reference recomputes per iteration.
    const float t_old = usv::seconds_f(OldImgTimeStampOtherCamera - OlderImgTimeStampOtherCamera);
    const float t_cur = usv::seconds_f(ImgTimeStampOtherCamera - OldImgTimeStampOtherCamera);
    const float t_ahead = usv::seconds_f(ImgTimeStampThisCamera - ImgTimeStampOtherCamera);
    for (size_t i = 0; i < triples.size(); ++i) {
        const Point2f cur = usv::pick(VectorCenter_pointOtherCamera, triples[i].x);
        const Point2f old = usv::pick(OldVectorCenter_pointOtherCamera, triples[i].y);
        const Point2f older = usv::pick(OlderVectorCenter_pointOtherCamera, triples[i].z);
        // constant-acceleration extrapolation to this camera's time stamp (lines 61-65)
        const Point2f vel_old = (old - older) / t_old;
        const Point2f vel_cur = (cur - old) / t_cur;
        const Point2f accel = (vel_cur - vel_old) / t_cur;
        const Point2f vel_ahead = vel_cur + (accel * t_ahead);
        interp.push_back((vel_ahead * t_ahead) + cur);
        int disp = 0;
        if (!thisPts.empty() && thisPts.size() > i) {  // lines 72-73
            // interp[i], not interp.back(): the reference indexes its by-value copy
            const int dx = CameraSide == LeftCam ? (int)(thisPts[i].x - interp[i].x)
                                                 : (int)(-thisPts[i].x + interp[i].x);
            const int dy = (int)(thisPts[i].y - interp[i].y);
            disp = (int)sqrt(pow(dx, 2) + pow(dy, 2));
        }
        dist.push_back(usv::distance_cm(disp));
    }
}

namespace usv {
// CooridinatePositionCalculator with the CoordinateDisplay gate as a parameter
// (the C ABI passes it explicitly so it stays reentrant).
void coordinate_position(bool CameraSide, const std::vector<double>& dist,
                         const std::vector<Point2f>& VectorCenter_pointThisCamera, bool display,
                         std::vector<Point3d>& PoscmFromReferencePointVector) {
    const double half_base = (double)(CameraDistcm / 2);
    for (size_t i = 0; dist.size() > i && VectorCenter_pointThisCamera.size() > i && display; ++i) {
        const double r = dist[i];
        const Point2f c = VectorCenter_pointThisCamera[i];
        // horizontal bearing, with the reference's empirical per-camera calibrations (lines 105-111)
        double bearing = ((double)c.x / (double)XPixelDimensions) * (double)XYFOVangle;
        if (CameraSide == LeftCam)
            bearing = -(141.08 * pow(r, -0.254) - bearing + (55 - rad2deg(acos(10.08 / r))));
        else
            bearing = (11.815 * log(r) - 31.397 - bearing + (125 - rad2deg(acos(10.08 / r))));
        const double cam_angle = (double)125 - bearing;
        const double deviation = rad2deg(asin((sin(deg2rad(cam_angle)) / r) * half_base));
        const double ref_angle = (double)180 - (cam_angle + deviation);
        const double cam_range = (half_base / sin(deg2rad(deviation))) * sin(deg2rad(ref_angle));
        const double x_cam = cam_range * tan(deg2rad((double)90 - cam_angle));
        double x = CameraSide == LeftCam ? x_cam - half_base : x_cam + half_base;
        x = CameraSide == LeftCam ? (x + 24.401) / -1.6257 : (x - 34.3) / 1.6834;
        const double y = sqrt(pow(r, 2) - pow(x, 2));
        const double elev = (double)45 - (((double)c.y / (double)YPixelDimensions) * (double)ZYFOVangle);
        double z = r * tan(deg2rad(elev));
        z = CameraSide == LeftCam ? (z - 0.6112) / 2.228 : (z - 6.3706) / 2.5771;
        PoscmFromReferencePointVector.push_back({x, y, z});
    }
}
}  // namespace usv

void CooridinatePositionCalculator(bool CameraSide, std::vector<double> dist,
                                   std::vector<Point2f> VectorCenter_pointThisCamera,
                                   vector<Point3d>& PoscmFromReferencePointVector) {
    usv::coordinate_position(CameraSide, dist, VectorCenter_pointThisCamera, CoordinateDisplay,
                             PoscmFromReferencePointVector);
}

// ---- C ABI over the same C++ functions ------------------------------------

extern "C" usv_status usv_distance_lut_cm(int model, double* lut_out) {
    if (!lut_out) return USV_ERR_INVALID_ARG;
    if (model != USV_DIST_MOVING_OBJECT && model != USV_DIST_CANNY) return USV_ERR_UNSUPPORTED;
    for (int d = 0; d < 256; ++d)
        lut_out[d] = model == USV_DIST_MOVING_OBJECT ? usv::distance_cm(d) : usv::canny_distance_cm(d);
    return USV_OK;
}

// north_star quotes distance in mm: the same table times 10 (one double multiply per entry, so
// mm[d] / 10 is cm[d] to within one rounding; inf stays inf).
extern "C" usv_status usv_distance_lut_mm(int model, double* lut_out) {
    usv_status st = usv_distance_lut_cm(model, lut_out);
    if (st != USV_OK) return st;
    for (int d = 0; d < 256; ++d) lut_out[d] = lut_out[d] * 10.0;
    return USV_OK;
}

extern "C" usv_status usv_moving_object_distance(
    int camera_side_left, int64_t ts_this, const float* this_pts, int n_this, const float* cur_pts,
    int n_cur, const float* old_pts, int n_old, const float* older_pts, int n_older,
    const float* interp_in, int n_interp_in, const int* triples, int n_triples, int64_t ts_other,
    int64_t ts_other_old, int64_t ts_other_older, double* dist_out, float* interp_out, int* n_out) {
    if (!n_out || n_this < 0 || n_cur < 0 || n_old < 0 || n_older < 0 || n_triples < 0 ||
        n_interp_in < 0)
        return USV_ERR_INVALID_ARG;
    if ((n_this && !this_pts) || (n_cur && !cur_pts) || (n_old && !old_pts) ||
        (n_older && !older_pts) || (n_interp_in && !interp_in) ||
        (n_triples && (!triples || !dist_out)))
        return USV_ERR_INVALID_ARG;
    auto pts = [](const float* p, int n) {
        std::vector<Point2f> v;
        v.reserve(n);
        for (int i = 0; i < n; ++i) v.push_back(Point2f(p[2 * i], p[2 * i + 1]));
        return v;
    };
    std::vector<Point3i> tri;
    tri.reserve(n_triples);
    for (int i = 0; i < n_triples; ++i) tri.push_back(Point3i(triples[3 * i], triples[3 * i + 1], triples[3 * i + 2]));
    using tp = steady_clock::time_point;
    auto at = [](int64_t ns) { return tp(std::chrono::duration_cast<steady_clock::duration>(std::chrono::nanoseconds(ns))); };
    std::vector<double> dist;
    // the reference's caller passes an empty vector (P/Main.cpp:869-871); any other is honoured
    std::vector<Point2f> interp = pts(interp_in, n_interp_in);
    usv::moving_object_distance(camera_side_left != 0, at(ts_this), pts(this_pts, n_this),
                                pts(cur_pts, n_cur), pts(old_pts, n_old), pts(older_pts, n_older),
                                interp, tri, at(ts_other), at(ts_other_old), at(ts_other_older), dist);
    for (size_t i = 0; i < dist.size(); ++i) dist_out[i] = dist[i];
    if (interp_out)
        for (size_t i = 0; i < interp.size(); ++i) {
            interp_out[2 * i] = interp[i].x;
            interp_out[2 * i + 1] = interp[i].y;
        }
    *n_out = (int)dist.size();
    return USV_OK;
}

extern "C" usv_status usv_coordinate_position(int camera_side_left, const double* dist, int n_dist,
                                              const float* this_pts, int n_this,
                                              int coordinate_display, double* xyz_out, int* n_out) {
    if (!n_out || n_dist < 0 || n_this < 0 || (n_dist && !dist) || (n_this && !this_pts))
        return USV_ERR_INVALID_ARG;
    std::vector<double> dv(dist, dist + n_dist);
    std::vector<Point2f> pv;
    for (int i = 0; i < n_this; ++i) pv.push_back(Point2f(this_pts[2 * i], this_pts[2 * i + 1]));
    std::vector<Point3d> out;
    usv::coordinate_position(camera_side_left != 0, dv, pv, coordinate_display != 0, out);
    if (!out.empty() && !xyz_out) return USV_ERR_INVALID_ARG;
    for (size_t i = 0; i < out.size(); ++i) {
        xyz_out[3 * i] = out[i].x;
        xyz_out[3 * i + 1] = out[i].y;
        xyz_out[3 * i + 2] = out[i].z;
    }
    *n_out = (int)out.size();
    return USV_OK;
}
