/*
 * distance_oracle.c -- CPU ORACLE (test infrastructure only; see usv_oracle.h).
 *
 * Plain-C restatement of the reference's distance arithmetic.  Compiled with
 * -ffp-contract=off (an FMA-contracted build flips the (int)
 * truncation of the extrapolated disparity).  OpenCV's Point_<float>
 * operators are element-wise float ops (+, -, * float, / float), so each
 * component below is written as the same sequence of float operations.
 */
#include "usv_oracle.h"
#include <math.h>
#include <stddef.h>
#include <stdlib.h>

#define USV_PI 3.14159265 /* P/DistanceCalculator.hpp:25 -- NOT M_PI */
#define USV_CAMERA_DIST_CM 20.16
#define USV_XPIX 640
#define USV_YPIX 480
#define USV_XYFOV 70
#define USV_ZYFOV 70

static double deg2rad(double deg) { return deg * USV_PI / 180.0; } /* P/DistanceCalculator.cpp:8-10 */
static double rad2deg(double rad) { return rad * 180 / USV_PI; }   /* P/DistanceCalculator.cpp:11-13 */

/* P/DistanceCalculator.cpp:84: pow(((10760 * pow(disp, -0.877)) / 3.0752), (1 / 0.7791)) */
double usv_oracle_distance_cm(int disp) {
    return pow((10760 * pow((double)disp, -0.877)) / 3.0752, 1 / 0.7791);
}

/* P/Main.cpp:694: ((201.6 * 4) / (disp * 0.000043)) / 1000 */
double usv_oracle_canny_distance_cm(int disp) {
    return ((201.6 * 4) / (disp * 0.000043)) / 1000;
}

void usv_oracle_disparity_to_distance_cm(const uint8_t* disp, int W, int H, int disp_pitch,
                                         double* out, int out_pitch_elems) {
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            out[(size_t)y * out_pitch_elems + x] =
                usv_oracle_distance_cm(disp[(size_t)y * disp_pitch + x]);
}

/* steady_clock::duration -> float seconds, P/DistanceCalculator.cpp:57-59:
 *   float(count) * period::num / period::den   (num = 1, den = 1e9 on every
 *   platform the reference targets; float * integer promotes to float). */
static float ticks_to_seconds(int64_t ticks) {
    float t = (float)ticks;
    t = t * (float)1;
    t = t / (float)1000000000LL;
    return t;
}

int usv_oracle_moving_object_distance(int camera_side_left, int64_t ts_this,
                                      const float* this_pts, int n_this, const float* cur_pts,
                                      int n_cur, const float* old_pts, int n_old,
                                      const float* older_pts, int n_older,
                                      const float* interp_in, int n_interp_in,
                                      const int* triples, int n_triples, int64_t ts_other,
                                      int64_t ts_other_old, int64_t ts_other_older,
                                      double* dist_out) {
    /* P/DistanceCalculator.cpp:28 -- all three other-camera vectors non-empty */
    if (n_cur <= 0 || n_old <= 0 || n_older <= 0) return 0;
    if (n_interp_in < 0) n_interp_in = 0;
    /* The by-value InterpolatedVectorCenter_pointOtherCamera copy (line 19):
     * the caller's n_interp_in points, then one point pushed per triple
     * (line 67).  Line 75 reads element i of it. */
    float* grown = (float*)malloc(sizeof(float) * 2 * ((size_t)n_interp_in + (size_t)(n_triples > 0 ? n_triples : 0) + 1));
    if (!grown) return -1;
    for (int k = 0; k < 2 * n_interp_in; ++k) grown[k] = interp_in[k];
    int n_grown = n_interp_in;
    int appended = 0;
    for (int i = 0; i < n_triples; ++i) {
        int tx = triples[3 * i + 0], ty = triples[3 * i + 1], tz = triples[3 * i + 2];
        /* (unsigned) casts: a negative index is "out of range" -> (0,0), lines 34-51 */
        float cx = 0.f, cy = 0.f, ox = 0.f, oy = 0.f, qx = 0.f, qy = 0.f;
        if ((unsigned)n_cur > (unsigned)tx) { cx = cur_pts[2 * tx]; cy = cur_pts[2 * tx + 1]; }
        if ((unsigned)n_old > (unsigned)ty) { ox = old_pts[2 * ty]; oy = old_pts[2 * ty + 1]; }
        if ((unsigned)n_older > (unsigned)tz) { qx = older_pts[2 * tz]; qy = older_pts[2 * tz + 1]; }
        float t1 = ticks_to_seconds(ts_other_old - ts_other_older);
        float t2 = ticks_to_seconds(ts_other - ts_other_old);
        float t3 = ticks_to_seconds(ts_this - ts_other);
        /* lines 61-65, component-wise float ops in the operators' order */
        float v1x = (ox - qx) / t1, v1y = (oy - qy) / t1;
        float v2x = (cx - ox) / t2, v2y = (cy - oy) / t2;
        float ax = (v2x - v1x) / t2, ay = (v2y - v1y) / t2;
        float v3x = v2x + (ax * t3), v3y = v2y + (ay * t3);
        float px = (v3x * t3) + cx, py = (v3y * t3) + cy;
        /* line 67 pushes onto the by-value copy; line 75 then reads index i of
         * that copy: the caller's element i while i < n_interp_in, else the
         * point pushed at iteration i - n_interp_in (a reference quirk kept
         * here; with an empty caller vector that is this iteration's point). */
        grown[2 * n_grown] = px;
        grown[2 * n_grown + 1] = py;
        ++n_grown;
        float ix = grown[2 * i], iy = grown[2 * i + 1];
        /* lines 69-83 -- interp index i is always in range after the push */
        int dispx = 0, dispy = 0, disp = 0;
        if (n_this > 0 && n_this > i) {
            if (camera_side_left) dispx = (int)(this_pts[2 * i] - ix);
            else dispx = (int)(-this_pts[2 * i] + ix);
            dispy = (int)(this_pts[2 * i + 1] - iy);
            disp = (int)sqrt(pow((double)dispx, 2) + pow((double)dispy, 2));
        }
        dist_out[appended++] = usv_oracle_distance_cm(disp);
    }
    free(grown);
    return appended;
}

int usv_oracle_coordinate_position(int camera_side_left, const double* dist, int n_dist,
                                   const float* this_pts, int n_this, int coordinate_display,
                                   double* xyz_out) {
    int n = 0;
    /* P/DistanceCalculator.cpp:92 */
    for (int i = 0; i < n_dist && i < n_this && coordinate_display; ++i) {
        double d = dist[i];
        double px = (double)this_pts[2 * i], py = (double)this_pts[2 * i + 1];
        double view_xy = (px / (double)USV_XPIX) * (double)USV_XYFOV;
        if (camera_side_left)
            view_xy = -(141.08 * pow(d, -0.254) - view_xy + (55 - rad2deg(acos(10.08 / d))));
        else
            view_xy = (11.815 * log(d) - 31.397 - view_xy + (125 - rad2deg(acos(10.08 / d))));
        double cam2obj = (double)125 - view_xy;
        double dev = rad2deg(asin((sin(deg2rad(cam2obj)) / d) * (double)(USV_CAMERA_DIST_CM / 2)));
        double ref2obj = (double)180 - (cam2obj + dev);
        double c2o_dist = ((double)(USV_CAMERA_DIST_CM / 2) / sin(deg2rad(dev))) * sin(deg2rad(ref2obj));
        double centre_angle = (double)90 - cam2obj;
        double x_cam = c2o_dist * tan(deg2rad(centre_angle));
        double x_ref;
        if (camera_side_left) {
            x_ref = x_cam - (double)(USV_CAMERA_DIST_CM / 2);
            x_ref = (x_ref + 24.401) / -1.6257;
        } else {
            x_ref = x_cam + (double)(USV_CAMERA_DIST_CM / 2);
            x_ref = (x_ref - 34.3) / 1.6834;
        }
        double y_ref = sqrt(pow(d, 2) - pow(x_ref, 2));
        double view_zy = (double)45 - ((py / (double)USV_YPIX) * (double)USV_ZYFOV);
        double z_ref = d * tan(deg2rad(view_zy));
        if (camera_side_left) z_ref = (z_ref - 0.6112) / 2.228;
        else z_ref = (z_ref - 6.3706) / 2.5771;
        xyz_out[3 * n + 0] = x_ref;
        xyz_out[3 * n + 1] = y_ref;
        xyz_out[3 * n + 2] = z_ref;
        ++n;
    }
    return n;
}
