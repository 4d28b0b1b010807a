/*
 * usv_oracle.h -- CPU ORACLE for the stereo block-match / distance hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libusv.so, the Python
 * package) links, imports or calls this.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load liboracle.so, and only as the
 * checker / the timed CPU baseline.
 *
 * What it restates (reference = /root/reference, P/ = Unsynchronized_Stereo_Vision_Proj325/):
 *   - SAD/SSD block match + argmin.  The reference has NO
 *     per-pixel block matcher; the spec is the build's own.
 *     Nearest reference primitive: absdiff, P/Main.cpp:304.  Parity for this
 *     function means "bit-exact vs this naive restatement", pinned by
 *     known-answer tests (shifted synthetic pairs) and an independent
 *     pure-Python restatement in tests/.
 *   - per-object distance power law P/DistanceCalculator.cpp:84,
 *     constant-acceleration extrapolation P/DistanceCalculator.cpp:53-81,
 *     Canny-path distance P/Main.cpp:681-694, XYZ P/DistanceCalculator.cpp:90-141.
 *     Pinned against the golden values SURVEY.md §8(c) recorded from the
 *     reference's own functions (tests/golden/distance_golden.json).
 *   - ResolveMatchList P/Main.cpp:432-477 and IDMatcher P/Main.cpp:483-499,
 *     pinned by the SURVEY.md §8(c) golden vectors (duplicate-emitting
 *     conflict pass; comma-operator Point3i).
 *   - GenerateMatchingList P/Main.cpp:403-426 with OpenCV 3.0 matchShapes /
 *     moments / HuMoments / contourArea, and the centre points of
 *     P/Main.cpp:1120-1143 with convexHull / minAreaRect / RotatedRect::points
 *     (shape_oracle.c).  Restated from OpenCV 3.0.0's published algorithms;
 *     parity vs OpenCV itself unpinned (absent, and the reference has no fixtures).
 *   - SURVEY.md §8(f) rows 1 and 3 (rectify_oracle.c, preproc_oracle.c):
 *     initUndistortRectifyMap + remap (P/Main.cpp:351-359), BGR2HSV /
 *     equalizeHist / HSV2BGR / BGR2GRAY (P/Main.cpp:365-371, 919-921), the
 *     absdiff and inRange masks with their 5x5-ellipse erode + dilate
 *     (P/Main.cpp:289-327).  OpenCV 3.0 semantics restated; parity unpinned
 *     against OpenCV (absent), pinned by known-answer tests.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off).
 */
#ifndef USV_ORACLE_H
#define USV_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

enum { USV_ORACLE_SAD = 0, USV_ORACLE_SSD = 1 };

/* A1, definition-level triple loop.  O(W*H*D*w^2).  Returns 0 on success. */
int usv_oracle_sad_naive(const uint8_t* L, const uint8_t* R, int W, int H, int pitch,
                         int D, int w, int metric, uint8_t* disp, int disp_pitch);

/* A1, separable running sums, n_threads row bands (0 = all cores).  Must equal
 * the naive variant bit for bit.  This is the timed CPU baseline. */
int usv_oracle_sad_sliding(const uint8_t* L, const uint8_t* R, int W, int H, int pitch,
                           int D, int w, int metric, uint8_t* disp, int disp_pitch,
                           int n_threads);

/* Same as the sliding variant but only for output rows [y0, y1): bounded CPU sample. */
int usv_oracle_sad_sliding_rows(const uint8_t* L, const uint8_t* R, int W, int H, int pitch,
                                int D, int w, int metric, uint8_t* disp, int disp_pitch,
                                int y0, int y1, int n_threads);

/* P/DistanceCalculator.cpp:84 for one integer disparity (cm; disp 0 -> inf). */
double usv_oracle_distance_cm(int disp);
/* P/Main.cpp:694 Canny-path formula for one integer disparity (cm). */
double usv_oracle_canny_distance_cm(int disp);

/* Per-pixel distance map from a u8 disparity map. */
void usv_oracle_disparity_to_distance_cm(const uint8_t* disp, int W, int H, int disp_pitch,
                                         double* out, int out_pitch_elems);

/* P/DistanceCalculator.cpp:15-88 restated over plain arrays.
 *   pts arrays are interleaved float (x,y); triples are int (x,y,z);
 *   time stamps are steady_clock tick counts (nanoseconds).
 *   interp_in/n_interp_in: the caller's InterpolatedVectorCenter_pointOtherCamera
 *   (by value in the reference; usually empty).  Appends n_triples doubles to
 *   dist_out (if the three other-camera vectors are non-empty) and returns the
 *   count appended. */
int usv_oracle_moving_object_distance(int camera_side_left,
                                      int64_t ts_this,
                                      const float* this_pts, int n_this,
                                      const float* cur_pts, int n_cur,
                                      const float* old_pts, int n_old,
                                      const float* older_pts, int n_older,
                                      const float* interp_in, int n_interp_in,
                                      const int* triples, int n_triples,
                                      int64_t ts_other, int64_t ts_other_old,
                                      int64_t ts_other_older,
                                      double* dist_out);

/* P/DistanceCalculator.cpp:90-141; xyz_out gets 3 doubles per emitted point.
 * coordinate_display mirrors the global CoordinateDisplay (P/DistanceCalculator.cpp:6). */
int usv_oracle_coordinate_position(int camera_side_left, const double* dist, int n_dist,
                                   const float* this_pts, int n_this,
                                   int coordinate_display, double* xyz_out);

/* Match record, layout of P/Match.hpp:4-12 (unsigned, unsigned, double). */
typedef struct { unsigned left, right; double value; } usv_oracle_match;

/* P/Main.cpp:432-477; returns the number of tentative matches written. */
int usv_oracle_resolve_match_list(const usv_oracle_match* in, int n_in, usv_oracle_match* out);
/* P/Main.cpp:483-499; out gets 3 ints per triple; returns the triple count. */
int usv_oracle_id_matcher(const usv_oracle_match* cur, int n_cur,
                          const usv_oracle_match* old, int n_old, int* out_xyz);

/* ---- A4 / A7: OpenCV 3.0 contour functions (shape_oracle.c; parity vs OpenCV unpinned) ---- */
/* Contours are n int (x, y) points interleaved. */
void usv_oracle_hu_moments(const int* pts, int n, double* hu7);
double usv_oracle_match_shapes_i1(const int* pts_a, int n_a, const int* pts_b, int n_b);
double usv_oracle_contour_area(const int* pts, int n); /* unoriented */
/* P/Main.cpp:403-426; contour i of a set = pts[2*off[i] .. 2*off[i+1]); returns the count written. */
int usv_oracle_generate_matching_list(const int* pts_a, const int* off_a, int n_a, const int* pts_b,
                                      const int* off_b, int n_b, usv_oracle_match* out);
/* convexHull(clockwise = true, returnPoints = true): hull_xy gets 2 ints per hull point; returns the count. */
int usv_oracle_convex_hull_cw(const int* pts, int n, int* hull_xy);
/* minAreaRect: out5 = {cx, cy, width, height, angle deg}; returns the hull size. */
int usv_oracle_min_area_rect(const int* pts, int n, float* out5);
/* RotatedRect::points of out5: 4 corners, 8 floats. */
void usv_oracle_rect_points(const float* r5, float* pt8);
/* P/Main.cpp:1120-1143: centre point per match (out_xy 2 floats each); returns the count. */
int usv_oracle_match_centroids(const int* pts, const int* off, int n_contours, const usv_oracle_match* matches,
                               int n_matches, float* out_xy);

/* ---- §8(f) row 1: rectification (rectify_oracle.c) ---- */
/* 3x3 inverse, cv::invert n == 3 path; returns 0 when singular. */
int usv_oracle_invert3(const double* m, double* out);
/* params (25 doubles): ir[9], fx, fy, u0, v0, k1 k2 p1 p2 k3 k4 k5 k6 s1 s2 s3 s4.
 * K 3x3, dist n_dist in {0,4,5,8,12}, Rrect 3x3 (NULL = identity), P 3 x p_cols (3 or 4). */
int usv_oracle_rectify_params(const double* K, const double* dist, int n_dist, const double* Rrect,
                              const double* P, int p_cols, double* params);
/* CV_16SC2 map1 (2 int16 per pixel) + CV_16UC1 map2, dense W x H. */
int usv_oracle_rectify_map(const double* params, int W, int H, int16_t* map1, uint16_t* map2);
/* remap INTER_LINEAR, BORDER_CONSTANT 0, u8 with cn interleaved channels. */
int usv_oracle_remap_linear(const uint8_t* src, int sW, int sH, int spitch, int cn, const int16_t* map1,
                            const uint16_t* map2, int W, int H, uint8_t* dst, int dpitch);

/* ---- §8(f) row 3: colour chain and masks (preproc_oracle.c) ---- */
void usv_oracle_bgr2hsv(const uint8_t* bgr, int W, int H, int pitch, uint8_t* hsv, int hsv_pitch);
void usv_oracle_equalize_lut(const uint32_t* hist, int total, uint8_t* lut);
void usv_oracle_hsv2bgr(const uint8_t* hsv, int W, int H, int pitch, uint8_t* bgr, int bgr_pitch);
void usv_oracle_bgr2gray(const uint8_t* bgr, int W, int H, int pitch, uint8_t* gray, int gray_pitch);
/* bgr (pitch) -> dense hsv' (3W), bgr' (3W), gray (W). */
int usv_oracle_frame_prep(const uint8_t* bgr, int W, int H, int pitch, uint8_t* hsv_out, uint8_t* bgr_out,
                          uint8_t* gray_out);
int usv_oracle_motion_mask(const uint8_t* gray, const uint8_t* prev, int W, int H, int pitch, int thresh,
                           uint8_t* mask, int mask_pitch);
int usv_oracle_colour_mask(const uint8_t* hsv, int W, int H, int pitch, const int* lo1, const int* hi1,
                           const int* lo2, const int* hi2, uint8_t* mask, int mask_pitch);

#ifdef __cplusplus
}
#endif
#endif
