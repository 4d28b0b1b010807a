/*
 * usv.h -- C ABI of the MI355X (gfx950) stereo block-match + distance engine.
 *
 * Plain pointers and sizes only (no HIP, torch or OpenCV types), so any FFI can
 * bind it (see INTEGRATION.md for the ctypes stub and the C++ call sites).
 * Every entry point is thread-safe and reentrant: no global mutable state;
 * work is enqueued on the caller's HIP stream (passed as an opaque void*,
 * NULL = the default stream) and never synchronises the device.
 *
 * Drop-in map (reference = 6dwavenminer/Unsynchronized_Stereo_Vision_Proj325,
 * P/ = Unsynchronized_Stereo_Vision_Proj325/):
 *
 *   usv_sad_disparity*        NEW hot path: per-pixel SAD/SSD block match +
 *                             argmin.  The reference has no
 *                             such function; its only per-pixel abs-diff is the
 *                             motion mask absdiff at P/Main.cpp:304 and its
 *                             "disparity" is a centroid x-difference
 *                             (P/DistanceCalculator.cpp:69-81, P/Main.cpp:681-693).
 *   usv_distance_lut_cm       P/DistanceCalculator.cpp:84 (model 0) and
 *                             P/Main.cpp:694 (model 1), tabulated for d=0..255.
 *   usv_disparity_to_distance per-pixel form of P/DistanceCalculator.cpp:84
 *                             (SURVEY.md §8(a) A11).
 *   usv_moving_object_distance  array form of MovingObjectDistanceCalculator,
 *                             P/DistanceCalculator.hpp:37-46 / .cpp:15-88.
 *   usv_coordinate_position   array form of CooridinatePositionCalculator,
 *                             P/DistanceCalculator.hpp:48 / .cpp:90-141.
 *   usv_resolve_match_list    ResolveMatchList, P/Main.cpp:432-477.
 *   usv_id_matcher            IDMatcher, P/Main.cpp:483-499.
 *   usv_generate_matching_list GenerateMatchingList, P/Main.cpp:403-426
 *                             (OpenCV matchShapes/contourArea restated; parity
 *                             unpinned -- OpenCV 3.0 is absent).
 *
 * Status codes replace exceptions so the C++ layer (include/Match.hpp,
 * include/DistanceCalculator.hpp, include/Matching.hpp) can keep the
 * reference's no-throw void convention.
 */
#ifndef USV_H
#define USV_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    USV_OK = 0,
    USV_ERR_INVALID_ARG = 1,  /* null pointer, bad size, pitch < width, ... */
    USV_ERR_UNSUPPORTED = 2,  /* parameter outside the engine's range (D > 256, even w, ...) */
    USV_ERR_HIP = 3,          /* a HIP runtime call failed (launch, copy) */
    USV_ERR_NO_DEVICE = 4     /* no gfx950 device visible */
} usv_status;

typedef enum { USV_METRIC_SAD = 0, USV_METRIC_SSD = 1 } usv_metric;

typedef enum {
    USV_DIST_MOVING_OBJECT = 0, /* P/DistanceCalculator.cpp:84 power law (cm) */
    USV_DIST_CANNY = 1          /* P/Main.cpp:694 reciprocal law (cm) */
} usv_distance_model;

typedef enum {
    USV_KERNEL_AUTO = 0,   /* fast path when the shape allows it, else generic */
    USV_KERNEL_FAST = 1,   /* lane-per-disparity running-sum kernel; UNSUPPORTED if not applicable */
    USV_KERNEL_GENERIC = 2 /* direct-window kernel, any w <= 63, SAD or SSD */
} usv_kernel;

/* Library / device info. */
const char* usv_version(void);
/* Returns USV_OK when a gfx950 device is visible; *n_devices gets the HIP count. */
usv_status usv_device_check(int* n_devices);

/*
 * Disparity map of one rectified u8 pair, all pointers DEVICE pointers.
 *   L, R        : W x H, row pitch `pitch` bytes (pitch >= W)
 *   D           : disparities searched, 1..256 (d = 0..D-1, R sampled at x-d)
 *   w           : odd window width/height, 1..63
 *   metric      : USV_METRIC_SAD / USV_METRIC_SSD
 *   disp        : W x H u8 output, pitch disp_pitch bytes
 * Border rule: replicate (columns and rows clamped independently for L and R);
 * ties resolve to the smallest d.  Bit-exact with oracle/sad_oracle.c.
 */
usv_status usv_sad_disparity(const uint8_t* L, const uint8_t* R, int W, int H, int pitch,
                             int D, int w, int metric, uint8_t* disp, int disp_pitch,
                             void* stream);

/*
 * As usv_sad_disparity, plus (when dist_cm != NULL) the fused per-pixel
 * distance map dist_cm[y*dist_pitch + x] = lut_cm[disp[y][x]] (doubles;
 * lut_cm = DEVICE pointer to 256 doubles from usv_distance_lut_cm).
 * kernel selects the implementation (USV_KERNEL_AUTO normally).
 */
usv_status usv_sad_disparity_ex(const uint8_t* L, const uint8_t* R, int W, int H, int pitch,
                                int D, int w, int metric, uint8_t* disp, int disp_pitch,
                                double* dist_cm, int dist_pitch, const double* lut_cm,
                                int kernel, void* stream);

/*
 * Batch of `batch` independent pairs laid out back to back on one device
 * (pair b at L + b*pair_stride, same for R, disp at disp + b*disp_stride,
 * dist at dist_cm + b*dist_stride elements).  One launch for the batch.
 */
usv_status usv_sad_disparity_batch(const uint8_t* L, const uint8_t* R, int batch,
                                   size_t pair_stride, int W, int H, int pitch, int D, int w,
                                   int metric, uint8_t* disp, size_t disp_stride,
                                   int disp_pitch, double* dist_cm, size_t dist_stride,
                                   int dist_pitch, const double* lut_cm, void* stream);

/* HOST: lut_out[d] = distance(d) in cm for d = 0..255 (d = 0 -> +inf for model 0). */
usv_status usv_distance_lut_cm(int model, double* lut_out);

/* DEVICE: out[y*out_pitch + x] = lut_cm[disp[y*disp_pitch + x]] (doubles). */
usv_status usv_disparity_to_distance(const uint8_t* disp, int W, int H, int disp_pitch,
                                     const double* lut_cm, double* out, int out_pitch,
                                     void* stream);

/* ---- host-side object path (C ABI mirrors of the reference's C++ API) ---- */

/* Layout of P/Match.hpp:4-12: {unsigned LeftIndex; unsigned RightIndex; double MatchValue;} */
typedef struct {
    unsigned left_index;
    unsigned right_index;
    double match_value;
} usv_match;

/* ResolveMatchList; out must hold n_in entries; *n_out gets the count. */
usv_status usv_resolve_match_list(const usv_match* in, int n_in, usv_match* out, int* n_out);

/* IDMatcher; out_xyz must hold 3*n_cur*n_old ints; *n_out gets the triple count. */
usv_status usv_id_matcher(const usv_match* cur, int n_cur, const usv_match* old, int n_old,
                          int* out_xyz, int* n_out);

/*
 * GenerateMatchingList over two contour sets given as flattened int (x,y)
 * points: contour i of set A is pts_a[2*off_a[i] .. 2*off_a[i+1]).  Appends to
 * out (capacity `cap`), *n_out gets the count written.
 */
usv_status usv_generate_matching_list(const int* pts_a, const int* off_a, int n_a,
                                      const int* pts_b, const int* off_b, int n_b,
                                      usv_match* out, int cap, int* n_out);

/* Hu-moment I1 distance (OpenCV CONTOURS_MATCH_I1) and unoriented polygon area. */
double usv_match_shapes_i1(const int* pts_a, int n_a, const int* pts_b, int n_b);
double usv_contour_area(const int* pts, int n);

/*
 * MovingObjectDistanceCalculator over arrays (see oracle/usv_oracle.h for the
 * argument meaning).  Appends up to n_triples doubles to dist_out; *n_out gets
 * the count; interp_out (nullable, 2*n_triples floats) receives the
 * extrapolated other-camera centroids.
 */
usv_status usv_moving_object_distance(int camera_side_left, int64_t ts_this,
                                      const float* this_pts, int n_this,
                                      const float* cur_pts, int n_cur,
                                      const float* old_pts, int n_old,
                                      const float* older_pts, int n_older,
                                      const int* triples, int n_triples,
                                      int64_t ts_other, int64_t ts_other_old,
                                      int64_t ts_other_older,
                                      double* dist_out, float* interp_out, int* n_out);

/* CooridinatePositionCalculator; xyz_out gets 3 doubles per point. */
usv_status usv_coordinate_position(int camera_side_left, const double* dist, int n_dist,
                                   const float* this_pts, int n_this, int coordinate_display,
                                   double* xyz_out, int* n_out);

#ifdef __cplusplus
}
#endif
#endif /* USV_H */
