/*
 * usv.h -- C ABI of the MI355X (gfx950) stereo block-match + distance engine.
 *
 * Plain pointers and sizes only (no HIP, torch or OpenCV types), so any FFI can
 * bind it (see INTEGRATION.md for the ctypes stub and the C++ call sites).
 * Every entry point is thread-safe and reentrant; the only global state is a
 * mutex-guarded, append-only cache of device copies of host distance tables
 * (see usv_sad_disparity_ex).  Work is enqueued on the caller's HIP stream
 * (passed as an opaque void*, NULL = the default stream) and never
 * synchronises the device, except that cache's one-time fill.
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
 *   usv_distance_lut_cm/_mm   P/DistanceCalculator.cpp:84 (model 0) and
 *                             P/Main.cpp:694 (model 1), tabulated for d=0..255
 *                             (cm as the reference prints, P/Main.cpp:1265; mm = 10 cm).
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
 *   usv_min_area_rect,        minAreaRect + the per-match centre point,
 *   usv_match_centroids       P/Main.cpp:1120-1143 (A7; OpenCV restated, unpinned).
 *   usv_contour_descriptors,  GPU form of GenerateMatchingList's scores
 *   usv_contour_pair_scores   (SURVEY §8(f) row 2), descriptors once per contour.
 *   usv_rectify_params / _map initUndistortRectifyMap(..., CV_16SC2, ...),
 *                             P/Main.cpp:352,357 (the
 *                             reference rebuilds it every frame, we build once)
 *   usv_load_calibration,     LoadCalibrationData, P/Main.cpp:329-349 (FileStorage
 *   usv_calibration_rectify_params  XML read without OpenCV)
 *   usv_remap_linear_u8,      remap(INTER_LINEAR, BORDER_CONSTANT, Scalar()),
 *   usv_rectify_pair_u8       P/Main.cpp:353,358 (one launch for both cameras)
 *   usv_remap_pack_map,       the same remap through a 4-byte-per-pixel form of
 *   usv_*_packed_u8           the map (built once; results bit-identical)
 *   usv_bgr2hsv_hist_u8,      cvtColor BGR2HSV P/Main.cpp:919 + LightingCorrection
 *   usv_equalize_hsv_bgr_gray_u8  (split/equalizeHist/merge/HSV2BGR,
 *   usv_frame_prep_u8         P/Main.cpp:365-371) + cvtColor BGR2GRAY :921
 *   usv_motion_mask_u8        ABSDiffSearch P/Main.cpp:299-312 (absdiff,
 *                             threshold 40, MorphilogicalFilter :289-292)
 *   usv_colour_mask_u8        ColourSearch P/Main.cpp:318-327 (two inRange,
 *                             addWeighted, MorphilogicalFilter)
 *   (OpenCV 3.0 u8 semantics restated in oracle/; parity unpinned against
 *   OpenCV itself, which the image lacks -- SURVEY §8(c).)
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
    USV_ERR_NO_DEVICE = 4,    /* no gfx950 device visible */
    USV_ERR_COMM = 5          /* an RCCL call failed (multi-GPU engine) */
} usv_status;

typedef enum { USV_METRIC_SAD = 0, USV_METRIC_SSD = 1 } usv_metric;

typedef enum {
    USV_DIST_MOVING_OBJECT = 0, /* P/DistanceCalculator.cpp:84 power law (cm) */
    USV_DIST_CANNY = 1          /* P/Main.cpp:694 reciprocal law (cm) */
} usv_distance_model;

typedef enum {
    USV_KERNEL_AUTO = 0,    /* fast path when the shape allows it, else tiled, else generic */
    USV_KERNEL_FAST = 1,    /* lane-per-disparity running-sum kernels: SAD (w <= 15), SSD (11 <= w <= 15);
                               W % 4 == 0, W >= 48, 4-byte aligned bases / pitch; UNSUPPORTED otherwise */
    USV_KERNEL_GENERIC = 2, /* direct-window kernel, any w <= 63, SAD or SSD (reference-speed fallback) */
    USV_KERNEL_TILED = 3,   /* sliding-window kernel: SAD or SSD, any W / pitch / alignment, w <= 31 */
    USV_KERNEL_MATRIX = 4   /* SSD whose window cross term runs on the matrix cores (v_mfma_i32_16x16x64_i8):
                               w = 3 .. 13, D = 32 .. 160 in steps of 32, W >= 64; USV_KERNEL_AUTO takes it for
                               every SSD shape it supports */
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
 * distance map dist_cm[y*dist_pitch + x] = lut_cm[disp[y][x]] (doubles).
 * lut_cm = 256 doubles from usv_distance_lut_cm, in device memory, pinned host
 * memory, or ordinary HOST memory: a pageable host table is copied to a
 * library-owned device buffer on its first use (one synchronous 2 KB copy per
 * device and distinct contents, at most 64 tables; make that first call before
 * any hipGraph capture) and found again by value afterwards.
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

/* A prepared match for a caller that repeats the same match over the same buffers (a frame loop into
 * fixed device buffers): usv_match_plan_create takes usv_sad_disparity_batch's arguments plus the kernel
 * choice (kernel != USV_KERNEL_AUTO needs batch == 1), validates them, resolves the distance table and
 * the kernel once, and returns a plan; usv_match_plan_launch enqueues one match on the plan's stream with
 * no further checks (one pointer argument: the per-call host cost is the launch itself).  The buffers and
 * the stream must outlive the plan; a plan may be launched from one thread at a time.  Replaces nothing in
 * the reference; it is the C side of StereoBlockMatcher.bind. */
typedef struct usv_match_plan usv_match_plan;
usv_status usv_match_plan_create(const uint8_t* L, const uint8_t* R, int batch, size_t pair_stride, int W, int H,
                                 int pitch, int D, int w, int metric, uint8_t* disp, size_t disp_stride,
                                 int disp_pitch, double* dist_cm, size_t dist_stride, int dist_pitch,
                                 const double* lut_cm, int kernel, void* stream, usv_match_plan** out);
usv_status usv_match_plan_launch(const usv_match_plan* plan);
usv_status usv_match_plan_destroy(usv_match_plan* plan);

/* ---- multi-GPU: one process, one device + stream + RCCL communicator per GPU ----
 *
 * SURVEY.md §8(b)(2) / §8(e).  A batch of independent frame pairs (configs D
 * and E: 8 pairs over 8 GPUs) is split into contiguous shards (usv_shard_range:
 * pair i -> GPU i when batch == n), each GPU matches its shard with the
 * batched kernel, and ONE ncclGather (rccl.h:745) brings the u8 disparity maps
 * to devices[0]; the distance maps are expanded there from the 256-entry table
 * (never shipped).  Replaces nothing in the reference (its two camera threads,
 * P/Main.cpp:1407-1420, share one CPU); it is the entry a C++ caller uses to
 * shard frames over the node.  Not thread-safe per engine: one caller at a time.
 */
typedef struct usv_sharded_engine usv_sharded_engine;

/* HOST: shard [*first, *first + *count) of a batch of `batch` pairs for GPU k of n. */
usv_status usv_shard_range(int batch, int n_devices, int k, int* first, int* count);
/* HOST: where pair `pair` of the batch lands in the root's gather buffer, in units of frames:
 * GPU k's shard starts at slot k * per (per = ceil(max_pairs / n) of the engine). */
usv_status usv_shard_slot(int batch, int n_devices, int per, int pair, long long* slot);

/* Engine for up to max_pairs W x H pairs per call on the n_devices listed GPUs
 * (distinct HIP ordinals; devices[0] is the gather root).  Allocates each GPU's
 * dense input / output shard buffers (ceil(max_pairs / n) pairs, pitch W) and
 * calls ncclCommInitAll.  USV_ERR_NO_DEVICE without a GPU. */
usv_status usv_sharded_create(const int* devices, int n_devices, int max_pairs, int W, int H, int D, int w,
                              int metric, usv_sharded_engine** out);
usv_status usv_sharded_destroy(usv_sharded_engine* e);

/* DEVICE buffers of GPU k's shard inputs for the NEXT submit (dense, pitch W, pair j at j*W*H;
 * the engine alternates two buffer slots per GPU): fill them and pass L = R = NULL to
 * usv_batch_sharded(_submit) to match HBM-resident frames.  If that slot still holds a batch in
 * flight, this call completes it first (as a submit on a busy slot does), so the buffers returned
 * are never read by a running batch; that batch's status is reported by its own wait. */
usv_status usv_sharded_input_buffers(usv_sharded_engine* e, int k, uint8_t** L, uint8_t** R);

/* DEVICE results on devices[0] of the last COMPLETED batch: the gather buffer
 * (GPU k's shard at slot k, i.e. k * ceil(max_pairs / n) * W * H bytes; equal
 * to batch order when batch == n * ceil(max_pairs / n)) and the distance maps
 * in batch order (NULL until a call asked for them). */
usv_status usv_sharded_outputs(usv_sharded_engine* e, const uint8_t** disp, const double** dist_cm);

/* Match a batch (1 <= batch <= max_pairs) across the engine's GPUs.  BLOCKING:
 * returns when the results are in place.
 *   L, R      : HOST batch (pair b at L + b * pair_stride, row pitch `pitch`),
 *               or both NULL = the frames already sit in usv_sharded_input_buffers.
 *   disp      : nullable HOST output, batch x H x W dense u8, batch order.
 *   dist_cm   : nullable HOST output, batch x H x W doubles; with_distance != 0
 *               computes the maps on devices[0] even when dist_cm is NULL.
 *   lut_cm    : the 256-entry table (host or device) when distances are wanted.
 * The calling thread's current device is restored before returning. */
usv_status usv_batch_sharded(usv_sharded_engine* e, const uint8_t* L, const uint8_t* R, int batch,
                             size_t pair_stride, int pitch, uint8_t* disp, double* dist_cm,
                             const double* lut_cm, int with_distance);
/* The same in two halves, two batches in flight: submit enqueues a batch on the next of two buffer
 * slots and returns *ticket; wait completes that batch (disp / dist_cm filled).  Host inputs (even
 * pageable ones) have been copied when submit returns: the caller may reuse them at once.  A submit
 * (or usv_sharded_input_buffers) that needs a busy slot first completes the older batch there -- its
 * results are delivered, and the wait on its ticket then returns that completion's status (USV_OK,
 * or the error it hit) once; a ticket never submitted or already waited for is USV_ERR_INVALID_ARG.
 * Batch k+1's copies and kernels overlap batch k's gather, distance expansion and D2H.  The host
 * output buffers of a batch must stay valid until its wait (or its implicit completion). */
usv_status usv_batch_sharded_submit(usv_sharded_engine* e, const uint8_t* L, const uint8_t* R, int batch,
                                    size_t pair_stride, int pitch, uint8_t* disp, double* dist_cm,
                                    const double* lut_cm, int with_distance, long long* ticket);
usv_status usv_batch_sharded_wait(usv_sharded_engine* e, long long ticket);

/* ---- streaming host frames (the reference's caller hands over HOST frames per camera
 * thread, P/Main.cpp:876-921, 1238-1242) ----
 * `depth` (2..8) frames in flight on the current device: each slot owns pinned host staging,
 * device buffers and a HIP stream, so frame k+1's H2D, frame k's match and frame k-1's D2H
 * overlap.  Output: the u8 disparity map in pinned host memory (expand distances on the host
 * with usv_distance_expand_host); flag USV_STREAM_DEVICE_DIST also computes the f64 cm map on
 * the device (fused) and copies it back (8 B/px more over PCIe).  Not thread-safe: one caller
 * thread per stream object (one object per camera pair). */
typedef struct usv_frame_stream usv_frame_stream;
#define USV_STREAM_DEVICE_DIST 1
usv_status usv_frame_stream_create(int W, int H, int D, int w, int metric, int depth, int flags,
                                   usv_frame_stream** out);
usv_status usv_frame_stream_destroy(usv_frame_stream* s);
/* Pinned staging of the slot the NEXT submit uses (dense, pitch W): write the frames there and
 * pass these pointers to submit to skip the host-side copy.  INVALID_ARG while that slot's
 * previous frame has not been released. */
usv_status usv_frame_stream_next_inputs(usv_frame_stream* s, uint8_t** L, uint8_t** R);
/* Enqueue one pair (HOST pointers, row pitch `pitch`); returns at once with *ticket.  Buffers
 * other than the slot's staging are copied into it first.  INVALID_ARG when `depth` frames are
 * still held (release the oldest first). */
usv_status usv_frame_stream_submit(usv_frame_stream* s, const uint8_t* L, const uint8_t* R, int pitch,
                                   long long* ticket);
/* Block until frame `ticket` is done; *disp (and *dist_cm with USV_STREAM_DEVICE_DIST, else pass
 * NULL) point into the slot's pinned host memory, valid until usv_frame_stream_release. */
usv_status usv_frame_stream_wait(usv_frame_stream* s, long long ticket, const uint8_t** disp,
                                 const double** dist_cm);
usv_status usv_frame_stream_release(usv_frame_stream* s, long long ticket);
/* HOST: out[y*out_pitch + x] = lut[disp[y*disp_pitch + x]] over n_threads host threads (0 = 1). */
usv_status usv_distance_expand_host(const uint8_t* disp, int W, int H, int disp_pitch, const double* lut,
                                    double* out, int out_pitch, int n_threads);

/* HOST: lut_out[d] = distance(d) in cm for d = 0..255 (d = 0 -> +inf for model 0). */
usv_status usv_distance_lut_cm(int model, double* lut_out);
/* HOST: the same table in mm (north_star's unit): lut_out[d] = 10 * cm(d). */
usv_status usv_distance_lut_mm(int model, double* lut_out);

/* DEVICE: out[y*out_pitch + x] = lut_cm[disp[y*disp_pitch + x]] (doubles);
 * lut_cm in device or host memory, as for usv_sad_disparity_ex. */
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
 * minAreaRect (OpenCV 3.0 restated) of n int (x,y) points: out5 = {centre.x,
 * centre.y, width, height, angle in degrees}.  P/Main.cpp:1129.
 */
usv_status usv_min_area_rect(const int* pts, int n, float* out5);

/*
 * The centroid step of P/Main.cpp:1120-1143: for each match (in order) whose
 * left_index names one of the n_contours contours (flattened as for
 * usv_generate_matching_list), the centre of that contour's minAreaRect as
 * float (x, y) into out_xy (2*n_matches floats); *n_out gets the count.
 */
usv_status usv_match_centroids(const int* pts, const int* off, int n_contours, const usv_match* matches,
                               int n_matches, float* out_xy, int* n_out);

/*
 * GPU contour matcher (GenerateMatchingList's scores,
 * P/Main.cpp:408-424).  Device pointers, flattened as for
 * usv_generate_matching_list.  usv_contour_descriptors writes n x 8 doubles per
 * contour set: the 7 I1 terms 1/(sign(h) log10|h|) of its Hu invariants (NaN
 * where |h| <= 1e-5) and its unoriented area.  usv_contour_pair_scores writes
 * the n_a x n_b score matrix (i-major) = I1 + |(A_i - A_j)/((A_i + A_j)/2)|;
 * the caller keeps scores < 0.75 in i-major order.
 */
usv_status usv_contour_descriptors(const int* pts, const int* off, int n, double* desc, void* stream);
usv_status usv_contour_pair_scores(const double* desc_a, int n_a, const double* desc_b, int n_b, double* scores,
                                   void* stream);

/*
 * GenerateMatchingList on the device from HOST inputs and into a HOST list (the drop-in form of
 * usv_generate_matching_list; same arguments, same output order and capacity rule, scores equal to
 * the host restatement's within the device log10 rounding).  The matcher object owns pinned staging,
 * device buffers for up to max_contours contours and max_points points per set, and a stream: one call
 * = one H2D copy, five launches (descriptors of each set; one wave per row of the score matrix keeps
 * v < 0.75 and compacts the row in j order with a ballot; the row offsets; the rows gathered into one
 * i-major list), one D2H of the list's length and head (the previous call's length, at least 256
 * entries) and, only when the list is longer, one more D2H of the rest.  max_contours <= 16384; memory:
 * max_contours^2 x 16 B pinned host and twice that on the device.  The current device at create time is
 * the matcher's device; not thread-safe (one object per caller thread).  Replaces the per-pair loop of
 * P/Main.cpp:403-426.
 */
typedef struct usv_contour_matcher usv_contour_matcher;
usv_status usv_contour_matcher_create(int max_contours, int max_points, usv_contour_matcher** out);
usv_status usv_contour_matcher_destroy(usv_contour_matcher* m);
usv_status usv_generate_matching_list_gpu(usv_contour_matcher* m, const int* pts_a, const int* off_a, int n_a,
                                          const int* pts_b, const int* off_b, int n_b, usv_match* out, int cap,
                                          int* n_out);

/*
 * MovingObjectDistanceCalculator over arrays, arguments in the reference's
 * order (P/DistanceCalculator.hpp:37-46).  Points are interleaved float (x, y),
 * triples int (x, y, z), time stamps steady_clock ticks (ns).
 *   interp_in / n_interp_in : the caller's InterpolatedVectorCenter_pointOtherCamera
 *                (by value in the reference; P/Main.cpp passes it empty).  The
 *                reference pushes one extrapolated point per triple onto its copy
 *                and reads element i of the grown vector (P/DistanceCalculator.cpp:67,75-80),
 *                so a non-empty vector shifts which point triple i is measured against.
 * Appends up to n_triples doubles to dist_out; *n_out gets the count;
 * interp_out (nullable, 2*(n_interp_in + n_triples) floats) receives the grown
 * vector: the caller's points, then the extrapolated other-camera centroids.
 */
usv_status usv_moving_object_distance(int camera_side_left, int64_t ts_this,
                                      const float* this_pts, int n_this,
                                      const float* cur_pts, int n_cur,
                                      const float* old_pts, int n_old,
                                      const float* older_pts, int n_older,
                                      const float* interp_in, int n_interp_in,
                                      const int* triples, int n_triples,
                                      int64_t ts_other, int64_t ts_other_old,
                                      int64_t ts_other_older,
                                      double* dist_out, float* interp_out, int* n_out);

/* CooridinatePositionCalculator; xyz_out gets 3 doubles per point. */
usv_status usv_coordinate_position(int camera_side_left, const double* dist, int n_dist,
                                   const float* this_pts, int n_this, int coordinate_display,
                                   double* xyz_out, int* n_out);

/* ---- rectification ---- */

/*
 * HOST: the 25 doubles initUndistortRectifyMap derives from the calibration:
 *   params = {inverse(P[:,0:3] * Rrect) (9, row-major), fx, fy, u0, v0,
 *             k1 k2 p1 p2 k3 k4 k5 k6 s1 s2 s3 s4}
 * K: 3x3 camera matrix; dist: n_dist in {0, 4, 5, 8, 12} coefficients;
 * Rrect: 3x3 rectification rotation (NULL = identity); P: 3 x p_cols (3 or 4)
 * projection / new camera matrix.  All row-major doubles.
 */
usv_status usv_rectify_params(const double* K, const double* dist, int n_dist, const double* Rrect,
                              const double* P, int p_cols, double* params);

/* DEVICE: the CV_16SC2 map1 (W x H x 2 int16) and CV_16UC1 map2 (W x H uint16,
 * (v_frac << 5) | u_frac) for an output of W x H; params is a HOST array. */
usv_status usv_rectify_map(const double* params, int W, int H, int16_t* map1, uint16_t* map2,
                           void* stream);

/* DEVICE: remap INTER_LINEAR / BORDER_CONSTANT(0) of a u8 image with cn = 1 or 3
 * interleaved channels (sW x sH, spitch bytes) through dense maps of W x H. */
usv_status usv_remap_linear_u8(const uint8_t* src, int sW, int sH, int spitch, int cn,
                               const int16_t* map1, const uint16_t* map2, int W, int H,
                               uint8_t* dst, int dpitch, void* stream);

/* DEVICE: both cameras of a pair in one launch (same source / output geometry). */
usv_status usv_rectify_pair_u8(const uint8_t* srcL, const uint8_t* srcR, int sW, int sH, int spitch,
                               int cn, const int16_t* map1L, const uint16_t* map2L,
                               const int16_t* map1R, const uint16_t* map2R, int W, int H,
                               uint8_t* dstL, uint8_t* dstR, int dpitch, void* stream);

/* DEVICE: the map pair above (W x H, for a sW x sH source) packed into ONE uint32 per pixel (4 B
 * instead of 6; bits 0-9 the fraction index, 10-20 sx + 1, 21-31 sy + 1, a pixel with no tap inside
 * the source stored as 2047 / 2047).  Sources of at most 2046 x 2046 (USV_ERR_UNSUPPORTED above).
 * Built once per calibration; remapping through it is bit-identical to remapping through map1/map2
 * and reads a third fewer map bytes per frame (no reference counterpart: the reference rebuilds its
 * map every frame, P/Main.cpp:352). */
usv_status usv_remap_pack_map(const int16_t* map1, const uint16_t* map2, int W, int H, int sW, int sH,
                              uint32_t* pmap, void* stream);

/* DEVICE: usv_remap_linear_u8 / usv_rectify_pair_u8 through packed maps. */
usv_status usv_remap_packed_u8(const uint8_t* src, int sW, int sH, int spitch, int cn, const uint32_t* pmap,
                               int W, int H, uint8_t* dst, int dpitch, void* stream);
usv_status usv_rectify_pair_packed_u8(const uint8_t* srcL, const uint8_t* srcR, int sW, int sH, int spitch,
                                      int cn, const uint32_t* pmapL, const uint32_t* pmapR, int W, int H,
                                      uint8_t* dstL, uint8_t* dstR, int dpitch, void* stream);

/* LDS-tiled form of the packed remap: 64 x 16 output tiles, each tile's source box (precomputed once
 * per packed map by usv_remap_tile_boxes: 2 u32 per tile, ceil(W / 64) * ceil(H / 16) tiles, for
 * `cn` channels) staged in LDS by coalesced loads together with the map; pixels whose taps leave the
 * box take per-tap reads.  Bit-identical to usv_remap_packed_u8 / usv_rectify_pair_packed_u8; the
 * packed map must be 16-byte aligned. */
usv_status usv_remap_tile_boxes(const uint32_t* pmap, int W, int H, int sW, int sH, int cn, uint32_t* boxes,
                                void* stream);
usv_status usv_remap_packed_tiled_u8(const uint8_t* src, int sW, int sH, int spitch, int cn, const uint32_t* pmap,
                                     const uint32_t* boxes, int W, int H, uint8_t* dst, int dpitch, void* stream);
usv_status usv_rectify_pair_packed_tiled_u8(const uint8_t* srcL, const uint8_t* srcR, int sW, int sH, int spitch,
                                            int cn, const uint32_t* pmapL, const uint32_t* pmapR,
                                            const uint32_t* boxesL, const uint32_t* boxesR, int W, int H,
                                            uint8_t* dstL, uint8_t* dstR, int dpitch, void* stream);

/* ---- calibration file: LoadCalibrationData, P/Main.cpp:329-349 ---- */

/* A small dense matrix, row-major doubles (rows = cols = 0: empty, as an unread cv::Mat). */
typedef struct {
    int rows, cols;
    double data[16];
} usv_mat;

/* CalibrationDataParameters (P/Main.cpp:175-180) without the maps, the reference's spellings. */
typedef struct {
    usv_mat intrinsicL, distCoeffsL, intrinsicR, distCoeffsR;
    usv_mat RotationMat, TranslationMat, EssentailMat, FundamentalMat;
    usv_mat RectificationTransformMatL, RectificationTransformMatR, ProjectionMatL, ProjectionMatR,
        Disparity2DepthMappingMat;
} usv_calibration;

/* HOST: read the 13 matrices of an OpenCV FileStorage XML file (opencv_storage
 * root, type_id="opencv-matrix" nodes); absent names stay empty.  At most 16
 * elements per matrix (USV_ERR_UNSUPPORTED otherwise). */
usv_status usv_load_calibration(const char* path, usv_calibration* out);

/* HOST: usv_rectify_params from one camera's four matrices (left != 0: the L
 * set), the arguments of initUndistortRectifyMap at P/Main.cpp:352 / 357. */
usv_status usv_calibration_rectify_params(const usv_calibration* cal, int left, double* params);

/* ---- per-frame colour chain and masks, all DEVICE ---- */

/* Device workspace of the frame preparation: USV_FRAME_PREP_WORK_BYTES bytes
 * (per parity, eight partial 256-bin u32 histograms of V), 4-byte aligned,
 * ZERO-FILLED ONCE by the caller.  Consecutive frames alternate `parity` (0, 1, 0, ...): a call fills
 * histogram `parity` and clears the other one for the next frame.  One
 * workspace per stream in flight. */
#define USV_FRAME_PREP_WORK_BYTES (2 * 8 * 256 * 4)

/* BGR (3 B/px) -> HSV (H in [0,180)) and the 256-bin histogram of V into
 * histogram `parity` of work.  W * H <= 2^24. */
usv_status usv_bgr2hsv_hist_u8(const uint8_t* bgr, int W, int H, int pitch, uint8_t* hsv,
                               int hsv_pitch, void* work, int parity, void* stream);

/* equalizeHist of V from histogram `parity` (V rewritten in hsv), then
 * HSV2BGR into bgr_out and BGR2GRAY into gray. */
usv_status usv_equalize_hsv_bgr_gray_u8(const void* work, int parity, uint8_t* hsv, int W, int H,
                                        int hsv_pitch, uint8_t* bgr_out, int bgr_pitch,
                                        uint8_t* gray, int gray_pitch, void* stream);

/* The reference's frame preparation after rectification: the same outputs as the two calls above, in
 * two launches that do not materialise the intermediate HSV image (a V = max(B, G, R) histogram pass
 * that only reads the frame, then BGR2HSV + equalize + HSV2BGR + BGR2GRAY from the frame: 13 B per
 * pixel instead of 16).  bgr_out may alias bgr. */
usv_status usv_frame_prep_u8(const uint8_t* bgr, int W, int H, int pitch, uint8_t* hsv,
                             int hsv_pitch, uint8_t* bgr_out, int bgr_pitch, uint8_t* gray,
                             int gray_pitch, void* work, int parity, void* stream);

/* Both cameras of a pair in two launches (usv_frame_prep_u8's two passes, each camera with its own
 * half of `work`, which holds 2 * USV_FRAME_PREP_WORK_BYTES bytes). */
usv_status usv_frame_prep_pair_u8(const uint8_t* bgrL, const uint8_t* bgrR, int W, int H, int pitch, uint8_t* hsvL,
                                  uint8_t* hsvR, int hsv_pitch, uint8_t* bgr_outL, uint8_t* bgr_outR, int bgr_pitch,
                                  uint8_t* grayL, uint8_t* grayR, int gray_pitch, void* work, int parity,
                                  void* stream);
/* The whole per-frame stage of a pair in two launches (P/Main.cpp:913-921): rectification (BGR,
 * remap INTER_LINEAR of src with each camera's CV_16SC2 map) fused with BGR2HSV and the histogram,
 * then equalize + HSV2BGR + BGR2GRAY.  Bit-identical to usv_rectify_pair_u8 (cn = 3) followed by
 * usv_frame_prep_pair_u8, without the rectified-BGR intermediate (the reference overwrites it,
 * P/Main.cpp:370).  work: 2 * USV_FRAME_PREP_WORK_BYTES bytes (camera L, then R). */
usv_status usv_rectify_prep_pair_u8(const uint8_t* srcL, const uint8_t* srcR, int sW, int sH, int spitch,
                                    const int16_t* map1L, const uint16_t* map2L, const int16_t* map1R,
                                    const uint16_t* map2R, int W, int H, uint8_t* hsvL, uint8_t* hsvR, int hsv_pitch,
                                    uint8_t* bgr_outL, uint8_t* bgr_outR, int bgr_pitch, uint8_t* grayL,
                                    uint8_t* grayR, int gray_pitch, void* work, int parity, void* stream);
/* The same through packed maps (usv_remap_pack_map). */
usv_status usv_rectify_prep_pair_packed_u8(const uint8_t* srcL, const uint8_t* srcR, int sW, int sH, int spitch,
                                           const uint32_t* pmapL, const uint32_t* pmapR, int W, int H, uint8_t* hsvL,
                                           uint8_t* hsvR, int hsv_pitch, uint8_t* bgr_outL, uint8_t* bgr_outR,
                                           int bgr_pitch, uint8_t* grayL, uint8_t* grayR, int gray_pitch, void* work,
                                           int parity, void* stream);

/* |gray - prev| > thresh -> 255, then erode + dilate with the 5x5 ellipse
 * (gray and prev share pitch). */
usv_status usv_motion_mask_u8(const uint8_t* gray, const uint8_t* prev, int W, int H, int pitch,
                              int thresh, uint8_t* mask, int mask_pitch, void* stream);

/* inRange(hsv, lo1, hi1) | inRange(hsv, lo2, hi2), then erode + dilate (5x5
 * ellipse).  lo/hi: HOST arrays of 3 ints (H, S, V), inclusive. */
usv_status usv_colour_mask_u8(const uint8_t* hsv, int W, int H, int pitch, const int* lo1,
                              const int* hi1, const int* lo2, const int* hi2, uint8_t* mask,
                              int mask_pitch, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* USV_H */
