/*
 * shape_oracle.c -- CPU ORACLE (test infrastructure only; see usv_oracle.h).
 *
 * the OpenCV 3.0.0 functions the reference
 * calls on its contour path, restated in plain C from OpenCV 3.0.0's published
 * algorithms (the library is absent from the image and is a third-party
 * dependency of the reference: opencv_world300, P/Unsynchronized_Stereo_Vision_Proj325.vcxproj:97,136):
 *
 *   GenerateMatchingList  P/Main.cpp:403-426 -- per (i, j) pair, as the reference
 *                         does it: matchShapes(c1, c2, CONTOURS_MATCH_I1, 0)
 *                         + |(A_i - A_j) / ((A_i + A_j) / 2)|, kept if < 0.75.
 *     matchShapes         imgproc/src/contours.cpp (3.0.0): HuMoments(moments(c)),
 *                         method 1 = sum |1/(s_b log10|h_b|) - 1/(s_a log10|h_a|)|
 *                         over terms with |h| > 1e-5 on both sides.
 *     moments             imgproc/src/moments.cpp contourMoments (Green's theorem
 *                         sums a00..a03 in double, scaled by +-1/2, 1/6, 1/12,
 *                         1/24, 1/20, 1/60 by the sign of a00, zero when
 *                         |a00| <= FLT_EPSILON) + completeMomentState.
 *     HuMoments           imgproc/src/moments.cpp.
 *     contourArea         imgproc/src/shapedescr.cpp: float points, double
 *                         cross products, * 0.5, fabs (oriented = false).
 *   centre points         P/Main.cpp:1120-1143: minAreaRect, RotatedRect::points,
 *                         Point2f sum of the 4 corners, /= 4.
 *     convexHull          imgproc/src/convhull.cpp: pointers sorted by (x, y),
 *                         Sklansky's scan (int coordinates, int64 cross product)
 *                         on the upper and lower halves, clockwise, points.
 *     minAreaRect         imgproc/src/rotcalipers.cpp: hull as float points,
 *                         rotatingCalipers(CALIPERS_MINAREARECT) in float.
 *     RotatedRect::points core/src/matrix.cpp (3.0.0).
 *
 * Written independently of csrc/host/ (the product) from those algorithms; the
 * tests compare the product's host C++ and its GPU contour kernels against this
 * file.  Parity vs OpenCV itself stays UNPINNED: neither OpenCV nor any output
 * of it exists in this image or in the reference repository (it has no tests
 * and no fixtures).  Built with -ffp-contract=off.
 */
#include "usv_oracle.h"

#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---- moments / Hu / I1 / area -------------------------------------------- */

typedef struct {
    double m00, m10, m01, m20, m11, m02, m30, m21, m12, m03;
    double mu20, mu11, mu02, mu30, mu21, mu12, mu03;
    double nu20, nu11, nu02, nu30, nu21, nu12, nu03;
} moments_t;

static void complete_moment_state(moments_t* m) {
    double cx = 0, cy = 0, inv_m00 = 0;
    if (fabs(m->m00) > DBL_EPSILON) {
        inv_m00 = 1. / m->m00;
        cx = m->m10 * inv_m00;
        cy = m->m01 * inv_m00;
    }
    double mu20 = m->m20 - m->m10 * cx;
    double mu11 = m->m11 - m->m10 * cy;
    double mu02 = m->m02 - m->m01 * cy;
    m->mu20 = mu20;
    m->mu11 = mu11;
    m->mu02 = mu02;
    m->mu30 = m->m30 - cx * (3 * mu20 + cx * m->m10);
    mu11 += mu11;
    m->mu21 = m->m21 - cx * (mu11 + cx * m->m01) - cy * mu20;
    m->mu12 = m->m12 - cy * (mu11 + cy * m->m10) - cx * mu02;
    m->mu03 = m->m03 - cy * (3 * mu02 + cy * m->m01);
    double inv_sqrt_m00 = sqrt(fabs(inv_m00));
    double s2 = inv_m00 * inv_m00, s3 = s2 * inv_sqrt_m00;
    m->nu20 = m->mu20 * s2;
    m->nu11 = m->mu11 * s2;
    m->nu02 = m->mu02 * s2;
    m->nu30 = m->mu30 * s3;
    m->nu21 = m->mu21 * s3;
    m->nu12 = m->mu12 * s3;
    m->nu03 = m->mu03 * s3;
}

static moments_t contour_moments(const int* pts, int lpt) {
    moments_t m;
    memset(&m, 0, sizeof(m));
    if (lpt <= 0) return m;
    double a00 = 0, a10 = 0, a01 = 0, a20 = 0, a11 = 0, a02 = 0, a30 = 0, a21 = 0, a12 = 0, a03 = 0;
    double xi, yi, xi2, yi2, xi_1, yi_1, xi_12, yi_12, dxy, xii_1, yii_1;
    xi_1 = pts[2 * (lpt - 1)];
    yi_1 = pts[2 * (lpt - 1) + 1];
    xi_12 = xi_1 * xi_1;
    yi_12 = yi_1 * yi_1;
    for (int i = 0; i < lpt; i++) {
        xi = pts[2 * i];
        yi = pts[2 * i + 1];
        xi2 = xi * xi;
        yi2 = yi * yi;
        dxy = xi_1 * yi - xi * yi_1;
        xii_1 = xi_1 + xi;
        yii_1 = yi_1 + yi;
        a00 += dxy;
        a10 += dxy * xii_1;
        a01 += dxy * yii_1;
        a20 += dxy * (xi_1 * xii_1 + xi2);
        a11 += dxy * (xi_1 * (yii_1 + yi_1) + xi * (yii_1 + yi));
        a02 += dxy * (yi_1 * yii_1 + yi2);
        a30 += dxy * xii_1 * (xi_12 + xi2);
        a03 += dxy * yii_1 * (yi_12 + yi2);
        a21 += dxy * (xi_12 * (3 * yi_1 + yi) + 2 * xi * xi_1 * yii_1 + xi2 * (yi_1 + 3 * yi));
        a12 += dxy * (yi_12 * (3 * xi_1 + xi) + 2 * yi * yi_1 * xii_1 + yi2 * (xi_1 + 3 * xi));
        xi_1 = xi;
        yi_1 = yi;
        xi_12 = xi2;
        yi_12 = yi2;
    }
    if (fabs(a00) > FLT_EPSILON) {
        double db1_2, db1_6, db1_12, db1_24, db1_20, db1_60;
        if (a00 > 0) {
            db1_2 = 0.5;
            db1_6 = 0.16666666666666666666666666666667;
            db1_12 = 0.083333333333333333333333333333333;
            db1_24 = 0.041666666666666666666666666666667;
            db1_20 = 0.05;
            db1_60 = 0.016666666666666666666666666666667;
        } else {
            db1_2 = -0.5;
            db1_6 = -0.16666666666666666666666666666667;
            db1_12 = -0.083333333333333333333333333333333;
            db1_24 = -0.041666666666666666666666666666667;
            db1_20 = -0.05;
            db1_60 = -0.016666666666666666666666666666667;
        }
        m.m00 = a00 * db1_2;
        m.m10 = a10 * db1_6;
        m.m01 = a01 * db1_6;
        m.m20 = a20 * db1_12;
        m.m11 = a11 * db1_24;
        m.m02 = a02 * db1_12;
        m.m30 = a30 * db1_20;
        m.m21 = a21 * db1_60;
        m.m12 = a12 * db1_60;
        m.m03 = a03 * db1_20;
        complete_moment_state(&m);
    }
    return m;
}

static void hu_moments(const moments_t* m, double hu[7]) {
    double t0 = m->nu30 + m->nu12;
    double t1 = m->nu21 + m->nu03;
    double q0 = t0 * t0, q1 = t1 * t1;
    double n4 = 4 * m->nu11;
    double s = m->nu20 + m->nu02;
    double d = m->nu20 - m->nu02;
    hu[0] = s;
    hu[1] = d * d + n4 * m->nu11;
    hu[3] = q0 + q1;
    hu[5] = d * (q0 - q1) + n4 * t0 * t1;
    t0 *= q0 - 3 * q1;
    t1 *= 3 * q0 - q1;
    q0 = m->nu30 - 3 * m->nu12;
    q1 = 3 * m->nu21 - m->nu03;
    hu[2] = q0 * q0 + q1 * q1;
    hu[4] = q0 * t0 + q1 * t1;
    hu[6] = q1 * t0 - q0 * t1;
}

void usv_oracle_hu_moments(const int* pts, int n, double* hu7) {
    moments_t m = contour_moments(pts, n);
    hu_moments(&m, hu7);
}

double usv_oracle_match_shapes_i1(const int* pts_a, int n_a, const int* pts_b, int n_b) {
    double ma[7], mb[7];
    double eps = 1.e-5, result = 0;
    usv_oracle_hu_moments(pts_a, n_a, ma);
    usv_oracle_hu_moments(pts_b, n_b, mb);
    for (int i = 0; i < 7; i++) {
        double ama = fabs(ma[i]);
        double amb = fabs(mb[i]);
        int sma = ma[i] > 0 ? 1 : (ma[i] < 0 ? -1 : 0);
        int smb = mb[i] > 0 ? 1 : (mb[i] < 0 ? -1 : 0);
        if (ama > eps && amb > eps) {
            ama = 1. / (sma * log10(ama));
            amb = 1. / (smb * log10(amb));
            result += fabs(-ama + amb);
        }
    }
    return result;
}

double usv_oracle_contour_area(const int* pts, int npoints) {
    if (npoints <= 0) return 0.;
    double a00 = 0;
    float prev_x = (float)pts[2 * (npoints - 1)], prev_y = (float)pts[2 * (npoints - 1) + 1];
    for (int i = 0; i < npoints; i++) {
        float px = (float)pts[2 * i], py = (float)pts[2 * i + 1];
        a00 += (double)prev_x * py - (double)prev_y * px;
        prev_x = px;
        prev_y = py;
    }
    a00 *= 0.5;
    return fabs(a00);
}

/* P/Main.cpp:403-426, every score recomputed per pair exactly as the reference does */
int usv_oracle_generate_matching_list(const int* pts_a, const int* off_a, int n_a, const int* pts_b,
                                      const int* off_b, int n_b, usv_oracle_match* out) {
    int n = 0;
    if (n_a <= 0 || n_b <= 0) return 0; /* line 405: both lists non-empty */
    for (int i = 0; i < n_a; i++) {
        const int* ca = pts_a + 2 * off_a[i];
        int na = off_a[i + 1] - off_a[i];
        for (int j = 0; j < n_b; j++) {
            const int* cb = pts_b + 2 * off_b[j];
            int nb = off_b[j + 1] - off_b[j];
            double v = usv_oracle_match_shapes_i1(ca, na, cb, nb);                            /* line 413 */
            v = v + fabs((usv_oracle_contour_area(ca, na) - usv_oracle_contour_area(cb, nb)) /
                         ((usv_oracle_contour_area(ca, na) + usv_oracle_contour_area(cb, nb)) / 2)); /* line 414 */
            if (v < 0.75) {                                                                   /* line 417 */
                out[n].left = (unsigned)i;
                out[n].right = (unsigned)j;
                out[n].value = v;
                n++;
            }
        }
    }
    return n;
}

/* ---- convexHull (clockwise, points) -------------------------------------- */

static const int* g_sort_pts; /* qsort has no context argument; the oracle is single-threaded */

static int cmp_xy(const void* a, const void* b) {
    const int* p = g_sort_pts + 2 * *(const int*)a;
    const int* q = g_sort_pts + 2 * *(const int*)b;
    if (p[0] != q[0]) return p[0] < q[0] ? -1 : 1;
    if (p[1] != q[1]) return p[1] < q[1] ? -1 : 1;
    return 0;
}

static int sgn64(int64_t v) { return (v > 0) - (v < 0); }

/* Sklansky_<int, int64>; ptr[k] = index of the k-th sorted point */
static int sklansky_int(const int* pts, const int* ptr, int start, int end, int* stack, int nsign, int sign2) {
#define PX(k) pts[2 * ptr[k]]
#define PY(k) pts[2 * ptr[k] + 1]
    int incr = end > start ? 1 : -1;
    int pprev = start, pcur = pprev + incr, pnext = pcur + incr;
    int stacksize = 3;
    if (start == end || (PX(start) == PX(end) && PY(start) == PY(end))) {
        stack[0] = start;
        return 1;
    }
    stack[0] = pprev;
    stack[1] = pcur;
    stack[2] = pnext;
    end += incr;
    while (pnext != end) {
        int cury = PY(pcur);
        int nexty = PY(pnext);
        int by = nexty - cury;
        if (sgn64(by) != nsign) {
            int ax = PX(pcur) - PX(pprev);
            int bx = PX(pnext) - PX(pcur);
            int ay = cury - PY(pprev);
            int64_t convexity = (int64_t)ay * bx - (int64_t)ax * by;
            if (sgn64(convexity) == sign2 && (pprev != start || pcur != end)) {
                pprev = pcur;
                pcur = pnext;
                pnext += incr;
                stack[stacksize] = pnext;
                stacksize++;
            } else {
                if (pprev == start) {
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
            }
        } else {
            pnext += incr;
            stack[stacksize - 1] = pnext;
        }
    }
#undef PX
#undef PY
    return --stacksize;
}

int usv_oracle_convex_hull_cw(const int* pts, int total, int* hull_xy) {
    if (total <= 0) return 0;
    int* ptr = (int*)malloc(sizeof(int) * (size_t)total);
    int* stack = (int*)malloc(sizeof(int) * ((size_t)total + 2));
    int* hullbuf = (int*)malloc(sizeof(int) * (size_t)total);
    int nout = 0, miny_ind = 0, maxy_ind = 0;
    for (int i = 0; i < total; i++) ptr[i] = i;
    g_sort_pts = pts;
    qsort(ptr, (size_t)total, sizeof(int), cmp_xy);
    for (int i = 1; i < total; i++) {
        int y = pts[2 * ptr[i] + 1];
        if (pts[2 * ptr[miny_ind] + 1] > y) miny_ind = i;
        if (pts[2 * ptr[maxy_ind] + 1] < y) maxy_ind = i;
    }
    const int first = ptr[0], last = ptr[total - 1];
    if (pts[2 * first] == pts[2 * last] && pts[2 * first + 1] == pts[2 * last + 1]) {
        hullbuf[nout++] = ptr[0];
    } else {
        int* tl_stack = stack;
        int tl_count = sklansky_int(pts, ptr, 0, maxy_ind, tl_stack, -1, 1);
        int* tr_stack = stack + tl_count;
        int tr_count = sklansky_int(pts, ptr, total - 1, maxy_ind, tr_stack, -1, -1);
        /* clockwise: no swap of the upper chains */
        for (int i = 0; i < tl_count - 1; i++) hullbuf[nout++] = ptr[tl_stack[i]];
        for (int i = tr_count - 1; i > 0; i--) hullbuf[nout++] = ptr[tr_stack[i]];
        int stop_idx = tr_count > 2 ? tr_stack[1] : tl_count > 2 ? tl_stack[tl_count - 2] : -1;
        int* bl_stack = stack;
        int bl_count = sklansky_int(pts, ptr, 0, miny_ind, bl_stack, 1, -1);
        int* br_stack = stack + bl_count;
        int br_count = sklansky_int(pts, ptr, total - 1, miny_ind, br_stack, 1, 1);
        { /* clockwise: swap the lower chains */
            int* ts = bl_stack; bl_stack = br_stack; br_stack = ts;
            int tc = bl_count; bl_count = br_count; br_count = tc;
        }
        if (stop_idx >= 0) {
            int check_idx = bl_count > 2 ? bl_stack[1] : bl_count + br_count > 2 ? br_stack[2 - bl_count] : -1;
            if (check_idx == stop_idx ||
                (check_idx >= 0 && pts[2 * ptr[check_idx]] == pts[2 * ptr[stop_idx]] &&
                 pts[2 * ptr[check_idx] + 1] == pts[2 * ptr[stop_idx] + 1])) {
                bl_count = bl_count < 2 ? bl_count : 2;
                br_count = br_count < 2 ? br_count : 2;
            }
        }
        for (int i = 0; i < bl_count - 1; i++) hullbuf[nout++] = ptr[bl_stack[i]];
        for (int i = br_count - 1; i > 0; i--) hullbuf[nout++] = ptr[br_stack[i]];
    }
    for (int i = 0; i < nout; i++) {
        hull_xy[2 * i] = pts[2 * hullbuf[i]];
        hull_xy[2 * i + 1] = pts[2 * hullbuf[i] + 1];
    }
    free(ptr);
    free(stack);
    free(hullbuf);
    return nout;
}

/* ---- rotatingCalipers(CALIPERS_MINAREARECT) + minAreaRect ---------------- */

static void rotating_calipers_minarea(const float* points, int n, float* out) {
    float minarea = FLT_MAX;
    float buf[7];
    int buf_left = 0, buf_bottom = 0;
    float* inv_vect_length = (float*)malloc(sizeof(float) * (size_t)n);
    float* vect = (float*)malloc(sizeof(float) * 2 * (size_t)n);
    int left = 0, bottom = 0, right = 0, top = 0;
    int seq[4];
    float orientation = 0, base_a, base_b = 0;
    float left_x, right_x, top_y, bottom_y;
    float pt0x = points[0], pt0y = points[1];
    memset(buf, 0, sizeof(buf));
    left_x = right_x = pt0x;
    top_y = bottom_y = pt0y;
    for (int i = 0; i < n; i++) {
        double dx, dy;
        if (pt0x < left_x) left_x = pt0x, left = i;
        if (pt0x > right_x) right_x = pt0x, right = i;
        if (pt0y > top_y) top_y = pt0y, top = i;
        if (pt0y < bottom_y) bottom_y = pt0y, bottom = i;
        int nx = (i + 1) & (i + 1 < n ? -1 : 0);
        float ptx = points[2 * nx], pty = points[2 * nx + 1];
        dx = ptx - pt0x;
        dy = pty - pt0y;
        vect[2 * i] = (float)dx;
        vect[2 * i + 1] = (float)dy;
        inv_vect_length[i] = (float)(1. / sqrt(dx * dx + dy * dy));
        pt0x = ptx;
        pt0y = pty;
    }
    {
        double ax = vect[2 * (n - 1)], ay = vect[2 * (n - 1) + 1];
        for (int i = 0; i < n; i++) {
            double bx = vect[2 * i], by = vect[2 * i + 1];
            double convexity = ax * by - ay * bx;
            if (convexity != 0) {
                orientation = (convexity > 0) ? 1.f : (-1.f);
                break;
            }
            ax = bx;
            ay = by;
        }
    }
    base_a = orientation;
    seq[0] = bottom;
    seq[1] = right;
    seq[2] = top;
    seq[3] = left;
    for (int k = 0; k < n; k++) {
        float dp[4];
        dp[0] = +base_a * vect[2 * seq[0]] + base_b * vect[2 * seq[0] + 1];
        dp[1] = -base_b * vect[2 * seq[1]] + base_a * vect[2 * seq[1] + 1];
        dp[2] = -base_a * vect[2 * seq[2]] - base_b * vect[2 * seq[2] + 1];
        dp[3] = +base_b * vect[2 * seq[3]] - base_a * vect[2 * seq[3] + 1];
        float maxcos = dp[0] * inv_vect_length[seq[0]];
        int main_element = 0;
        for (int i = 1; i < 4; ++i) {
            float cosalpha = dp[i] * inv_vect_length[seq[i]];
            if (cosalpha > maxcos) {
                main_element = i;
                maxcos = cosalpha;
            }
        }
        {
            int pindex = seq[main_element];
            float lead_x = vect[2 * pindex] * inv_vect_length[pindex];
            float lead_y = vect[2 * pindex + 1] * inv_vect_length[pindex];
            switch (main_element) {
                case 0: base_a = lead_x; base_b = lead_y; break;
                case 1: base_a = lead_y; base_b = -lead_x; break;
                case 2: base_a = -lead_x; base_b = -lead_y; break;
                default: base_a = -lead_y; base_b = lead_x; break;
            }
        }
        seq[main_element] += 1;
        seq[main_element] = (seq[main_element] == n) ? 0 : seq[main_element];
        {
            float height, area;
            float dx = points[2 * seq[1]] - points[2 * seq[3]];
            float dy = points[2 * seq[1] + 1] - points[2 * seq[3] + 1];
            float width = dx * base_a + dy * base_b;
            dx = points[2 * seq[2]] - points[2 * seq[0]];
            dy = points[2 * seq[2] + 1] - points[2 * seq[0] + 1];
            height = -dx * base_b + dy * base_a;
            area = width * height;
            if (area <= minarea) {
                minarea = area;
                buf_left = seq[3];
                buf[1] = base_a;
                buf[2] = width;
                buf[3] = base_b;
                buf[4] = height;
                buf_bottom = seq[0];
                buf[6] = area;
            }
        }
    }
    {
        float A1 = buf[1], B1 = buf[3];
        float A2 = -buf[3], B2 = buf[1];
        float C1 = A1 * points[2 * buf_left] + points[2 * buf_left + 1] * B1;
        float C2 = A2 * points[2 * buf_bottom] + points[2 * buf_bottom + 1] * B2;
        float idet = 1.f / (A1 * B2 - A2 * B1);
        float px = (C1 * B2 - C2 * B1) * idet;
        float py = (A1 * C2 - A2 * C1) * idet;
        out[0] = px;
        out[1] = py;
        out[2] = A1 * buf[2];
        out[3] = B1 * buf[2];
        out[4] = A2 * buf[4];
        out[5] = B2 * buf[4];
    }
    free(inv_vect_length);
    free(vect);
}

/* out5 = {center.x, center.y, size.width, size.height, angle (degrees)} */
int usv_oracle_min_area_rect(const int* pts, int npts, float* out5) {
    float cx = 0, cy = 0, w = 0, h = 0, angle = 0;
    int* hull = (int*)malloc(sizeof(int) * 2 * (size_t)(npts > 0 ? npts : 1));
    int n = usv_oracle_convex_hull_cw(pts, npts, hull);
    float* hp = (float*)malloc(sizeof(float) * 2 * (size_t)(n > 0 ? n : 1));
    for (int i = 0; i < 2 * n; i++) hp[i] = (float)hull[i]; /* hull.convertTo(CV_32F) */
    if (n > 2) {
        float o[6];
        rotating_calipers_minarea(hp, n, o);
        cx = o[0] + (o[2] + o[4]) * 0.5f;
        cy = o[1] + (o[3] + o[5]) * 0.5f;
        w = (float)sqrt((double)o[2] * o[2] + (double)o[3] * o[3]);
        h = (float)sqrt((double)o[4] * o[4] + (double)o[5] * o[5]);
        angle = (float)atan2((double)o[3], (double)o[2]);
    } else if (n == 2) {
        cx = (hp[0] + hp[2]) * 0.5f;
        cy = (hp[1] + hp[3]) * 0.5f;
        double dx = hp[2] - hp[0];
        double dy = hp[3] - hp[1];
        w = (float)sqrt(dx * dx + dy * dy);
        h = 0;
        angle = (float)atan2(dy, dx);
    } else if (n == 1) {
        cx = hp[0];
        cy = hp[1];
    }
    angle = (float)(angle * 180 / 3.1415926535897932384626433832795); /* CV_PI */
    out5[0] = cx;
    out5[1] = cy;
    out5[2] = w;
    out5[3] = h;
    out5[4] = angle;
    free(hull);
    free(hp);
    return n;
}

/* RotatedRect::points: 4 corners as 8 floats */
void usv_oracle_rect_points(const float* r5, float* pt8) {
    double _angle = r5[4] * 3.1415926535897932384626433832795 / 180.;
    float b = (float)cos(_angle) * 0.5f;
    float a = (float)sin(_angle) * 0.5f;
    float cx = r5[0], cy = r5[1], w = r5[2], h = r5[3];
    pt8[0] = cx - a * h - b * w;
    pt8[1] = cy + b * h - a * w;
    pt8[2] = cx + a * h - b * w;
    pt8[3] = cy - b * h - a * w;
    pt8[4] = 2 * cx - pt8[0];
    pt8[5] = 2 * cy - pt8[1];
    pt8[6] = 2 * cx - pt8[2];
    pt8[7] = 2 * cy - pt8[3];
}

/* P/Main.cpp:1120-1143: per tentative match, Σ corners (Point2f +=) then /= 4 */
int usv_oracle_match_centroids(const int* pts, const int* off, int n_contours, const usv_oracle_match* matches,
                               int n_matches, float* out_xy) {
    int n = 0;
    for (int m = 0; m < n_matches; m++) {
        unsigned li = matches[m].left;
        if (li >= (unsigned)n_contours) continue; /* out of range is UB in the reference; skipped here */
        float r[5], c[8], sx = 0.f, sy = 0.f;
        usv_oracle_min_area_rect(pts + 2 * off[li], off[li + 1] - off[li], r);
        usv_oracle_rect_points(r, c);
        for (int j = 0; j < 4; j++) {
            sx = sx + c[2 * j];
            sy = sy + c[2 * j + 1];
        }
        out_xy[2 * n] = sx / 4;
        out_xy[2 * n + 1] = sy / 4;
        n++;
    }
    return n;
}
