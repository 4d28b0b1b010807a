/*
 * preproc_oracle.c -- CPU ORACLE (test infrastructure only; see usv_oracle.h).
 *
 * the per-frame colour chain and masks the reference
 * runs on every rectified frame, u8 semantics of OpenCV 3.0.0 restated from
 * its published sources (imgproc/color.cpp RGB2HSV_b / HSV2RGB_b / RGB2Gray,
 * imgproc/histogram.cpp equalizeHist, imgproc/thresh.cpp, imgproc/morph.cpp,
 * core/arithm.cpp absdiff / inRange / addWeighted).  OpenCV is not in this
 * image and the reference has no fixtures for these calls: PARITY UNPINNED
 * against OpenCV (the IPP-accelerated paths of an OpenCV build may round
 * differently; the plain C++ paths are what is restated).  The GPU kernels
 * (csrc/usv_preproc.hip) must equal this file bit for bit.
 *
 *   frame prep (P/Main.cpp:919-921 with LightingCorrection P/Main.cpp:365-371):
 *     hsv  = BGR2HSV(bgr)                         (H in [0,180), hsv_shift 12 tables)
 *     V'   = equalizeHist(V)                      (float scale, cvRound)
 *     hsv' = (H, S, V')                           (merge writes through the shared Mat)
 *     bgr' = HSV2BGR(hsv')                        (float path, cvRound)
 *     gray = BGR2GRAY(bgr')                       ((1868 B + 9617 G + 4899 R + 8192) >> 14)
 *   motion mask (ABSDiffSearch P/Main.cpp:299-312 + MorphilogicalFilter :289-292):
 *     m = absdiff(gray, prev) > 40 ? 255 : 0; erode(ellipse 5x5); dilate(ellipse 5x5)
 *   colour mask (ColourSearch P/Main.cpp:318-327):
 *     m = inRange(hsv, lo1, hi1) + inRange(hsv, lo2, hi2) (saturating); erode; dilate
 *   Morphology borders: OpenCV's default border value for erode / dilate is
 *   +/-infinity, i.e. pixels outside the image never win the min / max.
 *   Ellipse 5x5 (getStructuringElement MORPH_ELLIPSE): rows 0 and 4 hold only
 *   the centre column, rows 1-3 all five columns.
 */
#include "usv_oracle.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static int sat_u8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

void usv_oracle_bgr2hsv(const uint8_t* bgr, int W, int H, int pitch, uint8_t* hsv, int hsv_pitch) {
    enum { hsv_shift = 12 };
    int sdiv[256], hdiv[256];
    sdiv[0] = hdiv[0] = 0;
    for (int i = 1; i < 256; ++i) {
        sdiv[i] = (int)lrint((255 << hsv_shift) / (1. * i));
        hdiv[i] = (int)lrint((180 << hsv_shift) / (6. * i));
    }
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const uint8_t* s = bgr + (size_t)y * pitch + 3 * (size_t)x;
            const int b = s[0], g = s[1], r = s[2];
            int v = b, vmin = b;
            if (g > v) v = g;
            if (r > v) v = r;
            if (g < vmin) vmin = g;
            if (r < vmin) vmin = r;
            const int diff = v - vmin;
            const int vr = v == r ? -1 : 0, vg = v == g ? -1 : 0;
            const int sat = (diff * sdiv[v] + (1 << (hsv_shift - 1))) >> hsv_shift;
            int h = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + ((~vg) & (r - g + 4 * diff))));
            h = (h * hdiv[diff] + (1 << (hsv_shift - 1))) >> hsv_shift;
            h += h < 0 ? 180 : 0;
            uint8_t* d = hsv + (size_t)y * hsv_pitch + 3 * (size_t)x;
            d[0] = (uint8_t)sat_u8(h);
            d[1] = (uint8_t)sat;
            d[2] = (uint8_t)v;
        }
}

/* equalizeHist LUT from a 256-bin histogram of `total` pixels (lut entries below the first
 * occupied bin are never read; they are set to 0). */
void usv_oracle_equalize_lut(const uint32_t* hist, int total, uint8_t* lut) {
    memset(lut, 0, 256);
    int i = 0;
    while (i < 256 && !hist[i]) ++i;
    if (i == 256) return;
    if ((int)hist[i] == total) {
        lut[i] = (uint8_t)i; /* dst.setTo(i) */
        return;
    }
    const float scale = (256 - 1.f) / (total - (int)hist[i]);
    int sum = 0;
    for (lut[i++] = 0; i < 256; ++i) {
        sum += (int)hist[i];
        lut[i] = (uint8_t)sat_u8((int)lrintf(sum * scale));
    }
}

static void hsv2bgr_px(int H8, int S8, int V8, uint8_t* out) {
    float h = (float)H8, s = S8 * (1.f / 255.f), v = V8 * (1.f / 255.f);
    float b, g, r;
    if (s == 0) {
        b = g = r = v;
    } else {
        static const int sector_data[][3] = {{1, 3, 0}, {1, 0, 2}, {3, 0, 1}, {0, 2, 1}, {0, 1, 3}, {2, 1, 0}};
        float tab[4];
        const float hscale = 6.f / 180;
        h *= hscale;
        if (h < 0)
            do h += 6; while (h < 0);
        else if (h >= 6)
            do h -= 6; while (h >= 6);
        int sector = (int)floorf(h);
        h -= sector;
        if ((unsigned)sector >= 6u) {
            sector = 0;
            h = 0.f;
        }
        tab[0] = v;
        tab[1] = v * (1.f - s);
        tab[2] = v * (1.f - s * h);
        tab[3] = v * (1.f - s * (1.f - h));
        b = tab[sector_data[sector][0]];
        g = tab[sector_data[sector][1]];
        r = tab[sector_data[sector][2]];
    }
    out[0] = (uint8_t)sat_u8((int)lrintf(b * 255.f));
    out[1] = (uint8_t)sat_u8((int)lrintf(g * 255.f));
    out[2] = (uint8_t)sat_u8((int)lrintf(r * 255.f));
}

void usv_oracle_hsv2bgr(const uint8_t* hsv, int W, int H, int pitch, uint8_t* bgr, int bgr_pitch) {
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const uint8_t* s = hsv + (size_t)y * pitch + 3 * (size_t)x;
            hsv2bgr_px(s[0], s[1], s[2], bgr + (size_t)y * bgr_pitch + 3 * (size_t)x);
        }
}

void usv_oracle_bgr2gray(const uint8_t* bgr, int W, int H, int pitch, uint8_t* gray, int gray_pitch) {
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const uint8_t* s = bgr + (size_t)y * pitch + 3 * (size_t)x;
            gray[(size_t)y * gray_pitch + x] = (uint8_t)((s[0] * 1868 + s[1] * 9617 + s[2] * 4899 + (1 << 13)) >> 14);
        }
}

int usv_oracle_frame_prep(const uint8_t* bgr, int W, int H, int pitch, uint8_t* hsv_out, uint8_t* bgr_out,
                          uint8_t* gray_out) {
    /* outputs are dense: hsv / bgr pitch 3W, gray pitch W */
    if (!bgr || !hsv_out || !bgr_out || !gray_out || W <= 0 || H <= 0 || pitch < 3 * W) return -1;
    usv_oracle_bgr2hsv(bgr, W, H, pitch, hsv_out, 3 * W);
    uint32_t hist[256] = {0};
    for (size_t p = 0; p < (size_t)W * H; ++p) hist[hsv_out[3 * p + 2]]++;
    uint8_t lut[256];
    usv_oracle_equalize_lut(hist, W * H, lut);
    for (size_t p = 0; p < (size_t)W * H; ++p) hsv_out[3 * p + 2] = lut[hsv_out[3 * p + 2]];
    usv_oracle_hsv2bgr(hsv_out, W, H, 3 * W, bgr_out, 3 * W);
    usv_oracle_bgr2gray(bgr_out, W, H, 3 * W, gray_out, W);
    return 0;
}

/* 5x5 ellipse footprint: (dy, dx) offsets */
static const int kEll[17][2] = {{-2, 0},  {-1, -2}, {-1, -1}, {-1, 0}, {-1, 1}, {-1, 2}, {0, -2}, {0, -1}, {0, 0},
                                {0, 1},   {0, 2},   {1, -2},  {1, -1}, {1, 0},  {1, 1},  {1, 2},  {2, 0}};

static void morph_ellipse5(const uint8_t* in, int W, int H, uint8_t* out, int is_erode) {
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            int acc = is_erode ? 255 : 0;
            for (int k = 0; k < 17; ++k) {
                const int yy = y + kEll[k][0], xx = x + kEll[k][1];
                if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue; /* border never wins */
                const int v = in[(size_t)yy * W + xx];
                if (is_erode ? v < acc : v > acc) acc = v;
            }
            out[(size_t)y * W + x] = (uint8_t)acc;
        }
}

static int finish_mask(uint8_t* t, int W, int H, uint8_t* mask, int mask_pitch) {
    uint8_t* e = (uint8_t*)malloc((size_t)W * H);
    uint8_t* d = (uint8_t*)malloc((size_t)W * H);
    if (!e || !d) {
        free(e);
        free(d);
        return -2;
    }
    morph_ellipse5(t, W, H, e, 1);
    morph_ellipse5(e, W, H, d, 0);
    for (int y = 0; y < H; ++y) memcpy(mask + (size_t)y * mask_pitch, d + (size_t)y * W, (size_t)W);
    free(e);
    free(d);
    return 0;
}

int usv_oracle_motion_mask(const uint8_t* gray, const uint8_t* prev, int W, int H, int pitch, int thresh,
                           uint8_t* mask, int mask_pitch) {
    if (!gray || !prev || !mask || W <= 0 || H <= 0 || pitch < W || mask_pitch < W) return -1;
    uint8_t* t = (uint8_t*)malloc((size_t)W * H);
    if (!t) return -2;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const int a = gray[(size_t)y * pitch + x], b = prev[(size_t)y * pitch + x];
            t[(size_t)y * W + x] = (uint8_t)((a > b ? a - b : b - a) > thresh ? 255 : 0);
        }
    const int rc = finish_mask(t, W, H, mask, mask_pitch);
    free(t);
    return rc;
}

int usv_oracle_colour_mask(const uint8_t* hsv, int W, int H, int pitch, const int* lo1, const int* hi1,
                           const int* lo2, const int* hi2, uint8_t* mask, int mask_pitch) {
    if (!hsv || !lo1 || !hi1 || !lo2 || !hi2 || !mask || W <= 0 || H <= 0 || pitch < 3 * W || mask_pitch < W)
        return -1;
    uint8_t* t = (uint8_t*)malloc((size_t)W * H);
    if (!t) return -2;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const uint8_t* s = hsv + (size_t)y * pitch + 3 * (size_t)x;
            int a = 255, b = 255;
            for (int c = 0; c < 3; ++c) {
                if (s[c] < lo1[c] || s[c] > hi1[c]) a = 0;
                if (s[c] < lo2[c] || s[c] > hi2[c]) b = 0;
            }
            t[(size_t)y * W + x] = (uint8_t)sat_u8(a + b); /* addWeighted(a, 1, b, 1, 0) */
        }
    const int rc = finish_mask(t, W, H, mask, mask_pitch);
    free(t);
    return rc;
}
