/* orc_freak.c -- CPU restatement of OpenCV 2.4.9's FREAK descriptor extractor (features2d/src/freak.cpp),
 * the extractor DescriptorsMatcher builds for FeatureOptions ExtractorType FREAK (reference
 * DescriptorsMatcher/descriptorsmatcher.cpp:350-353: cv::FREAK() -- orientationNormalized, scaleNormalized,
 * patternScale 22, nOctaves 4, the default pairs), matched like ORB / BRISK rows (:64-66).
 *
 * TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py's cpu_baseline): the GPU library
 * never links or calls this file.  OpenCV is not in this image, so this restatement is unpinned against
 * OpenCV itself; tests/test_freak_oracle.py checks its pieces against independent numpy statements (the
 * pattern, the orientation weights, the integral box means, the bit layout, rotation behaviour).
 *
 * Steps (DescriptorExtractor::compute -> FREAK::computeImpl):
 *   pattern     buildPattern: 43 points on 8 concentric circles (6 each, the centre last; radius from
 *               bigR 2/3 down to smallR 2/24, sigma radius / 2, odd circles rotated by pi / 6), per
 *               scale s (64 of them, scalingFactor pow(pow(2, nOctaves / 64.), s)) and orientation
 *               (256): x = (float)(radius * cos(alpha) * scalingFactor * patternScale), the same for
 *               y (sin) and sigma; patternSizes[s] = max over points of ceil((radius + sigma) *
 *               scalingFactor * patternScale) + 1
 *   weights     per orientation pair (i, j) of the scale-0 unrotated points: dx / (dx^2 + dy^2) in
 *               float, int(* 4096.0 + 0.5)
 *   filter      DescriptorExtractor::compute's runByKeypointSize(FLT_EPSILON) (NaN sizes dropped too), then
 *               per keypoint (from the last to the first, erasing in place: the kept order is the
 *               input order) its scale max((int)(logf(size / 7) * (float)(64 / (ln2 * 4)) + 0.5), 0)
 *               (at most 63), removed when x <= size or y <= size or x >= cols - size or y >= rows -
 *               size (patternSizes of its scale, compared as floats)
 *   intensity   meanIntensity: the point at (kp.x + x, kp.y + y) in float; sigma >= 0.5: the integral
 *               box [int(xf - s + 0.5), int(xf + s + 1.5)) x [int(yf - s + 0.5), int(yf + s + 1.5)),
 *               its sum divided (int) by its area; below 0.5 the 1024-fixed-point bilinear sample
 *               (ret + 2^21) / 2^22 as freak.cpp writes it (not reached with patternScale 22)
 *   orientation the 43 unrotated intensities; direction0 / 1 = sum over the 45 pairs (m = 44 .. 0) of
 *               (I_i - I_j) * weight / 2048 in int (C division); angle = (float)(atan2f(d1, d0) *
 *               180 / pi); thetaIdx = int(256 * angle (float) * (1 / 360.0) + 0.5), wrapped to [0, 256)
 *   bits        the 43 intensities at thetaIdx; the SSE2 build's layout (the plain build emulates it):
 *               byte 16q + b, bit t = I_i >= I_j of pair 128q + 16t + 15 - b (q = 0..3, t, b as
 *               bytes / bits), 64 bytes per keypoint
 * atan2f is the float of the deterministic double atan2 (fm3d_cv_atan2f; glibc's atan2f differs from
 * the correctly rounded float only where the double lies within rounding noise of a float boundary);
 * cos / sin / pow / logf are this image's libm, as the library's host code calls them.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "fm3d_cvmath.h"
#include "fm3d_freak.h"

#define ORC_API __attribute__((visibility("default")))

typedef struct orc_kpt {
    float x, y, size, angle, response;
    int octave, class_id;
} orc_kpt;

enum { FREAK_SCALES = 64, FREAK_NORIENT = 256, FREAK_POINTS = 43, FREAK_BYTES = 64 };

/* buildPattern: lut[((s * 256 + r) * 43 + i) * 3 + {0: x, 1: y, 2: sigma}], sizes[64] */
ORC_API void orc_freak_pattern(float patternScale, int nOctaves, float *lut, int *sizes)
{
    const int n[8] = {6, 6, 6, 6, 6, 6, 6, 1};
    const double bigR = 2.0 / 3.0, smallR = 2.0 / 24.0;
    const double unitSpace = (bigR - smallR) / 21.0;
    const double radius[8] = {bigR, bigR - 6 * unitSpace, bigR - 11 * unitSpace, bigR - 15 * unitSpace,
                              bigR - 18 * unitSpace, bigR - 20 * unitSpace, smallR, 0.0};
    const double sigma[8] = {radius[0] / 2.0, radius[1] / 2.0, radius[2] / 2.0, radius[3] / 2.0,
                             radius[4] / 2.0, radius[5] / 2.0, radius[6] / 2.0, radius[6] / 2.0};
    const double scaleStep = pow(2.0, (double)nOctaves / FREAK_SCALES);
    for (int s = 0; s < FREAK_SCALES; s++) {
        const double scalingFactor = pow(scaleStep, (double)s);
        sizes[s] = 0;
        for (int r = 0; r < FREAK_NORIENT; r++) {
            const double theta = (double)r * 2 * M_PI / (double)FREAK_NORIENT;
            int p = 0;
            for (int i = 0; i < 8; i++)
                for (int k = 0; k < n[i]; k++) {
                    const double beta = M_PI / n[i] * (i % 2);
                    const double alpha = (double)k * 2 * M_PI / (double)n[i] + beta + theta;
                    float *q = lut + (((size_t)s * FREAK_NORIENT + r) * FREAK_POINTS + p) * 3;
                    q[0] = (float)(radius[i] * cos(alpha) * scalingFactor * patternScale);
                    q[1] = (float)(radius[i] * sin(alpha) * scalingFactor * patternScale);
                    q[2] = (float)(sigma[i] * scalingFactor * patternScale);
                    const int sizeMax = (int)ceil((radius[i] + sigma[i]) * scalingFactor * patternScale) + 1;
                    if (sizes[s] < sizeMax) sizes[s] = sizeMax;
                    p++;
                }
        }
    }
}

/* the orientation pairs' weights from the scale-0, orientation-0 points */
ORC_API void orc_freak_weights(const float *lut, int *wdx, int *wdy)
{
    for (int m = FM3D_FREAK_NB_ORIENPAIRS; m--;) {
        const int i = FM3D_FREAK_ORIENT_PAIRS[2 * m], j = FM3D_FREAK_ORIENT_PAIRS[2 * m + 1];
        const float dx = lut[3 * i] - lut[3 * j];
        const float dy = lut[3 * i + 1] - lut[3 * j + 1];
        const float norm_sq = dx * dx + dy * dy;
        wdx[m] = (int)((dx / norm_sq) * 4096.0 + 0.5);
        wdy[m] = (int)((dy / norm_sq) * 4096.0 + 0.5);
    }
}

ORC_API int orc_freak_kscale(float size, int nOctaves)
{
    const float sizeCst = (float)(FREAK_SCALES / (0.693147180559945 * nOctaves));
    int s = (int)(logf(size / 7) * sizeCst + 0.5);
    if (s < 0) s = 0;
    if (s >= FREAK_SCALES) s = FREAK_SCALES - 1;
    return s;
}

/* (h+1) x (w+1) int sums, first row and column 0 (cv::integral, CV_32S) */
ORC_API void orc_freak_integral(const uint8_t *img, int w, int h, int *sum)
{
    memset(sum, 0, sizeof(int) * (size_t)(w + 1));
    for (int y = 0; y < h; y++) {
        int row = 0;
        sum[(size_t)(y + 1) * (w + 1)] = 0;
        for (int x = 0; x < w; x++) {
            row += img[(size_t)y * w + x];
            sum[(size_t)(y + 1) * (w + 1) + x + 1] = sum[(size_t)y * (w + 1) + x + 1] + row;
        }
    }
}

ORC_API int orc_freak_mean_intensity(const uint8_t *img, const int *sum, int w, float kx, float ky, float px,
                                     float py, float radius)
{
    const float xf = px + kx, yf = py + ky;
    const int x = (int)xf, y = (int)yf;
    if (radius < 0.5) {
        const int r_x = (int)((xf - x) * 1024), r_y = (int)((yf - y) * 1024);
        const int r_x_1 = 1024 - r_x, r_y_1 = 1024 - r_y;
        const uint8_t *ptr = img + x + (size_t)y * w;
        unsigned ret = (unsigned)(r_x_1 * r_y_1 * (int)ptr[0]);
        ret += (unsigned)(r_x * r_y_1 * (int)ptr[1]);
        ret += (unsigned)(r_x * r_y * (int)ptr[w + 1]);
        ret += (unsigned)(r_x_1 * r_y * (int)ptr[w]);
        ret += 2 * 1024 * 1024;
        return (uint8_t)(ret / (4 * 1024 * 1024));
    }
    const int x_left = (int)(xf - radius + 0.5);
    const int y_top = (int)(yf - radius + 0.5);
    const int x_right = (int)(xf + radius + 1.5);
    const int y_bottom = (int)(yf + radius + 1.5);
    const size_t W = (size_t)w + 1;
    int ret = sum[y_bottom * W + x_right];
    ret -= sum[y_bottom * W + x_left];
    ret += sum[y_top * W + x_left];
    ret -= sum[y_top * W + x_right];
    ret = ret / ((x_right - x_left) * (y_bottom - y_top));
    return (uint8_t)ret;
}

static float *freak_lut = 0;
static int freak_sizes[FREAK_SCALES];

static void freak_init(void)
{
    if (freak_lut) return;
    float *lut = (float *)malloc(sizeof(float) * 3 * (size_t)FREAK_SCALES * FREAK_NORIENT * FREAK_POINTS);
    orc_freak_pattern(22.0f, 4, lut, freak_sizes);
    freak_lut = lut;
}

/* the compressed pair index k (FREAK::DEF_PAIRS or a caller table) -> (i, j): the k-th of the pairs
   (i, j < i) of the 43 points in generation order */
static void freak_pair(int k, int *i, int *j)
{
    int a = 1;
    while (k >= a) {
        k -= a;
        a++;
    }
    *i = a;
    *j = k;
}

/* FREAK::compute with the default parameters on given keypoints: kept keypoints (angle set), the input
   index of each, 64 bytes per kept keypoint.  pairs: 512 indices (NULL: FM3D_FREAK_DEF_PAIRS). */
ORC_API int orc_freak_compute(const uint8_t *img, int w, int h, const orc_kpt *kin, int n, const int *pairs,
                              orc_kpt *kout, int *kept, uint8_t *desc)
{
    freak_init();
    if (!pairs) pairs = FM3D_FREAK_DEF_PAIRS;
    int wdx[FM3D_FREAK_NB_ORIENPAIRS], wdy[FM3D_FREAK_NB_ORIENPAIRS];
    orc_freak_weights(freak_lut, wdx, wdy);
    int pi[FM3D_FREAK_NB_PAIRS], pj[FM3D_FREAK_NB_PAIRS];
    for (int k = 0; k < FM3D_FREAK_NB_PAIRS; k++) freak_pair(pairs[k], &pi[k], &pj[k]);
    int *sum = (int *)malloc(sizeof(int) * (size_t)(w + 1) * (h + 1));
    orc_freak_integral(img, w, h, sum);
    int m = 0;
    for (int q = 0; q < n; q++) {
        const orc_kpt k = kin[q];
        /* DescriptorExtractor::compute: runByImageBorder(0) (nothing), runByKeypointSize(FLT_EPSILON) */
        if (!(k.size >= FLT_EPSILON && k.size <= FLT_MAX)) continue;
        const int s = orc_freak_kscale(k.size, 4);
        const float ps = (float)freak_sizes[s];
        if (k.x <= ps || k.y <= ps || k.x >= w - ps || k.y >= h - ps) continue;
        uint8_t v[FREAK_POINTS];
        const float *base = freak_lut + (size_t)s * FREAK_NORIENT * FREAK_POINTS * 3;
        for (int i = FREAK_POINTS; i--;)
            v[i] = (uint8_t)orc_freak_mean_intensity(img, sum, w, k.x, k.y, base[3 * i], base[3 * i + 1],
                                                     base[3 * i + 2]);
        int d0 = 0, d1 = 0;
        for (int o = FM3D_FREAK_NB_ORIENPAIRS; o--;) {
            const int delta = v[FM3D_FREAK_ORIENT_PAIRS[2 * o]] - v[FM3D_FREAK_ORIENT_PAIRS[2 * o + 1]];
            d0 += delta * wdx[o] / 2048;
            d1 += delta * wdy[o] / 2048;
        }
        orc_kpt ko = k;
        ko.angle = (float)(fm3d_cv_atan2f((float)d1, (float)d0) * (180.0 / M_PI));
        int theta = (int)(FREAK_NORIENT * ko.angle * (1 / 360.0) + 0.5);
        if (theta < 0) theta += FREAK_NORIENT;
        if (theta >= FREAK_NORIENT) theta -= FREAK_NORIENT;
        const float *rot = base + (size_t)theta * FREAK_POINTS * 3;
        for (int i = FREAK_POINTS; i--;)
            v[i] = (uint8_t)orc_freak_mean_intensity(img, sum, w, k.x, k.y, rot[3 * i], rot[3 * i + 1],
                                                     rot[3 * i + 2]);
        uint8_t *d = desc + (size_t)m * FREAK_BYTES;
        memset(d, 0, FREAK_BYTES);
        for (int qq = 0; qq < 4; qq++)
            for (int t = 0; t < 8; t++)
                for (int b = 0; b < 16; b++) {
                    const int p = 128 * qq + 16 * t + 15 - b;
                    if (v[pi[p]] >= v[pj[p]]) d[16 * qq + b] |= (uint8_t)(1u << t);
                }
        kout[m] = ko;
        if (kept) kept[m] = q;
        m++;
    }
    free(sum);
    return m;
}

/* the pattern sizes (patternSizes) of the default parameters */
ORC_API int orc_freak_size(int scale)
{
    freak_init();
    return freak_sizes[scale];
}

/* one default-pattern point (scale, orientation, i): x, y, sigma */
ORC_API void orc_freak_point(int scale, int rot, int i, float *x, float *y, float *sg)
{
    freak_init();
    const float *q = freak_lut + (((size_t)scale * FREAK_NORIENT + rot) * FREAK_POINTS + i) * 3;
    *x = q[0];
    *y = q[1];
    *sg = q[2];
}
