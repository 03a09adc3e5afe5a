/* orc_brisk.c -- CPU restatement of OpenCV 2.4.9's BRISK descriptor extractor (features2d/src/brisk.cpp),
 * the extractor DescriptorsMatcher builds for FeatureOptions ExtractorType BRISK
 * (reference DescriptorsMatcher/descriptorsmatcher.cpp:343-348: cv::BRISK(BriskDetector.Threshold,
 * BriskDetector.Octaves); build/settings.yml:46-48 carries that block).  The threshold and octaves only
 * steer BRISK's own detector, which the reference never builds (generateDetector has no BRISK branch),
 * so the extractor is the default pattern (patternScale 1) on the caller's keypoints.
 *
 * TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py's cpu_baseline): the GPU
 * library never links or calls this file.  OpenCV is not in this image, so this restatement is
 * unpinned against OpenCV itself; tests/test_brisk_oracle.py checks it against independent numpy
 * statements (the pattern, the pairs, the box-filtered intensities as weighted pixel sums).
 *
 * Steps (DescriptorExtractor::compute -> BRISK::computeImpl -> computeDescriptorsAndOrOrientation with
 * provided keypoints, so without the orientation step):
 *   pattern     generateKernel: rings of radius {0, 2.9, 4.9, 7.4, 10.8} * 0.85 with {1, 10, 14, 15, 20}
 *               points, 64 scales 2^(s * log2(30) / 64), 1024 rotations; the point (float)(scale *
 *               radius * cos(alpha + theta)) and the smoothing sigma in OpenCV's float / double mix;
 *               sizeList[scale] = ceil(scale * radius + sigma) + 1 over the rings
 *   pairs       from the unrotated scale-0 points: long pairs (|d|^2 > dMin^2, dMin 8.2) and short
 *               pairs (|d|^2 < dMax^2, dMax 5.85), in (i, j < i) order; 512 short pairs, 64 bytes
 *   filter      runByKeypointSize(FLT_EPSILON), then per keypoint its scale
 *               max((int)(64 / lb(30) * (log(size / 7.2) / ln 2) + 0.5), 0) (at most 63) and the
 *               removal of keypoints within sizeList[scale] of the border (order kept)
 *   theta       0 for angle -1, else (int)(1024 * angle / 360 + 0.5) wrapped to [0, 1024)
 *   intensity   smoothedIntensity: a box of half width sigma around the rotated point, its border
 *               pixels weighted by their covered fraction, in the fixed point of OpenCV (scaling =
 *               (int)(4194304 / area), weights truncated to int), integer sums, rounded division;
 *               below sigma 0.5 a bilinear sample (not reached by the default pattern)
 *   bits        bit k of the 512 = intensity(i_k) > intensity(j_k), little-endian 32-bit words
 * log() of the keypoint scale is the float overload (logf): an assumption where brisk.cpp's
 * unqualified call is ambiguous; it matters only for sizes whose scale lands within an ulp of n + 0.5.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_API __attribute__((visibility("default")))

typedef struct orc_kpt {
    float x, y, size, angle, response;
    int octave, class_id;
} orc_kpt;

enum { BRISK_SCALES = 64, BRISK_NROT = 1024, BRISK_POINTS = 60, BRISK_BYTES = 64 };
static const int brisk_num[5] = {1, 10, 14, 15, 20};

static void brisk_radii(float *r)
{
    const double f = 0.85 * 1.0;
    r[0] = (float)(f * 0.);
    r[1] = (float)(f * 2.9);
    r[2] = (float)(f * 4.9);
    r[3] = (float)(f * 7.4);
    r[4] = (float)(f * 10.8);
}

ORC_API float orc_brisk_scale_factor(int scale)
{
    const float lb_scale = (float)(log(30.f) / log(2.0));
    const float lb_scale_step = lb_scale / BRISK_SCALES;
    return (float)pow(2.0, (double)(scale * lb_scale_step));
}

/* the pattern point (x, y, sigma) of (scale, rot, i) */
ORC_API void orc_brisk_point(int scale, int rot, int i, float *px, float *py, float *psigma)
{
    float r[5];
    const float sc = orc_brisk_scale_factor(scale);
    const float sigma_scale = 1.3f;
    const double theta = (double)rot * 2 * M_PI / (double)BRISK_NROT;
    int ring = 0, num = i;
    double alpha;
    brisk_radii(r);
    while (num >= brisk_num[ring]) num -= brisk_num[ring++];
    alpha = (double)num * 2 * M_PI / (double)brisk_num[ring];
    *px = (float)(sc * r[ring] * cos(alpha + theta));
    *py = (float)(sc * r[ring] * sin(alpha + theta));
    if (ring == 0)
        *psigma = sigma_scale * sc * 0.5f;
    else
        *psigma = (float)(sigma_scale * sc * (double)r[ring] * sin(M_PI / brisk_num[ring]));
}

ORC_API int orc_brisk_size(int scale)
{
    float r[5];
    const float sc = orc_brisk_scale_factor(scale);
    int i, best = 0;
    brisk_radii(r);
    for (i = 0; i < BRISK_POINTS; i++) {
        float x, y, sg;
        int ring = 0, num = i, size;
        while (num >= brisk_num[ring]) num -= brisk_num[ring++];
        orc_brisk_point(scale, 0, i, &x, &y, &sg);
        size = (int)ceilf(sc * r[ring] + sg) + 1;
        if (size > best) best = size;
    }
    return best;
}

/* short pairs (i, j) in generation order; returns their count (long pairs are the orientation's) */
ORC_API int orc_brisk_short_pairs(int *pi, int *pj)
{
    const float dMin = (float)(8.2 * 1.0), dMax = (float)(5.85 * 1.0);
    const float dMin_sq = dMin * dMin, dMax_sq = dMax * dMax;
    float X[BRISK_POINTS], Y[BRISK_POINTS], sg;
    int i, j, n = 0;
    for (i = 0; i < BRISK_POINTS; i++) orc_brisk_point(0, 0, i, &X[i], &Y[i], &sg);
    for (i = 1; i < BRISK_POINTS; i++)
        for (j = 0; j < i; j++) {
            const float dx = X[j] - X[i], dy = Y[j] - Y[i];
            const float norm_sq = dx * dx + dy * dy;
            if (norm_sq > dMin_sq) continue; /* a long pair */
            if (norm_sq < dMax_sq) {
                if (pi) {
                    pi[n] = i;
                    pj[n] = j;
                }
                n++;
            }
        }
    return n;
}

/* the keypoint's pattern scale, from its size */
ORC_API int orc_brisk_kscale(float size)
{
    const float log2c = 0.693147180559945f;
    const float lb_scalerange = (float)(logf(30.f) / log2c);
    const float basicSize06 = 12.0f * 0.6f;
    int scale = (int)(BRISK_SCALES / lb_scalerange * (logf(size / basicSize06) / log2c) + 0.5);
    if (scale < 0) scale = 0;
    if (scale >= BRISK_SCALES) scale = BRISK_SCALES - 1;
    return scale;
}

ORC_API int orc_brisk_theta(float angle)
{
    int theta;
    if (angle == -1) return 0;
    theta = (int)(BRISK_NROT * (angle / 360.0) + 0.5);
    if (theta < 0) theta += BRISK_NROT;
    if (theta >= BRISK_NROT) theta -= BRISK_NROT;
    return theta;
}

/* smoothedIntensity at (key + point) with the point's sigma; II: (h+1) x (w+1) integral of img */
ORC_API int orc_brisk_intensity(const uint8_t *img, const int *II, int w, float kx, float ky, float ptx, float pty,
                                float sigma_half)
{
    const float xf = ptx + kx, yf = pty + ky;
    const int x = (int)xf, y = (int)yf;
    const float area = 4.0f * sigma_half * sigma_half;
    int scaling, scaling2, x_left, y_top, x_right, y_bottom, dx, dy, A, B, C, D, rx1i, ry1i, rx_1i, ry_1i;
    float x_1, x1, y_1, y1, r_x_1, r_y_1, r_x1, r_y1;
    long long ret; /* OpenCV sums in int; the tests check it stays in range */
    int i, j;
    if (sigma_half < 0.5) {
        const int r_x = (int)((xf - x) * 1024), r_y = (int)((yf - y) * 1024);
        const int r_x_1 = 1024 - r_x, r_y_1 = 1024 - r_y;
        const uint8_t *p = img + (size_t)y * w + x;
        const int v = r_x_1 * r_y_1 * p[0] + r_x * r_y_1 * p[1] + r_x * r_y * p[w] + r_x_1 * r_y * p[w + 1];
        return (v + 512) / 1024;
    }
    scaling = (int)(4194304.0 / area);
    scaling2 = (int)((float)scaling * area / 1024.0);
    x_1 = xf - sigma_half;
    x1 = xf + sigma_half;
    y_1 = yf - sigma_half;
    y1 = yf + sigma_half;
    x_left = (int)(x_1 + 0.5);
    y_top = (int)(y_1 + 0.5);
    x_right = (int)(x1 + 0.5);
    y_bottom = (int)(y1 + 0.5);
    r_x_1 = (float)x_left - x_1 + 0.5f;
    r_y_1 = (float)y_top - y_1 + 0.5f;
    r_x1 = x1 - (float)x_right + 0.5f;
    r_y1 = y1 - (float)y_bottom + 0.5f;
    dx = x_right - x_left - 1;
    dy = y_bottom - y_top - 1;
    A = (int)((r_x_1 * r_y_1) * scaling);
    B = (int)((r_x1 * r_y_1) * scaling);
    C = (int)((r_x1 * r_y1) * scaling);
    D = (int)((r_x_1 * r_y1) * scaling);
    rx_1i = (int)(r_x_1 * scaling);
    ry_1i = (int)(r_y_1 * scaling);
    rx1i = (int)(r_x1 * scaling);
    ry1i = (int)(r_y1 * scaling);
    /* the corners, the four edges without them and the interior: OpenCV takes the edges and the
       interior from the integral image when dx + dy > 2 and sums pixels otherwise; both are the same
       integer */
    (void)II;
#define P(r, c) ((long long)img[(size_t)(r) * w + (c)])
    ret = A * P(y_top, x_left) + B * P(y_top, x_right) + C * P(y_bottom, x_right) + D * P(y_bottom, x_left);
    for (i = x_left + 1; i < x_right; i++) ret += ry_1i * P(y_top, i) + ry1i * P(y_bottom, i);
    for (j = y_top + 1; j < y_bottom; j++) {
        ret += rx_1i * P(j, x_left) + rx1i * P(j, x_right);
        for (i = x_left + 1; i < x_right; i++) ret += (long long)scaling * P(j, i);
    }
#undef P
    (void)dx;
    (void)dy;
    return (int)((ret + scaling2 / 2) / scaling2);
}

/* BRISK compute on the caller's keypoints: returns the kept count m; kout / kept (input index) / desc
 * (m x 64 bytes) */
ORC_API int orc_brisk_compute(const uint8_t *img, int w, int h, const orc_kpt *kin, int n, orc_kpt *kout, int *kept,
                              uint8_t *desc)
{
    int pi[BRISK_POINTS * (BRISK_POINTS - 1) / 2], pj[BRISK_POINTS * (BRISK_POINTS - 1) / 2];
    const int npairs = orc_brisk_short_pairs(pi, pj);
    int sizes[BRISK_SCALES], q, m = 0, s;
    for (s = 0; s < BRISK_SCALES; s++) sizes[s] = orc_brisk_size(s);
    for (q = 0; q < n; q++) {
        const orc_kpt k = kin[q];
        int scale, border, theta, i, vals[BRISK_POINTS];
        uint8_t *d;
        if (!(k.size >= FLT_EPSILON)) continue; /* runByKeypointSize */
        scale = orc_brisk_kscale(k.size);
        border = sizes[scale];
        /* RoiPredicate(border, border, cols - border, rows - border) */
        if (k.x < (float)border || k.x >= (float)(w - border) || k.y < (float)border || k.y >= (float)(h - border))
            continue;
        theta = orc_brisk_theta(k.angle);
        for (i = 0; i < BRISK_POINTS; i++) {
            float px, py, sg;
            orc_brisk_point(scale, theta, i, &px, &py, &sg);
            vals[i] = orc_brisk_intensity(img, NULL, w, k.x, k.y, px, py, sg);
        }
        d = desc + (size_t)m * BRISK_BYTES;
        memset(d, 0, BRISK_BYTES);
        for (i = 0; i < npairs && i < 8 * BRISK_BYTES; i++)
            if (vals[pi[i]] > vals[pj[i]]) d[i >> 3] |= (uint8_t)(1u << (i & 7));
        kout[m] = k;
        if (kept) kept[m] = q;
        m++;
    }
    return m;
}
