/* orc_orb.c -- CPU restatement of OpenCV 2.4.9's ORB (features2d/src/orb.cpp and what it calls),
 * the detector / extractor DescriptorsMatcher builds for FeatureOptions DetectorType / ExtractorType
 * ORB (reference DescriptorsMatcher/descriptorsmatcher.cpp:273-279, 336-341:
 * cv::ORB(NumFeatures, ScaleFactor, NumLevels), the other parameters OpenCV's defaults: edgeThreshold
 * 31, firstLevel 0, WTA_K 2, HARRIS_SCORE, patchSize 31).
 *
 * TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py's cpu_baseline): the GPU
 * library never links or calls this file.  OpenCV is not in this image, so the restatement is pinned
 * piece by piece by independent numpy restatements and by the real libstdc++ (tests/test_orb_oracle.py).
 *
 * Steps, in OpenCV's operation order:
 *   level sizes     getScale = (float)pow(scaleFactor, level); size cvRound(cols * (1 / scale))
 *   orb_resize      resize(INTER_LINEAR) of level l-1 to level l (imgproc/resize.cpp): fixed-point
 *                   coefficients (INTER_RESIZE_COEF_BITS 11), the horizontal pass in int, the vertical
 *                   pass as VResizeLinearVec_32s8u (SSE2: >> 4, mulhi, (+2) >> 2) on its columns and
 *                   FixedPtCast (+ 2^21) >> 22 on the rest
 *   fast_score      FAST_t<16> with non-maximum suppression (features2d/src/fast.cpp): the 9-of-16
 *                   arc test, cornerScore<16> = (largest of max-of-arc-mins / -min-of-arc-maxes) - 1
 *   retain_best     KeyPointsFilter::retainBest: std::nth_element (libstdc++ introselect, GCC >= 4.9)
 *                   + std::partition (libstdc++'s bidirectional __partition), restated below
 *   harris          HarrisResponses(blockSize 7, k 0.04) in int sums and float
 *   ic_angle        IC_Angle: integer moments over the circular patch (umax), fastAtan2
 *   orb_blur        GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) on 8U: fixed-point row kernel
 *                   (x256, int sums); the column pass as SymmColumnVec_32s8u (SSE2, float) on the
 *                   first floor(width/4)*4 columns, FixedPtCastEx (+2^15) >> 16 on the rest
 *   orb_desc        computeOrbDescriptor, WTA_K 2: 256 intensity comparisons at the rotated pattern
 *                   points (cvRound of float rotations) of the blurred level
 * The 512-point pattern is DATA: OpenCV's bit_pattern_31_ table (patchSize 31) is not in this image;
 * the caller passes it, else makeRandomPattern(patchSize) (cv::RNG(0x34985739), what OpenCV uses for
 * every other patchSize) is used.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "fm3d_detmath.h"

#define ORC_API __attribute__((visibility("default")))

typedef struct {
    float x, y, size, angle, response;
    int octave, class_id;
} orc_kpt;

float orc_fast_atan2(float y, float x); /* orc_surf.c */

static int cv_roundf(float v) { return (int)lrintf(v); }
static int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* ---------------------------------------------------------------- level geometry */
ORC_API float orc_orb_scale(double scaleFactor, int level) { return (float)pow(scaleFactor, (double)level); }

ORC_API void orc_orb_level_size(int w, int h, double scaleFactor, int level, int *lw, int *lh)
{
    const float scale = 1 / orc_orb_scale(scaleFactor, level);
    *lw = cv_roundf(w * scale);
    *lh = cv_roundf(h * scale);
}

/* ---------------------------------------------------------------- resize (INTER_LINEAR, 8U) */
/* the first column the scalar tail of VResizeLinear handles (VResizeLinearVec_32s8u's loops) */
ORC_API int orc_vresize_sse_end(int width)
{
    int x = 0;
    for (; x <= width - 16; x += 16) {}
    for (; x < width - 4; x += 4) {}
    return x;
}

static short sat_short(float v)
{
    const int i = cv_roundf(v);
    return (short)(i < -32768 ? -32768 : (i > 32767 ? 32767 : i));
}

/* the horizontal tables: xofs, (a0, a1) per destination column, and xmax */
ORC_API int orc_resize_xtab(int sw, int dw, int *xofs, short *alpha)
{
    const double scale_x = 1. / ((double)dw / sw);
    int dx, xmax = dw;
    for (dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)floorf(fx);
        fx -= sx;
        if (sx < 0) {
            fx = 0;
            sx = 0;
        }
        if (sx + 1 >= sw) {
            if (dx < xmax) xmax = dx;
            if (sx >= sw - 1) {
                fx = 0;
                sx = sw - 1;
            }
        }
        xofs[dx] = sx;
        alpha[2 * dx] = sat_short((1.f - fx) * 2048);
        alpha[2 * dx + 1] = sat_short(fx * 2048);
    }
    return xmax;
}

/* the vertical tables: source row sy (unclamped) and (b0, b1) per destination row */
ORC_API void orc_resize_ytab(int sh, int dh, int *yofs, short *beta)
{
    const double scale_y = 1. / ((double)dh / sh);
    int dy;
    for (dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        const int sy = (int)floorf(fy);
        fy -= sy;
        yofs[dy] = sy;
        beta[2 * dy] = sat_short((1.f - fy) * 2048);
        beta[2 * dy + 1] = sat_short(fy * 2048);
    }
}

ORC_API void orc_orb_resize(const uint8_t *src, int sw, int sh, uint8_t *dst, int dw, int dh)
{
    int *xofs = (int *)malloc(sizeof(int) * dw), *yofs = (int *)malloc(sizeof(int) * dh);
    short *alpha = (short *)malloc(sizeof(short) * 2 * dw), *beta = (short *)malloc(sizeof(short) * 2 * dh);
    int *D0 = (int *)malloc(sizeof(int) * dw), *D1 = (int *)malloc(sizeof(int) * dw);
    const int xmax = orc_resize_xtab(sw, dw, xofs, alpha), xs = orc_vresize_sse_end(dw);
    int dx, dy;
    orc_resize_ytab(sh, dh, yofs, beta);
    for (dy = 0; dy < dh; dy++) {
        const uint8_t *S0 = src + (size_t)clampi(yofs[dy], 0, sh - 1) * sw;
        const uint8_t *S1 = src + (size_t)clampi(yofs[dy] + 1, 0, sh - 1) * sw;
        const int b0 = beta[2 * dy], b1 = beta[2 * dy + 1];
        for (dx = 0; dx < dw; dx++) {
            const int sx = xofs[dx];
            if (dx < xmax) {
                D0[dx] = S0[sx] * alpha[2 * dx] + S0[sx + 1] * alpha[2 * dx + 1];
                D1[dx] = S1[sx] * alpha[2 * dx] + S1[sx + 1] * alpha[2 * dx + 1];
            } else {
                D0[dx] = S0[sx] * 2048;
                D1[dx] = S1[sx] * 2048;
            }
        }
        for (dx = 0; dx < dw; dx++) {
            int v;
            if (dx < xs) { /* SSE2: (S >> 4) as int16, mulhi by beta, saturating adds, (+2) >> 2, packus */
                v = (((D0[dx] >> 4) * b0) >> 16) + (((D1[dx] >> 4) * b1) >> 16);
                v = (v + 2) >> 2;
            } else {
                v = (b0 * D0[dx] + b1 * D1[dx] + (1 << 21)) >> 22;
            }
            dst[(size_t)dy * dw + dx] = (uint8_t)clampi(v, 0, 255);
        }
    }
    free(xofs);
    free(yofs);
    free(alpha);
    free(beta);
    free(D0);
    free(D1);
}

/* ---------------------------------------------------------------- FAST-9 (16-pixel circle) */
static const int FAST_CIRCLE[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1},  {2, -2}, {1, -3},
                                       {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

/* pixel (x, y) (3 <= x < w-3, 3 <= y < h-3): 1 and *score = cornerScore<16> if it is a corner at
   `thr` (9 contiguous circle pixels darker than v - thr or brighter than v + thr), else 0 */
static int fast_corner(const uint8_t *img, int w, int x, int y, int thr, int *score)
{
    const uint8_t *p = img + (size_t)y * w + x;
    const int v = p[0];
    int d[25], k, cd = 0, cb = 0, dark = 0, bright = 0;
    for (k = 0; k < 25; k++) {
        const int q = p[FAST_CIRCLE[k & 15][0] + FAST_CIRCLE[k & 15][1] * w];
        d[k] = v - q;
        if (q < v - thr) {
            if (++cd > 8) dark = 1;
        } else {
            cd = 0;
        }
        if (q > v + thr) {
            if (++cb > 8) bright = 1;
        } else {
            cb = 0;
        }
    }
    if (!dark && !bright) return 0;
    {
        int a0 = -1000, b0 = 1000, s;
        for (k = 0; k < 16; k++) {
            int j, mn = d[k], mx = d[k];
            for (j = 1; j <= 8; j++) {
                mn = d[k + j] < mn ? d[k + j] : mn;
                mx = d[k + j] > mx ? d[k + j] : mx;
            }
            a0 = mn > a0 ? mn : a0;
            b0 = mx < b0 ? mx : b0;
        }
        s = (a0 > -b0 ? a0 : -b0) - 1;
        *score = s;
    }
    return 1;
}

/* FAST(img, keypoints, thr, nonmaxSuppression): KeyPoint(x, y, 7, -1, score) in raster order, the
   score 0 without non-max suppression (FAST_t computes it only for the suppression); returns the
   count (out may be NULL to count).  FastFeatureDetector(thr, nonmax) (features2d/src/fast.cpp,
   descriptorsmatcher.cpp:215-222) is this on the image itself. */
ORC_API int orc_fast_detect(const uint8_t *img, int w, int h, int thr, int nonmax, orc_kpt *out, int cap)
{
    /* S: the (uchar) score of every corner, 0 elsewhere (FAST_t's row buffers); C: corner flags */
    uint8_t *S = (uint8_t *)calloc((size_t)w * h, 1), *C = (uint8_t *)calloc((size_t)w * h, 1);
    int x, y, n = 0;
    thr = clampi(thr, 0, 255);
    for (y = 3; y < h - 3; y++)
        for (x = 3; x < w - 3; x++) {
            int s;
            if (fast_corner(img, w, x, y, thr, &s)) {
                S[(size_t)y * w + x] = (uint8_t)s;
                C[(size_t)y * w + x] = 1;
            }
        }
    for (y = 3; y < h - 3; y++)
        for (x = 3; x < w - 3; x++) {
            const uint8_t *c = S + (size_t)y * w + x;
            const int s = c[0];
            if (!C[(size_t)y * w + x]) continue;
            if (nonmax && !(s > c[-1] && s > c[1] && s > c[-w - 1] && s > c[-w] && s > c[-w + 1] && s > c[w - 1] &&
                            s > c[w] && s > c[w + 1]))
                continue;
            if (out && n < cap) {
                orc_kpt k = {(float)x, (float)y, 7.f, -1.f, nonmax ? (float)s : 0.f, 0, -1};
                out[n] = k;
            }
            n++;
        }
    free(S);
    free(C);
    return n;
}

/* FAST(img, keypoints, thr, true) */
ORC_API int orc_fast9(const uint8_t *img, int w, int h, int thr, orc_kpt *out, int cap)
{
    return orc_fast_detect(img, w, h, thr, 1, out, cap);
}

/* KeyPointsFilter::runByImageBorder: stable, Rect(b, b, w - 2b, h - 2b).contains(pt), where pt
   reaches Rect_<int>::contains as a Point: saturate_cast<int> = cvRound of each coordinate */
static int in_border(float x, float y, int w, int h, int b)
{
    const int ix = cv_roundf(x), iy = cv_roundf(y);
    return ix >= b && ix < b + (w - 2 * b) && iy >= b && iy < b + (h - 2 * b);
}
ORC_API int orc_run_by_image_border(orc_kpt *k, int n, int w, int h, int b)
{
    int i, m = 0;
    if (b <= 0) return n;
    if (h <= 2 * b || w <= 2 * b) return 0;
    for (i = 0; i < n; i++)
        if (in_border(k[i].x, k[i].y, w, h, b)) k[m++] = k[i];
    return m;
}

/* ---------------------------------------------------------------- libstdc++ selection */
/* comp = KeypointResponseGreater: a.response > b.response */
#define GREATER(a, b) ((a).response > (b).response)
static void kswap(orc_kpt *a, orc_kpt *b)
{
    const orc_kpt t = *a;
    *a = *b;
    *b = t;
}

static void push_heap(orc_kpt *f, long hole, long top, orc_kpt value)
{
    long parent = (hole - 1) / 2;
    while (hole > top && GREATER(f[parent], value)) {
        f[hole] = f[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    f[hole] = value;
}

static void adjust_heap(orc_kpt *f, long hole, long len, orc_kpt value)
{
    const long top = hole;
    long second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (GREATER(f[second], f[second - 1])) second--;
        f[hole] = f[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        f[hole] = f[second - 1];
        hole = second - 1;
    }
    push_heap(f, hole, top, value);
}

static void make_heap(orc_kpt *f, long len)
{
    long parent;
    if (len < 2) return;
    for (parent = (len - 2) / 2;; parent--) {
        adjust_heap(f, parent, len, f[parent]);
        if (parent == 0) return;
    }
}

static void pop_heap(orc_kpt *f, long len, orc_kpt *result)
{
    const orc_kpt value = *result;
    *result = f[0];
    adjust_heap(f, 0, len, value);
}

static void heap_select(orc_kpt *f, orc_kpt *mid, orc_kpt *last)
{
    orc_kpt *i;
    make_heap(f, mid - f);
    for (i = mid; i < last; i++)
        if (GREATER(*i, *f)) pop_heap(f, mid - f, i);
}

/* test hook: std::__heap_select (tests/test_orb_oracle.py compares it with libstdc++'s) */
ORC_API void orc_heap_select(orc_kpt *f, long mid, long n) { heap_select(f, f + mid, f + n); }

static void move_median_to_first(orc_kpt *r, orc_kpt *a, orc_kpt *b, orc_kpt *c)
{
    if (GREATER(*a, *b)) {
        if (GREATER(*b, *c))
            kswap(r, b);
        else if (GREATER(*a, *c))
            kswap(r, c);
        else
            kswap(r, a);
    } else if (GREATER(*a, *c))
        kswap(r, a);
    else if (GREATER(*b, *c))
        kswap(r, c);
    else
        kswap(r, b);
}

static orc_kpt *unguarded_partition(orc_kpt *first, orc_kpt *last, orc_kpt *pivot)
{
    for (;;) {
        while (GREATER(*first, *pivot)) first++;
        last--;
        while (GREATER(*pivot, *last)) last--;
        if (!(first < last)) return first;
        kswap(first, last);
        first++;
    }
}

static void insertion_sort(orc_kpt *first, orc_kpt *last)
{
    orc_kpt *i;
    if (first == last) return;
    for (i = first + 1; i != last; i++) {
        if (GREATER(*i, *first)) {
            const orc_kpt val = *i;
            memmove(first + 1, first, (size_t)(i - first) * sizeof(orc_kpt));
            *first = val;
        } else {
            const orc_kpt val = *i;
            orc_kpt *l = i, *next = i - 1;
            while (GREATER(val, *next)) {
                *l = *next;
                l = next;
                next--;
            }
            *l = val;
        }
    }
}

static long lg(long n)
{
    long k = 0;
    while (n > 1) {
        n >>= 1;
        k++;
    }
    return k;
}

/* std::nth_element(first, nth, last, KeypointResponseGreater()) */
ORC_API void orc_nth_element(orc_kpt *first, long nth, long n)
{
    orc_kpt *last = first + n, *pn = first + nth;
    long depth;
    if (n == 0 || nth == n) return;
    depth = lg(n) * 2;
    while (last - first > 3) {
        orc_kpt *mid, *cut;
        if (depth == 0) {
            heap_select(first, pn + 1, last);
            kswap(first, pn);
            return;
        }
        depth--;
        mid = first + (last - first) / 2;
        move_median_to_first(first, first + 1, mid, last - 1);
        cut = unguarded_partition(first + 1, last, first);
        if (cut <= pn)
            first = cut;
        else
            last = cut;
    }
    insertion_sort(first, last);
}

/* std::partition(first, last, response >= thr) (libstdc++'s bidirectional __partition) */
ORC_API long orc_partition_ge(orc_kpt *base, long lo, long hi, float thr)
{
    orc_kpt *first = base + lo, *last = base + hi;
    for (;;) {
        for (;;)
            if (first == last)
                return first - base;
            else if (first->response >= thr)
                first++;
            else
                break;
        last--;
        for (;;)
            if (first == last)
                return first - base;
            else if (!(last->response >= thr))
                last--;
            else
                break;
        kswap(first, last);
        first++;
    }
}

/* KeyPointsFilter::retainBest: new count */
ORC_API int orc_retain_best(orc_kpt *k, int n, int npts)
{
    if (npts >= 0 && n > npts) {
        float amb;
        if (npts == 0) return 0;
        orc_nth_element(k, npts, n);
        amb = k[npts - 1].response;
        return (int)orc_partition_ge(k, npts, n, amb);
    }
    return n;
}

/* ---------------------------------------------------------------- Harris, orientation */
ORC_API void orc_harris(const uint8_t *img, int w, orc_kpt *k, int n, int blockSize, float harris_k)
{
    const int r = blockSize / 2;
    float scale = (1 << 2) * blockSize * 255.0f;
    float sq;
    int p;
    scale = 1.0f / scale;
    sq = scale * scale * scale * scale;
    for (p = 0; p < n; p++) {
        const int x0 = cv_roundf(k[p].x - r), y0 = cv_roundf(k[p].y - r);
        int a = 0, b = 0, c = 0, i, j;
        for (i = 0; i < blockSize; i++)
            for (j = 0; j < blockSize; j++) {
                const uint8_t *q = img + (size_t)(y0 + i) * w + x0 + j;
                const int Ix = (q[1] - q[-1]) * 2 + (q[-w + 1] - q[-w - 1]) + (q[w + 1] - q[w - 1]);
                const int Iy = (q[w] - q[-w]) * 2 + (q[w - 1] - q[-w - 1]) + (q[w + 1] - q[-w + 1]);
                a += Ix * Ix;
                b += Iy * Iy;
                c += Ix * Iy;
            }
        k[p].response = ((float)a * b - (float)c * c - harris_k * ((float)a + b) * ((float)a + b)) * sq;
    }
}

/* computeKeyPoints' umax: the end of each row of the circular patch, made symmetric */
ORC_API void orc_orb_umax(int halfPatchSize, int *umax)
{
    int v, v0;
    const int vmax = (int)floorf(halfPatchSize * sqrtf(2.f) / 2 + 1);
    const int vmin = (int)ceilf(halfPatchSize * sqrtf(2.f) / 2);
    for (v = 0; v <= vmax; ++v) umax[v] = (int)lrint(sqrt((double)halfPatchSize * halfPatchSize - v * v));
    for (v = halfPatchSize, v0 = 0; v >= vmin; --v) {
        while (umax[v0] == umax[v0 + 1]) ++v0;
        umax[v] = v0;
        ++v0;
    }
}

ORC_API float orc_ic_angle(const uint8_t *img, int w, int half_k, float px, float py, const int *umax)
{
    int m01 = 0, m10 = 0, u, v;
    const uint8_t *c = img + (size_t)cv_roundf(py) * w + cv_roundf(px);
    for (u = -half_k; u <= half_k; ++u) m10 += u * c[u];
    for (v = 1; v <= half_k; ++v) {
        int vsum = 0;
        const int d = umax[v];
        for (u = -d; u <= d; ++u) {
            const int vp = c[u + v * w], vm = c[u - v * w];
            vsum += vp - vm;
            m10 += u * (vp + vm);
        }
        m01 += v * vsum;
    }
    return orc_fast_atan2((float)m01, (float)m10);
}

/* ---------------------------------------------------------------- GaussianBlur 7x7, sigma 2 */
/* the fixed-point kernel: cvRound(getGaussianKernel(7, 2, CV_32F) * 256) */
ORC_API void orc_orb_blur_kernel(int *ik)
{
    float g[7];
    const double scale2X = -0.5 / (2.0 * 2.0);
    double sum = 0;
    int i;
    for (i = 0; i < 7; i++) {
        const double x = i - 3.0;
        g[i] = (float)exp(scale2X * x * x);
        sum += g[i];
    }
    sum = 1. / sum;
    for (i = 0; i < 7; i++) g[i] = (float)(g[i] * sum);
    for (i = 0; i < 7; i++) ik[i] = cv_roundf(g[i] * 256.f);
}

static int reflect101(int p, int n)
{
    if (n == 1) return 0;
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}

ORC_API void orc_orb_blur(const uint8_t *src, int w, int h, uint8_t *dst)
{
    int ik[7], x, y, k;
    float fk[4];
    int *R = (int *)malloc(sizeof(int) * (size_t)w * h);
    const int xs = (w / 4) * 4;
    orc_orb_blur_kernel(ik);
    for (k = 0; k < 4; k++) fk[k] = (float)(ik[3 + k] * (1. / 65536));
    for (y = 0; y < h; y++)
        for (x = 0; x < w; x++) {
            int s = 0;
            for (k = 0; k < 7; k++) s += ik[k] * src[(size_t)y * w + reflect101(x + k - 3, w)];
            R[(size_t)y * w + x] = s;
        }
    for (y = 0; y < h; y++)
        for (x = 0; x < w; x++) {
            int v;
            if (x < xs) { /* SymmColumnVec_32s8u: float */
                float s = (float)R[(size_t)y * w + x] * fk[0] + 0.f;
                for (k = 1; k <= 3; k++)
                    s = s + (float)(R[(size_t)reflect101(y + k, h) * w + x] + R[(size_t)reflect101(y - k, h) * w + x]) *
                                fk[k];
                v = (int)lrintf(s);
            } else { /* FixedPtCastEx<int, uchar>(16) */
                int s = ik[3] * R[(size_t)y * w + x];
                for (k = 1; k <= 3; k++)
                    s += ik[3 + k] * (R[(size_t)reflect101(y + k, h) * w + x] + R[(size_t)reflect101(y - k, h) * w + x]);
                v = (s + (1 << 15)) >> 16;
            }
            dst[(size_t)y * w + x] = (uint8_t)clampi(v, 0, 255);
        }
    free(R);
}

/* ---------------------------------------------------------------- descriptors */
/* makeRandomPattern: cv::RNG(0x34985739), RNG::uniform(-patchSize/2, patchSize/2 + 1), x then y */
ORC_API void orc_orb_random_pattern(int patchSize, int *xy, int npoints)
{
    uint64_t state = 0x34985739;
    const int a = -patchSize / 2, b = patchSize / 2 + 1;
    int i;
    for (i = 0; i < 2 * npoints; i++) {
        state = (uint64_t)(unsigned)state * 4164903690U + (unsigned)(state >> 32);
        xy[i] = (int)((unsigned)state % (unsigned)(b - a) + (unsigned)a);
    }
}

ORC_API void orc_orb_describe(const uint8_t *img, int w, const orc_kpt *k, const int *pattern, uint8_t *desc)
{
    float angle = k->angle, a, b;
    const uint8_t *c;
    int i, j;
    angle *= (float)(M_PI / 180.f);
    a = (float)fm3d_cos((double)angle);
    b = (float)fm3d_sin((double)angle);
    c = img + (size_t)cv_roundf(k->y) * w + cv_roundf(k->x);
    for (i = 0; i < 32; i++) {
        int val = 0;
        for (j = 0; j < 8; j++) {
            const int *p0 = pattern + (i * 16 + 2 * j) * 2, *p1 = p0 + 2;
            const float x0 = p0[0] * a - p0[1] * b, y0 = p0[0] * b + p0[1] * a;
            const float x1 = p1[0] * a - p1[1] * b, y1 = p1[0] * b + p1[1] * a;
            const int t0 = c[cv_roundf(y0) * w + cv_roundf(x0)], t1 = c[cv_roundf(y1) * w + cv_roundf(x1)];
            val |= (t0 < t1) << j;
        }
        desc[i] = (uint8_t)val;
    }
}

/* ---------------------------------------------------------------- the pyramid */
typedef struct {
    int L, *w, *h;
    uint8_t **img;
} pyramid;

static void build_pyramid(const uint8_t *img, int w, int h, double scaleFactor, int L, pyramid *P)
{
    int l;
    P->L = L;
    P->w = (int *)malloc(sizeof(int) * L);
    P->h = (int *)malloc(sizeof(int) * L);
    P->img = (uint8_t **)malloc(sizeof(uint8_t *) * L);
    for (l = 0; l < L; l++) {
        orc_orb_level_size(w, h, scaleFactor, l, &P->w[l], &P->h[l]);
        P->img[l] = (uint8_t *)malloc((size_t)P->w[l] * P->h[l] + 1);
        if (l == 0)
            memcpy(P->img[0], img, (size_t)w * h);
        else
            orc_orb_resize(P->img[l - 1], P->w[l - 1], P->h[l - 1], P->img[l], P->w[l], P->h[l]);
    }
}

static void free_pyramid(pyramid *P)
{
    int l;
    for (l = 0; l < P->L; l++) free(P->img[l]);
    free(P->img);
    free(P->w);
    free(P->h);
}

/* ORB::operator()(image, noArray(), keypoints, descriptors?) detection: level-major keypoints
   (level coordinates scaled back by getScale), descriptors (32 bytes each) when desc != NULL.
   Returns the count; out / desc hold min(count, cap). */
ORC_API int orc_orb_detect(const uint8_t *img, int w, int h, int nfeatures, double scaleFactor, int nlevels,
                           int edgeThreshold, int patchSize, int fastThreshold, const int *pattern, orc_kpt *out,
                           uint8_t *desc, int cap)
{
    pyramid P;
    int *nper = (int *)malloc(sizeof(int) * (nlevels > 0 ? nlevels : 1));
    int *umax = (int *)malloc(sizeof(int) * (patchSize / 2 + 2));
    int *pat = NULL;
    const int halfPatch = patchSize / 2;
    int l, total = 0, sum = 0;
    if (nlevels <= 0) {
        free(nper);
        free(umax);
        return 0;
    }
    if (desc && !pattern) {
        pat = (int *)malloc(sizeof(int) * 1024);
        orc_orb_random_pattern(patchSize, pat, 512);
        pattern = pat;
    }
    {
        const float factor = (float)(1.0 / scaleFactor);
        float nd = nfeatures * (1 - factor) / (1 - (float)pow((double)factor, (double)nlevels));
        for (l = 0; l < nlevels - 1; l++) {
            nper[l] = cv_roundf(nd);
            sum += nper[l];
            nd *= factor;
        }
        nper[nlevels - 1] = nfeatures - sum > 0 ? nfeatures - sum : 0;
    }
    orc_orb_umax(halfPatch, umax);
    build_pyramid(img, w, h, scaleFactor, nlevels, &P);
    for (l = 0; l < nlevels; l++) {
        const int lw = P.w[l], lh = P.h[l];
        int n = (lw > 0 && lh > 0) ? orc_fast9(P.img[l], lw, lh, fastThreshold, NULL, 0) : 0, i;
        orc_kpt *k = (orc_kpt *)malloc(sizeof(orc_kpt) * (n > 0 ? n : 1));
        const float sf = orc_orb_scale(scaleFactor, l);
        if (n > 0) orc_fast9(P.img[l], lw, lh, fastThreshold, k, n);
        n = orc_run_by_image_border(k, n, lw, lh, edgeThreshold);
        n = orc_retain_best(k, n, 2 * nper[l]);
        orc_harris(P.img[l], lw, k, n, 7, 0.04f);
        n = orc_retain_best(k, n, nper[l]);
        for (i = 0; i < n; i++) {
            k[i].octave = l;
            k[i].size = patchSize * sf;
            k[i].angle = orc_ic_angle(P.img[l], lw, halfPatch, k[i].x, k[i].y, umax);
        }
        if (desc && n > 0) {
            uint8_t *b = (uint8_t *)malloc((size_t)lw * lh);
            orc_orb_blur(P.img[l], lw, lh, b);
            for (i = 0; i < n; i++)
                if (total + i < cap) orc_orb_describe(b, lw, &k[i], pattern, desc + (size_t)(total + i) * 32);
            free(b);
        }
        for (i = 0; i < n; i++) {
            if (l != 0) {
                k[i].x *= sf;
                k[i].y *= sf;
            }
            if (out && total + i < cap) out[total + i] = k[i];
        }
        total += n;
        free(k);
    }
    free_pyramid(&P);
    free(nper);
    free(umax);
    free(pat);
    return total;
}

/* ORB::compute (DescriptorExtractor::compute: runByKeypointSize(FLT_EPSILON), then ORB::operator()
   with the provided keypoints: runByImageBorder(edgeThreshold), grouped by octave (level-major,
   input order within a level), pt / getScale(octave), descriptors on the blurred level, pt *
   getScale(octave)).  kept[m] = input index of output m.  Returns the count, or -1 for a negative
   octave (OpenCV indexes allKeypoints[-1]). */
ORC_API int orc_orb_compute(const uint8_t *img, int w, int h, const orc_kpt *kin, int n, double scaleFactor,
                            int edgeThreshold, int patchSize, const int *pattern, orc_kpt *kout, int *kept,
                            uint8_t *desc)
{
    orc_kpt *k;
    int *src, i, m = 0, L = 0, l, total = 0;
    int *pat = NULL;
    pyramid P;
    if (n <= 0 || w <= 0 || h <= 0) return 0;
    k = (orc_kpt *)malloc(sizeof(orc_kpt) * n);
    src = (int *)malloc(sizeof(int) * n);
    for (i = 0; i < n; i++) {
        const float s = kin[i].size;
        if (s < FLT_EPSILON || s > FLT_MAX) continue; /* SizePredicate (NaN is kept) */
        if (edgeThreshold > 0 && !in_border(kin[i].x, kin[i].y, w, h, edgeThreshold)) continue;
        if (kin[i].octave < 0) {
            free(k);
            free(src);
            return -1;
        }
        k[m] = kin[i];
        src[m++] = i;
    }
    if (edgeThreshold > 0 && (h <= 2 * edgeThreshold || w <= 2 * edgeThreshold)) m = 0;
    for (i = 0; i < m; i++) L = k[i].octave + 1 > L ? k[i].octave + 1 : L;
    if (m == 0) {
        free(k);
        free(src);
        return 0;
    }
    if (!pattern) {
        pat = (int *)malloc(sizeof(int) * 1024);
        orc_orb_random_pattern(patchSize, pat, 512);
        pattern = pat;
    }
    build_pyramid(img, w, h, scaleFactor, L, &P);
    for (l = 0; l < L; l++) {
        const float sf = orc_orb_scale(scaleFactor, l), inv = 1 / sf;
        uint8_t *b = NULL;
        for (i = 0; i < m; i++) {
            orc_kpt q;
            if (k[i].octave != l) continue;
            if (!b) {
                b = (uint8_t *)malloc((size_t)P.w[l] * P.h[l]);
                orc_orb_blur(P.img[l], P.w[l], P.h[l], b);
            }
            q = k[i];
            if (l != 0) {
                q.x *= inv;
                q.y *= inv;
            }
            orc_orb_describe(b, P.w[l], &q, pattern, desc + (size_t)total * 32);
            if (l != 0) {
                q.x *= sf;
                q.y *= sf;
            }
            kout[total] = q;
            if (kept) kept[total] = src[i];
            total++;
        }
        free(b);
    }
    free_pyramid(&P);
    free(k);
    free(src);
    free(pat);
    return total;
}
