/* orc_sift.c -- CPU restatement of OpenCV 2.4.9's SIFT (nonfree/src/sift.cpp and the core / imgproc
 * functions it calls), the detector / extractor DescriptorsMatcher builds for FeatureOptions
 * DetectorType / ExtractorType SIFT (reference DescriptorsMatcher/descriptorsmatcher.cpp:243-257,
 * 302-315: cv::SIFT(NumFeatures, NumOctaveLayers, ContrastThreshold, EdgeThreshold, Sigma); OpenCV's
 * defaults 0 / 3 / 0.04 / 10 / 1.6 when settings.yml names no values).
 *
 * TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py's cpu_baseline): the GPU
 * library never links or calls this file.  OpenCV (with its nonfree module) is not in this image, so
 * the restatement is pinned piece by piece by independent numpy restatements and exact properties
 * (tests/test_sift_oracle.py).  OpenCV 2.4.9's sift_wt is float (SIFT_FIXPT_SCALE 1).
 *
 * Steps, in OpenCV's operation order (x86-64 SSE2 build, no IPP):
 *   createInitialImage  gray -> float; doubled with resize(INTER_LINEAR) (float coefficients:
 *                       D = S0*a0 + S1*a1 per pass; x clamped with fx = 0 at the edges, y rows
 *                       clamped with fy kept) and GaussianBlur(sig_diff); or blurred in place
 *   GaussianBlur        getGaussianKernel(cvRound(sigma*8+1)|1, sigma, CV_32F); FilterEngine with
 *                       BORDER_REFLECT_101: RowFilter/RowVec_32f (sum over taps in order) then
 *                       SymmColumnFilter/SymmColumnVec_32f (f[0]*centre + 0, += f[k]*(up + down))
 *   buildGaussianPyramid  sig[i] = sqrt(sig_total^2 - sig_prev^2); octave bases by resize(INTER_NEAREST)
 *                       of level nOctaveLayers of the previous octave (cvFloor(x * (1 / inv_scale)))
 *   buildDoGPyramid     level i+1 - level i
 *   findScaleSpaceExtrema  |v| > cvFloor(0.5*ct/L*255) and >= / <= its 26 neighbours, scanned
 *                       octave, layer, row, column; adjustLocalExtrema (Matx33f::solve(DECOMP_LU) =
 *                       Cramer's rule with the float determinant, zeros when it is 0); calcOrientationHist
 *                       (cv::exp / fastAtan2 / magnitude over the compacted neighbourhood, 36 bins,
 *                       [1 4 6 4 1]/16 smoothing); one keypoint per peak >= 0.8 max
 *   removeDuplicated    KeyPoint_LessThan order (index as the last key), first of each equal group
 *   retainBest          std::nth_element + std::partition (orc_orb.c's libstdc++ restatement)
 *   firstOctave -1      octave byte - 1, pt and size * 0.5f
 *   compute             runByKeypointSize(FLT_EPSILON); the pyramid from firstOctave = min(0, octaves)
 *                       and nOctaves = max - first + 1; calcSIFTDescriptor (4x4x8, tri-linear, wrap,
 *                       0.2 clamp, * 512 / |.|, saturate_cast<uchar>)
 * cv::exp / fastAtan2 / cosf / sinf / powf come from include/fm3d_cvmath.h (shared with the GPU).
 */
#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "fm3d_cvmath.h"

#define ORC_API __attribute__((visibility("default")))

typedef struct {
    float x, y, size, angle, response;
    int octave, class_id;
} orc_kpt;

int orc_retain_best(orc_kpt *k, int n, int npts); /* orc_orb.c */

enum { SIFT_DESCR_WIDTH = 4, SIFT_DESCR_HIST_BINS = 8, SIFT_IMG_BORDER = 5, SIFT_MAX_INTERP_STEPS = 5,
       SIFT_ORI_HIST_BINS = 36 };
#define SIFT_INIT_SIGMA 0.5f
#define SIFT_ORI_SIG_FCTR 1.5f
#define SIFT_ORI_RADIUS (3 * SIFT_ORI_SIG_FCTR)
#define SIFT_ORI_PEAK_RATIO 0.8f
#define SIFT_DESCR_SCL_FCTR 3.f
#define SIFT_DESCR_MAG_THR 0.2f
#define SIFT_INT_DESCR_FCTR 512.f

typedef struct {
    int w, h;
    float *p;
} fimg;

/* 1: cosf / sinf / powf from this image's libm instead of the correctly rounded deterministic ones
   (a parity-risk variant: glibc's float functions are not correctly rounded, and which glibc the
   reference ran is not recorded) */
static int g_libm = 0;
ORC_API void orc_sift_set_libm(int on) { g_libm = on; }
static float s_cosf(float x) { return g_libm ? cosf(x) : fm3d_cv_cosf(x); }
static float s_sinf(float x) { return g_libm ? sinf(x) : fm3d_cv_sinf(x); }
static float s_exp2f(float y) { return g_libm ? powf(2.f, y) : fm3d_cv_exp2f(y); }

static float at(const fimg *m, int y, int x) { return m->p[(size_t)y * m->w + x]; }

/* ---------------------------------------------------------------- filters */
/* getGaussianKernel(n, sigma, CV_32F) */
ORC_API int orc_sift_gauss_ksize(double sigma) { return fm3d_cv_round(sigma * 4 * 2 + 1) | 1; }

ORC_API int orc_sift_gauss_kernel(double sigma, float *cf)
{
    const int n = orc_sift_gauss_ksize(sigma);
    const double scale2X = -0.5 / (sigma * sigma);
    double sum = 0;
    int i;
    for (i = 0; i < n; i++) {
        const double x = i - (n - 1) * 0.5;
        cf[i] = (float)exp(scale2X * x * x);
        sum += cf[i];
    }
    sum = 1. / sum;
    for (i = 0; i < n; i++) cf[i] = (float)(cf[i] * sum);
    return n;
}

/* GaussianBlur(src, dst, Size(), sigma, sigma) on a float image (src == dst allowed) */
ORC_API void orc_sift_blur(const float *src, float *dst, int w, int h, double sigma)
{
    float *f = (float *)malloc(sizeof(float) * (size_t)orc_sift_gauss_ksize(sigma));
    const int n = orc_sift_gauss_kernel(sigma, f), r = n / 2;
    float *tmp = (float *)malloc(sizeof(float) * (size_t)w * h);
    float *out = (float *)malloc(sizeof(float) * (size_t)w * h);
    int y;
#pragma omp parallel for schedule(static)
    for (y = 0; y < h; y++) {
        const float *S = src + (size_t)y * w;
        int x, k;
        for (x = 0; x < w; x++) {
            float s = f[0] * S[fm3d_cv_reflect101(x - r, w)];
            for (k = 1; k < n; k++) s += f[k] * S[fm3d_cv_reflect101(x - r + k, w)];
            tmp[(size_t)y * w + x] = s;
        }
    }
#pragma omp parallel for schedule(static)
    for (y = 0; y < h; y++) {
        int x, k;
        for (x = 0; x < w; x++) {
            float s = f[r] * tmp[(size_t)y * w + x] + 0.f;
            for (k = 1; k <= r; k++)
                s += f[r + k] * (tmp[(size_t)fm3d_cv_reflect101(y + k, h) * w + x] +
                                 tmp[(size_t)fm3d_cv_reflect101(y - k, h) * w + x]);
            out[(size_t)y * w + x] = s;
        }
    }
    memcpy(dst, out, sizeof(float) * (size_t)w * h);
    free(f);
    free(tmp);
    free(out);
}

/* resize(INTER_LINEAR) of a float image */
ORC_API void orc_sift_resize_linear(const float *src, int sw, int sh, float *dst, int dw, int dh)
{
    const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
    int *xofs = (int *)malloc(sizeof(int) * dw);
    float *alpha = (float *)malloc(sizeof(float) * 2 * dw);
    float *R0 = (float *)malloc(sizeof(float) * dw), *R1 = (float *)malloc(sizeof(float) * dw);
    int dx, dy, xmax = dw;
    for (dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = fm3d_cv_floorf(fx);
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
        alpha[2 * dx] = 1.f - fx;
        alpha[2 * dx + 1] = fx;
    }
    for (dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        const int sy = fm3d_cv_floorf(fy);
        const float *S0, *S1;
        float b0, b1;
        fy -= sy;
        b0 = 1.f - fy;
        b1 = fy;
        S0 = src + (size_t)(sy < 0 ? 0 : (sy >= sh ? sh - 1 : sy)) * sw;
        S1 = src + (size_t)(sy + 1 < 0 ? 0 : (sy + 1 >= sh ? sh - 1 : sy + 1)) * sw;
        for (dx = 0; dx < dw; dx++) {
            const int sx = xofs[dx];
            if (dx < xmax) {
                R0[dx] = S0[sx] * alpha[2 * dx] + S0[sx + 1] * alpha[2 * dx + 1];
                R1[dx] = S1[sx] * alpha[2 * dx] + S1[sx + 1] * alpha[2 * dx + 1];
            } else {
                R0[dx] = S0[sx];
                R1[dx] = S1[sx];
            }
        }
        for (dx = 0; dx < dw; dx++) dst[(size_t)dy * dw + dx] = R0[dx] * b0 + R1[dx] * b1;
    }
    free(xofs);
    free(alpha);
    free(R0);
    free(R1);
}

/* resize(INTER_NEAREST) */
ORC_API void orc_sift_resize_nn(const float *src, int sw, int sh, float *dst, int dw, int dh)
{
    const double ifx = 1. / ((double)dw / sw), ify = 1. / ((double)dh / sh);
    int x, y;
    for (y = 0; y < dh; y++) {
        int sy = (int)floor(y * ify);
        if (sy > sh - 1) sy = sh - 1;
        for (x = 0; x < dw; x++) {
            int sx = (int)floor(x * ifx);
            if (sx > sw - 1) sx = sw - 1;
            dst[(size_t)y * dw + x] = src[(size_t)sy * sw + sx];
        }
    }
}

/* ---------------------------------------------------------------- pyramids */
typedef struct {
    int L, nOct, firstOctave;
    fimg *g; /* nOct * (L + 3) */
    fimg *d; /* nOct * (L + 2), or NULL */
} pyr_t;

static void pyr_free(pyr_t *P)
{
    int i;
    if (P->g)
        for (i = 0; i < P->nOct * (P->L + 3); i++) free(P->g[i].p);
    if (P->d)
        for (i = 0; i < P->nOct * (P->L + 2); i++) free(P->d[i].p);
    free(P->g);
    free(P->d);
    P->g = P->d = NULL;
}

/* the octave count detection uses: cvRound(log(min(cols, rows)) / log(2) - 2) - firstOctave */
ORC_API int orc_sift_num_octaves(int w, int h, int firstOctave)
{
    const int bw = firstOctave < 0 ? 2 * w : w, bh = firstOctave < 0 ? 2 * h : h;
    return fm3d_cv_round(log((double)(bw < bh ? bw : bh)) / log(2.) - 2) - firstOctave;
}

/* sig[i] of buildGaussianPyramid */
ORC_API void orc_sift_sigmas(int L, double sigma, double *sig)
{
    const double k = pow(2., 1. / L);
    int i;
    sig[0] = sigma;
    for (i = 1; i < L + 3; i++) {
        const double sig_prev = pow(k, (double)(i - 1)) * sigma;
        const double sig_total = sig_prev * k;
        sig[i] = sqrt(sig_total * sig_total - sig_prev * sig_prev);
    }
}

/* createInitialImage + buildGaussianPyramid (+ buildDoGPyramid).  0, or -1 when an octave would be
   empty (OpenCV's resize asserts there) */
static int build_pyramids(const uint8_t *img, int w, int h, int firstOctave, int nOct, int L, double sigmaD, int dog,
                          pyr_t *P)
{
    const float sigma = (float)sigmaD; /* createInitialImage(img, first < 0, (float)sigma) */
    const int nl = L + 3;
    double sig[64];
    int o, i, bw, bh;
    float *gray;
    memset(P, 0, sizeof(*P));
    P->L = L;
    P->nOct = nOct;
    P->firstOctave = firstOctave;
    if (nOct < 1) return 0;
    P->g = (fimg *)calloc((size_t)nOct * nl, sizeof(fimg));
    if (dog) P->d = (fimg *)calloc((size_t)nOct * (L + 2), sizeof(fimg));
    gray = (float *)malloc(sizeof(float) * (size_t)w * h);
    for (i = 0; i < w * h; i++) gray[i] = (float)img[i];
    if (firstOctave < 0) {
        const float sig_diff = sqrtf(fmaxf(sigma * sigma - SIFT_INIT_SIGMA * SIFT_INIT_SIGMA * 4, 0.01f));
        bw = 2 * w;
        bh = 2 * h;
        P->g[0].p = (float *)malloc(sizeof(float) * (size_t)bw * bh);
        orc_sift_resize_linear(gray, w, h, P->g[0].p, bw, bh);
        orc_sift_blur(P->g[0].p, P->g[0].p, bw, bh, sig_diff);
        free(gray);
    } else {
        const float sig_diff = sqrtf(fmaxf(sigma * sigma - SIFT_INIT_SIGMA * SIFT_INIT_SIGMA, 0.01f));
        bw = w;
        bh = h;
        orc_sift_blur(gray, gray, w, h, sig_diff);
        P->g[0].p = gray;
    }
    P->g[0].w = bw;
    P->g[0].h = bh;
    orc_sift_sigmas(L, sigmaD, sig); /* buildGaussianPyramid: the double member */
    for (o = 0; o < nOct; o++)
        for (i = 0; i < nl; i++) {
            fimg *dst = &P->g[o * nl + i];
            if (o == 0 && i == 0) continue;
            if (i == 0) {
                const fimg *src = &P->g[(o - 1) * nl + L];
                dst->w = src->w / 2;
                dst->h = src->h / 2;
                if (dst->w < 1 || dst->h < 1) {
                    pyr_free(P);
                    return -1;
                }
                dst->p = (float *)malloc(sizeof(float) * (size_t)dst->w * dst->h);
                orc_sift_resize_nn(src->p, src->w, src->h, dst->p, dst->w, dst->h);
            } else {
                const fimg *src = &P->g[o * nl + i - 1];
                dst->w = src->w;
                dst->h = src->h;
                dst->p = (float *)malloc(sizeof(float) * (size_t)dst->w * dst->h);
                orc_sift_blur(src->p, dst->p, src->w, src->h, sig[i]);
            }
        }
    if (dog)
        for (o = 0; o < nOct; o++)
            for (i = 0; i < L + 2; i++) {
                const fimg *a = &P->g[o * nl + i], *b = &P->g[o * nl + i + 1];
                fimg *d = &P->d[o * (L + 2) + i];
                size_t q, np = (size_t)a->w * a->h;
                d->w = a->w;
                d->h = a->h;
                d->p = (float *)malloc(sizeof(float) * np);
                for (q = 0; q < np; q++) d->p[q] = b->p[q] - a->p[q];
            }
    return 0;
}

/* the Gaussian (dog = 0) or DoG (dog = 1) levels of a pyramid, concatenated octave-major; sizes:
   (w, h) per level.  Returns the number of floats (out / sizes may be NULL to ask). */
ORC_API long orc_sift_pyramid(const uint8_t *img, int w, int h, int firstOctave, int nOct, int L, double sigma,
                              int dog, float *out, int *sizes)
{
    pyr_t P;
    long tot = 0;
    int i, nl = dog ? L + 2 : L + 3;
    if (build_pyramids(img, w, h, firstOctave, nOct, L, sigma, dog, &P)) return -1;
    for (i = 0; i < nOct * nl; i++) {
        const fimg *m = dog ? &P.d[i] : &P.g[i];
        if (sizes) {
            sizes[2 * i] = m->w;
            sizes[2 * i + 1] = m->h;
        }
        if (out) memcpy(out + tot, m->p, sizeof(float) * (size_t)m->w * m->h);
        tot += (long)m->w * m->h;
    }
    pyr_free(&P);
    return tot;
}

/* ---------------------------------------------------------------- detection */
/* Matx<float,3,3>::solve(b, DECOMP_LU) = Matx_FastSolveOp<float,3,1>: Cramer's rule with the float
   determinant (Matx_DetOp<float,3>), zeros when it is 0 */
ORC_API void orc_sift_solve3(const float *a, const float *b, float *x)
{
#define A(i, j) a[(i) * 3 + (j)]
    float d = A(0, 0) * (A(1, 1) * A(2, 2) - A(2, 1) * A(1, 2)) - A(0, 1) * (A(1, 0) * A(2, 2) - A(2, 0) * A(1, 2)) +
              A(0, 2) * (A(1, 0) * A(2, 1) - A(2, 0) * A(1, 1));
    if (d == 0) {
        x[0] = x[1] = x[2] = 0;
        return;
    }
    d = 1 / d;
    x[0] = d * (b[0] * (A(1, 1) * A(2, 2) - A(1, 2) * A(2, 1)) - A(0, 1) * (b[1] * A(2, 2) - A(1, 2) * b[2]) +
                A(0, 2) * (b[1] * A(2, 1) - A(1, 1) * b[2]));
    x[1] = d * (A(0, 0) * (b[1] * A(2, 2) - A(1, 2) * b[2]) - b[0] * (A(1, 0) * A(2, 2) - A(1, 2) * A(2, 0)) +
                A(0, 2) * (A(1, 0) * b[2] - b[1] * A(2, 0)));
    x[2] = d * (A(0, 0) * (A(1, 1) * b[2] - b[1] * A(2, 1)) - A(0, 1) * (A(1, 0) * b[2] - b[1] * A(2, 0)) +
                b[0] * (A(1, 0) * A(2, 1) - A(1, 1) * A(2, 0)));
#undef A
}

/* adjustLocalExtrema; D: the DoG levels (nOct * (L + 2)) */
static int adjust_local_extrema(const fimg *D, orc_kpt *kpt, int octv, int *layer_, int *r_, int *c_, int L,
                                float contrastThreshold, float edgeThreshold, float sigma)
{
    const float img_scale = 1.f / (255 * 1);
    const float deriv_scale = img_scale * 0.5f;
    const float second_deriv_scale = img_scale;
    const float cross_deriv_scale = img_scale * 0.25f;
    float xi = 0, xr = 0, xc = 0, contr = 0;
    int i = 0, layer = *layer_, r = *r_, c = *c_;
    for (; i < SIFT_MAX_INTERP_STEPS; i++) {
        const int idx = octv * (L + 2) + layer;
        const fimg *img = &D[idx], *prev = &D[idx - 1], *next = &D[idx + 1];
        float dD[3], H[9], X[3];
        float v2, dxx, dyy, dss, dxy, dxs, dys;
        dD[0] = (at(img, r, c + 1) - at(img, r, c - 1)) * deriv_scale;
        dD[1] = (at(img, r + 1, c) - at(img, r - 1, c)) * deriv_scale;
        dD[2] = (at(next, r, c) - at(prev, r, c)) * deriv_scale;
        v2 = at(img, r, c) * 2;
        dxx = (at(img, r, c + 1) + at(img, r, c - 1) - v2) * second_deriv_scale;
        dyy = (at(img, r + 1, c) + at(img, r - 1, c) - v2) * second_deriv_scale;
        dss = (at(next, r, c) + at(prev, r, c) - v2) * second_deriv_scale;
        dxy = (at(img, r + 1, c + 1) - at(img, r + 1, c - 1) - at(img, r - 1, c + 1) + at(img, r - 1, c - 1)) *
              cross_deriv_scale;
        dxs = (at(next, r, c + 1) - at(next, r, c - 1) - at(prev, r, c + 1) + at(prev, r, c - 1)) * cross_deriv_scale;
        dys = (at(next, r + 1, c) - at(next, r - 1, c) - at(prev, r + 1, c) + at(prev, r - 1, c)) * cross_deriv_scale;
        H[0] = dxx; H[1] = dxy; H[2] = dxs;
        H[3] = dxy; H[4] = dyy; H[5] = dys;
        H[6] = dxs; H[7] = dys; H[8] = dss;
        orc_sift_solve3(H, dD, X);
        xi = -X[2];
        xr = -X[1];
        xc = -X[0];
        if (fabsf(xi) < 0.5f && fabsf(xr) < 0.5f && fabsf(xc) < 0.5f) break;
        if (fabsf(xi) > (float)(INT_MAX / 3) || fabsf(xr) > (float)(INT_MAX / 3) || fabsf(xc) > (float)(INT_MAX / 3))
            return 0;
        c += fm3d_cv_roundf(xc);
        r += fm3d_cv_roundf(xr);
        layer += fm3d_cv_roundf(xi);
        if (layer < 1 || layer > L || c < SIFT_IMG_BORDER || c >= img->w - SIFT_IMG_BORDER || r < SIFT_IMG_BORDER ||
            r >= img->h - SIFT_IMG_BORDER)
            return 0;
    }
    if (i >= SIFT_MAX_INTERP_STEPS) return 0;
    {
        const int idx = octv * (L + 2) + layer;
        const fimg *img = &D[idx], *prev = &D[idx - 1], *next = &D[idx + 1];
        const float d0 = (at(img, r, c + 1) - at(img, r, c - 1)) * deriv_scale;
        const float d1 = (at(img, r + 1, c) - at(img, r - 1, c)) * deriv_scale;
        const float d2 = (at(next, r, c) - at(prev, r, c)) * deriv_scale;
        float t = 0, v2, dxx, dyy, dxy, tr, det;
        t += d0 * xc;
        t += d1 * xr;
        t += d2 * xi;
        contr = at(img, r, c) * img_scale + t * 0.5f;
        if (fabsf(contr) * L < contrastThreshold) return 0;
        v2 = at(img, r, c) * 2.f;
        dxx = (at(img, r, c + 1) + at(img, r, c - 1) - v2) * second_deriv_scale;
        dyy = (at(img, r + 1, c) + at(img, r - 1, c) - v2) * second_deriv_scale;
        dxy = (at(img, r + 1, c + 1) - at(img, r + 1, c - 1) - at(img, r - 1, c + 1) + at(img, r - 1, c - 1)) *
              cross_deriv_scale;
        tr = dxx + dyy;
        det = dxx * dyy - dxy * dxy;
        if (det <= 0 || tr * tr * edgeThreshold >= (edgeThreshold + 1) * (edgeThreshold + 1) * det) return 0;
    }
    kpt->x = (c + xc) * (1 << octv);
    kpt->y = (r + xr) * (1 << octv);
    kpt->octave = octv + (layer << 8) + (fm3d_cv_round((xi + 0.5) * 255) << 16);
    kpt->size = sigma * s_exp2f((layer + xi) / L) * (1 << octv) * 2;
    kpt->response = fabsf(contr);
    *layer_ = layer;
    *r_ = r;
    *c_ = c;
    return 1;
}

/* calcOrientationHist; returns the largest smoothed bin */
ORC_API float orc_sift_ori_hist(const float *imgp, int w, int h, int px, int py, int radius, float sigma, float *hist,
                                int n)
{
    const fimg im = {w, h, (float *)imgp}, *img = &im;
    int i, j, k, len = (radius * 2 + 1) * (radius * 2 + 1);
    const float expf_scale = -1.f / (2.f * sigma * sigma);
    float *X = (float *)malloc(sizeof(float) * (size_t)len * 3 + 16), *Y = X + len, *W = Y + len;
    float th[64 + 4], *temphist = th + 2, maxval;
    for (i = 0; i < n; i++) temphist[i] = 0.f;
    for (i = -radius, k = 0; i <= radius; i++) {
        const int y = py + i;
        if (y <= 0 || y >= img->h - 1) continue;
        for (j = -radius; j <= radius; j++) {
            const int x = px + j;
            if (x <= 0 || x >= img->w - 1) continue;
            X[k] = at(img, y, x + 1) - at(img, y, x - 1);
            Y[k] = at(img, y - 1, x) - at(img, y + 1, x);
            W[k] = (i * i + j * j) * expf_scale;
            k++;
        }
    }
    len = k;
    for (k = 0; k < len; k++) {
        const float wk = fm3d_cv_exp_at(W[k], k, len);
        const float ori = fm3d_cv_atan2_deg(Y[k], X[k]);
        const float mag = sqrtf(X[k] * X[k] + Y[k] * Y[k]);
        int bin = fm3d_cv_roundf((n / 360.f) * ori);
        if (bin >= n) bin -= n;
        if (bin < 0) bin += n;
        temphist[bin] += wk * mag;
    }
    free(X);
    temphist[-1] = temphist[n - 1];
    temphist[-2] = temphist[n - 2];
    temphist[n] = temphist[0];
    temphist[n + 1] = temphist[1];
    for (i = 0; i < n; i++)
        hist[i] = (temphist[i - 2] + temphist[i + 2]) * (1.f / 16.f) + (temphist[i - 1] + temphist[i + 1]) * (4.f / 16.f) +
                  temphist[i] * (6.f / 16.f);
    maxval = hist[0];
    for (i = 1; i < n; i++) maxval = fmaxf(maxval, hist[i]);
    return maxval;
}

typedef struct {
    orc_kpt *k;
    int n, cap;
} kvec;

static void kpush(kvec *v, const orc_kpt *k)
{
    if (v->n == v->cap) {
        v->cap = v->cap ? 2 * v->cap : 1024;
        v->k = (orc_kpt *)realloc(v->k, sizeof(orc_kpt) * v->cap);
    }
    v->k[v->n++] = *k;
}

/* extremum test of findScaleSpaceExtrema at (r, c) of DoG layer idx */
static int is_extremum(const fimg *D, int idx, int r, int c, int threshold)
{
    const fimg *img = &D[idx], *prev = &D[idx - 1], *next = &D[idx + 1];
    const float val = at(img, r, c);
    int dy, dx;
    if (!(fabsf(val) > threshold)) return 0;
    if (val > 0) {
        for (dy = -1; dy <= 1; dy++)
            for (dx = -1; dx <= 1; dx++) {
                if (!(val >= at(img, r + dy, c + dx))) return 0;
                if (!(val >= at(prev, r + dy, c + dx))) return 0;
                if (!(val >= at(next, r + dy, c + dx))) return 0;
            }
        return 1;
    }
    if (val < 0) {
        for (dy = -1; dy <= 1; dy++)
            for (dx = -1; dx <= 1; dx++) {
                if (!(val <= at(img, r + dy, c + dx))) return 0;
                if (!(val <= at(prev, r + dy, c + dx))) return 0;
                if (!(val <= at(next, r + dy, c + dx))) return 0;
            }
        return 1;
    }
    return 0;
}

static void find_scale_space_extrema(const pyr_t *P, double contrastThreshold, double edgeThreshold, double sigma,
                                     kvec *out)
{
    const int L = P->L, n = SIFT_ORI_HIST_BINS;
    const int threshold = (int)floor(0.5 * contrastThreshold / L * 255 * 1);
    int o, i;
    for (o = 0; o < P->nOct; o++)
        for (i = 1; i <= L; i++) {
            const int idx = o * (L + 2) + i;
            const fimg *img = &P->d[idx];
            int r, c;
            for (r = SIFT_IMG_BORDER; r < img->h - SIFT_IMG_BORDER; r++)
                for (c = SIFT_IMG_BORDER; c < img->w - SIFT_IMG_BORDER; c++) {
                    orc_kpt kpt;
                    float hist[SIFT_ORI_HIST_BINS], scl_octv, omax, mag_thr;
                    const fimg *g;
                    int r1 = r, c1 = c, layer = i, j;
                    if (!is_extremum(P->d, idx, r, c, threshold)) continue;
                    memset(&kpt, 0, sizeof(kpt));
                    kpt.class_id = -1;
                    if (!adjust_local_extrema(P->d, &kpt, o, &layer, &r1, &c1, L, (float)contrastThreshold,
                                              (float)edgeThreshold, (float)sigma))
                        continue;
                    scl_octv = kpt.size * 0.5f / (1 << o);
                    g = &P->g[o * (L + 3) + layer];
                    omax = orc_sift_ori_hist(g->p, g->w, g->h, c1, r1, fm3d_cv_roundf(SIFT_ORI_RADIUS * scl_octv),
                                             SIFT_ORI_SIG_FCTR * scl_octv, hist, n);
                    mag_thr = omax * SIFT_ORI_PEAK_RATIO;
                    for (j = 0; j < n; j++) {
                        const int l = j > 0 ? j - 1 : n - 1;
                        const int r2 = j < n - 1 ? j + 1 : 0;
                        if (hist[j] > hist[l] && hist[j] > hist[r2] && hist[j] >= mag_thr) {
                            float bin = j + 0.5f * (hist[l] - hist[r2]) / (hist[l] - 2 * hist[j] + hist[r2]);
                            bin = bin < 0 ? n + bin : (bin >= n ? bin - n : bin);
                            kpt.angle = 360.f - (float)((360.f / n) * bin);
                            if (fabsf(kpt.angle - 360.f) < FLT_EPSILON) kpt.angle = 0.f;
                            kpush(out, &kpt);
                        }
                    }
                }
        }
}

/* KeyPoint_LessThan, the index as the last key */
static const orc_kpt *g_lt_k;
static int kp_less(int i, int j)
{
    const orc_kpt *a = &g_lt_k[i], *b = &g_lt_k[j];
    if (a->x != b->x) return a->x < b->x;
    if (a->y != b->y) return a->y < b->y;
    if (a->size != b->size) return a->size > b->size;
    if (a->angle != b->angle) return a->angle < b->angle;
    if (a->response != b->response) return a->response > b->response;
    if (a->octave != b->octave) return a->octave > b->octave;
    if (a->class_id != b->class_id) return a->class_id > b->class_id;
    return i < j;
}
static int kp_cmp(const void *pa, const void *pb)
{
    const int i = *(const int *)pa, j = *(const int *)pb;
    return kp_less(i, j) ? -1 : (kp_less(j, i) ? 1 : 0);
}

/* KeyPointsFilter::removeDuplicated */
ORC_API int orc_remove_duplicated(orc_kpt *k, int n)
{
    int *idx, i, j;
    unsigned char *mask;
    if (n < 2) return n;
    idx = (int *)malloc(sizeof(int) * n);
    mask = (unsigned char *)malloc(n);
    for (i = 0; i < n; i++) {
        idx[i] = i;
        mask[i] = 1;
    }
    g_lt_k = k;
    qsort(idx, n, sizeof(int), kp_cmp);
    for (i = 1, j = 0; i < n; i++) {
        const orc_kpt *a = &k[idx[i]], *b = &k[idx[j]];
        if (a->x != b->x || a->y != b->y || a->size != b->size || a->angle != b->angle)
            j = i;
        else
            mask[idx[i]] = 0;
    }
    for (i = j = 0; i < n; i++)
        if (mask[i]) {
            if (i != j) k[j] = k[i];
            j++;
        }
    free(idx);
    free(mask);
    return j;
}

/* ---------------------------------------------------------------- description */
/* calcSIFTDescriptor(img, ptf, ori, scl, d = 4, n = 8, dst) */
ORC_API void orc_sift_descriptor(const float *imgp, int w, int h, float ptx, float pty, float ori, float scl, float *dst)
{
    const int d = SIFT_DESCR_WIDTH, n = SIFT_DESCR_HIST_BINS;
    const fimg im = {w, h, (float *)imgp}, *img = &im;
    const int ptX = fm3d_cv_roundf(ptx), ptY = fm3d_cv_roundf(pty);
    float cos_t = s_cosf(ori * (float)(3.141592653589793238462643383279502884 / 180));
    float sin_t = s_sinf(ori * (float)(3.141592653589793238462643383279502884 / 180));
    const float bins_per_rad = n / 360.f;
    const float exp_scale = -1.f / (d * d * 0.5f);
    const float hist_width = SIFT_DESCR_SCL_FCTR * scl;
    int radius = fm3d_cv_roundf(hist_width * 1.4142135623730951f * (d + 1) * 0.5f);
    const int rows = img->h, cols = img->w;
    int i, j, k, len, histlen = (d + 2) * (d + 2) * (n + 2);
    float *X, *Y, *W, *RBin, *CBin, *hist, nrm2, thr;
    {
        const int diag = (int)sqrt((double)img->w * img->w + img->h * img->h);
        if (radius > diag) radius = diag;
    }
    cos_t /= hist_width;
    sin_t /= hist_width;
    len = (radius * 2 + 1) * (radius * 2 + 1);
    X = (float *)malloc(sizeof(float) * ((size_t)len * 5 + histlen));
    Y = X + len;
    W = Y + len;
    RBin = W + len;
    CBin = RBin + len;
    hist = CBin + len;
    for (i = 0; i < histlen; i++) hist[i] = 0.f;
    for (i = -radius, k = 0; i <= radius; i++)
        for (j = -radius; j <= radius; j++) {
            const float c_rot = j * cos_t - i * sin_t;
            const float r_rot = j * sin_t + i * cos_t;
            const float rbin = r_rot + d / 2 - 0.5f;
            const float cbin = c_rot + d / 2 - 0.5f;
            const int r = ptY + i, c = ptX + j;
            if (rbin > -1 && rbin < d && cbin > -1 && cbin < d && r > 0 && r < rows - 1 && c > 0 && c < cols - 1) {
                X[k] = at(img, r, c + 1) - at(img, r, c - 1);
                Y[k] = at(img, r - 1, c) - at(img, r + 1, c);
                RBin[k] = rbin;
                CBin[k] = cbin;
                W[k] = (c_rot * c_rot + r_rot * r_rot) * exp_scale;
                k++;
            }
        }
    len = k;
    for (k = 0; k < len; k++) {
        float rbin = RBin[k], cbin = CBin[k];
        const float Ori = fm3d_cv_atan2_deg(Y[k], X[k]);
        const float Mag = sqrtf(X[k] * X[k] + Y[k] * Y[k]);
        const float Wk = fm3d_cv_exp_at(W[k], k, len);
        float obin = (Ori - ori) * bins_per_rad;
        const float mag = Mag * Wk;
        const int r0 = fm3d_cv_floorf(rbin), c0 = fm3d_cv_floorf(cbin);
        int o0 = fm3d_cv_floorf(obin), idx;
        float v_r1, v_r0, v_rc11, v_rc10, v_rc01, v_rc00;
        float v_rco111, v_rco110, v_rco101, v_rco100, v_rco011, v_rco010, v_rco001, v_rco000;
        rbin -= r0;
        cbin -= c0;
        obin -= o0;
        if (o0 < 0) o0 += n;
        if (o0 >= n) o0 -= n;
        v_r1 = mag * rbin;
        v_r0 = mag - v_r1;
        v_rc11 = v_r1 * cbin;
        v_rc10 = v_r1 - v_rc11;
        v_rc01 = v_r0 * cbin;
        v_rc00 = v_r0 - v_rc01;
        v_rco111 = v_rc11 * obin;
        v_rco110 = v_rc11 - v_rco111;
        v_rco101 = v_rc10 * obin;
        v_rco100 = v_rc10 - v_rco101;
        v_rco011 = v_rc01 * obin;
        v_rco010 = v_rc01 - v_rco011;
        v_rco001 = v_rc00 * obin;
        v_rco000 = v_rc00 - v_rco001;
        idx = ((r0 + 1) * (d + 2) + c0 + 1) * (n + 2) + o0;
        hist[idx] += v_rco000;
        hist[idx + 1] += v_rco001;
        hist[idx + (n + 2)] += v_rco010;
        hist[idx + (n + 3)] += v_rco011;
        hist[idx + (d + 2) * (n + 2)] += v_rco100;
        hist[idx + (d + 2) * (n + 2) + 1] += v_rco101;
        hist[idx + (d + 3) * (n + 2)] += v_rco110;
        hist[idx + (d + 3) * (n + 2) + 1] += v_rco111;
    }
    for (i = 0; i < d; i++)
        for (j = 0; j < d; j++) {
            const int idx = ((i + 1) * (d + 2) + (j + 1)) * (n + 2);
            hist[idx] += hist[idx + n];
            hist[idx + 1] += hist[idx + n + 1];
            for (k = 0; k < n; k++) dst[(i * d + j) * n + k] = hist[idx + k];
        }
    len = d * d * n;
    nrm2 = 0;
    for (k = 0; k < len; k++) nrm2 += dst[k] * dst[k];
    thr = sqrtf(nrm2) * SIFT_DESCR_MAG_THR;
    for (i = 0, nrm2 = 0; i < k; i++) {
        const float val = fminf(dst[i], thr);
        dst[i] = val;
        nrm2 += val * val;
    }
    nrm2 = SIFT_INT_DESCR_FCTR / fmaxf(sqrtf(nrm2), FLT_EPSILON);
    for (k = 0; k < len; k++) {
        const int v = fm3d_cv_roundf(dst[k] * nrm2);
        dst[k] = (float)(v < 0 ? 0 : (v > 255 ? 255 : v));
    }
    free(X);
}

static void unpack_octave(const orc_kpt *k, int *octave, int *layer, float *scale)
{
    int o = k->octave & 255;
    *layer = (k->octave >> 8) & 255;
    o = o < 128 ? o : (-128 | o);
    *octave = o;
    *scale = o >= 0 ? 1.f / (1 << o) : (float)(1 << -o);
}

/* DescriptorExtractor::compute with the SIFT extractor: runByKeypointSize(FLT_EPSILON), then
   SIFT::operator()(img, Mat(), kpts, desc, true).  kout / kept: capacity n.  Returns the kept count,
   or -1 when OpenCV asserts (firstOctave < -1, a layer above nOctaveLayers + 2 or an octave
   the image cannot hold) */
ORC_API int orc_sift_compute(const uint8_t *img, int w, int h, int L, double sigma, const orc_kpt *kin, int n,
                             orc_kpt *kout, int *kept, float *desc)
{
    int i, m = 0, firstOctave = 0, maxOctave = INT_MIN, actualNLayers = 0;
    pyr_t P;
    for (i = 0; i < n; i++)
        if (!(kin[i].size < FLT_EPSILON || kin[i].size > FLT_MAX)) {
            kout[m] = kin[i];
            if (kept) kept[m] = i;
            m++;
        }
    if (m == 0) return 0;
    for (i = 0; i < m; i++) {
        int octave, layer;
        float scale;
        unpack_octave(&kout[i], &octave, &layer, &scale);
        if (octave < firstOctave) firstOctave = octave;
        if (octave > maxOctave) maxOctave = octave;
        if (layer - 2 > actualNLayers) actualNLayers = layer - 2;
    }
    if (firstOctave > 0) firstOctave = 0;
    if (firstOctave < -1 || actualNLayers > L) return -1;
    if (build_pyramids(img, w, h, firstOctave, maxOctave - firstOctave + 1, L, sigma, 0, &P)) return -1;
    for (i = 0; i < m; i++) {
        int octave, layer;
        float scale;
        unpack_octave(&kout[i], &octave, &layer, &scale);
        if (!(octave >= firstOctave && layer <= L + 2)) {
            pyr_free(&P);
            return -1;
        }
    }
#pragma omp parallel for schedule(dynamic, 16)
    for (i = 0; i < m; i++) {
        const orc_kpt *kp = &kout[i];
        int octave, layer;
        float scale, size, angle;
        const fimg *g;
        unpack_octave(kp, &octave, &layer, &scale);
        size = kp->size * scale;
        g = &P.g[(octave - firstOctave) * (L + 3) + layer];
        angle = 360.f - kp->angle;
        if (fabsf(angle - 360.f) < FLT_EPSILON) angle = 0.f;
        orc_sift_descriptor(g->p, g->w, g->h, kp->x * scale, kp->y * scale, angle, size * 0.5f, desc + (size_t)i * 128);
    }
    pyr_free(&P);
    return m;
}

/* FeatureDetector::detect with the SIFT detector (SIFT::operator()(img, Mat(), kpts, noArray())).
   stage 1: the raw findScaleSpaceExtrema list (doubled-image coordinates, before removeDuplicated).
   Returns the number of keypoints (all of them; min(n, cap) written). */
ORC_API int orc_sift_detect(const uint8_t *img, int w, int h, int nfeatures, int L, double contrastThreshold,
                            double edgeThreshold, double sigma, int stage, orc_kpt *out, int cap)
{
    const int firstOctave = -1;
    pyr_t P;
    kvec v = {NULL, 0, 0};
    int i, n;
    const int nOct = orc_sift_num_octaves(w, h, firstOctave);
    if (build_pyramids(img, w, h, firstOctave, nOct, L, sigma, 1, &P)) return -1;
    find_scale_space_extrema(&P, contrastThreshold, edgeThreshold, sigma, &v);
    pyr_free(&P);
    n = v.n;
    if (stage != 1) {
        n = orc_remove_duplicated(v.k, n);
        if (nfeatures > 0) n = orc_retain_best(v.k, n, nfeatures);
        for (i = 0; i < n; i++) {
            orc_kpt *k = &v.k[i];
            const float scale = 1.f / (float)(1 << -firstOctave);
            k->octave = (k->octave & ~255) | ((k->octave + firstOctave) & 255);
            k->x *= scale;
            k->y *= scale;
            k->size *= scale;
        }
    }
    for (i = 0; i < n && i < cap; i++) out[i] = v.k[i];
    free(v.k);
    return n;
}

/* float primitives, for the tests */
ORC_API float orc_cv_exp_at(float x, int k, int n) { return fm3d_cv_exp_at(x, k, n); }
ORC_API float orc_cv_exp2f(float y) { return fm3d_cv_exp2f(y); }
ORC_API float orc_cv_cosf(float x) { return fm3d_cv_cosf(x); }
ORC_API float orc_cv_sinf(float x) { return fm3d_cv_sinf(x); }
ORC_API float orc_cv_atan2_deg(float y, float x) { return fm3d_cv_atan2_deg(y, x); }
