/*
 * orc_surf.c -- CPU ORACLE of the reference's feature detection + description.
 *
 * TEST INFRASTRUCTURE ONLY (same rules as fm3d_oracle.c: loaded by tests/ and the cpu_baseline
 * leg only; the product never links it).
 *
 * The reference builds a SURF detector and extractor from build/settings.yml:37-49
 * (DescriptorsMatcher::generateDetector / generateExtractor, descriptorsmatcher.cpp:176-359:
 * HessianThreshold 400, NumOctaves 4, NumOctaveLayers 2, Extended 1, Upright 1) and calls
 * detect + compute on both images (compareWithNNDR, :110-115) and on the exported patches
 * (extractDescriptorsFromPatches, :133-174).  SURF lives in OpenCV 2.4's nonfree module, which is
 * not in this image; this file restates its published 2.4 algorithm (nonfree/src/surf.cpp):
 *   integral(img, sum, CV_32S);
 *   fastHessianDetector: (nOctaveLayers+2)*nOctaves layers, size (9 + 6*layer) << octave, sample
 *     step 1 << octave; calcLayerDetAndTrace with the resized Haar patterns (resizeHaarPattern);
 *     findMaximaInLayer: threshold, 3x3x3 non-maximum suppression, interpolateKeypoint (Matx33f
 *     solve = Cramer's rule with the float determinant); sort by KeypointGreater;
 *   SURFInvoker (upright): keypoints whose 2*cvRound(2s) wavelet exceeds the integral image are
 *     dropped; the 21s x 21s window (border replicated, rotated by 270 degrees), resize to 21x21 with
 *     INTER_AREA (the integer-scale fast path or computeResizeAreaTab), 2x2 Haar gradients weighted
 *     by a 20x20 Gaussian (sigma 3.3), 4x4 subregions of 8 (extended) or 4 sums, unit length.
 * Float / double types and operation order follow that source, no FMA contraction.  Choices where
 * the 2.4.x releases differ: the 2x2 fast area path rounds (sum + 2) >> 2 for the first 16 of the 21
 * outputs of a row (the SSE2 build's 8-wide steps) and cvRound(sum / 4) for the rest; ties of
 * KeypointGreater keep the sequential (layer, row, column) discovery order.
 * Parity vs OpenCV itself: UNPINNED (no OpenCV here); see DESIGN.md.
 */
#include <float.h>
#include <math.h>
#include "fm3d_detmath.h"
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_API __attribute__((visibility("default")))

typedef struct orc_kpt {
    float x, y, size, angle, response;
    int octave, class_id;
} orc_kpt;

typedef struct {
    int p0, p1, p2, p3;
    float w;
} orc_hf;

/* cvRound: round to nearest, ties to even (cvtsd2si in the default rounding mode) */
static int cv_round(double v) { return (int)lrint(v); }

static void resize_haar(const int src[][5], orc_hf *dst, int n, int oldSize, int newSize, int widthStep)
{
    const float ratio = (float)newSize / oldSize;
    int k;
    for (k = 0; k < n; k++) {
        const int dx1 = cv_round(ratio * src[k][0]);
        const int dy1 = cv_round(ratio * src[k][1]);
        const int dx2 = cv_round(ratio * src[k][2]);
        const int dy2 = cv_round(ratio * src[k][3]);
        dst[k].p0 = dy1 * widthStep + dx1;
        dst[k].p1 = dy2 * widthStep + dx1;
        dst[k].p2 = dy1 * widthStep + dx2;
        dst[k].p3 = dy2 * widthStep + dx2;
        dst[k].w = src[k][4] / ((float)(dx2 - dx1) * (dy2 - dy1));
    }
}

static float haar(const int *origin, const orc_hf *f, int n)
{
    double d = 0;
    int k;
    for (k = 0; k < n; k++) d += (origin[f[k].p0] + origin[f[k].p3] - origin[f[k].p1] - origin[f[k].p2]) * f[k].w;
    return (float)d;
}

static const int DX_S[3][5] = {{0, 2, 3, 7, 1}, {3, 2, 6, 7, -2}, {6, 2, 9, 7, 1}};
static const int DY_S[3][5] = {{2, 0, 7, 3, 1}, {2, 3, 7, 6, -2}, {2, 6, 7, 9, 1}};
static const int DXY_S[4][5] = {{1, 1, 4, 4, 1}, {5, 1, 8, 4, -1}, {1, 5, 4, 8, -1}, {5, 5, 8, 8, 1}};
/* SURFInvoker's orientation wavelets (dx_s / dy_s, 4x4 base size) */
static const int DXO_S[2][5] = {{0, 0, 2, 4, -1}, {2, 0, 4, 4, 1}};
static const int DYO_S[2][5] = {{0, 0, 4, 2, 1}, {0, 2, 4, 4, -1}};

ORC_API void orc_integral(const uint8_t *img, int w, int h, int *sum)
{
    int x, y;
    for (x = 0; x <= w; x++) sum[x] = 0;
    for (y = 0; y < h; y++) {
        int s = 0;
        int *row = sum + (size_t)(y + 1) * (w + 1);
        const int *prev = row - (w + 1);
        row[0] = 0;
        for (x = 0; x < w; x++) {
            s += img[(size_t)y * w + x];
            row[x + 1] = prev[x + 1] + s;
        }
    }
}

/* Matx33f::solve(b, DECOMP_LU) for 3x1: Matx_FastSolveOp<float, 3, 1> (Cramer's rule) */
static int solve3(const float a[9], const float b[3], float x[3])
{
#define A_(i, j) a[(i)*3 + (j)]
    float d = (float)(A_(0, 0) * (A_(1, 1) * A_(2, 2) - A_(2, 1) * A_(1, 2)) -
                      A_(0, 1) * (A_(1, 0) * A_(2, 2) - A_(2, 0) * A_(1, 2)) +
                      A_(0, 2) * (A_(1, 0) * A_(2, 1) - A_(2, 0) * A_(1, 1)));
    if (d == 0) {
        x[0] = x[1] = x[2] = 0;
        return 0;
    }
    d = 1 / d;
    x[0] = d * (b[0] * (A_(1, 1) * A_(2, 2) - A_(1, 2) * A_(2, 1)) - A_(0, 1) * (b[1] * A_(2, 2) - A_(1, 2) * b[2]) +
                A_(0, 2) * (b[1] * A_(2, 1) - A_(1, 1) * b[2]));
    x[1] = d * (A_(0, 0) * (b[1] * A_(2, 2) - A_(1, 2) * b[2]) - b[0] * (A_(1, 0) * A_(2, 2) - A_(1, 2) * A_(2, 0)) +
                A_(0, 2) * (A_(1, 0) * b[2] - b[1] * A_(2, 0)));
    x[2] = d * (A_(0, 0) * (A_(1, 1) * b[2] - b[1] * A_(2, 1)) - A_(0, 1) * (A_(1, 0) * b[2] - b[1] * A_(2, 0)) +
                b[0] * (A_(1, 0) * A_(2, 1) - A_(1, 1) * A_(2, 0)));
#undef A_
    return 1;
}

/* interpolateKeypoint: one Newton step of the 3D quadratic through the 3x3x3 samples */
static int interpolate(const float N9[3][9], int dx, int dy, int ds, orc_kpt *k)
{
    const float b[3] = {-(N9[1][5] - N9[1][3]) / 2, -(N9[1][7] - N9[1][1]) / 2, -(N9[2][4] - N9[0][4]) / 2};
    const float dxx = N9[1][3] - 2 * N9[1][4] + N9[1][5];
    const float dxy = (N9[1][8] - N9[1][6] - N9[1][2] + N9[1][0]) / 4;
    const float dxs = (N9[2][5] - N9[2][3] - N9[0][5] + N9[0][3]) / 4;
    const float dyy = N9[1][1] - 2 * N9[1][4] + N9[1][7];
    const float dys = (N9[2][7] - N9[2][1] - N9[0][7] + N9[0][1]) / 4;
    const float dss = N9[0][4] - 2 * N9[1][4] + N9[2][4];
    const float A[9] = {dxx, dxy, dxs, dxy, dyy, dys, dxs, dys, dss};
    float x[3];
    int ok;
    solve3(A, b, x);
    ok = (x[0] != 0 || x[1] != 0 || x[2] != 0) && fabsf(x[0]) <= 1 && fabsf(x[1]) <= 1 && fabsf(x[2]) <= 1;
    if (ok) {
        k->x += x[0] * dx;
        k->y += x[1] * dy;
        k->size = (float)cv_round(k->size + x[2] * ds);
    }
    return ok;
}

typedef struct {
    orc_kpt k;
    long long seq; /* discovery order (middle layer, row, column) */
} kseq;

/* KeypointGreater (response, size, octave descending; y, x descending), then discovery order */
static int kcmp(const void *pa, const void *pb)
{
    const kseq *a = (const kseq *)pa, *b = (const kseq *)pb;
    if (a->k.response > b->k.response) return -1;
    if (a->k.response < b->k.response) return 1;
    if (a->k.size > b->k.size) return -1;
    if (a->k.size < b->k.size) return 1;
    if (a->k.octave > b->k.octave) return -1;
    if (a->k.octave < b->k.octave) return 1;
    if (a->k.y < b->k.y) return 1;
    if (a->k.y > b->k.y) return -1;
    if (a->k.x > b->k.x) return -1;
    if (a->k.x < b->k.x) return 1;
    return a->seq < b->seq ? -1 : (a->seq > b->seq ? 1 : 0);
}

/* fastHessianDetector + the detect-time SURFInvoker pass (upright: angle 270, oversized wavelets
   dropped).  Returns the number of keypoints (<= cap written). */
static int surf_orientation(const int *sum, int w, int h, orc_kpt *k);
ORC_API int orc_surf_detect2(const uint8_t *img, int w, int h, float thr, int nOctaves, int nOctaveLayers,
                             int upright, orc_kpt *out, int cap)
{
    const int W1 = w + 1, nTotal = (nOctaveLayers + 2) * nOctaves;
    int *sum = (int *)malloc(sizeof(int) * (size_t)W1 * (h + 1));
    float **det = (float **)calloc(nTotal, sizeof(float *)), **tr = (float **)calloc(nTotal, sizeof(float *));
    int *sizes = (int *)malloc(sizeof(int) * nTotal), *steps = (int *)malloc(sizeof(int) * nTotal);
    kseq *ks = NULL;
    size_t nk = 0, capk = 0;
    int o, l, idx = 0, n = 0;
    size_t q;
    orc_integral(img, w, h, sum);
    for (o = 0; o < nOctaves; o++)
        for (l = 0; l < nOctaveLayers + 2; l++, idx++) {
            const int step = 1 << o, rows = h / step, cols = w / step;
            sizes[idx] = (9 + 6 * l) << o;
            steps[idx] = step;
            det[idx] = (float *)calloc((size_t)rows * cols + 1, sizeof(float));
            tr[idx] = (float *)calloc((size_t)rows * cols + 1, sizeof(float));
        }
    /* calcLayerDetAndTrace */
    for (idx = 0; idx < nTotal; idx++) {
        const int size = sizes[idx], step = steps[idx], cols = w / step;
        orc_hf Dx[3], Dy[3], Dxy[4];
        int i, j, si, sj, margin;
        if (size > h || size > w) continue;
        resize_haar(DX_S, Dx, 3, 9, size, W1);
        resize_haar(DY_S, Dy, 3, 9, size, W1);
        resize_haar(DXY_S, Dxy, 4, 9, size, W1);
        si = 1 + (h - size) / step;
        sj = 1 + (w - size) / step;
        margin = (size / 2) / step;
        for (i = 0; i < si; i++)
            for (j = 0; j < sj; j++) {
                const int *origin = sum + (size_t)i * step * W1 + (size_t)j * step;
                const float dx = haar(origin, Dx, 3), dy = haar(origin, Dy, 3), dxy = haar(origin, Dxy, 4);
                det[idx][(size_t)(i + margin) * cols + j + margin] = dx * dy - 0.81f * dxy * dxy;
                tr[idx][(size_t)(i + margin) * cols + j + margin] = dx + dy;
            }
    }
    /* findMaximaInLayer for every middle layer, in (octave, layer) order */
    for (o = 0; o < nOctaves; o++)
        for (l = 1; l <= nOctaveLayers; l++) {
            const int L = o * (nOctaveLayers + 2) + l, size = sizes[L], step = steps[L];
            const int rows = h / step, cols = w / step, margin = (sizes[L + 1] / 2) / step + 1;
            int i, j;
            for (i = margin; i < rows - margin; i++)
                for (j = margin; j < cols - margin; j++) {
                    const float val0 = det[L][(size_t)i * cols + j];
                    float N9[3][9];
                    int a, b, c, ismax = 1;
                    if (!(val0 > thr)) continue;
                    for (a = 0; a < 3; a++)
                        for (b = -1; b <= 1; b++)
                            for (c = -1; c <= 1; c++) N9[a][(b + 1) * 3 + c + 1] = det[L - 1 + a][(size_t)(i + b) * cols + j + c];
                    for (a = 0; a < 3 && ismax; a++)
                        for (b = 0; b < 9; b++)
                            if (!(a == 1 && b == 4) && !(val0 > N9[a][b])) {
                                ismax = 0;
                                break;
                            }
                    if (!ismax) continue;
                    {
                        const int sum_i = step * (i - (size / 2) / step), sum_j = step * (j - (size / 2) / step);
                        const float ci = sum_i + (size - 1) * 0.5f, cj = sum_j + (size - 1) * 0.5f;
                        const float t = tr[L][(size_t)i * cols + j];
                        orc_kpt k;
                        k.x = cj;
                        k.y = ci;
                        k.size = (float)sizes[L];
                        k.angle = -1;
                        k.response = val0;
                        k.octave = o;
                        k.class_id = (t > 0) - (t < 0);
                        if (interpolate((const float(*)[9])N9, step, step, size - sizes[L - 1], &k)) {
                            if (nk == capk) {
                                capk = capk ? 2 * capk : 1024;
                                ks = (kseq *)realloc(ks, capk * sizeof(kseq));
                            }
                            ks[nk].k = k;
                            ks[nk].seq = ((long long)L << 42) | ((long long)i << 21) | j;
                            nk++;
                        }
                    }
                }
        }
    if (nk > 1) qsort(ks, nk, sizeof(kseq), kcmp);
    /* SURFInvoker (detect): the gradient wavelet must fit the integral image; upright angle 270,
       else the dominant orientation (no orientation sample inside the image: dropped) */
    for (q = 0; q < nk; q++) {
        orc_kpt k = ks[q].k;
        const float s = k.size * 1.2f / 9.0f;
        const int gws = 2 * cv_round(2 * s);
        if (h + 1 < gws || w + 1 < gws) continue;
        if (upright) k.angle = 360.f - 90.f;
        else if (!surf_orientation(sum, w, h, &k)) continue;
        if (n < cap) out[n] = k;
        n++;
    }
    for (idx = 0; idx < nTotal; idx++) {
        free(det[idx]);
        free(tr[idx]);
    }
    free(det);
    free(tr);
    free(sizes);
    free(steps);
    free(sum);
    free(ks);
    return n;
}
ORC_API int orc_surf_detect(const uint8_t *img, int w, int h, float thr, int nOctaves, int nOctaveLayers,
                            orc_kpt *out, int cap)
{
    return orc_surf_detect2(img, w, h, thr, nOctaves, nOctaveLayers, 1, out, cap);
}

/* getGaussianKernel(n, sigma, CV_32F) */
static void gaussian_kernel(int n, double sigma, float *cf)
{
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
}

/* cv::fastAtan2 (OpenCV 2.4.9+ core/mathfuncs.cpp; FastAtan2_32f's SSE2 and scalar paths compute the
   same float operations): degrees in [0, 360) */
#define ORC_ATAN2_P1 (0.9997878412794807f * (float)(180 / M_PI))
#define ORC_ATAN2_P3 (-0.3258083974640975f * (float)(180 / M_PI))
#define ORC_ATAN2_P5 (0.1555786518463281f * (float)(180 / M_PI))
#define ORC_ATAN2_P7 (-0.04432655554792128f * (float)(180 / M_PI))
static float fast_atan2f(float y, float x)
{
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((ORC_ATAN2_P7 * c2 + ORC_ATAN2_P5) * c2 + ORC_ATAN2_P3) * c2 + ORC_ATAN2_P1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((ORC_ATAN2_P7 * c2 + ORC_ATAN2_P5) * c2 + ORC_ATAN2_P3) * c2 + ORC_ATAN2_P1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}
ORC_API float orc_fast_atan2(float y, float x) { return fast_atan2f(y, x); }

/* the orientation samples of the SURFInvoker constructor: the disc of radius ORI_RADIUS = 6
   (i outer = x, j inner = y), weights G(i) * G(j) with G = getGaussianKernel(13, 2.5, CV_32F) */
enum { ORI_RADIUS = 6, ORI_SAMPLES_MAX = (2 * 6 + 1) * (2 * 6 + 1), ORI_SEARCH_INC = 5, ORI_WIN = 60 };
static void gaussian_kernel(int n, double sigma, float *cf);
static int ori_samples(int apt[][2], float *aptw)
{
    float g[2 * ORI_RADIUS + 1];
    int i, j, n = 0;
    gaussian_kernel(2 * ORI_RADIUS + 1, 2.5, g);
    for (i = -ORI_RADIUS; i <= ORI_RADIUS; i++)
        for (j = -ORI_RADIUS; j <= ORI_RADIUS; j++)
            if (i * i + j * j <= ORI_RADIUS * ORI_RADIUS) {
                apt[n][0] = i;
                apt[n][1] = j;
                aptw[n++] = g[i + ORI_RADIUS] * g[j + ORI_RADIUS];
            }
    return n;
}
ORC_API int orc_surf_ori_samples(int *apt, float *aptw) { return ori_samples((int(*)[2])apt, aptw); }

/* SURFInvoker's dominant orientation (upright == 0): Haar responses of size 2*cvRound(2s) at the
   disc samples scaled by s, Gaussian weighted, their angles (cvCartToPolar in degrees = the
   fastAtan2 polynomial), the 60-degree window of largest |sum| over 72 steps of 5 degrees, angle
   fastAtan2(-besty, bestx).  Returns 0 when no sample fits the integral image (the keypoint is
   dropped: kp.size = -1). */
static int surf_orientation(const int *sum, int w, int h, orc_kpt *k)
{
    int apt[ORI_SAMPLES_MAX][2], nOri;
    float aptw[ORI_SAMPLES_MAX];
    const int W1 = w + 1, H1 = h + 1;
    const float s = k->size * 1.2f / 9.0f;
    const int gws = 2 * cv_round(2 * s);
    float X[ORI_SAMPLES_MAX], Y[ORI_SAMPLES_MAX], ang[ORI_SAMPLES_MAX];
    float bestx = 0, besty = 0, descriptor_mod = 0;
    orc_hf dxt[2], dyt[2];
    int kk, nangle = 0, i, j;
    nOri = ori_samples(apt, aptw);
    resize_haar(DXO_S, dxt, 2, 4, gws, W1);
    resize_haar(DYO_S, dyt, 2, 4, gws, W1);
    for (kk = 0; kk < nOri; kk++) {
        const int x = cv_round(k->x + apt[kk][0] * s - (float)(gws - 1) / 2);
        const int y = cv_round(k->y + apt[kk][1] * s - (float)(gws - 1) / 2);
        const int *ptr;
        if (y < 0 || y >= H1 - gws || x < 0 || x >= W1 - gws) continue;
        ptr = sum + (size_t)y * W1 + x;
        X[nangle] = haar(ptr, dxt, 2) * aptw[kk];
        Y[nangle] = haar(ptr, dyt, 2) * aptw[kk];
        nangle++;
    }
    if (nangle == 0) return 0;
    for (j = 0; j < nangle; j++) ang[j] = fast_atan2f(Y[j], X[j]);
    for (i = 0; i < 360; i += ORI_SEARCH_INC) {
        float sumx = 0, sumy = 0, temp_mod;
        for (j = 0; j < nangle; j++) {
            const int d = abs(cv_round(ang[j]) - i);
            if (d < ORI_WIN / 2 || d > 360 - ORI_WIN / 2) {
                sumx += X[j];
                sumy += Y[j];
            }
        }
        temp_mod = sumx * sumx + sumy * sumy;
        if (temp_mod > descriptor_mod) {
            descriptor_mod = temp_mod;
            bestx = sumx;
            besty = sumy;
        }
    }
    k->angle = fast_atan2f(-besty, bestx);
    return 1;
}

/* the 20x20 descriptor weights DW (SURFInvoker constructor) */
ORC_API void orc_surf_dw(float *dw)
{
    float g[20];
    int i, j;
    gaussian_kernel(20, 3.3, g);
    for (i = 0; i < 20; i++)
        for (j = 0; j < 20; j++) dw[i * 20 + j] = g[i] * g[j];
}

typedef struct {
    int di, si;
    float alpha;
} decim;

/* computeResizeAreaTab */
static int area_tab(int ssize, int dsize, double scale, decim *tab)
{
    int k = 0, dx;
    for (dx = 0; dx < dsize; dx++) {
        const double fsx1 = dx * scale, fsx2 = fsx1 + scale;
        const double cellWidth = scale < ssize - fsx1 ? scale : ssize - fsx1;
        int sx1 = (int)ceil(fsx1), sx2 = (int)floor(fsx2), sx;
        sx2 = sx2 < ssize - 1 ? sx2 : ssize - 1;
        sx1 = sx1 < sx2 ? sx1 : sx2;
        if (sx1 - fsx1 > 1e-3) {
            tab[k].di = dx;
            tab[k].si = sx1 - 1;
            tab[k++].alpha = (float)((sx1 - fsx1) / cellWidth);
        }
        for (sx = sx1; sx < sx2; sx++) {
            tab[k].di = dx;
            tab[k].si = sx;
            tab[k++].alpha = (float)(1.0 / cellWidth);
        }
        if (fsx2 - sx2 > 1e-3) {
            double a = fsx2 - sx2;
            a = a < 1. ? a : 1.;
            a = a < cellWidth ? a : cellWidth;
            tab[k].di = dx;
            tab[k].si = sx2;
            tab[k++].alpha = (float)(a / cellWidth);
        }
    }
    return k;
}

static uint8_t sat_u8(float v)
{
    const int iv = cv_round(v);
    return (uint8_t)(iv < 0 ? 0 : (iv > 255 ? 255 : iv));
}

/* resize(win (W x W, u8), patch (21 x 21), INTER_AREA) as OpenCV 2.4 for scale >= 1 */
void resize_area(const uint8_t *src, int W, uint8_t *dst);
ORC_API void orc_resize_area21(const uint8_t *src, int W, uint8_t *dst) { resize_area(src, W, dst); }
void resize_area(const uint8_t *src, int W, uint8_t *dst)
{
    const int D = 21;
    const double inv_scale = (double)D / W, scale = 1. / inv_scale;
    const int iscale = cv_round(scale);
    int dx, dy;
    if (fabs(scale - iscale) < DBL_EPSILON) {
        /* resizeAreaFast_: per destination pixel the iscale x iscale block */
        const int area = iscale * iscale;
        const float fs = 1.f / area;
        for (dy = 0; dy < D; dy++)
            for (dx = 0; dx < D; dx++) {
                const uint8_t *S = src + (size_t)dy * iscale * W + (size_t)dx * iscale;
                int sum = 0, a, b;
                if (iscale == 2 && dx < 16) {
                    /* ResizeAreaFastVec_SIMD_8u: 8 outputs per step, (sum + 2) >> 2; the 5 left of
                       the 21 take the scalar cvRound(sum * 0.25f) below */
                    dst[dy * D + dx] = (uint8_t)((S[0] + S[1] + S[W] + S[W + 1] + 2) >> 2);
                    continue;
                }
                /* ofs order: sy outer, sx inner; unrolled by 4 as sum += s0 + s1 + s2 + s3 */
                {
                    int k = 0, v[4096];
                    for (a = 0; a < iscale; a++)
                        for (b = 0; b < iscale; b++) v[k++] = S[(size_t)a * W + b];
                    for (k = 0; k <= area - 4; k += 4) sum += v[k] + v[k + 1] + v[k + 2] + v[k + 3];
                    for (; k < area; k++) sum += v[k];
                }
                dst[dy * D + dx] = sat_u8(sum * fs);
            }
        return;
    }
    {
        decim *xt = (decim *)malloc(sizeof(decim) * 2 * W), *yt = (decim *)malloc(sizeof(decim) * 2 * W);
        const int nx = area_tab(W, D, scale, xt), ny = area_tab(W, D, scale, yt);
        float buf[21], sum[21];
        int j, k, prev = yt[0].di;
        for (dx = 0; dx < D; dx++) sum[dx] = 0;
        for (j = 0; j < ny; j++) {
            const float beta = yt[j].alpha;
            const int ddy = yt[j].di;
            const uint8_t *S = src + (size_t)yt[j].si * W;
            for (dx = 0; dx < D; dx++) buf[dx] = 0;
            for (k = 0; k < nx; k++) buf[xt[k].di] += S[xt[k].si] * xt[k].alpha;
            if (ddy != prev) {
                for (dx = 0; dx < D; dx++) {
                    dst[prev * D + dx] = sat_u8(sum[dx]);
                    sum[dx] = beta * buf[dx];
                }
                prev = ddy;
            } else {
                for (dx = 0; dx < D; dx++) sum[dx] += beta * buf[dx];
            }
        }
        for (dx = 0; dx < D; dx++) dst[prev * D + dx] = sat_u8(sum[dx]);
        free(xt);
        free(yt);
    }
}

/* the W x W window of SURFInvoker around keypoint k: upright (angle 270: border-replicated pixels,
   rows = x) or rotated by k.angle (degrees): the subpixel version, bilinear inside the image and
   nearest (clamped) outside, start positions accumulated in float and the positions along a row in
   double, as the source does.  sin / cos of the float angle in radians: correctly rounded float
   values (fm3d_detmath in double, rounded; glibc's sinf / cosf give the same floats in practice). */
static void surf_window(const uint8_t *img, int w, int h, const orc_kpt *k, int upright, int W, uint8_t *win)
{
    const float win_offset = -(float)(W - 1) / 2;
    int i, j;
    if (upright) {
        int start_x = cv_round(k->x + win_offset), start_y = cv_round(k->y - win_offset);
        for (i = 0; i < W; i++, start_x++) {
            int pixel_x = start_x, pixel_y = start_y;
            for (j = 0; j < W; j++, pixel_y--) {
                int x = pixel_x > 0 ? pixel_x : 0, y = pixel_y > 0 ? pixel_y : 0;
                x = x < w - 1 ? x : w - 1;
                y = y < h - 1 ? y : h - 1;
                win[(size_t)i * W + j] = img[(size_t)y * w + x];
            }
        }
        return;
    }
    {
        const float dir = k->angle * (float)(M_PI / 180);
        const float sin_dir = -(float)fm3d_sin((double)dir), cos_dir = (float)fm3d_cos((double)dir);
        float start_x = k->x + win_offset * cos_dir + win_offset * sin_dir;
        float start_y = k->y - win_offset * sin_dir + win_offset * cos_dir;
        const int ncols1 = w - 1, nrows1 = h - 1;
        for (i = 0; i < W; i++, start_x += sin_dir, start_y += cos_dir) {
            double pixel_x = start_x, pixel_y = start_y;
            for (j = 0; j < W; j++, pixel_x += cos_dir, pixel_y -= sin_dir) {
                const int ix = (int)floor(pixel_x), iy = (int)floor(pixel_y);
                uint8_t v;
                if ((unsigned)ix < (unsigned)ncols1 && (unsigned)iy < (unsigned)nrows1) {
                    const float a = (float)(pixel_x - ix), b = (float)(pixel_y - iy);
                    const uint8_t *p = img + (size_t)iy * w + ix;
                    v = (uint8_t)cv_round(p[0] * (1.f - a) * (1.f - b) + p[1] * a * (1.f - b) + p[w] * (1.f - a) * b +
                                          p[w + 1] * a * b);
                } else {
                    int x = cv_round(pixel_x), y = cv_round(pixel_y);
                    x = x > 0 ? x : 0;
                    y = y > 0 ? y : 0;
                    x = x < ncols1 ? x : ncols1;
                    y = y < nrows1 ? y : nrows1;
                    v = img[(size_t)y * w + x];
                }
                win[(size_t)i * W + j] = v;
            }
        }
    }
}

static short sat_short2048(float v)
{
    const int i = (int)lrintf(v * 2048);
    return (short)(i < -32768 ? -32768 : (i > 32767 ? 32767 : i));
}

/* resize(src W x W, dst D x D, INTER_AREA) with W < D (OpenCV 2.4.9 imgproc/resize.cpp): INTER_AREA only
 * averages when shrinking; enlarging runs the generic linear path with area-mode coefficients:
 * s = floor(d * scale), f = (float)((d + 1) - (s + 1) / scale), f = f <= 0 ? 0 : f - floor(f), the
 * coefficients (1 - f, f) * 2048 rounded to short.  Columns: s + 1 >= W ends the interpolated range
 * (xmax) and s >= W - 1 becomes (W - 1, f = 0); rows: s and s + 1 clamped to [0, W - 1].
 * HResizeLinear in int (S[s] * 2048 from xmax on), VResizeLinear as VResizeLinearVec_32s8u's SSE2
 * arithmetic ((S >> 4) mulhi b, (+2) >> 2) on its columns and FixedPtCast ((+2^21) >> 22) on the rest. */
ORC_API void orc_resize_area_up(const uint8_t *src, int W, int D, uint8_t *dst)
{
    const double inv = (double)D / W, scale = 1. / inv;
    int xo[64], yo[64], H0[64], H1[64], xmax = D, xs = 0, d;
    short xa[128], yb[128];
    for (; xs <= D - 16; xs += 16) {}
    for (; xs < D - 4; xs += 4) {}
    for (d = 0; d < D; d++) {
        int sx = (int)floor(d * scale);
        float f = (float)((d + 1) - (sx + 1) * inv);
        f = f <= 0 ? 0.f : f - floorf(f);
        yo[d] = sx;
        yb[2 * d] = sat_short2048(1.f - f);
        yb[2 * d + 1] = sat_short2048(f);
        if (sx + 1 >= W) {
            if (d < xmax) xmax = d;
            if (sx >= W - 1) {
                f = 0;
                sx = W - 1;
            }
        }
        xo[d] = sx;
        xa[2 * d] = sat_short2048(1.f - f);
        xa[2 * d + 1] = sat_short2048(f);
    }
    for (d = 0; d < D; d++) {
        const int r0 = yo[d] < 0 ? 0 : (yo[d] > W - 1 ? W - 1 : yo[d]);
        const int r1 = yo[d] + 1 < 0 ? 0 : (yo[d] + 1 > W - 1 ? W - 1 : yo[d] + 1);
        const uint8_t *S0 = src + (size_t)r0 * W, *S1 = src + (size_t)r1 * W;
        const int b0 = yb[2 * d], b1 = yb[2 * d + 1];
        int dx;
        for (dx = 0; dx < D; dx++) {
            const int sx = xo[dx];
            if (dx < xmax) {
                H0[dx] = S0[sx] * xa[2 * dx] + S0[sx + 1] * xa[2 * dx + 1];
                H1[dx] = S1[sx] * xa[2 * dx] + S1[sx + 1] * xa[2 * dx + 1];
            } else {
                H0[dx] = S0[sx] * 2048;
                H1[dx] = S1[sx] * 2048;
            }
        }
        for (dx = 0; dx < D; dx++) {
            int v;
            if (dx < xs)
                v = ((((H0[dx] >> 4) * b0) >> 16) + (((H1[dx] >> 4) * b1) >> 16) + 2) >> 2;
            else
                v = (b0 * H0[dx] + b1 * H1[dx] + (1 << 21)) >> 22;
            dst[(size_t)d * D + dx] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
        }
    }
}

/* SURFInvoker descriptors for given keypoints (SURF::operator() with useProvidedKeypoints, via
   DescriptorExtractor::compute): size < FLT_EPSILON dropped first, then keypoints whose wavelet
   exceeds the integral image, and (upright == 0) those without an orientation sample; the others get
   angle 270 (upright) or their dominant orientation.  Compacted with their descriptors, kept[] gets
   the input index of each survivor.  desc: n x (128 | 64).  A window narrower than the 21 x 21 patch
   (size < 7.5) is enlarged by orc_resize_area_up; returns -1 for an empty window (size < 0.36: OpenCV's
   resize asserts). */
ORC_API int orc_surf_describe2(const uint8_t *img, int w, int h, const orc_kpt *kin, int n, int extended, int upright,
                               orc_kpt *kout, int *kept, float *desc)
{
    const int dsize = extended ? 128 : 64;
    float DW[400];
    int q, m = 0;
    int *sum = NULL;
    orc_surf_dw(DW);
    if (!upright) {
        sum = (int *)malloc(sizeof(int) * (size_t)(w + 1) * (h + 1));
        orc_integral(img, w, h, sum);
    }
    for (q = 0; q < n; q++) {
        orc_kpt k = kin[q];
        const float s = k.size * 1.2f / 9.0f;
        const int gws = 2 * cv_round(2 * s);
        int win_size, i, j, kk;
        float *vec;
        uint8_t *win, patch[21 * 21];
        float DXa[400], DYa[400];
        double square_mag = 0;
        float scale;
        /* DescriptorExtractor::compute: KeyPointsFilter::runByKeypointSize(FLT_EPSILON) first
           (runByImageBorder with border 0 removes nothing), then the SURFInvoker wavelet drop */
        if (!(k.size >= FLT_EPSILON)) continue;
        if (h + 1 < gws || w + 1 < gws) continue;
        if (upright) k.angle = 360.f - 90.f;
        else if (!surf_orientation(sum, w, h, &k)) continue;
        win_size = (int)((20 + 1) * s);
        if (win_size < 1) { free(sum); return -1; } /* resize of an empty Mat: OpenCV asserts */
        win = (uint8_t *)malloc((size_t)win_size * win_size);
        surf_window(img, w, h, &k, upright, win_size, win);
        if (win_size < 21)
            orc_resize_area_up(win, win_size, 21, patch);
        else
            resize_area(win, win_size, patch);
        free(win);
        for (i = 0; i < 20; i++)
            for (j = 0; j < 20; j++) {
                const float dw = DW[i * 20 + j];
                DXa[i * 20 + j] = (patch[i * 21 + j + 1] - patch[i * 21 + j] + patch[(i + 1) * 21 + j + 1] -
                                   patch[(i + 1) * 21 + j]) * dw;
                DYa[i * 20 + j] = (patch[(i + 1) * 21 + j] - patch[i * 21 + j] + patch[(i + 1) * 21 + j + 1] -
                                   patch[i * 21 + j + 1]) * dw;
            }
        vec = desc + (size_t)m * dsize;
        for (kk = 0; kk < dsize; kk++) vec[kk] = 0;
        for (i = 0; i < 4; i++)
            for (j = 0; j < 4; j++) {
                int y, x;
                for (y = i * 5; y < i * 5 + 5; y++)
                    for (x = j * 5; x < j * 5 + 5; x++) {
                        const float tx = DXa[y * 20 + x], ty = DYa[y * 20 + x];
                        if (extended) {
                            if (ty >= 0) {
                                vec[0] += tx;
                                vec[1] += (float)fabs(tx);
                            } else {
                                vec[2] += tx;
                                vec[3] += (float)fabs(tx);
                            }
                            if (tx >= 0) {
                                vec[4] += ty;
                                vec[5] += (float)fabs(ty);
                            } else {
                                vec[6] += ty;
                                vec[7] += (float)fabs(ty);
                            }
                        } else {
                            vec[0] += tx;
                            vec[1] += ty;
                            vec[2] += (float)fabs(tx);
                            vec[3] += (float)fabs(ty);
                        }
                    }
                for (kk = 0; kk < (extended ? 8 : 4); kk++) square_mag += vec[kk] * vec[kk];
                vec += extended ? 8 : 4;
            }
        vec = desc + (size_t)m * dsize;
        scale = (float)(1. / (sqrt(square_mag) + DBL_EPSILON));
        for (kk = 0; kk < dsize; kk++) vec[kk] *= scale;
        kout[m] = k;
        if (kept) kept[m] = q;
        m++;
    }
    free(sum);
    return m;
}
ORC_API int orc_surf_describe(const uint8_t *img, int w, int h, const orc_kpt *kin, int n, int extended,
                              orc_kpt *kout, int *kept, float *desc)
{
    return orc_surf_describe2(img, w, h, kin, n, extended, 1, kout, kept, desc);
}
