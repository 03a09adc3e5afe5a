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
ORC_API int orc_surf_detect(const uint8_t *img, int w, int h, float thr, int nOctaves, int nOctaveLayers,
                            orc_kpt *out, int cap)
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
    /* SURFInvoker (detect): upright angle; the gradient wavelet must fit the integral image */
    for (q = 0; q < nk; q++) {
        orc_kpt k = ks[q].k;
        const float s = k.size * 1.2f / 9.0f;
        const int gws = 2 * cv_round(2 * s);
        if (h + 1 < gws || w + 1 < gws) continue;
        k.angle = 360.f - 90.f;
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

/* SURFInvoker descriptors of the upright extractor for given keypoints (SURF::operator() with
   useProvidedKeypoints): keypoints whose wavelet exceeds the integral image are dropped (compacted
   with their descriptors, kept[] gets the input index of each survivor).  desc: n x (128 | 64). */
ORC_API int orc_surf_describe(const uint8_t *img, int w, int h, const orc_kpt *kin, int n, int extended,
                              orc_kpt *kout, int *kept, float *desc)
{
    const int dsize = extended ? 128 : 64;
    float DW[400];
    int q, m = 0;
    orc_surf_dw(DW);
    for (q = 0; q < n; q++) {
        orc_kpt k = kin[q];
        const float s = k.size * 1.2f / 9.0f;
        const int gws = 2 * cv_round(2 * s);
        int win_size, start_x, start_y, i, j, kk;
        float win_offset, *vec;
        uint8_t *win, patch[21 * 21];
        float DXa[400], DYa[400];
        double square_mag = 0;
        float scale;
        /* DescriptorExtractor::compute: KeyPointsFilter::runByKeypointSize(FLT_EPSILON) first
           (runByImageBorder with border 0 removes nothing), then the SURFInvoker wavelet drop */
        if (!(k.size >= FLT_EPSILON)) continue;
        if (h + 1 < gws || w + 1 < gws) continue;
        k.angle = 360.f - 90.f;
        win_size = (int)((20 + 1) * s);
        if (win_size < 21) return -1; /* OpenCV's INTER_AREA upscale branch: not restated */
        win_offset = -(float)(win_size - 1) / 2;
        start_x = cv_round(k.x + win_offset);
        start_y = cv_round(k.y - win_offset);
        win = (uint8_t *)malloc((size_t)win_size * win_size);
        for (i = 0; i < win_size; i++, start_x++) {
            int pixel_x = start_x, pixel_y = start_y;
            for (j = 0; j < win_size; j++, pixel_y--) {
                int x = pixel_x > 0 ? pixel_x : 0, y = pixel_y > 0 ? pixel_y : 0;
                x = x < w - 1 ? x : w - 1;
                y = y < h - 1 ? y : h - 1;
                win[(size_t)i * win_size + j] = img[(size_t)y * w + x];
            }
        }
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
    return m;
}
