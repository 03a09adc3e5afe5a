/* orc_star.c -- CPU restatement of OpenCV 2.4.9's StarDetector (CenSurE; features2d/src/stardetector.cpp),
 * the detector DescriptorsMatcher builds for FeatureOptions DetectorType STAR
 * (reference DescriptorsMatcher/descriptorsmatcher.cpp:204-213: cv::StarFeatureDetector(MaxSize,
 * Response, LineThreshold, LineBinarized, Suppression)) and that AdjusterAdapter::create("STAR") runs
 * in the ADAPTIVE mode (:185-200; StarAdjuster: StarFeatureDetector(16, cvRound(thresh), 10, 8, 3)).
 *
 * TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py's cpu_baseline): the GPU
 * library never links or calls this file.  OpenCV is not in this image, so this restatement of its
 * published algorithm is unpinned against OpenCV itself; tests/test_star_oracle.py checks it against
 * independent numpy statements of the same definitions (box sums from the plain integral image,
 * brute-force tile maxima).
 *
 * Steps, in OpenCV's operation order:
 *   integrals   computeIntegralImages: the upright sum S, the 45-degree "tilted" sum T and the
 *               "flat tilted" sum F, (h+1) x (w+1) int32, by OpenCV's row recursions (rows 0 and 1
 *               and columns 0, 1 and w have their own formulas)
 *   responses   StarDetectorComputeResponses: the bi-level star (an upright square plus a 45-degree
 *               square) at 17 sizes; per pixel every pattern's box sum from 8 integral reads (int),
 *               then per inner/outer pair  inner/innerArea - outer/outerArea  in float, the pair with
 *               the largest |response| (the first on ties) giving the response and the size; sizes at
 *               the ends of the range are negated so that the non-maximum stage rejects them.  The
 *               SSE2 block of four columns forms outer = float(vals) - float(inner) where the scalar
 *               tail converts the int difference; both are restated (they differ only above 2^24)
 *   nonmax      StarDetectorSuppressNonmax: tiles of (Suppression/2 + 1)^2 pixels; in each the
 *               largest response above +Response and the smallest below -Response (raster order,
 *               first wins), each kept if no other pixel of its (2*delta+1)^2 window reaches it, its
 *               size is >= 4 and StarDetectorSuppressLines does not reject it (the Harris-like test
 *               on response gradients sampled every size/4 pixels, float, then on the binarised size
 *               map, int); KeyPoint(x, y, size, -1, maxResponse) -- the minimum's keypoint carries the
 *               tile's maxResponse as OpenCV 2.4.9 writes it
 * Undefined in OpenCV and refused here (returns -1): min(w, h) <= 6 (its pattern count loop then
 * reads pairs[-1]) and MaxSize > 128 (it reads sizes0[-1]).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_API __attribute__((visibility("default")))

typedef struct orc_kpt {
    float x, y, size, angle, response;
    int octave, class_id;
} orc_kpt;

static const int star_sizes0[17] = {1, 2, 3, 4, 6, 8, 11, 12, 16, 22, 23, 32, 45, 46, 64, 90, 128};
/* (outer, inner) pattern index pairs; each inner pattern is half its outer one */
static const int star_pairs[12][2] = {{1, 0}, {3, 1}, {4, 2}, {5, 3}, {7, 4}, {8, 5},
                                      {9, 6}, {11, 8}, {13, 10}, {14, 11}, {15, 12}, {16, 14}};

ORC_API void orc_star_integrals(const uint8_t *I, int w, int h, int *S, int *T, int *F)
{
    const int st = w + 1;
    int x, y;
    for (x = 0; x <= w; x++) S[x] = T[x] = F[x] = 0;
    {
        int *s = S + st, *t = T + st, *f = F + st;
        s[0] = t[0] = 0;
        f[0] = I[0];
        for (x = 1; x < w; x++) {
            s[x] = s[x - 1] + I[x - 1];
            t[x] = I[x - 1];
            f[x] = I[x] + I[x - 1];
        }
        s[w] = s[w - 1] + I[w - 1];
        t[w] = f[w] = I[w - 1];
    }
    for (y = 2; y <= h; y++) {
        const uint8_t *a = I + (size_t)(y - 1) * w, *b = a - w; /* image rows y-1 and y-2 */
        int *s = S + (size_t)y * st, *t = T + (size_t)y * st, *f = F + (size_t)y * st;
        const int *s1 = s - st, *t1 = t - st, *t2 = t1 - st, *f1 = f - st, *f2 = f1 - st;
        s[0] = s1[0];
        s[1] = s1[1] + a[0];
        t[0] = t1[1];
        t[1] = f[0] = t1[2] + b[0] + a[0];
        f[1] = f1[2] + b[0] + a[1] + a[0];
        for (x = 2; x < w; x++) {
            s[x] = s[x - 1] + s1[x] - s1[x - 1] + a[x - 1];
            t[x] = t1[x - 1] + t1[x + 1] - t2[x] + b[x - 1] + a[x - 1];
            f[x] = f1[x - 1] + f1[x + 1] - f2[x] + a[x] + a[x - 1];
        }
        s[w] = s[w - 1] + s1[w] - s1[w - 1] + a[w - 1];
        t[w] = f[w] = t1[w - 1] + b[w - 1] + a[w - 1];
    }
}

/* the pattern set of StarDetectorComputeResponses: returns the number of pairs (0: undefined input) and
 * fills maxIdx, border, the signed sizes, the per-pattern integral offsets (8 per pattern, relative to
 * y*(w+1)+x; 0-3 into S, 4 and 7 into T, 5 and 6 into F) and the pairs' float reciprocal areas */
ORC_API int orc_star_patterns(int w, int h, int maxSize, int *maxIdx, int *border, int *sizes1, int *ofs,
                              float *inv)
{
    const int st = w + 1, mn = w < h ? w : h;
    int np = 0, i, area[17];
    if (maxSize > 128 || mn <= 6) return 0;
    while (np < 12 && !(star_sizes0[star_pairs[np][0]] >= maxSize ||
                        star_sizes0[star_pairs[np + 1][0]] + star_sizes0[star_pairs[np + 1][0]] / 2 >= mn))
        np++;
    if (np == 0) return 0;
    np += 1; /* the first pattern past the range is kept for the size rejection */
    if (np > 12) np = 12;
    *maxIdx = star_pairs[np - 1][0];
    for (i = 0; i <= *maxIdx; i++) {
        const int u = star_sizes0[i], t = u + u / 2;
        int *o = ofs + 8 * i;
        o[0] = (u + 1) * st + u + 1;
        o[1] = -u * st + u + 1;
        o[2] = (u + 1) * st - u;
        o[3] = -u * st - u;
        o[4] = (t + 1) * st + 1;
        o[5] = -t;
        o[6] = t + 1;
        o[7] = -t * st + 1;
        area[i] = (2 * u + 1) * (2 * u + 1) + t * t + (t + 1) * (t + 1);
        sizes1[i] = u;
    }
    sizes1[0] = -sizes1[0];
    sizes1[1] = -sizes1[1];
    sizes1[*maxIdx] = -sizes1[*maxIdx];
    *border = star_sizes0[*maxIdx] + star_sizes0[*maxIdx] / 2;
    for (i = 0; i < np; i++) {
        const int inner = area[star_pairs[i][1]], outer = area[star_pairs[i][0]] - inner;
        inv[2 * i] = 1.f / (float)outer;
        inv[2 * i + 1] = 1.f / (float)inner;
    }
    return np;
}

/* responses (float) and sizes (short) over the whole image; returns the border, -1 if undefined */
ORC_API int orc_star_responses(const uint8_t *img, int w, int h, int maxSize, float *resp, short *sizes)
{
    const int st = w + 1;
    int maxIdx, border, sizes1[17], ofs[17 * 8], np, x, y, i, nsimd;
    float inv[24];
    int *S, *T, *F;
    memset(resp, 0, sizeof(float) * (size_t)w * h);
    memset(sizes, 0, sizeof(short) * (size_t)w * h);
    np = orc_star_patterns(w, h, maxSize, &maxIdx, &border, sizes1, ofs, inv);
    if (np == 0) return -1;
    S = (int *)malloc(sizeof(int) * (size_t)st * (h + 1));
    T = (int *)malloc(sizeof(int) * (size_t)st * (h + 1));
    F = (int *)malloc(sizeof(int) * (size_t)st * (h + 1));
    orc_star_integrals(img, w, h, S, T, F);
    /* the SSE2 loop takes x = border, border + 4, ... while x <= w - border - 4 */
    nsimd = w - 2 * border >= 0 ? 4 * ((w - 2 * border) / 4) : 0;
    for (y = border; y < h - border; y++)
        for (x = border; x < w - border; x++) {
            const int o = y * st + x, simd = x - border < nsimd;
            int vals[17];
            float best = 0;
            int bestSize = 0;
            for (i = 0; i <= maxIdx; i++) {
                const int *p = ofs + 8 * i;
                vals[i] = S[o + p[0]] - S[o + p[1]] - S[o + p[2]] + S[o + p[3]] + T[o + p[4]] - F[o + p[5]] -
                          F[o + p[6]] + T[o + p[7]];
            }
            for (i = 0; i < np; i++) {
                const int in = vals[star_pairs[i][1]];
                float outer, r;
                if (simd)
                    outer = (float)vals[star_pairs[i][0]] - (float)in;
                else
                    outer = (float)(vals[star_pairs[i][0]] - in);
                r = (float)in * inv[2 * i + 1] - outer * inv[2 * i];
                if (fabsf(r) > fabsf(best)) {
                    best = r;
                    bestSize = sizes1[star_pairs[i][0]];
                }
            }
            resp[(size_t)y * w + x] = best;
            sizes[(size_t)y * w + x] = (short)bestSize;
        }
    free(S);
    free(T);
    free(F);
    return border;
}

/* StarDetectorSuppressLines: 1 = reject */
static int star_lines(const float *R, const short *Z, int w, int x0, int y0, int lineProj, int lineBin)
{
    const int sz = Z[(size_t)y0 * w + x0], d = sz / 4, rad = d * 4;
    float Lxx = 0, Lyy = 0, Lxy = 0;
    int Bxx = 0, Byy = 0, Bxy = 0, x, y;
    for (y = y0 - rad; y <= y0 + rad; y += d)
        for (x = x0 - rad; x <= x0 + rad; x += d) {
            const float Lx = R[(size_t)y * w + x + 1] - R[(size_t)y * w + x - 1];
            const float Ly = R[(size_t)(y + 1) * w + x] - R[(size_t)(y - 1) * w + x];
            Lxx += Lx * Lx;
            Lyy += Ly * Ly;
            Lxy += Lx * Ly;
        }
    if ((Lxx + Lyy) * (Lxx + Lyy) >= (float)lineProj * (Lxx * Lyy - Lxy * Lxy)) return 1;
    for (y = y0 - rad; y <= y0 + rad; y += d)
        for (x = x0 - rad; x <= x0 + rad; x += d) {
            const int bx = (Z[(size_t)y * w + x + 1] == sz) - (Z[(size_t)y * w + x - 1] == sz);
            const int by = (Z[(size_t)(y + 1) * w + x] == sz) - (Z[(size_t)(y - 1) * w + x] == sz);
            Bxx += bx * bx;
            Byy += by * by;
            Bxy += bx * by;
        }
    if ((Bxx + Byy) * (Bxx + Byy) >= lineBin * (Bxx * Byy - Bxy * Bxy)) return 1;
    return 0;
}

/* StarDetector(maxSize, responseThreshold, lineThresholdProjected, lineThresholdBinarized,
 * suppressNonmaxSize)(img, keypoints): returns the keypoint count (written up to cap), -1 when
 * undefined (see the header) */
ORC_API int orc_star_detect(const uint8_t *img, int w, int h, int maxSize, int respThr, int lineProj, int lineBin,
                            int supp, orc_kpt *out, int cap)
{
    float *R;
    short *Z;
    int border, n = 0, x, y, x1, y1;
    const int delta = supp / 2;
    if (w <= 0 || h <= 0) return -1;
    R = (float *)malloc(sizeof(float) * (size_t)w * h);
    Z = (short *)malloc(sizeof(short) * (size_t)w * h);
    border = orc_star_responses(img, w, h, maxSize, R, Z);
    if (border < 0 || delta > border) {
        free(R);
        free(Z);
        return -1;
    }
    for (y = border; y < h - border; y += delta + 1)
        for (x = border; x < w - border; x += delta + 1) {
            float maxR = (float)respThr, minR = (float)-respThr;
            int mx = -1, my = -1, nx = -1, ny = -1, pass, sz;
            const int ey = y + delta < h - border - 1 ? y + delta : h - border - 1;
            const int ex = x + delta < w - border - 1 ? x + delta : w - border - 1;
            for (y1 = y; y1 <= ey; y1++)
                for (x1 = x; x1 <= ex; x1++) {
                    const float v = R[(size_t)y1 * w + x1];
                    if (maxR < v) {
                        maxR = v;
                        mx = x1;
                        my = y1;
                    } else if (minR > v) {
                        minR = v;
                        nx = x1;
                        ny = y1;
                    }
                }
            for (pass = 0; pass < 2; pass++) {
                const int px = pass ? nx : mx, py = pass ? ny : my;
                int ok = px >= 0;
                for (y1 = py - delta; ok && y1 <= py + delta; y1++)
                    for (x1 = px - delta; x1 <= px + delta; x1++) {
                        const float v = R[(size_t)y1 * w + x1];
                        if ((pass ? v <= minR : v >= maxR) && (y1 != py || x1 != px)) {
                            ok = 0;
                            break;
                        }
                    }
                if (!ok) continue;
                sz = Z[(size_t)py * w + px];
                if (sz >= 4 && !star_lines(R, Z, w, px, py, lineProj, lineBin)) {
                    if (n < cap) {
                        orc_kpt k = {(float)px, (float)py, (float)sz, -1.f, maxR, 0, -1};
                        out[n] = k;
                    }
                    n++;
                }
            }
        }
    free(R);
    free(Z);
    return n;
}
