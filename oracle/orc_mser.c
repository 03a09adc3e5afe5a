/* orc_mser.c -- CPU restatement of OpenCV 2.4.9's MSER detector on 8-bit grey images
 * (features2d/src/mser.cpp), the detector DescriptorsMatcher builds for FeatureOptions DetectorMode
 * STATIC + DetectorType MSER (reference DescriptorsMatcher/descriptorsmatcher.cpp:258-272:
 * cv::MserFeatureDetector(Delta, MinArea, MaxArea, MaxVariation, MinDiversity, MaxEvolution,
 * AreaThreshold, MinMargin, EdgeBlurSize); the last four only steer the colour-image algorithm).
 *
 * TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py's cpu_baseline): the GPU library
 * never links or calls this file.  OpenCV is not in this image, so this restatement is unpinned against
 * OpenCV itself; tests/test_mser_oracle.py checks it against an independent pure-Python restatement of
 * the flood on small images and against numpy (extremal-region properties, least squares, ellipse
 * moments).  This file keeps mser.cpp's pointer structure; the GPU (csrc/fm3d_mser.hip) is a separate
 * index-based statement of the same steps.
 *
 * Steps (FeatureDetector::detect -> MSER::detectImpl -> MSER::operator() -> extractMSER_8UC1):
 *   layout    preprocessMSER_8UC1: an int image `step` wide (the power of two >= width + 2, at least 8)
 *             with a -1 border; pixel = grey value, 0x80000000 = visited, bits 16..18 = next direction
 *             (right, down, left, up); one LIFO bucket per grey level in one heap array
 *   passes    pass 1 on 255 - I (colour -1), pass 2 on I (colour +1; preprocess inverts the image in
 *             place both times), both starting at pixel (0, 0)
 *   flood     extractMSER_8UC1_Pass: Nister & Stewenius' linear-time flood with a component stack
 *             (grey levels decreasing towards the top, a 256 sentinel at the bottom); a lower neighbour
 *             pushes the current pixel back and opens a component; a finished pixel joins the top
 *             component's linked point list; when the current level's bucket is empty the next
 *             non-empty level decides between raising the top component (stability check, new
 *             history) and merging it down the stack (the larger component's history continues; equal
 *             sizes keep the upper one's)
 *   stability MSERStableCheck: history size in (MinArea, MaxArea); div = (size - stable) / size (float);
 *             var = (size - size at level - delta) / that size along the history shortcuts
 *             (MSERVariationCalc); stable when the variation's derivative turns (dvar && !comp->dvar),
 *             comp->var < MaxVariation and div > MinDiversity; the region is the first history->size
 *             points of the component's list (MSERToContour)
 *   keypoint  MserFeatureDetector::detectImpl: RotatedRect = fitEllipse(points) (imgproc cvFitEllipse2:
 *             a float centroid, then cvSolve(CV_SVD) of the 5-parameter conic, of the 2x2 centre system
 *             and of the 3-parameter re-fit); diam = sqrtf(w * h); kept when diam > FLT_EPSILON and
 *             Rect(0, 0, cols, rows) contains the centre rounded (cvRound) to int; KeyPoint(centre, diam):
 *             angle -1, response 0, octave 0, class -1
 *   solve     cv::solve(DECOMP_SVD): At = A^T, JacobiSVDImpl_ (one-sided Jacobi on At's rows, eps
 *             10 DBL_EPSILON, rotation from hypot(2p, a - b), sorted singular values, U rows = At rows /
 *             w), SVBkSbImpl_ (threshold 2 DBL_EPSILON * sum(w)).  The scalar build's loop order: the sums
 *             run over the points in region-list order.  hypot is sqrt(p^2 + beta^2) and atan2 / sin are
 *             fm3d_detmath.h's (the GPU evaluates the same expressions); a zero singular value's left
 *             vector (OpenCV draws a random one) is never used by the back substitution and is left as is.
 * The centroid's float sums run in region-list order (OpenCV's).  The GPU sums lane-strided + tree
 * where every partial sum stays below 2^24 (exact integers: any order gives these bits) and in list
 * order on one lane elsewhere (wide images with large regions).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "fm3d_detmath.h"

typedef struct orc_lpt {
    struct orc_lpt *prev, *next;
    int x, y;
} orc_lpt;

typedef struct orc_hist {
    struct orc_hist *shortcut, *child;
    int stable, val, size;
} orc_hist;

typedef struct {
    orc_lpt *head, *tail;
    orc_hist *history;
    unsigned long grey_level;
    int size, dvar;
    float var;
} orc_comp;

typedef struct {
    int delta, minArea, maxArea;
    double maxVariation, minDiversity;
} orc_mser_params;

/* one emitted region: colour, first list node, point count */
typedef struct {
    int color, count;
    orc_lpt *head;
} orc_region;

static void comp_init(orc_comp *c) {
    c->size = 0;
    c->var = 0;
    c->dvar = 1;
    c->history = NULL;
}

static void new_history(orc_comp *comp, orc_hist *h) {
    h->child = h;
    if (!comp->history) {
        h->shortcut = h;
        h->stable = 0;
    } else {
        comp->history->child = h;
        h->shortcut = comp->history->shortcut;
        h->stable = comp->history->stable;
    }
    h->val = (int)comp->grey_level;
    h->size = comp->size;
    comp->history = h;
}

/* MSERMergeComp(comp1, comp2, comp = comp2, history) */
static void merge_comp(orc_comp *c1, orc_comp *c2, orc_comp *comp, orc_hist *h) {
    orc_lpt *head, *tail;
    orc_comp *win = c1->size >= c2->size ? c1 : c2, *lose = win == c1 ? c2 : c1;
    comp->grey_level = c2->grey_level;
    h->child = h;
    if (!win->history) {
        h->shortcut = h;
        h->stable = 0;
    } else {
        win->history->child = h;
        h->shortcut = win->history->shortcut;
        h->stable = win->history->stable;
    }
    if (lose->history && lose->history->stable > h->stable) h->stable = lose->history->stable;
    h->val = (int)win->grey_level;
    h->size = win->size;
    comp->var = win->var;
    comp->dvar = win->dvar;
    /* the winner's points first, then the other's */
    if (c1->size > 0 && c2->size > 0) {
        win->tail->next = lose->head;
        lose->head->prev = win->tail;
    }
    head = win->size > 0 ? win->head : lose->head;
    tail = lose->size > 0 ? lose->tail : win->tail;
    comp->head = head;
    comp->tail = tail;
    comp->history = h;
    comp->size = c1->size + c2->size;
}

static float variation(orc_comp *comp, int delta) {
    orc_hist *history = comp->history;
    int val = (int)comp->grey_level;
    if (history) {
        orc_hist *shortcut = history->shortcut, *child;
        while (shortcut != shortcut->shortcut && shortcut->val + delta > val) shortcut = shortcut->shortcut;
        child = shortcut->child;
        while (child != child->child && child->val + delta <= val) {
            shortcut = child;
            child = child->child;
        }
        history->shortcut = shortcut;
        return (float)(comp->size - shortcut->size) / (float)shortcut->size;
    }
    return 1.f;
}

static int stable_check(orc_comp *comp, const orc_mser_params *p) {
    float div, var;
    int dvar, stable;
    if (!comp->history || comp->history->size <= p->minArea || comp->history->size >= p->maxArea) return 0;
    div = (float)(comp->history->size - comp->history->stable) / (float)comp->history->size;
    var = variation(comp, p->delta);
    dvar = comp->var < var || (unsigned long)(comp->history->val + 1) < comp->grey_level;
    stable = dvar && !comp->dvar && comp->var < p->maxVariation && div > p->minDiversity;
    comp->var = var;
    comp->dvar = dvar;
    if (stable) comp->history->stable = comp->history->size;
    return stable;
}

static void accumulate(orc_comp *comp, orc_lpt *pt) {
    if (comp->size > 0) {
        pt->prev = comp->tail;
        comp->tail->next = pt;
        pt->next = NULL;
    } else {
        pt->prev = NULL;
        pt->next = NULL;
        comp->head = pt;
    }
    comp->tail = pt;
    comp->size++;
}

/* preprocessMSER_8UC1 without a mask: src inverted in place; returns the start pixel */
static int *preprocess(int *img, int step, int ***heap_cur, uint8_t *src, int w, int h) {
    int level_size[256], i, j;
    int *p = img;
    for (i = 0; i < 256; i++) level_size[i] = 0;
    for (i = 0; i < w + 2; i++) *p++ = -1;
    p += step - w - 2;
    for (i = 0; i < h; i++) {
        *p++ = -1;
        for (j = 0; j < w; j++) {
            uint8_t *s = src + (size_t)i * w + j;
            *s = (uint8_t)(0xff - *s);
            level_size[*s]++;
            *p++ = *s;
        }
        *p = -1;
        p += step - w - 1;
    }
    for (i = 0; i < w + 2; i++) *p++ = -1;
    heap_cur[0][0] = 0;
    for (i = 1; i < 256; i++) {
        heap_cur[i] = heap_cur[i - 1] + level_size[i - 1] + 1;
        heap_cur[i][0] = 0;
    }
    return img + step + 1;
}

/* the emitted regions (grown as needed) */
typedef struct {
    orc_region *r;
    int n, cap;
} orc_regs;

/* emit: the stable top component (MSERToContour keeps the first history->size points) */
static void emit(orc_comp *comp, int color, orc_regs *out) {
    if (out->n == out->cap) {
        out->cap = out->cap ? 2 * out->cap : 256;
        out->r = (orc_region *)realloc(out->r, sizeof(orc_region) * (size_t)out->cap);
    }
    out->r[out->n].color = color;
    out->r[out->n].count = comp->history->size;
    out->r[out->n].head = comp->head;
    out->n++;
}

static void mser_pass(int *ioptr, int *imgptr, int ***heap_cur, orc_lpt *ptsptr, orc_hist *histptr, orc_comp *comptr,
                      int step, int stepmask, int stepgap, const orc_mser_params *p, int color, orc_regs *out) {
    int dir[4];
    dir[0] = 1;
    dir[1] = step;
    dir[2] = -1;
    dir[3] = -step;
    comptr->grey_level = 256;
    comptr++;
    comptr->grey_level = (unsigned long)(*imgptr & 0xff);
    comp_init(comptr);
    *imgptr |= (int)0x80000000;
    heap_cur += *imgptr & 0xff;
    for (;;) {
        while ((*imgptr & 0x70000) < 0x40000) {
            int *nbr = imgptr + dir[(*imgptr & 0x70000) >> 16];
            if (*nbr >= 0) {
                *nbr |= (int)0x80000000;
                if ((*nbr & 0xff) < (*imgptr & 0xff)) {
                    (*heap_cur)++;
                    **heap_cur = imgptr;
                    *imgptr += 0x10000;
                    heap_cur += (*nbr & 0xff) - (*imgptr & 0xff);
                    imgptr = nbr;
                    comptr++;
                    comp_init(comptr);
                    comptr->grey_level = (unsigned long)(*imgptr & 0xff);
                    continue;
                } else {
                    int d = (*nbr & 0xff) - (*imgptr & 0xff);
                    heap_cur[d]++;
                    *heap_cur[d] = nbr;
                }
            }
            *imgptr += 0x10000;
        }
        {
            int imsk = (int)(imgptr - ioptr);
            ptsptr->x = imsk & stepmask;
            ptsptr->y = imsk >> stepgap;
        }
        accumulate(comptr, ptsptr);
        ptsptr++;
        if (**heap_cur) {
            imgptr = **heap_cur;
            (*heap_cur)--;
        } else {
            unsigned long pixel_val = 0, i;
            heap_cur++;
            for (i = (unsigned long)((*imgptr & 0xff) + 1); i < 256; i++) {
                if (**heap_cur) {
                    pixel_val = i;
                    break;
                }
                heap_cur++;
            }
            if (!pixel_val) break;
            imgptr = **heap_cur;
            (*heap_cur)--;
            if (pixel_val < comptr[-1].grey_level) {
                if (stable_check(comptr, p)) emit(comptr, color, out);
                new_history(comptr, histptr);
                comptr[0].grey_level = pixel_val;
                histptr++;
            } else {
                for (;;) {
                    comptr--;
                    merge_comp(comptr + 1, comptr, comptr, histptr);
                    histptr++;
                    if (pixel_val <= comptr[0].grey_level) break;
                    if (pixel_val < comptr[-1].grey_level) {
                        if (stable_check(comptr, p)) emit(comptr, color, out);
                        new_history(comptr, histptr);
                        comptr[0].grey_level = pixel_val;
                        histptr++;
                        break;
                    }
                }
            }
        }
    }
}

int orc_mser_step(int w) {
    int step = 8;
    while (step < w + 2) step <<= 1;
    return step;
}

/* ---------------- cv::solve(A, b, x, DECOMP_SVD) for one right-hand side ---------------- */
/* At: n rows of m (A transposed); destroyed (becomes U^T).  x: n. */
static void orc_svd_solve(double *At, int m, int n, const double *b, double *x) {
    double W[8], Vt[64], sd, threshold = 0;
    const double eps = DBL_EPSILON * 10;
    int i, j, k, iter, max_iter = m > 30 ? m : 30;
    for (i = 0; i < n; i++) {
        for (k = 0, sd = 0; k < m; k++) sd += At[i * m + k] * At[i * m + k];
        W[i] = sd;
        for (k = 0; k < n; k++) Vt[i * n + k] = 0;
        Vt[i * n + i] = 1;
    }
    for (iter = 0; iter < max_iter; iter++) {
        int changed = 0;
        for (i = 0; i < n - 1; i++)
            for (j = i + 1; j < n; j++) {
                double *Ai = At + i * m, *Aj = At + j * m;
                double a = W[i], pp = 0, bb = W[j], beta, gamma, c, s;
                for (k = 0; k < m; k++) pp += Ai[k] * Aj[k];
                if (fabs(pp) <= eps * sqrt(a * bb)) continue;
                pp *= 2;
                beta = a - bb;
                gamma = sqrt(pp * pp + beta * beta);
                if (beta < 0) {
                    double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = pp / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = pp / (gamma * c * 2);
                }
                a = bb = 0;
                for (k = 0; k < m; k++) {
                    double t0 = c * Ai[k] + s * Aj[k];
                    double t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0;
                    Aj[k] = t1;
                    a += t0 * t0;
                    bb += t1 * t1;
                }
                W[i] = a;
                W[j] = bb;
                changed = 1;
                {
                    double *Vi = Vt + i * n, *Vj = Vt + j * n;
                    for (k = 0; k < n; k++) {
                        double t0 = c * Vi[k] + s * Vj[k];
                        double t1 = -s * Vi[k] + c * Vj[k];
                        Vi[k] = t0;
                        Vj[k] = t1;
                    }
                }
            }
        if (!changed) break;
    }
    for (i = 0; i < n; i++) {
        for (k = 0, sd = 0; k < m; k++) sd += At[i * m + k] * At[i * m + k];
        W[i] = sqrt(sd);
    }
    for (i = 0; i < n - 1; i++) {
        j = i;
        for (k = i + 1; k < n; k++)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            double t = W[i];
            W[i] = W[j];
            W[j] = t;
            for (k = 0; k < m; k++) {
                t = At[i * m + k];
                At[i * m + k] = At[j * m + k];
                At[j * m + k] = t;
            }
            for (k = 0; k < n; k++) {
                t = Vt[i * n + k];
                Vt[i * n + k] = Vt[j * n + k];
                Vt[j * n + k] = t;
            }
        }
    }
    for (i = 0; i < n; i++) {
        double t;
        if (W[i] <= DBL_MIN) continue; /* OpenCV's random left vector: unused below */
        t = 1. / W[i];
        for (k = 0; k < m; k++) At[i * m + k] *= t;
    }
    /* SVBkSbImpl_, nb = 1 */
    for (i = 0; i < n; i++) x[i] = 0;
    for (i = 0; i < n; i++) threshold += W[i];
    threshold *= DBL_EPSILON * 2;
    for (i = 0; i < n; i++) {
        double wi = W[i], s = 0;
        if (fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        for (k = 0; k < m; k++) s += At[i * m + k] * b[k];
        s *= wi;
        for (k = 0; k < n; k++) x[k] = x[k] + s * Vt[i * n + k];
    }
}

/* cvFitEllipse2's three solves on integer points: sol = {cx, cy, A..E of the conic, the centre (2), the
 * re-fit's A..C} (12 doubles; cx, cy hold floats); -1 when n < 5 */
int orc_fit_ellipse_solves(const int *xy, int n, double *sol) {
    double *Ad, *bd, gfp[5], rp[2];
    float cx = 0, cy = 0;
    int i;
    if (n < 5) return -1;
    Ad = (double *)malloc(sizeof(double) * 5 * (size_t)n);
    bd = (double *)malloc(sizeof(double) * (size_t)n);
    for (i = 0; i < n; i++) {
        cx += (float)xy[2 * i];
        cy += (float)xy[2 * i + 1];
    }
    cx /= n;
    cy /= n;
    /* A (n x 5) stored transposed: column c of A is At[c * n ..] */
    for (i = 0; i < n; i++) {
        float px = (float)xy[2 * i] - cx, py = (float)xy[2 * i + 1] - cy;
        bd[i] = 10000.0;
        Ad[0 * n + i] = -(double)px * px;
        Ad[1 * n + i] = -(double)py * py;
        Ad[2 * n + i] = -(double)px * py;
        Ad[3 * n + i] = px;
        Ad[4 * n + i] = py;
    }
    orc_svd_solve(Ad, n, 5, bd, gfp);
    {
        double A2[4], b2[2];
        /* A = [[2 g0, g2], [g2, 2 g1]] transposed (symmetric) */
        A2[0] = 2 * gfp[0];
        A2[1] = A2[2] = gfp[2];
        A2[3] = 2 * gfp[1];
        b2[0] = gfp[3];
        b2[1] = gfp[4];
        orc_svd_solve(A2, 2, 2, b2, rp);
    }
    sol[0] = cx;
    sol[1] = cy;
    for (i = 0; i < 5; i++) sol[2 + i] = gfp[i];
    sol[7] = rp[0];
    sol[8] = rp[1];
    for (i = 0; i < n; i++) {
        float px = (float)xy[2 * i] - cx, py = (float)xy[2 * i + 1] - cy;
        bd[i] = 1.0;
        Ad[0 * n + i] = (px - rp[0]) * (px - rp[0]);
        Ad[1 * n + i] = (py - rp[1]) * (py - rp[1]);
        Ad[2 * n + i] = (px - rp[0]) * (py - rp[1]);
    }
    orc_svd_solve(Ad, n, 3, bd, sol + 9);
    free(Ad);
    free(bd);
    return 0;
}

/* the RotatedRect from the solves: box = {cx, cy, width, height, angle} */
void orc_ellipse_box(const double *sol, float *box) {
    const double min_eps = 1e-6, *gfp = sol + 9;
    double rp[5], t;
    float bw, bh, ang = 0;
    rp[0] = sol[7];
    rp[1] = sol[8];
    rp[4] = -0.5 * fm3d_atan2(gfp[2], gfp[1] - gfp[0]);
    t = fm3d_sin(-2.0 * rp[4]);
    if (fabs(t) > fabs(gfp[2]) * min_eps)
        t = gfp[2] / t;
    else
        t = gfp[1] - gfp[0];
    rp[2] = fabs(gfp[0] + gfp[1] - t);
    if (rp[2] > min_eps) rp[2] = sqrt(2.0 / rp[2]);
    rp[3] = fabs(gfp[0] + gfp[1] + t);
    if (rp[3] > min_eps) rp[3] = sqrt(2.0 / rp[3]);
    box[0] = (float)rp[0] + (float)sol[0];
    box[1] = (float)rp[1] + (float)sol[1];
    bw = (float)(rp[2] * 2);
    bh = (float)(rp[3] * 2);
    if (bw > bh) {
        float tmp = bw;
        bw = bh;
        bh = tmp;
        ang = (float)(90 + rp[4] * 180 / M_PI);
    }
    if (ang < -180) ang += 360;
    if (ang > 360) ang -= 360;
    box[2] = bw;
    box[3] = bh;
    box[4] = ang;
}

/* cvFitEllipse2 on integer points: box = {cx, cy, width, height, angle}; -1 when n < 5 */
int orc_fit_ellipse(const int *xy, int n, float *box) {
    double sol[12];
    if (orc_fit_ellipse_solves(xy, n, sol) < 0) return -1;
    orc_ellipse_box(sol, box);
    return 0;
}

/* Both passes.  Regions: color[i], count[i] and their points (x, y) concatenated in pts_out (capacity
 * ptcap pairs).  Returns the region count (all of them; min(count, cap) written) or -1 on bad input.
 * *npts = total points (all). */
int orc_mser_regions(const uint8_t *img, int w, int h, int delta, int minArea, int maxArea, double maxVariation,
                     double minDiversity, int *color, int *count, int cap, int *pts_out, long long ptcap,
                     long long *npts) {
    orc_mser_params p;
    int step, stepgap = 3, nreg = 0, pass, i;
    int *im, **heap, ***heap_cur;
    orc_lpt *pts;
    orc_hist *hist;
    orc_comp comp[257];
    uint8_t *src;
    orc_regs out = {NULL, 0, 0};
    long long tot = 0;
    const size_t N = (size_t)w * h;
    if (w <= 0 || h <= 0 || !img) return -1;
    p.delta = delta;
    p.minArea = minArea;
    p.maxArea = maxArea;
    p.maxVariation = maxVariation;
    p.minDiversity = minDiversity;
    step = 8;
    while (step < w + 2) {
        step <<= 1;
        stepgap++;
    }
    im = (int *)malloc(sizeof(int) * (size_t)(h + 2) * step);
    heap = (int **)malloc(sizeof(int *) * (N + 256));
    heap_cur = (int ***)malloc(sizeof(int **) * 256);
    pts = (orc_lpt *)malloc(sizeof(orc_lpt) * N * 2); /* one list per pass: regions are walked after both */
    /* mser.cpp allocates w * h histories; a raise per accumulated pixel plus a merge per opened
     * component can exceed that, so this allocates the bound (2 w h + 2) */
    hist = (orc_hist *)malloc(sizeof(orc_hist) * (2 * N + 2));
    src = (uint8_t *)malloc(N);
    memcpy(src, img, N);
    for (pass = 0; pass < 2; pass++) {
        int *start;
        heap_cur[0] = heap;
        start = preprocess(im, step, heap_cur, src, w, h);
        mser_pass(im + step + 1, start, heap_cur, pts + (size_t)pass * N, hist, comp, step, step - 1, stepgap, &p,
                  pass == 0 ? -1 : 1, &out);
    }
    nreg = out.n;
    for (i = 0; i < nreg; i++) {
        orc_lpt *q = out.r[i].head;
        int k;
        if (i < cap) {
            color[i] = out.r[i].color;
            count[i] = out.r[i].count;
        }
        for (k = 0; k < out.r[i].count; k++, q = q->next) {
            if (pts_out && tot < ptcap) {
                pts_out[2 * tot] = q->x;
                pts_out[2 * tot + 1] = q->y;
            }
            tot++;
        }
    }
    *npts = tot;
    free(im);
    free(heap);
    free(heap_cur);
    free(pts);
    free(hist);
    free(src);
    free(out.r);
    return nreg;
}

/* cv::MserFeatureDetector(...).detect: keypoints {x, y, size, angle -1, response 0, octave 0, class -1}
 * as 7 floats-ish fields of fm3d_keypoint order (x, y, size, angle, response, octave, class_id).
 * Returns the keypoint count (min(count, cap) written) or -1 (bad input / a region below 5 points:
 * OpenCV's fitEllipse throws). */
typedef struct {
    float x, y, size, angle, response;
    int octave, class_id;
} orc_mser_kp;

int orc_mser_detect(const uint8_t *img, int w, int h, int delta, int minArea, int maxArea, double maxVariation,
                    double minDiversity, orc_mser_kp *kp, int cap) {
    int nreg, cap2, i, nk = 0;
    int *color, *count, *pts;
    long long npts = 0, off = 0;
    nreg = orc_mser_regions(img, w, h, delta, minArea, maxArea, maxVariation, minDiversity, NULL, NULL, 0, NULL, 0,
                            &npts);
    if (nreg < 0) return -1;
    cap2 = nreg > 0 ? nreg : 1;
    color = (int *)malloc(sizeof(int) * cap2);
    count = (int *)malloc(sizeof(int) * cap2);
    pts = (int *)malloc(sizeof(int) * 2 * (size_t)(npts > 0 ? npts : 1));
    orc_mser_regions(img, w, h, delta, minArea, maxArea, maxVariation, minDiversity, color, count, cap2, pts, npts,
                     &npts);
    for (i = 0; i < nreg; i++) {
        float box[5], diam;
        int rx, ry;
        if (orc_fit_ellipse(pts + 2 * off, count[i], box) < 0) {
            nk = -1;
            break;
        }
        off += count[i];
        diam = sqrtf(box[3] * box[2]);
        /* Rect::contains(Point(cvRound(cx), cvRound(cy))): cvRound of a NaN, an infinity or a value
         * past the int range is INT_MIN (SSE2 conversion), never inside; compared as floats here */
        {
            const float fx = rintf(box[0]), fy = rintf(box[1]);
            rx = fx >= 0.f && fx < (float)w;
            ry = fy >= 0.f && fy < (float)h;
        }
        if (diam > FLT_EPSILON && rx && ry) {
            if (nk < cap) {
                kp[nk].x = box[0];
                kp[nk].y = box[1];
                kp[nk].size = diam;
                kp[nk].angle = -1;
                kp[nk].response = 0;
                kp[nk].octave = 0;
                kp[nk].class_id = -1;
            }
            nk++;
        }
    }
    free(color);
    free(count);
    free(pts);
    return nk;
}
