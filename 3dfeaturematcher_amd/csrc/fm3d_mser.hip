// fm3d_mser.hip -- the MSER detector on gfx950.
//
// Reference: DescriptorsMatcher's DetectorType MSER (descriptorsmatcher.cpp:258-272:
// cv::MserFeatureDetector(Delta, MinArea, MaxArea, MaxVariation, MinDiversity, MaxEvolution,
// AreaThreshold, MinMargin, EdgeBlurSize) of OpenCV 2.4.9; on grey images only the first five steer
// the result).  Restated in oracle/orc_mser.c (pointer form, as mser.cpp); this file is an index-based
// statement of the same steps and equals the oracle bit for bit.
//
// MSER's linear-time flood (Nister & Stewenius, as mser.cpp implements it) is one priority flood per
// pass whose visiting order decides which component's history continues at equal-size merges, which
// point list comes first, and the order the regions come out in -- all part of the detector's output.
// It is sequential by construction, so each pass is one lane (the two passes run side by side, one
// workgroup each); the rest of the workgroup lays out the padded int image and the grey-level
// histogram first.  The component stack (257 entries) and the 256 bucket tops live in LDS; the padded
// image, the bucket heap, the point nodes and the histories in HBM (L2-resident at VGA sizes).
// fitEllipse then runs one lane per region (its three least-squares solves are OpenCV's scalar
// one-sided Jacobi SVD, sums in the region list's order), all regions in parallel.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "fm3d_detmath.h"
#include "fm3d_kernels.h"

namespace fm3d {

MserLayout mser_layout(int w, int h) {
    MserLayout L;
    L.w = w;
    L.h = h;
    L.step = 8;
    L.stepgap = 3;
    while (L.step < w + 2) {
        L.step <<= 1;
        L.stepgap++;
    }
    const long long N = (long long)w * h;
    L.imgInts = (long long)(h + 2) * L.step;
    L.heapInts = N + 256;
    L.nodes = N;
    L.hists = 2 * N + 2;
    L.regCap = N + 1;
    return L;
}

namespace {

struct Comp {  // MSERConnectedComp by index
    int head, tail, hist, level, size, dvar;
    float var;
};

constexpr int kMserThreads = 256;

__device__ __forceinline__ void comp_init(Comp& c) {
    c.size = 0;
    c.var = 0.f;
    c.dvar = 1;
    c.hist = -1;
}

// MSERNewHistory
__device__ __forceinline__ void new_history(Comp& c, MserHist* hist, int hi) {
    MserHist r;
    r.child = hi;
    if (c.hist < 0) {
        r.shortcut = hi;
        r.stable = 0;
    } else {
        hist[c.hist].child = hi;
        r.shortcut = hist[c.hist].shortcut;
        r.stable = hist[c.hist].stable;
    }
    r.val = c.level;
    r.size = c.size;
    hist[hi] = r;
    c.hist = hi;
}

// MSERMergeComp(top, below, below, history): the larger keeps its history (the top one on a tie);
// its point list comes first
__device__ __forceinline__ void merge(const Comp& top, Comp& below, MserHist* hist, int2* node, int hi) {
    const bool topWins = top.size >= below.size;
    const Comp win = topWins ? top : below, lose = topWins ? below : top;
    MserHist r;
    r.child = hi;
    if (win.hist < 0) {
        r.shortcut = hi;
        r.stable = 0;
    } else {
        hist[win.hist].child = hi;
        r.shortcut = hist[win.hist].shortcut;
        r.stable = hist[win.hist].stable;
    }
    if (lose.hist >= 0) {
        const int ls = hist[lose.hist].stable;
        if (ls > r.stable) r.stable = ls;
    }
    r.val = win.level;
    r.size = win.size;
    hist[hi] = r;
    if (top.size > 0 && below.size > 0) node[win.tail].x = lose.head;
    Comp m;
    m.level = below.level;
    m.var = win.var;
    m.dvar = win.dvar;
    m.head = win.size > 0 ? win.head : lose.head;
    m.tail = lose.size > 0 ? lose.tail : win.tail;
    m.hist = hi;
    m.size = top.size + below.size;
    below = m;
}

// MSERStableCheck (with MSERVariationCalc)
__device__ __forceinline__ bool stable_check(Comp& c, MserHist* hist, const MserParams& P) {
    if (c.hist < 0) return false;
    MserHist H = hist[c.hist];
    if (H.size <= P.minArea || H.size >= P.maxArea) return false;
    const float div = (float)(H.size - H.stable) / (float)H.size;
    int sc = H.shortcut;
    MserHist S = hist[sc];
    while (sc != S.shortcut && S.val + P.delta > c.level) {
        sc = S.shortcut;
        S = hist[sc];
    }
    int ch = S.child;
    MserHist C = hist[ch];
    while (ch != C.child && C.val + P.delta <= c.level) {
        sc = ch;
        S = C;
        ch = C.child;
        C = hist[ch];
    }
    hist[c.hist].shortcut = sc;
    const float var = (float)(c.size - S.size) / (float)S.size;
    const bool dvar = c.var < var || (unsigned)(H.val + 1) < (unsigned)c.level;
    const bool stable = dvar && !c.dvar && (double)c.var < P.maxVariation && (double)div > P.minDiversity;
    c.var = var;
    c.dvar = dvar ? 1 : 0;
    if (stable) hist[c.hist].stable = H.size;
    return stable;
}

__global__ __launch_bounds__(kMserThreads) void mser_flood_kernel(const uint8_t* __restrict__ src, MserLayout L,
                                                                   MserParams P, int* work, int* heapAll,
                                                                   int2* nodeAll, MserHist* histAll, int4* regAll,
                                                                   int* nreg) {
    const int pass = blockIdx.x, tid = threadIdx.x;
    int* img = work + (size_t)pass * L.imgInts;
    int* heap = heapAll + (size_t)pass * L.heapInts;
    int2* node = nodeAll + (size_t)pass * L.nodes;
    MserHist* hist = histAll + (size_t)pass * L.hists;
    int4* reg = regAll + (size_t)pass * L.regCap;
    __shared__ int hcur[256];
    __shared__ int lsize[256];
    __shared__ Comp comp[257];
    for (int i = tid; i < 256; i += kMserThreads) lsize[i] = 0;
    __syncthreads();
    // preprocessMSER_8UC1: -1 border, grey value (255 - I on pass 0) inside, the level histogram
    const int smask = L.step - 1;
    for (long long i = tid; i < L.imgInts; i += kMserThreads) {
        const int y = (int)(i >> L.stepgap), x = (int)(i & smask);
        int v = -1;
        if (y >= 1 && y <= L.h && x >= 1 && x <= L.w) {
            const int g = src[(size_t)(y - 1) * L.w + (x - 1)];
            v = pass == 0 ? 255 - g : g;
            atomicAdd(&lsize[v], 1);
        }
        img[i] = v;
    }
    __syncthreads();
    if (tid != 0) return;
    {
        int base = 0;
        hcur[0] = 0;
        heap[0] = 0;
        for (int i = 1; i < 256; i++) {
            base += lsize[i - 1] + 1;
            hcur[i] = base;
            heap[base] = 0;
        }
    }
    const int color = pass == 0 ? -1 : 1, ioff = L.step + 1;
    const long long regCap = L.regCap;
    int nnode = 0, nhist = 0, nr = 0;
    int cur = ioff;
    int cv = img[cur];
    int top = 1;
    comp[0].level = 256;
    comp_init(comp[1]);
    comp[1].level = cv & 0xff;
    cv |= (int)0x80000000;
    img[cur] = cv;
    int lev = cv & 0xff;
    for (;;) {
        bool descended = false;
        while ((cv & 0x70000) < 0x40000) {
            const int d = (cv & 0x70000) >> 16;
            const int nb = cur + (d == 0 ? 1 : d == 1 ? L.step : d == 2 ? -1 : -L.step);
            int nv = img[nb];
            if (nv >= 0) {
                nv |= (int)0x80000000;
                img[nb] = nv;
                if ((nv & 0xff) < (cv & 0xff)) {
                    // push the current pixel back and open a component at the neighbour's level
                    const int t = ++hcur[lev];
                    heap[t] = cur;
                    cv += 0x10000;
                    img[cur] = cv;
                    lev = nv & 0xff;
                    cur = nb;
                    cv = nv;
                    top++;
                    comp_init(comp[top]);
                    comp[top].level = lev;
                    descended = true;
                    break;
                }
                const int b = nv & 0xff;
                const int t = ++hcur[b];
                heap[t] = nb;
            }
            cv += 0x10000;
        }
        if (descended) continue;
        // accumulateMSERComp: the finished pixel joins the top component's list
        {
            Comp& c = comp[top];
            node[nnode] = make_int2(-1, cur - ioff);
            if (c.size > 0)
                node[c.tail].x = nnode;
            else
                c.head = nnode;
            c.tail = nnode;
            c.size++;
            nnode++;
        }
        {
            const int t = hcur[lev];
            const int nx = heap[t];
            if (nx) {
                cur = nx;
                hcur[lev] = t - 1;
                cv = img[cur];
                continue;
            }
        }
        int pv = 0;
        for (int i = (cv & 0xff) + 1; i < 256; i++)
            if (heap[hcur[i]]) {
                pv = i;
                break;
            }
        if (!pv) break;
        lev = pv;
        {
            const int t = hcur[lev];
            cur = heap[t];
            hcur[lev] = t - 1;
            cv = img[cur];
        }
        if (pv < comp[top - 1].level) {
            if (stable_check(comp[top], hist, P)) {
                if (nr < regCap) reg[nr] = make_int4(color, comp[top].head, hist[comp[top].hist].size, 0);
                nr++;
            }
            new_history(comp[top], hist, nhist++);
            comp[top].level = pv;
        } else {
            for (;;) {
                top--;
                merge(comp[top + 1], comp[top], hist, node, nhist++);
                if (pv <= comp[top].level) break;
                if (pv < comp[top - 1].level) {
                    if (stable_check(comp[top], hist, P)) {
                        if (nr < regCap) reg[nr] = make_int4(color, comp[top].head, hist[comp[top].hist].size, 0);
                        nr++;
                    }
                    new_history(comp[top], hist, nhist++);
                    comp[top].level = pv;
                    break;
                }
            }
        }
    }
    nreg[pass] = nr;
}

// cv::solve(A, b, DECOMP_SVD) with At = A^T (n rows of m), b constant (bval): JacobiSVDImpl_ + SVBkSbImpl_
__device__ void svd_solve(double* At, int m, int n, double bval, double* x) {
    double W[5], Vt[25];
    const double eps = DBL_EPSILON * 10;
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) sd += At[i * m + k] * At[i * m + k];
        W[i] = sd;
        for (int k = 0; k < n; k++) Vt[i * n + k] = 0;
        Vt[i * n + i] = 1;
    }
    const int max_iter = m > 30 ? m : 30;
    for (int iter = 0; iter < max_iter; iter++) {
        bool changed = false;
        for (int i = 0; i < n - 1; i++)
            for (int j = i + 1; j < n; j++) {
                double* Ai = At + i * m;
                double* Aj = At + j * m;
                double a = W[i], pp = 0, bb = W[j];
                for (int k = 0; k < m; k++) pp += Ai[k] * Aj[k];
                if (fabs(pp) <= eps * sqrt(a * bb)) continue;
                pp *= 2;
                const double beta = a - bb, gamma = sqrt(pp * pp + beta * beta);
                double c, s;
                if (beta < 0) {
                    const double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = pp / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = pp / (gamma * c * 2);
                }
                a = bb = 0;
                for (int k = 0; k < m; k++) {
                    const double t0 = c * Ai[k] + s * Aj[k];
                    const double t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0;
                    Aj[k] = t1;
                    a += t0 * t0;
                    bb += t1 * t1;
                }
                W[i] = a;
                W[j] = bb;
                changed = true;
                for (int k = 0; k < n; k++) {
                    const double t0 = c * Vt[i * n + k] + s * Vt[j * n + k];
                    const double t1 = -s * Vt[i * n + k] + c * Vt[j * n + k];
                    Vt[i * n + k] = t0;
                    Vt[j * n + k] = t1;
                }
            }
        if (!changed) break;
    }
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) sd += At[i * m + k] * At[i * m + k];
        W[i] = sqrt(sd);
    }
    for (int i = 0; i < n - 1; i++) {
        int j = i;
        for (int k = i + 1; k < n; k++)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            double t = W[i];
            W[i] = W[j];
            W[j] = t;
            for (int k = 0; k < m; k++) {
                t = At[i * m + k];
                At[i * m + k] = At[j * m + k];
                At[j * m + k] = t;
            }
            for (int k = 0; k < n; k++) {
                t = Vt[i * n + k];
                Vt[i * n + k] = Vt[j * n + k];
                Vt[j * n + k] = t;
            }
        }
    }
    for (int i = 0; i < n; i++) {
        if (W[i] <= DBL_MIN) continue;  // OpenCV's random left vector: unused below
        const double t = 1. / W[i];
        for (int k = 0; k < m; k++) At[i * m + k] *= t;
    }
    double threshold = 0;
    for (int i = 0; i < n; i++) x[i] = 0;
    for (int i = 0; i < n; i++) threshold += W[i];
    threshold *= DBL_EPSILON * 2;
    for (int i = 0; i < n; i++) {
        double wi = W[i], s = 0;
        if (fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        for (int k = 0; k < m; k++) s += At[i * m + k] * bval;
        s *= wi;
        for (int k = 0; k < n; k++) x[k] = x[k] + s * Vt[i * n + k];
    }
}

__global__ __launch_bounds__(64) void mser_fit_kernel(const int4* __restrict__ reg, long long regCap, int n0, int n,
                                                      const int2* __restrict__ nodeAll, long long nodes,
                                                      const long long* __restrict__ off, MserLayout L, int2* xyAll,
                                                      double* scratch, fm3d_keypoint* kp, int* flag, float* boxOut) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int pass = r < n0 ? 0 : 1;
    const int4 R = reg[pass * regCap + (pass ? r - n0 : r)];
    const int2* node = nodeAll + pass * nodes;
    const int m = R.z;
    int2* xy = xyAll + off[r];
    double* At = scratch + 5 * off[r];
    {
        int q = R.y;
        for (int k = 0; k < m; k++) {
            const int2 nd = node[q];
            xy[k] = make_int2(nd.y & (L.step - 1), nd.y >> L.stepgap);
            q = nd.x;
        }
    }
    float cx = 0.f, cy = 0.f;
    for (int k = 0; k < m; k++) {
        cx = __fadd_rn(cx, (float)xy[k].x);
        cy = __fadd_rn(cy, (float)xy[k].y);
    }
    cx = cx / (float)m;
    cy = cy / (float)m;
    for (int k = 0; k < m; k++) {
        const float px = __fsub_rn((float)xy[k].x, cx), py = __fsub_rn((float)xy[k].y, cy);
        At[0 * m + k] = -(double)px * (double)px;
        At[1 * m + k] = -(double)py * (double)py;
        At[2 * m + k] = -(double)px * (double)py;
        At[3 * m + k] = px;
        At[4 * m + k] = py;
    }
    double gfp[5], rp[5];
    svd_solve(At, m, 5, 10000.0, gfp);
    {
        double A2[4], x2[2];
        A2[0] = 2 * gfp[0];
        A2[1] = A2[2] = gfp[2];
        A2[3] = 2 * gfp[1];
        // b = (gfp[3], gfp[4]) is not constant: the 2 x 2 solve inline
        double W2[2], V2[4];
        {
            // same steps as svd_solve with m = n = 2 and a vector right-hand side
            double* At2 = A2;
            const double eps = DBL_EPSILON * 10;
            for (int i = 0; i < 2; i++) {
                double sd = 0;
                for (int k = 0; k < 2; k++) sd += At2[i * 2 + k] * At2[i * 2 + k];
                W2[i] = sd;
                V2[i * 2] = 0;
                V2[i * 2 + 1] = 0;
                V2[i * 2 + i] = 1;
            }
            for (int iter = 0; iter < 30; iter++) {
                bool changed = false;
                double a = W2[0], pp = 0, bb = W2[1];
                for (int k = 0; k < 2; k++) pp += At2[k] * At2[2 + k];
                if (!(fabs(pp) <= eps * sqrt(a * bb))) {
                    pp *= 2;
                    const double beta = a - bb, gamma = sqrt(pp * pp + beta * beta);
                    double c, s;
                    if (beta < 0) {
                        const double delta = (gamma - beta) * 0.5;
                        s = sqrt(delta / gamma);
                        c = pp / (gamma * s * 2);
                    } else {
                        c = sqrt((gamma + beta) / (gamma * 2));
                        s = pp / (gamma * c * 2);
                    }
                    a = bb = 0;
                    for (int k = 0; k < 2; k++) {
                        const double t0 = c * At2[k] + s * At2[2 + k];
                        const double t1 = -s * At2[k] + c * At2[2 + k];
                        At2[k] = t0;
                        At2[2 + k] = t1;
                        a += t0 * t0;
                        bb += t1 * t1;
                    }
                    W2[0] = a;
                    W2[1] = bb;
                    changed = true;
                    for (int k = 0; k < 2; k++) {
                        const double t0 = c * V2[k] + s * V2[2 + k];
                        const double t1 = -s * V2[k] + c * V2[2 + k];
                        V2[k] = t0;
                        V2[2 + k] = t1;
                    }
                }
                if (!changed) break;
            }
            for (int i = 0; i < 2; i++) {
                double sd = 0;
                for (int k = 0; k < 2; k++) sd += At2[i * 2 + k] * At2[i * 2 + k];
                W2[i] = sqrt(sd);
            }
            if (W2[0] < W2[1]) {
                double t = W2[0];
                W2[0] = W2[1];
                W2[1] = t;
                for (int k = 0; k < 2; k++) {
                    t = At2[k];
                    At2[k] = At2[2 + k];
                    At2[2 + k] = t;
                    t = V2[k];
                    V2[k] = V2[2 + k];
                    V2[2 + k] = t;
                }
            }
            for (int i = 0; i < 2; i++) {
                if (W2[i] <= DBL_MIN) continue;
                const double t = 1. / W2[i];
                for (int k = 0; k < 2; k++) At2[i * 2 + k] *= t;
            }
            const double b2[2] = {gfp[3], gfp[4]};
            double threshold = 0;
            x2[0] = x2[1] = 0;
            threshold += W2[0];
            threshold += W2[1];
            threshold *= DBL_EPSILON * 2;
            for (int i = 0; i < 2; i++) {
                double wi = W2[i], s = 0;
                if (fabs(wi) <= threshold) continue;
                wi = 1 / wi;
                for (int k = 0; k < 2; k++) s += At2[i * 2 + k] * b2[k];
                s *= wi;
                for (int k = 0; k < 2; k++) x2[k] = x2[k] + s * V2[i * 2 + k];
            }
        }
        rp[0] = x2[0];
        rp[1] = x2[1];
    }
    for (int k = 0; k < m; k++) {
        const float px = __fsub_rn((float)xy[k].x, cx), py = __fsub_rn((float)xy[k].y, cy);
        At[0 * m + k] = ((double)px - rp[0]) * ((double)px - rp[0]);
        At[1 * m + k] = ((double)py - rp[1]) * ((double)py - rp[1]);
        At[2 * m + k] = ((double)px - rp[0]) * ((double)py - rp[1]);
    }
    double g[3];
    svd_solve(At, m, 3, 1.0, g);
    const double min_eps = 1e-6;
    rp[4] = -0.5 * fm3d_atan2(g[2], g[1] - g[0]);
    double t = fm3d_sin(-2.0 * rp[4]);
    if (fabs(t) > fabs(g[2]) * min_eps)
        t = g[2] / t;
    else
        t = g[1] - g[0];
    rp[2] = fabs(g[0] + g[1] - t);
    if (rp[2] > min_eps) rp[2] = sqrt(2.0 / rp[2]);
    rp[3] = fabs(g[0] + g[1] + t);
    if (rp[3] > min_eps) rp[3] = sqrt(2.0 / rp[3]);
    const float bx = __fadd_rn((float)rp[0], cx), by = __fadd_rn((float)rp[1], cy);
    float bw = (float)(rp[2] * 2), bh = (float)(rp[3] * 2), ang = 0.f;
    if (bw > bh) {
        const float tmp = bw;
        bw = bh;
        bh = tmp;
        ang = (float)(90 + rp[4] * 180 / M_PI);
    }
    if (ang < -180) ang = __fadd_rn(ang, 360.f);
    if (ang > 360) ang = __fsub_rn(ang, 360.f);
    const float diam = sqrtf(bh * bw);
    const int rx = (int)rintf(bx), ry = (int)rintf(by);
    fm3d_keypoint k;
    k.x = bx;
    k.y = by;
    k.size = diam;
    k.angle = -1.f;
    k.response = 0.f;
    k.octave = 0;
    k.class_id = -1;
    kp[r] = k;
    flag[r] = diam > FLT_EPSILON && rx >= 0 && rx < L.w && ry >= 0 && ry < L.h;
    if (boxOut) {
        boxOut[5 * r + 0] = bx;
        boxOut[5 * r + 1] = by;
        boxOut[5 * r + 2] = bw;
        boxOut[5 * r + 3] = bh;
        boxOut[5 * r + 4] = ang;
    }
}

}  // namespace

void launch_mser_flood(const uint8_t* img, const MserLayout& L, const MserParams& P, int* work, int* heap, int2* node,
                       MserHist* hist, int4* reg, int* nreg, hipStream_t s) {
    mser_flood_kernel<<<2, kMserThreads, 0, s>>>(img, L, P, work, heap, node, hist, reg, nreg);
}

void launch_mser_fit(const int4* reg, long long regCap, int n0, int n, const int2* node, long long nodes,
                     const long long* off, const MserLayout& L, int2* xy, double* scratch, fm3d_keypoint* kp, int* flag,
                     float* box, hipStream_t s) {
    if (n <= 0) return;
    mser_fit_kernel<<<(n + 63) / 64, 64, 0, s>>>(reg, regCap, n0, n, node, nodes, off, L, xy, scratch, kp, flag, box);
}

}  // namespace fm3d
