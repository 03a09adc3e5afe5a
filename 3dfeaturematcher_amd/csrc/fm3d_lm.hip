// fm3d_lm.hip -- NormalOptimizer::computeOptimizedNormals on gfx950.
//
// Reference: Triangulator/normaloptimizer.cpp:223-452 (optimize_pyramid, optimize,
// computeOptimizedNormals), the residual evaluateNormal (:65-149) and the
// SingleCameraTriangulator geometry it calls (singlecameratriangulator.cpp:341-665),
// minimised by lmfit's lmmin (MINPACK lmdif with lmfit's lm_control_double).
//
// Design: one LANE per keypoint.  The LM trajectory of a point
// is decided at the rounding-noise level (ftol = xtol = 30*DBL_EPSILON), so any
// reordering of the m_dat-long sums (fnorm, column norms, Householder dot
// products) changes which steps are accepted and moves the final normal by up
// to 1e-2 on ~15 % of points (measured with the oracle).  Each lane
// therefore runs the reference's sequential algorithm for its own point: every
// sum is accumulated in pixel-index order exactly as MINPACK does, so results
// are bit-identical to the oracle.  The 64 lanes of a wave stream their per-pixel
// arrays from a slab laid out [pixel][lane] (one 512-byte line per double
// array and pixel), so every load and store is fully coalesced; the image
// samples are gathers served from L2.  Lanes fetch new points from a global
// queue when they finish one, so a wave stays full until the queue drains.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "fm3d_device.h"
#include "fm3d_kernels.h"

namespace fm3d {

namespace {

constexpr int kWave = 64;

enum LaneState { S_NEED_POINT = 0, S_INIT, S_LEVEL, S_EVAL, S_QR, S_DONE };
enum EvalKind { E_INITIAL = 0, E_JAC0, E_JAC1, E_TRIAL };

constexpr double kEpsmch = DBL_EPSILON;
constexpr double kDwarf = DBL_MIN;

// ---- MINPACK qrsolv / lmpar for n = 2 (lmfit lm_qrsolv / lm_lmpar) ----
// r: 2x2 column-major (ldr = 2).  Op order identical to oracle/fm3d_oracle.c.
__device__ inline void qrsolv2(double* r, const int* ipvt, const double* diag, const double* qtb, double* x,
                               double* sdiag, double* wa) {
    const int n = 2;
#define R_(i, j) r[(j)*2 + (i)]
    for (int j = 0; j < n; j++) {
        for (int i = j; i < n; i++) R_(i, j) = R_(j, i);
        x[j] = R_(j, j);
        wa[j] = qtb[j];
    }
    for (int j = 0; j < n; j++) {
        int l = ipvt[j];
        if (diag[l] != 0.) {
            for (int k = j; k < n; k++) sdiag[k] = 0.;
            sdiag[j] = diag[l];
            double qtbpj = 0.;
            for (int k = j; k < n; k++) {
                if (sdiag[k] == 0.) continue;
                double sn, cs;
                if (fabs(R_(k, k)) < fabs(sdiag[k])) {
                    double ct = R_(k, k) / sdiag[k];
                    sn = 0.5 / sqrt(0.25 + 0.25 * ct * ct);
                    cs = sn * ct;
                } else {
                    double tn = sdiag[k] / R_(k, k);
                    cs = 0.5 / sqrt(0.25 + 0.25 * tn * tn);
                    sn = cs * tn;
                }
                R_(k, k) = cs * R_(k, k) + sn * sdiag[k];
                double temp = cs * wa[k] + sn * qtbpj;
                qtbpj = -sn * wa[k] + cs * qtbpj;
                wa[k] = temp;
                for (int i = k + 1; i < n; i++) {
                    temp = cs * R_(i, k) + sn * sdiag[i];
                    sdiag[i] = -sn * R_(i, k) + cs * sdiag[i];
                    R_(i, k) = temp;
                }
            }
        }
        sdiag[j] = R_(j, j);
        R_(j, j) = x[j];
    }
    int nsing = n;
    for (int j = 0; j < n; j++) {
        if (sdiag[j] == 0. && nsing == n) nsing = j;
        if (nsing < n) wa[j] = 0.;
    }
    for (int k = 0; k < nsing; k++) {
        int j = nsing - k - 1;
        double sum = 0.;
        for (int i = j + 1; i < nsing; i++) sum += R_(i, j) * wa[i];
        wa[j] = (wa[j] - sum) / sdiag[j];
    }
    for (int j = 0; j < n; j++) x[ipvt[j]] = wa[j];
#undef R_
}

__device__ inline void lmpar2(double* r, const int* ipvt, const double* diag, const double* qtb, double delta,
                              double* par, double* x, double* sdiag, double* wa1, double* wa2) {
    const int n = 2;
    const double p1 = 0.1, p001 = 0.001;
    int iter, nsing;
    double dxnorm, fp, gnorm, parc, parl, paru, sum, temp;
#define R_(i, j) r[(j)*2 + (i)]
    nsing = n;
    for (int j = 0; j < n; j++) {
        wa1[j] = qtb[j];
        if (R_(j, j) == 0. && nsing == n) nsing = j;
        if (nsing < n) wa1[j] = 0.;
    }
    for (int i = 0; i < nsing; i++) {
        int j = nsing - i - 1;
        wa1[j] = wa1[j] / R_(j, j);
        temp = wa1[j];
        for (int l = 0; l < j; l++) wa1[l] -= R_(l, j) * temp;
    }
    for (int j = 0; j < n; j++) x[ipvt[j]] = wa1[j];
    iter = 0;
    for (int j = 0; j < n; j++) wa2[j] = diag[j] * x[j];
    dxnorm = enorm2(wa2);
    fp = dxnorm - delta;
    if (fp <= p1 * delta) goto done;
    parl = 0.;
    if (nsing >= n) {
        for (int j = 0; j < n; j++) {
            int l = ipvt[j];
            wa1[j] = diag[l] * (wa2[l] / dxnorm);
        }
        for (int j = 0; j < n; j++) {
            sum = 0.;
            for (int i = 0; i < j; i++) sum += R_(i, j) * wa1[i];
            wa1[j] = (wa1[j] - sum) / R_(j, j);
        }
        temp = enorm2(wa1);
        parl = ((fp / delta) / temp) / temp;
    }
    for (int j = 0; j < n; j++) {
        sum = 0.;
        for (int i = 0; i <= j; i++) sum += R_(i, j) * qtb[i];
        int l = ipvt[j];
        wa1[j] = sum / diag[l];
    }
    gnorm = enorm2(wa1);
    paru = gnorm / delta;
    if (paru == 0.) paru = kDwarf / (delta < p1 ? delta : p1);
    *par = *par > parl ? *par : parl;
    *par = *par < paru ? *par : paru;
    if (*par == 0.) *par = gnorm / dxnorm;
    for (;;) {
        iter++;
        if (*par == 0.) *par = (kDwarf > p001 * paru) ? kDwarf : p001 * paru;
        temp = sqrt(*par);
        for (int j = 0; j < n; j++) wa1[j] = temp * diag[j];
        qrsolv2(r, ipvt, wa1, qtb, x, sdiag, wa2);
        for (int j = 0; j < n; j++) wa2[j] = diag[j] * x[j];
        dxnorm = enorm2(wa2);
        temp = fp;
        fp = dxnorm - delta;
        if (fabs(fp) <= p1 * delta || (parl == 0. && fp <= temp && temp < 0.) || iter == 10) break;
        for (int j = 0; j < n; j++) {
            int l = ipvt[j];
            wa1[j] = diag[l] * (wa2[l] / dxnorm);
        }
        for (int j = 0; j < n; j++) {
            wa1[j] = wa1[j] / sdiag[j];
            temp = wa1[j];
            for (int i = j + 1; i < n; i++) wa1[i] -= R_(i, j) * temp;
        }
        temp = enorm2(wa1);
        parc = ((fp / delta) / temp) / temp;
        if (fp > 0.) parl = parl > *par ? parl : *par;
        if (fp < 0.) paru = paru < *par ? paru : *par;
        *par = parl > *par + parc ? parl : *par + parc;
    }
done:
    if (iter == 0) *par = 0.;
#undef R_
}

// all LM bookkeeping of one lane (registers)
struct LM {
    double x[2], fnorm, par, delta, xnorm, gnorm, diag[2], acnorm[2], r[4], qtf[2], h[2];
    double wa1[2], wa2[2], pnorm;
    int iter, nfev, ipvt[2];
};

// MINPACK lmdif inner-loop head: lmpar, trial point (lmdif "determine the
// levenberg-marquardt parameter" ... "at first call adjust the step bound").
__device__ inline void lm_inner_step(LM& s) {
    double rr[4] = {s.r[0], s.r[1], s.r[2], s.r[3]};
    double sdiag[2], lw[2], wa3[2];
    lmpar2(rr, s.ipvt, s.diag, s.qtf, s.delta, &s.par, s.wa1, sdiag, lw, wa3);
    for (int j = 0; j < 2; j++) {
        s.wa1[j] = -s.wa1[j];
        s.wa2[j] = s.x[j] + s.wa1[j];
        wa3[j] = s.diag[j] * s.wa1[j];
    }
    s.pnorm = enorm2(wa3);
    if (s.iter == 1) s.delta = s.delta < s.pnorm ? s.delta : s.pnorm;
}

// MINPACK lmdif after a trial evaluation.  Returns info (0 = continue); *accepted
// tells whether x moved (then the next step is a new Jacobian).
__device__ inline int lm_after_trial(LM& s, double fnorm1, bool* accepted) {
    const double ftol = 30 * kEpsmch, xtol = 30 * kEpsmch;
    const double p1 = 0.1, p5 = 0.5, p25 = 0.25, p75 = 0.75, p0001 = 1.0e-4;
    double actred = -1., temp, wa3[2];
    if (p1 * fnorm1 < s.fnorm) actred = 1. - (fnorm1 / s.fnorm) * (fnorm1 / s.fnorm);
    for (int j = 0; j < 2; j++) {
        wa3[j] = 0.;
        int l = s.ipvt[j];
        temp = s.wa1[l];
        for (int i = 0; i <= j; i++) wa3[i] += s.r[j * 2 + i] * temp;
    }
    double temp1 = enorm2(wa3) / s.fnorm;
    double temp2 = (sqrt(s.par) * s.pnorm) / s.fnorm;
    double prered = temp1 * temp1 + temp2 * temp2 / p5;
    double dirder = -(temp1 * temp1 + temp2 * temp2);
    double ratio = 0.;
    if (prered != 0.) ratio = actred / prered;
    if (ratio <= p25) {
        if (actred >= 0.)
            temp = p5;
        else
            temp = p5 * dirder / (dirder + p5 * actred);
        if (p1 * fnorm1 >= s.fnorm || temp < p1) temp = p1;
        s.delta = temp * (s.delta < s.pnorm / p1 ? s.delta : s.pnorm / p1);
        s.par = s.par / temp;
    } else if (s.par == 0. || ratio >= p75) {
        s.delta = s.pnorm / p5;
        s.par = p5 * s.par;
    }
    *accepted = false;
    if (ratio >= p0001) {
        double w2[2];
        for (int j = 0; j < 2; j++) {
            s.x[j] = s.wa2[j];
            w2[j] = s.diag[j] * s.x[j];
        }
        s.xnorm = enorm2(w2);
        s.fnorm = fnorm1;
        s.iter++;
        *accepted = true;
    }
    int info = 0;
    if (fabs(actred) <= ftol && prered <= ftol && p5 * ratio <= 1.) info = 1;
    if (s.delta <= xtol * s.xnorm) info = 2;
    if (fabs(actred) <= ftol && prered <= ftol && p5 * ratio <= 1. && info == 2) info = 3;
    if (info != 0) return info;
    if (s.nfev >= 300) info = 5;  // maxfev = patience(100) * (n + 1)
    if (fabs(actred) <= kEpsmch && prered <= kEpsmch && p5 * ratio <= 1.) info = 6;
    if (s.delta <= kEpsmch * s.xnorm) info = 7;
    if (s.gnorm <= kEpsmch) info = 8;
    if (info != 0) return info;
    if (ratio < p0001) *accepted = false;
    return 0;
}

// lmdif after the QR factorisation: first-iteration scaling, gradient test.
// Returns info (4 if gnorm <= gtol) or 0.
__device__ inline int lm_after_qr(LM& s) {
    const double gtol = 30 * kEpsmch, factor = 100.;
    if (s.iter == 1) {
        for (int j = 0; j < 2; j++) {
            s.diag[j] = s.acnorm[j];
            if (s.acnorm[j] == 0.) s.diag[j] = 1.;
        }
        double wa3[2] = {s.diag[0] * s.x[0], s.diag[1] * s.x[1]};
        s.xnorm = enorm2(wa3);
        s.delta = factor * s.xnorm;
        if (s.delta == 0.) s.delta = factor;
    }
    s.gnorm = 0.;
    if (s.fnorm != 0.) {
        for (int j = 0; j < 2; j++) {
            int l = s.ipvt[j];
            if (s.acnorm[l] == 0.) continue;
            double sum = 0.;
            for (int i = 0; i <= j; i++) sum += s.r[j * 2 + i] * (s.qtf[i] / s.fnorm);
            double temp = fabs(sum / s.acnorm[l]);
            s.gnorm = s.gnorm > temp ? s.gnorm : temp;
        }
    }
    if (s.gnorm <= gtol) return 4;
    for (int j = 0; j < 2; j++) s.diag[j] = s.diag[j] > s.acnorm[j] ? s.diag[j] : s.acnorm[j];
    return 0;
}

// getBilinearInterpPix32f (tools.cpp:129-142) arithmetic on four gathered bytes
__device__ inline float bilinear4(uint8_t b00_, uint8_t b01_, uint8_t b10_, uint8_t b11_, float x, float y) {
    float x0 = (float)(int)floor((double)x), y0 = (float)(int)floor((double)y);
    float b00 = (float)b00_, b10 = (float)b10_, b01 = (float)b01_, b11 = (float)b11_;
    float xm0 = 1.0f - (x - x0), xm1 = (x - x0);
    float ym0 = 1.0f - (y - y0), ym1 = (y - y0);
    return xm0 * (b00 * ym0 + b10 * ym1) + xm1 * (b01 * ym0 + b11 * ym1);
}

__device__ inline void sph2car_det(double phi, double theta, double& n0, double& n1, double& n2) {
    // tools.cpp:772-777 with the deterministic transcendentals
    n0 = fm3d_cos(theta) * fm3d_cos(phi);
    n1 = fm3d_cos(theta) * fm3d_sin(phi);
    n2 = fm3d_sin(theta);
}

}  // namespace

// Pixel loops run in chunks of kCh pixels: all slab loads of a chunk are issued
// first, then the geometry, then all image gathers, then the in-order
// accumulation -- so each wave keeps ~3*kCh 512-byte loads and 4*kCh gathers in
// flight instead of three dependent round trips per pixel.
constexpr int kCh = 8;

__global__ __launch_bounds__(256) void lm_kernel(LMParams p) {
    const int lane = threadIdx.x & (kWave - 1);
    const long wave = (long)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
    if (wave >= p.nWaves) return;  // whole wave exits together
    const int nOffPad = p.nOffPad;  // multiple of kCh; padded offsets are never valid pixels
    const size_t plane = (size_t)nOffPad * kWave;
    double* __restrict__ RX = p.slab + (size_t)wave * 5 * plane;
    double* __restrict__ RY = RX + plane;
    double* __restrict__ F = RY + plane;
    double* __restrict__ J0 = F + plane;
    double* __restrict__ J1 = J0 + plane;
    float* __restrict__ I1 = p.slabI1 + (size_t)wave * plane;
    const double eps = sqrt(p.epsfcn > kEpsmch ? p.epsfcn : kEpsmch);
    const double cm = (double)p.cmax;
    const double Ident[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    const double Zero[3] = {0, 0, 0};

    int st = S_NEED_POINT;
    int pidx = -1;
    double X0 = 0, X1 = 0, X2 = 0, ccx = 0, ccy = 0, nrm0 = 0, nrm1 = 0, nrm2 = 0;
    int m = 0, kfirst = 0, ksecond = 0, L = 0;
    bool i1ok = true;
    double scale = 1.;
    // lanes without a point still execute the (masked-out) gathers of a chunk:
    // keep their image pointers valid
    LevelDesc lv = p.lvl[0];
    LM s{};
    int ekind = E_INITIAL;
    double ex0 = 0, ex1 = 0;
    long long cnt_eval = 0, cnt_pix = 0;

    auto finish_point = [&](int code) {
        p.status[pidx] = code;
        p.normals[3 * pidx + 0] = nrm0;
        p.normals[3 * pidx + 1] = nrm1;
        p.normals[3 * pidx + 2] = nrm2;
        p.mdat[pidx] = m;
        st = S_NEED_POINT;
    };
    auto level_done = [&](int info) {
        p.info[8 * pidx + L] = info;
        p.nfev[8 * pidx + L] = s.nfev;
        sph2car_det(s.x[0], s.x[1], nrm0, nrm1, nrm2);
        L--;
        if (L < 0)
            finish_point(FM3D_ST_OK);
        else
            st = S_LEVEL;
    };
    auto abort_level = [&](int code) {
        p.info[8 * pidx + L] = -code;
        p.nfev[8 * pidx + L] = s.nfev;
        finish_point(code);
    };
    auto request_eval = [&](int kind, double a, double b) {
        ekind = kind;
        ex0 = a;
        ex1 = b;
        st = S_EVAL;
    };

    long long iterations = 0;
    for (;;) {
        if (++iterations > p.maxIter) {  // cannot happen for a correct state machine; never hang the GPU
            if (lane == 0) atomicExch(p.overflow, 1);
            break;
        }
        // ---------------- fetch points ----------------
        if (st == S_NEED_POINT) {
            pidx = atomicAdd(p.queue, 1);
            if (pidx >= p.P) {
                st = S_DONE;
            } else {
                X0 = p.points[3 * pidx + 0];
                X1 = p.points[3 * pidx + 1];
                X2 = p.points[3 * pidx + 2];
                // extractPixelsContour(Vec3d) (:376-397): project with r = t = 0
                project1(p.cam, Ident, Zero, X0, X1, X2, ccx, ccy);
                for (int l = 0; l < 8; l++) {
                    p.info[8 * pidx + l] = 0;
                    p.nfev[8 * pidx + l] = 0;
                }
                st = S_INIT;
            }
        }
        if (__all(st == S_DONE)) break;

        // ---------------- neighbourhood + undistorted rays (once per point) ----------------
        if (__any(st == S_INIT)) {
            const bool act = (st == S_INIT);
            int cnt = 0, kf = -1, ks = -1;
            for (int k0 = 0; k0 < nOffPad; k0 += kCh) {
#pragma unroll
                for (int c = 0; c < kCh; c++) {
                    const int k = k0 + c;
                    const int2 o2 = p.offsets[k];
                    if (act) {
                        // extractPixelsContour(Vec2d) (:341-374): keep 0 <= p < (boundW, boundH)
                        double px = ccx + (double)o2.x, py = ccy + (double)o2.y;
                        const size_t o = (size_t)k * kWave + lane;
                        if (px < 0 || py < 0 || px >= p.boundW || py >= p.boundH) {
                            RX[o] = __builtin_nan("");
                        } else {
                            double ux, uy;
                            undistort1(p.cam, px, py, ux, uy);
                            RX[o] = ux;
                            RY[o] = uy;
                            if (kf < 0)
                                kf = k;
                            else if (ks < 0)
                                ks = k;
                            cnt++;
                        }
                    }
                }
            }
            if (act) {
                m = cnt;
                kfirst = kf;
                ksecond = ks;
                // initial guess: X / norm(X) == X * (1/norm) (Vec3d operator/)
                double nr = sqrt(X0 * X0 + X1 * X1 + X2 * X2);
                double inv = 1. / nr;
                nrm0 = X0 * inv;
                nrm1 = X1 * inv;
                nrm2 = X2 * inv;
                if (m <= 0) {
                    finish_point(FM3D_ST_NO_PIXELS);
                } else {
                    L = p.levels;
                    st = S_LEVEL;
                }
            }
        }

        // ---------------- level start: image-1 intensities, car2sph, lmdif init ----------------
        if (__any(st == S_LEVEL)) {
            const bool act = (st == S_LEVEL);
            if (act) {
                lv = p.lvl[L];
                scale = ldexp(1.0, -L);  // 1.0 / float(2^L)  (optimize_pyramid, :225-241)
                i1ok = true;
            }
            for (int k0 = 0; k0 < nOffPad; k0 += kCh) {
                double rx[kCh];
                const uint8_t* g[kCh];
                float fx[kCh], fy[kCh];
                bool use[kCh];
#pragma unroll
                for (int c = 0; c < kCh; c++) rx[c] = RX[(size_t)(k0 + c) * kWave + lane];
#pragma unroll
                for (int c = 0; c < kCh; c++) {
                    const int2 o2 = p.offsets[k0 + c];
                    double px = ccx + (double)o2.x, py = ccy + (double)o2.y;
                    bool valid = act && (rx[c] == rx[c]);
                    bool good = pixel_good(px, py, scale, lv.w, lv.h);
                    if (valid && !good) i1ok = false;  // updateImage1PixelsIntensity (:580-584)
                    use[c] = valid && good;
                    fx[c] = (float)(scale * px);
                    fy[c] = (float)(scale * py);
                    g[c] = use[c] ? lv.img1 + (long)(int)floor((double)fy[c]) * lv.w + (int)floor((double)fx[c])
                                  : lv.img1;
                }
                uint8_t b00[kCh], b01[kCh], b10[kCh], b11[kCh];
#pragma unroll
                for (int c = 0; c < kCh; c++) {
                    b00[c] = g[c][0];
                    b01[c] = g[c][1];
                    b10[c] = g[c][lv.w];
                    b11[c] = g[c][lv.w + 1];
                }
#pragma unroll
                for (int c = 0; c < kCh; c++) {
                    if (use[c]) I1[(size_t)(k0 + c) * kWave + lane] = bilinear4(b00[c], b01[c], b10[c], b11[c], fx[c], fy[c]);
                }
            }
            if (act) {
                // car2sph (tools.cpp:767-771)
                s.x[1] = fm3d_atan2(nrm2, sqrt(nrm0 * nrm0 + nrm1 * nrm1));
                s.x[0] = fm3d_atan2(nrm1, nrm0);
                s.nfev = 0;
                s.iter = 1;
                s.par = 0.;
                s.delta = 0.;
                s.xnorm = 0.;
                if (m < 2)
                    level_done(0);  // lmdif: m < n -> improper input, info 0, no evaluation
                else
                    request_eval(E_INITIAL, s.x[0], s.x[1]);
            }
        }

        // ---------------- one residual evaluation per lane ----------------
        if (__any(st == S_EVAL)) {
            const bool act = (st == S_EVAL);
            double n0 = 0, n1 = 0, n2 = 0, mm = 0, w = 1.0, hj = 1.0;
            int fail = 0, ph1 = 0;
            bool ph3 = false;
            Enorm en;
            en.init(m > 0 ? m : 1);
            double* __restrict__ out = F;
            const bool isjac = (ekind == E_JAC0 || ekind == E_JAC1);
            if (act) {
                s.nfev++;
                cnt_eval++;
                cnt_pix += m;
                sph2car_det(ex0, ex1, n0, n1, n2);  // par = (phi, theta)
                if (n2 != n2 || n1 != n1 || n0 != n0) fail = FM3D_ST_NAN_NORMAL;
                mm = n0 * X0 + n1 * X1 + n2 * X2;
                double w_theta = 1.0, w_phi = 1.0;
                if (fabs(ex1) - M_PI / 2 > 0 || fabs(ex0) - M_PI > 0) {
                    w_theta = fm3d_exp(fabs(ex1) - M_PI / 2) + 1;
                    w_phi = fm3d_exp(fabs(ex0) - M_PI + 1) + 1;
                }
                w = w_phi * w_theta;
                if (ekind == E_JAC0) {
                    hj = s.h[0];
                    out = J0;
                } else if (ekind == E_JAC1) {
                    hj = s.h[1];
                    out = J1;
                }
            }
            const bool run = act && fail == 0;
            if (__any(run)) {
                for (int k0 = 0; k0 < nOffPad; k0 += kCh) {
                    double rx[kCh], ry[kCh], fk[kCh];
                    float i1[kCh];
#pragma unroll
                    for (int c = 0; c < kCh; c++) {
                        const size_t o = (size_t)(k0 + c) * kWave + lane;
                        rx[c] = RX[o];
                        ry[c] = RY[o];
                        i1[c] = I1[o];
                        fk[c] = F[o];
                    }
                    // geometry: projectPointToPlane (:421-470), isInBoundingBox (:646-655),
                    // projectPointsToImage2 (:591-644)
                    unsigned char code1[kCh];  // 0 ok, 1 invalid pixel, 2 NaN plane, 3 bbox
                    bool good[kCh];
                    float fx[kCh], fy[kCh];
                    const uint8_t* g[kCh];
#pragma unroll
                    for (int c = 0; c < kCh; c++) {
                        const double ux = rx[c], uy = ry[c];
                        double nn = n0 * ux + n1 * uy + n2 * 1.;
                        double kk = mm / nn;
                        double P0 = kk * ux, P1 = kk * uy, P2 = kk * 1.;
                        unsigned char cd = 0;
                        if (ux != ux)
                            cd = 1;
                        else if (P0 != P0 || P1 != P1 || P2 != P2)
                            cd = 2;
                        else if (!((P0 > -cm && P0 < cm) && (P1 > -cm && P1 < cm) && (P2 > 0. && P2 < cm)))
                            cd = 3;
                        code1[c] = cd;
                        double u, v;
                        project1(p.cam, p.R2, p.t2, P0, P1, P2, u, v);
                        bool gd = (cd == 0) && pixel_good(u, v, scale, lv.w, lv.h);
                        good[c] = gd;
                        fx[c] = (float)(scale * u);
                        fy[c] = (float)(scale * v);
                        g[c] = gd ? lv.img2 + (long)(int)floor((double)fy[c]) * lv.w + (int)floor((double)fx[c])
                                  : lv.img2;
                    }
                    uint8_t b00[kCh], b01[kCh], b10[kCh], b11[kCh];
#pragma unroll
                    for (int c = 0; c < kCh; c++) {
                        b00[c] = g[c][0];
                        b01[c] = g[c][1];
                        b10[c] = g[c][lv.w];
                        b11[c] = g[c][lv.w + 1];
                    }
                    // residuals in pixel order (evaluateNormal :145-148 / fdjac2)
#pragma unroll
                    for (int c = 0; c < kCh; c++) {
                        if (run && ph1 == 0 && code1[c] != 1) {
                            if (code1[c] == 2) {
                                ph1 = FM3D_ST_NAN_PLANE;
                            } else if (code1[c] == 3) {
                                ph1 = FM3D_ST_ABORT_BBOX;
                            } else if (i1ok && !ph3) {
                                if (!good[c]) {
                                    ph3 = true;
                                } else {
                                    float I2 = bilinear4(b00[c], b01[c], b10[c], b11[c], fx[c], fy[c]);
                                    float dI = i1[c] - I2;
                                    double r = w * (double)dI;
                                    double val = r;
                                    if (isjac) val = (r - fk[c]) / hj;
                                    out[(size_t)(k0 + c) * kWave + lane] = val;
                                    en.add(val);
                                }
                            }
                        }
                    }
                }
            }
            if (act) {
                int code = fail ? fail : ph1 ? ph1 : (!i1ok ? FM3D_ST_ABORT_PIX1 : (ph3 ? FM3D_ST_ABORT_PIX2 : 0));
                if (code) {
                    abort_level(code);
                } else {
                    double nrm = en.finish();
                    if (ekind == E_INITIAL) {
                        s.fnorm = nrm;
                        s.h[0] = eps * fabs(s.x[0]);
                        if (s.h[0] == 0.) s.h[0] = eps;
                        request_eval(E_JAC0, s.x[0] + s.h[0], s.x[1]);
                    } else if (ekind == E_JAC0) {
                        s.acnorm[0] = nrm;
                        s.h[1] = eps * fabs(s.x[1]);
                        if (s.h[1] == 0.) s.h[1] = eps;
                        request_eval(E_JAC1, s.x[0], s.x[1] + s.h[1]);
                    } else if (ekind == E_JAC1) {
                        s.acnorm[1] = nrm;
                        st = S_QR;
                    } else {
                        bool accepted;
                        int info = lm_after_trial(s, nrm, &accepted);
                        if (info) {
                            level_done(info);
                        } else if (accepted) {
                            s.h[0] = eps * fabs(s.x[0]);
                            if (s.h[0] == 0.) s.h[0] = eps;
                            request_eval(E_JAC0, s.x[0] + s.h[0], s.x[1]);
                        } else {
                            lm_inner_step(s);
                            request_eval(E_TRIAL, s.wa2[0], s.wa2[1]);
                        }
                    }
                }
            }
        }

        // ---------------- Householder QR (qrfac, pivoting) + Q^T fvec, n = 2 ----------------
        if (__any(st == S_QR)) {
            const bool act = (st == S_QR);
            int pc = 0;
            double ajn0 = 0, ajn0s = 1, apf = 0, aqf = 0, ff = 0, aps = 0, fs = 0, vfirst = 0;
            const double* Jp = J0;
            const double* Jq = J1;
            bool t0 = false;
            if (act) {
                pc = (s.acnorm[1] > s.acnorm[0]) ? 1 : 0;
                s.ipvt[0] = pc;
                s.ipvt[1] = 1 - pc;
                Jp = pc ? J1 : J0;
                Jq = pc ? J0 : J1;
                ajn0 = s.acnorm[pc];  // enorm of the pivot column == its acnorm (same elements, same order)
                const size_t of = (size_t)kfirst * kWave + lane, os = (size_t)ksecond * kWave + lane;
                apf = Jp[of];
                aqf = Jq[of];
                ff = F[of];
                aps = Jp[os];
                fs = F[os];
                t0 = (ajn0 != 0.);
                ajn0s = (t0 && apf < 0.) ? -ajn0 : ajn0;
                if (!t0) ajn0s = 1.;  // unused
                vfirst = t0 ? (apf / ajn0s) + 1. : apf;
            }
            // P1: sum_i v_i a_q[i] (qrfac) and sum_i v_i f[i] (lmdif qtf, j = 0)
            double dot = 0., s0 = 0.;
            const bool run1 = act && t0;
            if (__any(run1)) {
                for (int k0 = 0; k0 < nOffPad; k0 += kCh) {
                    double rx[kCh], ap[kCh], aq[kCh], fk[kCh];
#pragma unroll
                    for (int c = 0; c < kCh; c++) {
                        const size_t o = (size_t)(k0 + c) * kWave + lane;
                        rx[c] = RX[o];
                        ap[c] = Jp[o];
                        aq[c] = Jq[o];
                        fk[c] = F[o];
                    }
#pragma unroll
                    for (int c = 0; c < kCh; c++) {
                        if (run1 && rx[c] == rx[c]) {
                            double v = ap[c] / ajn0s;
                            if (k0 + c == kfirst) v = v + 1.;
                            dot += v * aq[c];
                            s0 += v * fk[c];
                        }
                    }
                }
            }
            double tq = 0., r01 = aqf, tq0 = 0., qtf0 = ff;
            bool q0 = false;
            if (act) {
                if (t0) {
                    tq = dot / vfirst;
                    r01 = aqf - tq * vfirst;
                }
                q0 = (vfirst != 0.);
                if (q0) {
                    tq0 = -s0 / vfirst;
                    qtf0 = ff + vfirst * tq0;
                }
            }
            // P2: ajnorm of the transformed second column, elements 1..m-1
            Enorm e2;
            e2.init(m > 1 ? m - 1 : 1);
            double aqs1 = 0.;
            if (__any(act)) {
                for (int k0 = 0; k0 < nOffPad; k0 += kCh) {
                    double rx[kCh], ap[kCh], aq[kCh];
#pragma unroll
                    for (int c = 0; c < kCh; c++) {
                        const size_t o = (size_t)(k0 + c) * kWave + lane;
                        rx[c] = RX[o];
                        ap[c] = Jp[o];
                        aq[c] = Jq[o];
                    }
#pragma unroll
                    for (int c = 0; c < kCh; c++) {
                        const int k = k0 + c;
                        if (act && k > kfirst && rx[c] == rx[c]) {
                            double a = aq[c];
                            if (t0) {
                                double v = ap[c] / ajn0s;
                                a = a - tq * v;
                            }
                            e2.add(a);
                            if (k == ksecond) aqs1 = a;
                        }
                    }
                }
            }
            double ajn1 = 0, ajn1s = 1, usecond = 0;
            bool t1 = false;
            if (act) {
                ajn1 = e2.finish();
                t1 = (ajn1 != 0.);
                ajn1s = (t1 && aqs1 < 0.) ? -ajn1 : ajn1;
                if (!t1) ajn1s = 1.;  // unused
                usecond = t1 ? (aqs1 / ajn1s) + 1. : aqs1;
            }
            // P3: lmdif qtf, j = 1: sum_{i>=1} u_i wa4_i
            double s1 = 0.;
            const bool run3 = act && usecond != 0.;
            if (__any(run3)) {
                for (int k0 = 0; k0 < nOffPad; k0 += kCh) {
                    double rx[kCh], ap[kCh], aq[kCh], fk[kCh];
#pragma unroll
                    for (int c = 0; c < kCh; c++) {
                        const size_t o = (size_t)(k0 + c) * kWave + lane;
                        rx[c] = RX[o];
                        ap[c] = Jp[o];
                        aq[c] = Jq[o];
                        fk[c] = F[o];
                    }
#pragma unroll
                    for (int c = 0; c < kCh; c++) {
                        const int k = k0 + c;
                        if (run3 && k > kfirst && rx[c] == rx[c]) {
                            double v = t0 ? ap[c] / ajn0s : 0.;
                            double a = aq[c];
                            if (t0) a = a - tq * v;
                            double u = t1 ? a / ajn1s : a;
                            if (t1 && k == ksecond) u = u + 1.;
                            double wa = fk[c];
                            if (q0) wa = wa + v * tq0;
                            s1 += u * wa;
                        }
                    }
                }
            }
            if (act) {
                double wa4s = q0 ? fs + (aps / ajn0s) * tq0 : fs;
                double qtf1 = wa4s;
                if (usecond != 0.) {
                    double tq1 = -s1 / usecond;
                    qtf1 = wa4s + usecond * tq1;
                }
                s.r[0] = t0 ? -ajn0s : 0.;
                s.r[1] = 0.;
                s.r[2] = r01;
                s.r[3] = t1 ? -ajn1s : 0.;
                s.qtf[0] = qtf0;
                s.qtf[1] = qtf1;
                int info = lm_after_qr(s);
                if (info) {
                    level_done(info);
                } else {
                    lm_inner_step(s);
                    request_eval(E_TRIAL, s.wa2[0], s.wa2[1]);
                }
            }
        }
    }

    // statistics: one atomic per wave
    for (int off = 32; off > 0; off >>= 1) {
        cnt_eval += __shfl_down(cnt_eval, off);
        cnt_pix += __shfl_down(cnt_pix, off);
    }
    if (lane == 0) {
        atomicAdd(p.statEval, (unsigned long long)cnt_eval);
        atomicAdd(p.statPix, (unsigned long long)cnt_pix);
    }
}

}  // namespace fm3d
