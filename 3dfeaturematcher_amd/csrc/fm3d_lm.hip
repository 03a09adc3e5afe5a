// fm3d_lm.hip -- NormalOptimizer::computeOptimizedNormals on gfx950.
//
// Reference: Triangulator/normaloptimizer.cpp:223-452 (optimize_pyramid, optimize,
// computeOptimizedNormals), the residual evaluateNormal (:65-149) and the
// SingleCameraTriangulator geometry it calls (singlecameratriangulator.cpp:341-665),
// minimised by lmfit's lmmin (MINPACK lmdif with lmfit's lm_control_double).
//
// Design.  The LM trajectory of a point is decided at the
// rounding-noise level (ftol = xtol = 30*DBL_EPSILON): any reordering of the
// m_dat-long sums (fnorm, column norms, Householder dot products) changes which
// steps are accepted and moves the final normal by up to 1e-2 on ~15 % of
// points (measured with the oracle).  So every sum is replayed in
// MINPACK's pixel order, bit for bit -- but only the ADDS are sequential:
//
//   * a workgroup (256 threads) serves kG = 4 points ("slots");
//   * each pass over the neighbourhood runs in chunks of kC pixels: all 256
//     threads compute the per-(pixel, slot) terms in parallel -- the residual
//     (plane intersection, distorted projection, bilinear samples), Jacobian
//     columns, Householder products -- and park them in LDS;
//   * one "chain" lane per slot (lanes 0..3 of wave 0) then adds the chunk's
//     terms in pixel order (MINPACK enorm / dot-product order) and runs the
//     slot's lmdif bookkeeping between passes;
//   * per-pixel state (undistorted rays, I1, fvec, Jacobian) lives in a
//     per-workgroup slab laid out [pixel][slot] (coalesced 2 KB per load
//     instruction); slots fetch new points from a global queue.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "fm3d_device.h"
#include "fm3d_kernels.h"

namespace fm3d {

namespace {


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

constexpr int kG = kLMSlots;                  // points (slots) per workgroup
constexpr int kThreads = kLMThreads;
constexpr int kC = kLMChunk;                  // pixels per chunk
constexpr int kPer = kC * kG / kThreads;      // entries per thread per chunk (8)
constexpr int kSub = 4;                       // entries in flight per thread (register budget)

enum PassKind { P_IDLE = 0, P_INIT, P_LEVEL, P_EVAL, P_QR1, P_QR2, P_QR3, P_DONE };

// parameters of a slot's current pass (LDS; written by the slot's chain lane)
struct SlotP {
    int pass, ekind, kfirst, ksecond, t0, t1, q0, pivot, lw, lh;
    double n0, n1, n2, mm, w, hj, scale, ccx, ccy, ajn0s, tq, ajn1s, tq0, agiant;
    const uint8_t* img1;
    const uint8_t* img2;
};

// persistent state of a slot (LDS; only its chain lane touches it)
struct SlotS {
    LM s;
    double X0, X1, X2, ccx, ccy, nrm0, nrm1, nrm2;
    double apf, aqf, ff, aps, fs, vfirst, r01, tq0, qtf0, wa4s, usecond, ajn0s, tq, ajn1s;
    int pidx, m, kfirst, ksecond, L, i1ok, ekind, t0, q0, t1;
};

// per-pass results the chain lane hands to the bookkeeping
struct PassOut {
    double nrm;          // EVAL / QR2: enorm of the pass's values
    double sumA, sumB;   // QR1 / QR3 dot products
    double aqs1;         // QR2: transformed a_q at the second kept pixel
    int cnt, kmin, fail, ph3, i1fail;
};

// lmdif bookkeeping of one slot (chain lane only).  Kept out of line so that the
// register budget of the data-parallel part of the kernel is not set by it.
struct Ctl {
    const LMParams* p;
    double* F;
    double* J0;
    double* J1;
    double eps;
    long long cnt_eval, cnt_pix;

    __device__ void fetch(SlotS& S, SlotP& P) {
        int pidx = atomicAdd(p->queue, 1);
        if (pidx >= p->P) {
            P.pass = P_DONE;
            return;
        }
        S.pidx = pidx;
        S.X0 = p->points[3 * pidx + 0];
        S.X1 = p->points[3 * pidx + 1];
        S.X2 = p->points[3 * pidx + 2];
        const double Ident[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        const double Zero[3] = {0, 0, 0};
        double cx, cy;
        project1(p->cam, Ident, Zero, S.X0, S.X1, S.X2, cx, cy);  // extractPixelsContour(Vec3d) :376-397
        S.ccx = cx;
        S.ccy = cy;
        for (int l = 0; l < 8; l++) {
            p->info[8 * pidx + l] = 0;
            p->nfev[8 * pidx + l] = 0;
        }
        P.pass = P_INIT;
        P.ccx = cx;
        P.ccy = cy;
    }
    __device__ void start_level(SlotS& S, SlotP& P) {
        const LevelDesc lv = p->lvl[S.L];
        P.pass = P_LEVEL;
        P.scale = ldexp(1.0, -S.L);  // 1.0 / float(2^L)  (optimize_pyramid, :225-241)
        P.img1 = lv.img1;
        P.img2 = lv.img2;
        P.lw = lv.w;
        P.lh = lv.h;
    }
    __device__ void finish_point(SlotS& S, SlotP& P, int code) {
        p->status[S.pidx] = code;
        p->normals[3 * S.pidx + 0] = S.nrm0;
        p->normals[3 * S.pidx + 1] = S.nrm1;
        p->normals[3 * S.pidx + 2] = S.nrm2;
        p->mdat[S.pidx] = S.m;
        fetch(S, P);
    }
    __device__ void level_done(SlotS& S, SlotP& P, int info) {
        p->info[8 * S.pidx + S.L] = info;
        p->nfev[8 * S.pidx + S.L] = S.s.nfev;
        sph2car_det(S.s.x[0], S.s.x[1], S.nrm0, S.nrm1, S.nrm2);
        S.L--;
        if (S.L < 0)
            finish_point(S, P, FM3D_ST_OK);
        else
            start_level(S, P);
    }
    __device__ void abort_level(SlotS& S, SlotP& P, int code) {
        p->info[8 * S.pidx + S.L] = -code;
        p->nfev[8 * S.pidx + S.L] = S.s.nfev;
        finish_point(S, P, code);
    }
    // evaluateNormal (normaloptimizer.cpp:65-149), per-call part
    __device__ void eval_pass(SlotS& S, SlotP& P, int kind, double a, double b) {
        S.s.nfev++;
        cnt_eval++;
        cnt_pix += S.m;
        double n0, n1, n2;
        sph2car_det(a, b, n0, n1, n2);  // par = (phi, theta)
        if (n2 != n2 || n1 != n1 || n0 != n0) {
            abort_level(S, P, FM3D_ST_NAN_NORMAL);
            return;
        }
        double w_theta = 1.0, w_phi = 1.0;
        if (fabs(b) - M_PI / 2 > 0 || fabs(a) - M_PI > 0) {
            w_theta = fm3d_exp(fabs(b) - M_PI / 2) + 1;
            w_phi = fm3d_exp(fabs(a) - M_PI + 1) + 1;
        }
        S.ekind = kind;
        P.pass = P_EVAL;
        P.ekind = kind;
        P.n0 = n0;
        P.n1 = n1;
        P.n2 = n2;
        P.mm = n0 * S.X0 + n1 * S.X1 + n2 * S.X2;
        P.w = w_phi * w_theta;
        P.hj = kind == E_JAC0 ? S.s.h[0] : kind == E_JAC1 ? S.s.h[1] : 1.0;
        P.agiant = 1.304e19 / (double)S.m;
    }
    __device__ void jac0(SlotS& S, SlotP& P) {
        LM& s = S.s;
        s.h[0] = eps * fabs(s.x[0]);
        if (s.h[0] == 0.) s.h[0] = eps;
        eval_pass(S, P, E_JAC0, s.x[0] + s.h[0], s.x[1]);
    }
    __device__ void finalize_qr(SlotS& S, SlotP& P, double qtf1) {
        S.s.r[0] = S.t0 ? -S.ajn0s : 0.;
        S.s.r[1] = 0.;
        S.s.r[2] = S.r01;
        S.s.r[3] = S.t1 ? -S.ajn1s : 0.;
        S.s.qtf[0] = S.qtf0;
        S.s.qtf[1] = qtf1;
        int info = lm_after_qr(S.s);
        if (info) {
            level_done(S, P, info);
        } else {
            lm_inner_step(S.s);
            eval_pass(S, P, E_TRIAL, S.s.wa2[0], S.s.wa2[1]);
        }
    }
    // qrfac with column pivoting for n = 2, on the Jacobian columns left in the slab
    __device__ void start_qr(SlotS& S, SlotP& P, int slot) {
        LM& s = S.s;
        const int pc = (s.acnorm[1] > s.acnorm[0]) ? 1 : 0;  // pivot column = larger norm
        s.ipvt[0] = pc;
        s.ipvt[1] = 1 - pc;
        const double* Jpp = pc ? J1 : J0;
        const double* Jqq = pc ? J0 : J1;
        const size_t of = (size_t)S.kfirst * kG + slot, os = (size_t)S.ksecond * kG + slot;
        S.apf = Jpp[of];
        S.aqf = Jqq[of];
        S.ff = F[of];
        S.aps = Jpp[os];
        S.fs = F[os];
        const double ajn0 = s.acnorm[pc];  // == enorm of the pivot column (same elements, same order)
        S.t0 = ajn0 != 0.;
        S.ajn0s = (S.t0 && S.apf < 0.) ? -ajn0 : ajn0;
        if (!S.t0) S.ajn0s = 1.;  // unused
        S.vfirst = S.t0 ? (S.apf / S.ajn0s) + 1. : S.apf;
        P.pivot = pc;
        P.kfirst = S.kfirst;
        P.ksecond = S.ksecond;
        P.t0 = S.t0;
        P.ajn0s = S.ajn0s;
        if (S.t0) {
            P.pass = P_QR1;
        } else {
            S.tq = 0.;
            S.r01 = S.aqf;
            S.q0 = 0;  // vfirst == apf == 0
            S.tq0 = 0.;
            S.qtf0 = S.ff;
            qr2(S, P);
        }
    }
    __device__ void qr2(SlotS& S, SlotP& P) {
        P.pass = P_QR2;
        P.tq = S.tq;
        P.agiant = 1.304e19 / (double)(S.m - 1);
    }

    __device__ __noinline__ void after_pass(SlotS& S, SlotP& P, const PassOut& o, int slot) {
        const int ps = P.pass;
        if (ps == P_INIT) {
            S.m = o.cnt;
            S.kfirst = o.kmin;
            // second kept pixel: next offset after kfirst inside the bounds
            int ks = -1;
            for (int k = S.kfirst + 1; S.m > 1 && k < p->nOff; k++) {
                const int2 o2 = p->offsets[k];
                const double px = S.ccx + (double)o2.x, py = S.ccy + (double)o2.y;
                if (!(px < 0 || py < 0 || px >= p->boundW || py >= p->boundH)) {
                    ks = k;
                    break;
                }
            }
            S.ksecond = ks;
            // initial guess: X / norm(X) == X * (1/norm) (Vec3d operator/, :342-343)
            double nr = sqrt(S.X0 * S.X0 + S.X1 * S.X1 + S.X2 * S.X2);
            double inv = 1. / nr;
            S.nrm0 = S.X0 * inv;
            S.nrm1 = S.X1 * inv;
            S.nrm2 = S.X2 * inv;
            if (S.m <= 0) {
                finish_point(S, P, FM3D_ST_NO_PIXELS);
            } else {
                S.L = p->levels;
                start_level(S, P);
            }
        } else if (ps == P_LEVEL) {
            S.i1ok = o.i1fail ? 0 : 1;
            // car2sph (tools.cpp:767-771) -> lmdif from the current normal
            S.s.x[1] = fm3d_atan2(S.nrm2, sqrt(S.nrm0 * S.nrm0 + S.nrm1 * S.nrm1));
            S.s.x[0] = fm3d_atan2(S.nrm1, S.nrm0);
            S.s.nfev = 0;
            S.s.iter = 1;
            S.s.par = 0.;
            S.s.delta = 0.;
            S.s.xnorm = 0.;
            if (S.m < 2)
                level_done(S, P, 0);  // lmdif: m < n -> improper input, info 0, no evaluation
            else
                eval_pass(S, P, E_INITIAL, S.s.x[0], S.s.x[1]);
        } else if (ps == P_EVAL) {
            int code = 0;
            if (o.fail != 0x7fffffff)  // first failing pixel in index order decides (:455-470, :557-560)
                code = (o.fail & 3) == 2 ? FM3D_ST_NAN_PLANE : FM3D_ST_ABORT_BBOX;
            else if (!S.i1ok)
                code = FM3D_ST_ABORT_PIX1;
            else if (o.ph3)
                code = FM3D_ST_ABORT_PIX2;
            if (code) {
                abort_level(S, P, code);
                return;
            }
            LM& s = S.s;
            if (S.ekind == E_INITIAL) {
                s.fnorm = o.nrm;
                jac0(S, P);
            } else if (S.ekind == E_JAC0) {
                s.acnorm[0] = o.nrm;
                s.h[1] = eps * fabs(s.x[1]);
                if (s.h[1] == 0.) s.h[1] = eps;
                eval_pass(S, P, E_JAC1, s.x[0], s.x[1] + s.h[1]);
            } else if (S.ekind == E_JAC1) {
                s.acnorm[1] = o.nrm;
                start_qr(S, P, slot);
            } else {
                bool accepted;
                int info = lm_after_trial(s, o.nrm, &accepted);
                if (info) {
                    level_done(S, P, info);
                } else if (accepted) {
                    jac0(S, P);
                } else {
                    lm_inner_step(s);
                    eval_pass(S, P, E_TRIAL, s.wa2[0], s.wa2[1]);
                }
            }
        } else if (ps == P_QR1) {
            // qrfac j = 0: temp = sum v a_q / v_first; lmdif qtf j = 0: temp = -sum v f / v_first
            S.tq = o.sumA / S.vfirst;
            S.r01 = S.aqf - S.tq * S.vfirst;
            S.q0 = S.vfirst != 0.;
            S.tq0 = 0.;
            S.qtf0 = S.ff;
            if (S.q0) {
                S.tq0 = -o.sumB / S.vfirst;
                S.qtf0 = S.ff + S.vfirst * S.tq0;
            }
            qr2(S, P);
        } else if (ps == P_QR2) {
            const double ajn1 = o.nrm;
            S.t1 = ajn1 != 0.;
            S.ajn1s = (S.t1 && o.aqs1 < 0.) ? -ajn1 : ajn1;
            if (!S.t1) S.ajn1s = 1.;  // unused
            S.usecond = S.t1 ? (o.aqs1 / S.ajn1s) + 1. : o.aqs1;
            S.wa4s = S.q0 ? S.fs + (S.aps / S.ajn0s) * S.tq0 : S.fs;
            if (S.usecond != 0.) {
                P.pass = P_QR3;
                P.t1 = S.t1;
                P.ajn1s = S.ajn1s;
                P.q0 = S.q0;
                P.tq0 = S.tq0;
            } else {
                finalize_qr(S, P, S.wa4s);
            }
        } else if (ps == P_QR3) {
            const double tq1 = -o.sumA / S.usecond;
            finalize_qr(S, P, S.wa4s + S.usecond * tq1);
        }
    }
};

__device__ __noinline__ void ctl_fetch(Ctl& c, SlotS& S, SlotP& P) { c.fetch(S, P); }

// enorm terms: x^2 for MINPACK's "intermediate" range (the branch almost every value
// takes), 0 otherwise; values outside that range raise the chunk's slow flag
__device__ inline double enorm_term(double x, double agiant, int* slow) {
    const double xa = fabs(x);
    if (xa > 3.834e-20 && xa < agiant) return xa * xa;
    if (xa != 0.) *slow = 1;
    return 0.;
}

__global__ __launch_bounds__(kThreads) void lm_kernel(LMParams p) {
    __shared__ double term[2][kG][kC];
    __shared__ SlotP sp[kG];
    __shared__ SlotS ss[kG];
    __shared__ int shCnt[kG], shKmin[kG], shFail[kG], shPh3[kG], shI1fail[kG], shSlow[kG];
    __shared__ double shAqs1[kG];
    __shared__ int shStop;

    const int tid = threadIdx.x;
    const int slot = tid & (kG - 1);
    const int prow = tid >> 2;  // pixel row of this thread inside a chunk (+64 i)
    const size_t ents = (size_t)p.nOffPad * kG;
    double* __restrict__ RX = p.slab + (size_t)blockIdx.x * 5 * ents;
    double* __restrict__ RY = RX + ents;
    double* __restrict__ F = RY + ents;
    double* __restrict__ J0 = F + ents;
    double* __restrict__ J1 = J0 + ents;
    float* __restrict__ I1 = p.slabI1 + (size_t)blockIdx.x * ents;
    const double cm = (double)p.cmax;
    const bool chain = tid < kG;  // chain / control lane of slot `tid`

    Ctl ctl;
    ctl.p = &p;
    ctl.F = F;
    ctl.J0 = J0;
    ctl.J1 = J1;
    ctl.eps = sqrt(p.epsfcn > kEpsmch ? p.epsfcn : kEpsmch);
    ctl.cnt_eval = 0;
    ctl.cnt_pix = 0;
    if (chain) ctl_fetch(ctl, ss[tid], sp[tid]);

    // chain accumulators (chain lanes)
    Enorm en;
    en.init(1);
    double sumA = 0., sumB = 0.;

    long long iterations = 0;
    const unsigned long long tStart = wall_clock64();
    if (tid == 0) shStop = 0;
    for (;;) {
        if (tid == 0 && (++iterations > p.maxIter || (long long)(wall_clock64() - tStart) > p.maxTicks)) {
            // cannot happen for a correct state machine; never hang the GPU
            shStop = 1;
            atomicExch(p.overflow, 1);
        }
        if (chain) {
            shCnt[tid] = 0;
            shKmin[tid] = 0x7fffffff;
            shFail[tid] = 0x7fffffff;
            shPh3[tid] = 0;
            shI1fail[tid] = 0;
            shSlow[tid] = 0;
            en.init(1);
            en.agiant = sp[tid].agiant;
            sumA = 0.;
            sumB = 0.;
        }
        __syncthreads();
        bool allDone = true;
        for (int q = 0; q < kG; q++) allDone = allDone && sp[q].pass == P_DONE;
        if (shStop || allDone) break;
        // this thread's slot parameters
        const SlotP& P = sp[slot];  // read from LDS on use (keeps VGPRs for the pixel data)
        const bool isjac = (P.ekind == E_JAC0 || P.ekind == E_JAC1);
        double* __restrict__ outArr = P.ekind == E_JAC0 ? J0 : P.ekind == E_JAC1 ? J1 : F;
        const double* __restrict__ Jp = P.pivot ? J1 : J0;
        const double* __restrict__ Jq = P.pivot ? J0 : J1;
        const bool i1ok = ss[slot].i1ok != 0;

        for (int k0 = 0; k0 < p.nOffPad; k0 += kC) {
            // ---------------- parallel terms of this chunk ----------------
            if (P.pass == P_EVAL) {
#pragma unroll 1
                for (int i0 = 0; i0 < kPer; i0 += kSub) {
                    double rx[kSub], ry[kSub], fk[kSub];
                    float i1v[kSub];
                    bool valid[kSub];
#pragma unroll
                    for (int i = 0; i < kSub; i++) {
                        const int k = k0 + prow + 64 * (i0 + i);
                        const size_t e = (size_t)k * kG + slot;
                        const int2 o2 = p.offsets[k];
                        const double px = P.ccx + (double)o2.x, py = P.ccy + (double)o2.y;
                        valid[i] = !(px < 0 || py < 0 || px >= p.boundW || py >= p.boundH);
                        rx[i] = RX[e];
                        ry[i] = RY[e];
                        i1v[i] = I1[e];
                        fk[i] = isjac ? F[e] : 0.;
                    }
                    unsigned char code1[kSub];
                    float fx[kSub], fy[kSub];
                    const uint8_t* g[kSub];
#pragma unroll
                    for (int i = 0; i < kSub; i++) {
                        // projectPointToPlane (:421-470) + isInBoundingBox (:646-655)
                        const double ux = rx[i], uy = ry[i];
                        double nn = P.n0 * ux + P.n1 * uy + P.n2 * 1.;
                        double kk = P.mm / nn;
                        double P0 = kk * ux, P1 = kk * uy, P2 = kk * 1.;
                        unsigned char cd = 0;
                        if (!valid[i])
                            cd = 1;
                        else if (P0 != P0 || P1 != P1 || P2 != P2)
                            cd = 2;
                        else if (!((P0 > -cm && P0 < cm) && (P1 > -cm && P1 < cm) && (P2 > 0. && P2 < cm)))
                            cd = 3;
                        // projectPointsToImage2 (:591-644)
                        double u, v;
                        project1(p.cam, p.R2, p.t2, P0, P1, P2, u, v);
                        if (cd == 0 && !pixel_good(u, v, P.scale, P.lw, P.lh)) cd = 4;
                        code1[i] = cd;
                        fx[i] = (float)(P.scale * u);
                        fy[i] = (float)(P.scale * v);
                        g[i] = cd == 0 ? P.img2 + (long)(int)floor((double)fy[i]) * P.lw + (int)floor((double)fx[i])
                                       : P.img2;
                    }
                    uint8_t b00[kSub], b01[kSub], b10[kSub], b11[kSub];
#pragma unroll
                    for (int i = 0; i < kSub; i++) {
                        b00[i] = g[i][0];
                        b01[i] = g[i][1];
                        b10[i] = g[i][P.lw];
                        b11[i] = g[i][P.lw + 1];
                    }
#pragma unroll
                    for (int i = 0; i < kSub; i++) {
                        const int pl = prow + 64 * (i0 + i);
                        const int k = k0 + pl;
                        double t1 = 0., t2 = __builtin_nan("");
                        if (code1[i] == 2 || code1[i] == 3) {
                            atomicMin(&shFail[slot], k * 4 + code1[i]);  // first failing pixel decides
                        } else if (code1[i] == 4) {
                            shPh3[slot] = 1;
                        } else if (code1[i] == 0 && i1ok) {
                            float I2 = bilinear4(b00[i], b01[i], b10[i], b11[i], fx[i], fy[i]);
                            float dI = i1v[i] - I2;
                            double r = P.w * (double)dI;                    // evaluateNormal :145-148
                            double val = isjac ? (r - fk[i]) / P.hj : r;  // fdjac2 forward difference
                            outArr[(size_t)k * kG + slot] = val;
                            t1 = enorm_term(val, P.agiant, &shSlow[slot]);
                            t2 = val;
                        }
                        term[0][slot][pl] = t1;
                        term[1][slot][pl] = t2;
                    }
                }
            } else if (P.pass == P_QR1 || P.pass == P_QR2 || P.pass == P_QR3) {
#pragma unroll 1
                for (int i0 = 0; i0 < kPer; i0 += kSub) {
                    double ap[kSub], aq[kSub], fv[kSub];
                    bool valid[kSub];
#pragma unroll
                    for (int i = 0; i < kSub; i++) {
                        const int k = k0 + prow + 64 * (i0 + i);
                        const size_t e = (size_t)k * kG + slot;
                        const int2 o2 = p.offsets[k];
                        const double px = P.ccx + (double)o2.x, py = P.ccy + (double)o2.y;
                        valid[i] = !(px < 0 || py < 0 || px >= p.boundW || py >= p.boundH);
                        ap[i] = Jp[e];
                        aq[i] = Jq[e];
                        fv[i] = P.pass == P_QR2 ? 0. : F[e];
                    }
#pragma unroll
                    for (int i = 0; i < kSub; i++) {
                        const int pl = prow + 64 * (i0 + i);
                        const int k = k0 + pl;
                        double t1 = __builtin_nan(""), t2 = __builtin_nan("");
                        if (P.pass == P_QR1) {
                            // qrfac column j = 0: v = a_p / ajnorm (+1 on the diagonal); sum v*a_q, sum v*f
                            if (valid[i]) {
                                double v = ap[i] / P.ajn0s;
                                if (k == P.kfirst) v = v + 1.;
                                t1 = v * aq[i];
                                t2 = v * fv[i];
                            }
                        } else if (P.pass == P_QR2) {
                            // a_q' = a_q - temp * v below the diagonal -> ajnorm of column 1
                            t1 = 0.;
                            if (valid[i] && k > P.kfirst) {
                                double a = aq[i];
                                if (P.t0) {
                                    double v = ap[i] / P.ajn0s;
                                    a = a - P.tq * v;
                                }
                                if (k == P.ksecond) shAqs1[slot] = a;
                                t1 = enorm_term(a, P.agiant, &shSlow[slot]);
                                t2 = a;
                            }
                        } else {
                            // lmdif qtf, j = 1: u_i * wa4_i
                            if (valid[i] && k > P.kfirst) {
                                double v = P.t0 ? ap[i] / P.ajn0s : 0.;
                                double a = aq[i];
                                if (P.t0) a = a - P.tq * v;
                                double u = P.t1 ? a / P.ajn1s : a;
                                if (P.t1 && k == P.ksecond) u = u + 1.;
                                double wa = fv[i];
                                if (P.q0) wa = wa + v * P.tq0;
                                t1 = u * wa;
                            }
                        }
                        term[0][slot][pl] = t1;
                        term[1][slot][pl] = t2;
                    }
                }
            } else if (P.pass == P_INIT) {
#pragma unroll 1
                for (int i = 0; i < kPer; i++) {
                    const int k = k0 + prow + 64 * i;
                    const size_t e = (size_t)k * kG + slot;
                    const int2 o2 = p.offsets[k];
                    // extractPixelsContour(Vec2d) (:341-374): keep 0 <= p < (boundW, boundH)
                    const double px = P.ccx + (double)o2.x, py = P.ccy + (double)o2.y;
                    if (!(px < 0 || py < 0 || px >= p.boundW || py >= p.boundH)) {
                        double ux, uy;
                        undistort1(p.cam, px, py, ux, uy);  // get3dPointsFromImage1Pixels :542
                        RX[e] = ux;
                        RY[e] = uy;
                        atomicAdd(&shCnt[slot], 1);
                        atomicMin(&shKmin[slot], k);
                    }
                }
            } else if (P.pass == P_LEVEL) {
#pragma unroll 1
                for (int i = 0; i < kPer; i++) {
                    const int k = k0 + prow + 64 * i;
                    const size_t e = (size_t)k * kG + slot;
                    const int2 o2 = p.offsets[k];
                    const double px = P.ccx + (double)o2.x, py = P.ccy + (double)o2.y;
                    if (!(px < 0 || py < 0 || px >= p.boundW || py >= p.boundH)) {
                        // updateImage1PixelsIntensity (:576-589)
                        if (!pixel_good(px, py, P.scale, P.lw, P.lh)) {
                            shI1fail[slot] = 1;
                        } else {
                            const float fx = (float)(P.scale * px), fy = (float)(P.scale * py);
                            const uint8_t* g = P.img1 + (long)(int)floor((double)fy) * P.lw + (int)floor((double)fx);
                            I1[e] = bilinear4(g[0], g[1], g[P.lw], g[P.lw + 1], fx, fy);
                        }
                    }
                }
            }
            __syncthreads();
            // ---------------- sequential sums in MINPACK's pixel order ----------------
            if (chain) {
                const int ps = sp[tid].pass;
                const double* tA = term[0][tid];
                const double* tB = term[1][tid];
                if (ps == P_EVAL || ps == P_QR2) {
                    if (!shSlow[tid]) {
                        double s2 = en.s2;
#pragma unroll 16
                        for (int q = 0; q < kC; q++) s2 += tA[q];
                        en.s2 = s2;
                    } else {
                        for (int q = 0; q < kC; q++) {
                            const double x = tB[q];
                            if (x == x) en.add(x);
                        }
                    }
                    shSlow[tid] = 0;  // ordered before the next chunk by the barrier below
                } else if (ps == P_QR1) {
#pragma unroll 8
                    for (int q = 0; q < kC; q++) {
                        const double a = tA[q], b = tB[q];
                        if (a == a) {
                            sumA += a;
                            sumB += b;
                        }
                    }
                } else if (ps == P_QR3) {
#pragma unroll 8
                    for (int q = 0; q < kC; q++) {
                        const double a = tA[q];
                        if (a == a) sumA += a;
                    }
                }
            }
            __syncthreads();
        }

        // ---------------- per-slot lmdif bookkeeping ----------------
        if (chain) {
            PassOut o;
            o.nrm = en.finish();
            o.sumA = sumA;
            o.sumB = sumB;
            o.aqs1 = shAqs1[tid];
            o.cnt = shCnt[tid];
            o.kmin = shKmin[tid];
            o.fail = shFail[tid];
            o.ph3 = shPh3[tid];
            o.i1fail = shI1fail[tid];
            ctl.after_pass(ss[tid], sp[tid], o, tid);
        }
    }

    if (chain) {
        atomicAdd(p.statEval, (unsigned long long)ctl.cnt_eval);
        atomicAdd(p.statPix, (unsigned long long)ctl.cnt_pix);
    }
}

}  // namespace fm3d
