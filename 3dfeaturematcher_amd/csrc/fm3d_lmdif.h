// fm3d_lmdif.h -- MINPACK lmdif for n = 2 (lmfit lmmin with lm_control_double), device side.
//
// Reference: Triangulator/normaloptimizer.cpp:247-292 calls lmfit's lmmin, a C restatement of
// MINPACK lmdif / lmpar / qrsolv / qrfac.  lmfit is not vendored in the reference; the
// restatement follows MINPACK with lmfit-4 defaults (ftol = xtol = gtol = 30*DBL_EPSILON,
// stepbound 100, patience 100 -> maxfev 300) and is pinned by scipy.optimize.leastsq
// (tests/golden/lm.npz).  Operation order identical to oracle/fm3d_oracle.c.
#pragma once

#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "fm3d_device.h"
#include "fm3d_crmath.h"

namespace fm3d {
namespace lmdif {


// E_JAC evaluates both forward-difference columns (fdjac2's j = 0 and j = 1
// calls) in one pass: they are independent evaluations at (x0+h0, x1), (x0, x1+h1).
enum EvalKind { E_INITIAL = 0, E_JAC, E_TRIAL };

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
    // tools.cpp:772-777 with the 1-ulp deterministic transcendentals (the NCC hypotheses)
    n0 = fm3d_cos(theta) * fm3d_cos(phi);
    n1 = fm3d_cos(theta) * fm3d_sin(phi);
    n2 = fm3d_sin(theta);
}
// tools.cpp:772-777 with the correctly rounded transcendentals (fm3d_crmath.h): the LM path, whose
// reference values are libm's, and libm is correctly rounded on ~99.8 % of the LM's arguments
__device__ inline void sph2car_cr(double phi, double theta, double& n0, double& n1, double& n2) {
    const double ct = fm3d_cos_cr(theta);
    n0 = ct * fm3d_cos_cr(phi);
    n1 = ct * fm3d_sin_cr(phi);
    n2 = fm3d_sin_cr(theta);
}

}  // namespace lmdif
}  // namespace fm3d
