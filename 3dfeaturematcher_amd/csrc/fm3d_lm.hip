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
//   * a workgroup serves kG = 4 points ("slots") with 3 "term" waves and one
//     "chain" wave;
//   * a pass over the neighbourhood (one residual evaluation, the two-column
//     forward-difference Jacobian, or one Householder product) runs in chunks
//     of kC pixels.  The term waves compute every (slot, pixel) term of a chunk
//     in parallel -- plane intersection, distorted projection, bilinear
//     samples, Jacobian columns, Householder products -- into a double-buffered
//     LDS tile, while the chain wave adds the previous chunk's terms in pixel
//     order (one lane per slot and sum: MINPACK's enorm / dot-product order);
//   * between passes the chain lanes run the slot's lmdif bookkeeping;
//   * the first pass of a point compacts its neighbourhood: the pixels inside
//     the image bounds, in reference order, become entries 0..m_dat-1 of the
//     slot's slab rows (undistorted rays, I1, fvec, Jacobian columns; layout
//     [array][slot][entry]), so every later pass streams exactly m_dat entries
//     with contiguous 512-byte wave loads and no bounds tests;
//   * each term thread owns one entry of every slot per chunk and issues the
//     loads (then the image gathers) of all slots before consuming any, so a
//     wave keeps 4 slots' memory traffic in flight.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "fm3d_device.h"
#include "fm3d_kernels.h"
#include "fm3d_lmdif.h"

namespace fm3d {

namespace {

using namespace lmdif;

}  // namespace

typedef __attribute__((address_space(1))) double gdouble;
typedef __attribute__((address_space(1))) float gfloat;
typedef __attribute__((address_space(1))) int gint;
typedef __attribute__((address_space(1))) const long long gi64;  // an int2 offset (x low, y high)
typedef __attribute__((address_space(1))) const uint8_t gu8;

constexpr int kG = kLMSlots;                   // points (slots) per workgroup
constexpr int kTermThreads = kLMThreads - 64;  // term waves; the last wave is the chain wave
constexpr int kC = kLMChunk;                   // entries per slot per chunk: one per term thread
static_assert(kC == kTermThreads, "one entry per term thread and slot");
constexpr int kB = 2;  // slots per batch: a term thread keeps two batches' loads in flight

enum PassKind { P_IDLE = 0, P_INIT, P_LEVEL, P_EVAL, P_QR1, P_QR2, P_QR3, P_DONE };

// parameters of a slot's current pass (LDS; written by the slot's chain lane)
struct SlotP {
    int pass, ekind, nev, len, t0, t1, q0, pivot, lw, lh;
    double n0[2], n1[2], n2[2], mm[2], w[2], hj[2];
    double scale, xmax, ymax, ccx, ccy, ajn0s, tq, ajn1s, tq0, agiant;  // xmax = (1/scale)*cols (isPixelGood)
    const uint8_t* img1;
    const uint8_t* img2;
};

// persistent state of a slot (LDS; only its chain lane touches it)
struct SlotS {
    LM s;
    double X0, X1, X2, ccx, ccy, nrm0, nrm1, nrm2;
    double apf, aqf, ff, aps, fs, vfirst, r01, tq0, qtf0, wa4s, usecond, ajn0s, tq, ajn1s;
    int pidx, m, L, i1ok, ekind, t0, q0, t1, bNaN;
    int slot, passes;  // passes spent on the current point (heavy-point scheduling)
};

// per-pass results the chain lanes hand to the bookkeeping
struct PassOut {
    double nrm[2];  // EVAL (per evaluation) / QR2: enorm of the pass's values
    double sum[2];  // QR1 (a_q and fvec products) / QR3 dot products
    double aqs1;    // QR2: transformed a_q at the second kept pixel
    int cnt, fail[2], ph3[2], i1fail;
};

// lmdif bookkeeping of one slot (chain lane only).  Kept out of line so that the
// register budget of the data-parallel part of the kernel is not set by it.
// Entry indices are compact: entry 0 is the first kept pixel, entry 1 the second.
struct Ctl {
    const LMParams* p;  // a private copy: the kernel's own accesses stay on the kernarg segment
    const double* F;
    const double* J0;
    const double* J1;
    double eps;
    long long cnt_eval, cnt_pix;
    int* heavy;  // LDS: passes spent by each slot's current point (0 = none)

    // Heavy-point scheduling: once one slot's point has taken more than heavyPasses
    // passes, the other slots take no new points until it is done, so the group's
    // term waves serve that point alone (4 rows per chunk, ~4x shorter passes) and a
    // long point cannot stretch the end of the launch.  Only the order of work changes.
    __device__ bool other_heavy(const SlotS& S) const {
        if (p->heavyPasses <= 0) return false;
        for (int q = 0; q < kG; q++)
            if (q != S.slot && heavy[q] > p->heavyPasses) return true;
        return false;
    }
    __device__ void next_point(SlotS& S, SlotP& P) {
        if (p->trace && S.pidx >= 0 && S.passes > 0) {
            p->trace[4 * S.pidx + 1] = (long long)wall_clock64();
            p->trace[4 * S.pidx + 2] += S.passes;
            p->trace[4 * S.pidx + 3] = blockIdx.x;
        }
        heavy[S.slot] = 0;
        S.passes = 0;
        if (other_heavy(S)) {
            P.pass = P_IDLE;
            return;
        }
        fetch(S, P);
    }
    __device__ void fetch(SlotS& S, SlotP& P) {
        const int q = atomicAdd(p->queue, 1);
        if (q >= (p->order ? *p->nOrder : p->P)) {
            P.pass = P_DONE;
            return;
        }
        const int pidx = p->order ? p->order[q] : q;
        S.pidx = pidx;
        if (p->trace) p->trace[4 * pidx + 0] = (long long)wall_clock64();
        S.X0 = p->points[3 * pidx + 0];
        S.X1 = p->points[3 * pidx + 1];
        S.X2 = p->points[3 * pidx + 2];
        const double Ident[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        const double Zero[3] = {0, 0, 0};
        double cx, cy;
        project1(p->cam, Ident, Zero, S.X0, S.X1, S.X2, cx, cy);  // extractPixelsContour(Vec3d) :376-397
        S.ccx = cx;
        S.ccy = cy;
        P.pass = P_INIT;
        P.len = p->nOffPad;
        P.ccx = cx;
        P.ccy = cy;
    }
    __device__ void start_level(SlotS& S, SlotP& P) {
        const LevelDesc lv = p->lvl[S.L];
        P.pass = P_LEVEL;
        P.len = S.m;
        P.scale = ldexp(1.0, -S.L);  // 1.0 / float(2^L)  (optimize_pyramid, :225-241)
        P.xmax = (1 / P.scale) * lv.w;
        P.ymax = (1 / P.scale) * lv.h;
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
        next_point(S, P);
    }
    __device__ void level_done(SlotS& S, SlotP& P, int info) {
        p->info[8 * S.pidx + S.L] = info;
        p->nfev[8 * S.pidx + S.L] = S.s.nfev;
        sph2car_det(S.s.x[0], S.s.x[1], S.nrm0, S.nrm1, S.nrm2);
        S.L--;
        if (S.L < 0) {
            finish_point(S, P, FM3D_ST_OK);
        } else if (S.L < p->levelLo) {
            // end of this launch's level range: park the warm-start normal (status stays running)
            p->normals[3 * S.pidx + 0] = S.nrm0;
            p->normals[3 * S.pidx + 1] = S.nrm1;
            p->normals[3 * S.pidx + 2] = S.nrm2;
            next_point(S, P);
        } else {
            start_level(S, P);
        }
    }
    __device__ void abort_level(SlotS& S, SlotP& P, int code) {
        p->info[8 * S.pidx + S.L] = -code;
        p->nfev[8 * S.pidx + S.L] = S.s.nfev;
        finish_point(S, P, code);
    }
    // evaluateNormal (normaloptimizer.cpp:65-149), per-call part, for evaluation slot ev.
    // Returns false if the normal is NaN (the call aborts before touching a pixel).
    __device__ bool setup_eval(SlotS& S, SlotP& P, int ev, double a, double b, double hj) {
        double n0, n1, n2;
        sph2car_det(a, b, n0, n1, n2);  // par = (phi, theta)
        if (n2 != n2 || n1 != n1 || n0 != n0) return false;
        double w_theta = 1.0, w_phi = 1.0;
        if (fabs(b) - M_PI / 2 > 0 || fabs(a) - M_PI > 0) {
            w_theta = fm3d_exp(fabs(b) - M_PI / 2) + 1;
            w_phi = fm3d_exp(fabs(a) - M_PI + 1) + 1;
        }
        P.n0[ev] = n0;
        P.n1[ev] = n1;
        P.n2[ev] = n2;
        P.mm[ev] = n0 * S.X0 + n1 * S.X1 + n2 * S.X2;
        P.w[ev] = w_phi * w_theta;
        P.hj[ev] = hj;
        return true;
    }
    __device__ void count_eval(SlotS& S) {
        S.s.nfev++;
        cnt_eval++;
        cnt_pix += S.m;
    }
    __device__ void eval_pass(SlotS& S, SlotP& P, int kind, double a, double b) {
        count_eval(S);
        if (!setup_eval(S, P, 0, a, b, 1.0)) {
            abort_level(S, P, FM3D_ST_NAN_NORMAL);
            return;
        }
        S.ekind = kind;
        P.pass = P_EVAL;
        P.len = S.m;
        P.ekind = kind;
        P.nev = 1;
        P.agiant = 1.304e19 / (double)S.m;
    }
    // fdjac2: column j = 0 at (x0 + h0, x1), column j = 1 at (x0, x1 + h1)
    __device__ void jac_pass(SlotS& S, SlotP& P) {
        LM& s = S.s;
        s.h[0] = eps * fabs(s.x[0]);
        if (s.h[0] == 0.) s.h[0] = eps;
        s.h[1] = eps * fabs(s.x[1]);
        if (s.h[1] == 0.) s.h[1] = eps;
        count_eval(S);
        if (!setup_eval(S, P, 0, s.x[0] + s.h[0], s.x[1], s.h[0])) {
            abort_level(S, P, FM3D_ST_NAN_NORMAL);
            return;
        }
        // column 1's call only happens if column 0's succeeds: counted after the pass
        S.bNaN = !setup_eval(S, P, 1, s.x[0], s.x[1] + s.h[1], s.h[1]);
        S.ekind = E_JAC;
        P.pass = P_EVAL;
        P.len = S.m;
        P.ekind = E_JAC;
        P.nev = S.bNaN ? 1 : 2;
        P.agiant = 1.304e19 / (double)S.m;
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
        const size_t base = (size_t)slot * p->nOffPad;
        const double* Jpp = (pc ? J1 : J0) + base;
        const double* Jqq = (pc ? J0 : J1) + base;
        S.apf = Jpp[0];
        S.aqf = Jqq[0];
        S.ff = F[base + 0];
        S.aps = Jpp[1];
        S.fs = F[base + 1];
        const double ajn0 = s.acnorm[pc];  // == enorm of the pivot column (same elements, same order)
        S.t0 = ajn0 != 0.;
        S.ajn0s = (S.t0 && S.apf < 0.) ? -ajn0 : ajn0;
        if (!S.t0) S.ajn0s = 1.;  // unused
        S.vfirst = S.t0 ? (S.apf / S.ajn0s) + 1. : S.apf;
        P.pivot = pc;
        P.len = S.m;
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
    __device__ static int fail_code(int fail, int ph3, int i1ok) {
        if (fail != 0x7fffffff)  // first failing pixel in index order decides (:455-470, :557-560)
            return (fail & 3) == 2 ? FM3D_ST_NAN_PLANE : FM3D_ST_ABORT_BBOX;
        if (!i1ok) return FM3D_ST_ABORT_PIX1;
        if (ph3) return FM3D_ST_ABORT_PIX2;
        return 0;
    }

    __device__ __noinline__ void after_pass(SlotS& S, SlotP& P, const PassOut& o, int slot) {
        const int ps = P.pass;
        heavy[slot] = ++S.passes;
        if (ps == P_INIT) {
            S.m = o.cnt;
            if (p->levelHi == p->levels) {
                // initial guess: X / norm(X) == X * (1/norm) (Vec3d operator/, :342-343)
                double nr = sqrt(S.X0 * S.X0 + S.X1 * S.X1 + S.X2 * S.X2);
                double inv = 1. / nr;
                S.nrm0 = S.X0 * inv;
                S.nrm1 = S.X1 * inv;
                S.nrm2 = S.X2 * inv;
            } else {  // warm start parked by the previous level's launch
                S.nrm0 = p->normals[3 * S.pidx + 0];
                S.nrm1 = p->normals[3 * S.pidx + 1];
                S.nrm2 = p->normals[3 * S.pidx + 2];
            }
            if (S.m <= 0) {
                finish_point(S, P, FM3D_ST_NO_PIXELS);
            } else {
                S.L = p->levelHi;
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
            int code = fail_code(o.fail[0], o.ph3[0], S.i1ok);
            if (code) {
                abort_level(S, P, code);
                return;
            }
            LM& s = S.s;
            if (S.ekind == E_INITIAL) {
                s.fnorm = o.nrm[0];
                jac_pass(S, P);
            } else if (S.ekind == E_JAC) {
                s.acnorm[0] = o.nrm[0];
                count_eval(S);  // fdjac2's call for column 1
                if (S.bNaN) {
                    abort_level(S, P, FM3D_ST_NAN_NORMAL);
                    return;
                }
                code = fail_code(o.fail[1], o.ph3[1], S.i1ok);
                if (code) {
                    abort_level(S, P, code);
                    return;
                }
                s.acnorm[1] = o.nrm[1];
                start_qr(S, P, slot);
            } else {
                bool accepted;
                int info = lm_after_trial(s, o.nrm[0], &accepted);
                if (info) {
                    level_done(S, P, info);
                } else if (accepted) {
                    jac_pass(S, P);
                } else {
                    lm_inner_step(s);
                    eval_pass(S, P, E_TRIAL, s.wa2[0], s.wa2[1]);
                }
            }
        } else if (ps == P_QR1) {
            // qrfac j = 0: temp = sum v a_q / v_first; lmdif qtf j = 0: temp = -sum v f / v_first
            S.tq = o.sum[0] / S.vfirst;
            S.r01 = S.aqf - S.tq * S.vfirst;
            S.q0 = S.vfirst != 0.;
            S.tq0 = 0.;
            S.qtf0 = S.ff;
            if (S.q0) {
                S.tq0 = -o.sum[1] / S.vfirst;
                S.qtf0 = S.ff + S.vfirst * S.tq0;
            }
            qr2(S, P);
        } else if (ps == P_QR2) {
            const double ajn1 = o.nrm[0];
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
            const double tq1 = -o.sum[0] / S.usecond;
            finalize_qr(S, P, S.wa4s + S.usecond * tq1);
        }
    }

    // Slow path of a chunk's enorm (values outside MINPACK's intermediate range
    // occurred): replay enorm over the chunk's raw values, re-read from the slab
    // (EVAL) or recomputed with the term waves' exact expression (QR2).
    __device__ __forceinline__ void enorm_slow(Enorm& en, const SlotP& P, int slot, int which, int e0, int n) const {
        const size_t base = (size_t)slot * p->nOffPad;
        const int e1 = e0 + n < P.len ? e0 + n : P.len;
        for (int e = e0; e < e1; e++) {
            if (P.pass == P_EVAL) {
                const double* arr = P.ekind == E_JAC ? (which ? J1 : J0) : F;
                en.add(arr[base + e]);
            } else if (e > 0) {  // QR2: elements below the diagonal
                const double* Jp = P.pivot ? J1 : J0;
                const double* Jq = P.pivot ? J0 : J1;
                double a = Jq[base + e];
                if (P.t0) {
                    double v = Jp[base + e] / P.ajn0s;
                    a = a - P.tq * v;
                }
                en.add(a);
            }
        }
    }
};

__device__ __noinline__ void ctl_fetch(Ctl& c, SlotS& S, SlotP& P) { c.next_point(S, P); }

// enorm terms: x^2 for MINPACK's "intermediate" range (the branch almost every value
// takes), +0 otherwise (an exact no-op on the non-negative sum); values outside that
// range raise the chunk's slow flag and the chain lane replays the chunk with enorm.
__device__ inline double enorm_term(double x, double agiant, int* slow) {
    const double xa = fabs(x);
    if (xa > 3.834e-20 && xa < agiant) return xa * xa;
    if (xa != 0.) *slow = 1;
    return 0.;
}

// sum += t[0..kC) in index order.  Skipped entries hold +0.0, an exact no-op: a
// running sum that starts at +0.0 can never become -0.0.
__device__ inline double chain_sum(double sum, const double* t) {
    const double2* t2 = reinterpret_cast<const double2*>(t);
    double2 cur[8], nxt[8];
#pragma unroll
    for (int i = 0; i < 8; i++) cur[i] = t2[i];
    for (int q = 16; q < kC; q += 16) {
#pragma unroll
        for (int i = 0; i < 8; i++) nxt[i] = t2[q / 2 + i];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            sum += cur[i].x;
            sum += cur[i].y;
        }
#pragma unroll
        for (int i = 0; i < 8; i++) cur[i] = nxt[i];
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
        sum += cur[i].x;
        sum += cur[i].y;
    }
    return sum;
}

template <int kMinWavesPerSimd>
__global__ __launch_bounds__(kLMThreads, kMinWavesPerSimd) void lm_kernel(LMParams p) {
    __shared__ double term[2][2][kG][kC];  // [buffer][sum][row][entry]
    __shared__ SlotP sp[kG];
    __shared__ SlotS ss[kG];
    __shared__ int shCnt[kG], shFail[2][kG], shPh3[2][kG], shI1fail[kG], shSlow[2][2][kG];
    __shared__ double shAqs1[kG];
    __shared__ int shStop, shHeavy[kG];
    __shared__ LMParams shP;
    __shared__ Ctl shCtl[kG];
    __shared__ PassOut shOut[kG];

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const bool chainWave = tid >= kTermThreads;
    const int cl = tid - kTermThreads;  // chain lane: slot cl & 3, sum cl >> 2
    const bool chain = chainWave && cl < 2 * kG;
    const int cslot = cl & (kG - 1), cwhich = cl >> 2;
    const int nOffPad = p.nOffPad;
    const size_t ents = (size_t)nOffPad * kG;
    gdouble* __restrict__ RX = (gdouble*)(p.slab + (size_t)blockIdx.x * 5 * ents);
    gdouble* __restrict__ RY = RX + ents;
    gdouble* __restrict__ F = RY + ents;
    gdouble* __restrict__ J0 = F + ents;
    gdouble* __restrict__ J1 = J0 + ents;
    gfloat* __restrict__ I1 = (gfloat*)(p.slabI1 + (size_t)blockIdx.x * 2 * ents);
    gint* __restrict__ KI = (gint*)(I1 + ents);  // compact entry -> neighbourhood offset index
    const gi64* __restrict__ offsets = (const gi64*)p.offsets;
    const double cm = (double)p.cmax;
    const unsigned long long ltMask = (1ull << lane) - 1;

    // The bookkeeping works on LDS copies of the parameters and of its own state: taking
    // the address of a private object would put it in scratch (and a kernel with a large
    // scratch footprint gets fewer resident waves), taking &p would demote every access.
    if (tid == 0) shP = p;
    __syncthreads();
    Ctl& ctl = shCtl[cslot];
    if (chain && cwhich == 0) {
        ctl.p = &shP;
        ctl.F = (const double*)F;
        ctl.J0 = (const double*)J0;
        ctl.J1 = (const double*)J1;
        ctl.eps = sqrt(p.epsfcn > kEpsmch ? p.epsfcn : kEpsmch);
        ctl.cnt_eval = 0;
        ctl.cnt_pix = 0;
        ctl.heavy = shHeavy;
        shHeavy[cslot] = 0;
        ss[cslot].slot = cslot;
        ss[cslot].passes = 0;
        ss[cslot].pidx = -1;
        ctl_fetch(ctl, ss[cslot], sp[cslot]);
    }
    // the chain wave's dependent adds bound a pass once few slots are left: let it issue first
    if (chainWave) __builtin_amdgcn_s_setprio(3);

    // residual / Householder passes: a batch of kB slots' slab entries (loaded one
    // batch ahead), then their geometry, gathers and terms
    struct Ld {
        double a[kB], b[kB], c[kB];
        float i[kB];
    };
    // term rows of a chunk: row r holds kC consecutive entries of one slot.  With one or
    // two busy slots each gets 4 or 2 rows, so a lone point's pass takes 4x fewer steps.
    struct Rows {
        int slot[kG];  // -1: unused row (wave-uniform)
        int e0, rps;   // this thread's entry in row r: e0 + (r % rps) * kC
    };
    auto load_batch = [&](Ld& L, const int h, const Rows& R) {
#pragma unroll
        for (int s = 0; s < kB; s++) {
            L.a[s] = L.b[s] = L.c[s] = 0.;
            L.i[s] = 0.f;
            const int slot = R.slot[h + s], e = R.e0 + ((h + s) % R.rps) * kC;
            if (slot < 0) continue;
            const SlotP& P = sp[slot];
            const int ps = P.pass;
            if (ps < P_EVAL || ps > P_QR3 || e >= P.len) continue;
            const size_t sb = (size_t)slot * nOffPad;
            if (ps == P_EVAL) {
                L.a[s] = RX[sb + e];
                L.b[s] = RY[sb + e];
                L.i[s] = I1[sb + e];
                if (P.ekind == E_JAC) L.c[s] = F[sb + e];
            } else {
                const gdouble* Jp = P.pivot ? J1 : J0;
                const gdouble* Jq = P.pivot ? J0 : J1;
                L.a[s] = Jp[sb + e];
                L.b[s] = Jq[sb + e];
                if (ps != P_QR2) L.c[s] = F[sb + e];
            }
        }
    };
    auto process_batch = [&](const Ld& L, const int h, const Rows& R, const int buf) {
        // geometry of every evaluation: projectPointToPlane (:421-470), isInBoundingBox
        // (:646-655), projectPointsToImage2 (:591-644) -> gather addresses
        unsigned char code[kB][2];
        float fx[kB][2], fy[kB][2];
        const gu8* g[kB][2];
#pragma unroll
        for (int s = 0; s < kB; s++) {
#pragma unroll
            for (int ev = 0; ev < 2; ev++) {
                const int slot = R.slot[h + s], e = R.e0 + ((h + s) % R.rps) * kC;
                const SlotP& P = sp[slot < 0 ? 0 : slot];
                code[s][ev] = 1;
                fx[s][ev] = fy[s][ev] = 0.f;
                g[s][ev] = (const gu8*)P.img2;
                if (slot < 0 || P.pass != P_EVAL || ev >= P.nev || e >= P.len) continue;
                const double ux = L.a[s], uy = L.b[s];
                double nn = P.n0[ev] * ux + P.n1[ev] * uy + P.n2[ev] * 1.;
                double kk = P.mm[ev] / nn;
                double P0 = kk * ux, P1 = kk * uy, P2 = kk * 1.;
                unsigned char cd = 0;
                if (P0 != P0 || P1 != P1 || P2 != P2)
                    cd = 2;
                else if (!((P0 > -cm && P0 < cm) && (P1 > -cm && P1 < cm) && (P2 > 0. && P2 < cm)))
                    cd = 3;
                double u, v;
                project1(p.cam, p.R2, p.t2, P0, P1, P2, u, v);
                if (cd == 0 && !pixel_good_b(u, v, P.xmax, P.ymax)) cd = 4;
                code[s][ev] = cd;
                fx[s][ev] = (float)(P.scale * u);
                fy[s][ev] = (float)(P.scale * v);
                if (cd == 0)
                    g[s][ev] += (long)(int)floor((double)fy[s][ev]) * P.lw + (int)floor((double)fx[s][ev]);
            }
        }
        uint8_t b00[kB][2], b01[kB][2], b10[kB][2], b11[kB][2];
#pragma unroll
        for (int s = 0; s < kB; s++) {
#pragma unroll
            for (int ev = 0; ev < 2; ev++) {
                b00[s][ev] = b01[s][ev] = b10[s][ev] = b11[s][ev] = 0;
                if (code[s][ev] != 0) continue;
                const int lw = sp[R.slot[h + s]].lw;
                b00[s][ev] = g[s][ev][0];
                b01[s][ev] = g[s][ev][1];
                b10[s][ev] = g[s][ev][lw];
                b11[s][ev] = g[s][ev][lw + 1];
            }
        }
        // ---- terms ----
#pragma unroll
        for (int s = 0; s < kB; s++) {
            const int slot = R.slot[h + s], e = R.e0 + ((h + s) % R.rps) * kC, row = h + s;
            if (slot < 0) continue;
            const SlotP& P = sp[slot];
            const int ps = P.pass;
            if (ps < P_EVAL || ps > P_QR3) continue;
            const size_t sb = (size_t)slot * nOffPad;
            const bool in = e < P.len;
            if (ps == P_EVAL) {
                const bool jac = P.ekind == E_JAC;
                const bool i1ok = ss[slot].i1ok != 0;
#pragma unroll
                for (int ev = 0; ev < 2; ev++) {
                    if (ev >= P.nev) continue;
                    const unsigned char cd = code[s][ev];
                    double t = 0.;
                    if (!in) {
                    } else if (cd == 2 || cd == 3) {
                        atomicMin(&shFail[ev][slot], e * 4 + cd);  // first failing pixel decides
                    } else if (cd == 4) {
                        shPh3[ev][slot] = 1;
                    } else if (i1ok) {
                        float I2 = bilinear4(b00[s][ev], b01[s][ev], b10[s][ev], b11[s][ev], fx[s][ev],
                                             fy[s][ev]);
                        float dI = L.i[s] - I2;
                        double r = P.w[ev] * (double)dI;                   // evaluateNormal :145-148
                        double val = jac ? (r - L.c[s]) / P.hj[ev] : r;  // fdjac2 forward difference
                        (jac ? (ev ? J1 : J0) : F)[sb + e] = val;
                        t = enorm_term(val, P.agiant, &shSlow[buf][ev][slot]);
                    }
                    term[buf][ev][row][tid] = t;
                }
            } else {
                const double ap = L.a[s], aq = L.b[s], fv = L.c[s];
                double t0 = 0., t1 = 0.;
                if (ps == P_QR1) {
                    // qrfac column j = 0: v = a_p / ajnorm (+1 on the diagonal); v*a_q, v*f
                    if (in) {
                        double v = ap / P.ajn0s;
                        if (e == 0) v = v + 1.;
                        t0 = v * aq;
                        t1 = v * fv;
                    }
                    term[buf][1][row][tid] = t1;
                } else if (ps == P_QR2) {
                    // a_q' = a_q - temp * v below the diagonal -> ajnorm of column 1
                    if (in && e > 0) {
                        double a = aq;
                        if (P.t0) {
                            double v = ap / P.ajn0s;
                            a = a - P.tq * v;
                        }
                        if (e == 1) shAqs1[slot] = a;
                        t0 = enorm_term(a, P.agiant, &shSlow[buf][0][slot]);
                    }
                } else {
                    // lmdif qtf, j = 1: u_i * wa4_i
                    if (in && e > 0) {
                        double v = P.t0 ? ap / P.ajn0s : 0.;
                        double a = aq;
                        if (P.t0) a = a - P.tq * v;
                        double u = P.t1 ? a / P.ajn1s : a;
                        if (P.t1 && e == 1) u = u + 1.;
                        double wa = fv;
                        if (P.q0) wa = wa + v * P.tq0;
                        t0 = u * wa;
                    }
                }
                term[buf][0][row][tid] = t0;
            }
        }
    };

    long long iterations = 0;
    unsigned long long cyTerms = 0, cyChain = 0, cyCtl = 0;
    const unsigned long long tStart = wall_clock64(), cyStart = clock64();
    // per pass class (any JAC / any other evaluation / Householder only / once-per-point):
    // group passes and cycles, counted by thread 0
    unsigned long long clsCnt[4] = {0, 0, 0, 0}, clsCyc[4] = {0, 0, 0, 0};
    unsigned long long passStart = 0;
    int passCls = 0;
    if (tid == 0) {
        shStop = 0;
        atomicMin(p.statPass + 17, tStart);
    }
    for (;;) {
        if (tid == 0 && (++iterations > p.maxIter || (long long)(wall_clock64() - tStart) > p.maxTicks)) {
            // cannot happen for a correct state machine; never hang the GPU
            shStop = 1;
            atomicExch(p.overflow, 1);
        }
        if (chain && cwhich == 0) {
            if (sp[cslot].pass == P_IDLE) ctl_fetch(ctl, ss[cslot], sp[cslot]);  // waiting on a heavy point
            shCnt[cslot] = 0;
            shFail[0][cslot] = shFail[1][cslot] = 0x7fffffff;
            shPh3[0][cslot] = shPh3[1][cslot] = 0;
            shI1fail[cslot] = 0;
            for (int b = 0; b < 2; b++) shSlow[b][0][cslot] = shSlow[b][1][cslot] = 0;
        }
        __syncthreads();
        bool allDone = true, rare = false;
        unsigned actMask = 0;
#pragma unroll
        for (int q = 0; q < kG; q++) {
            const int ps = sp[q].pass;
            allDone = allDone && ps == P_DONE;
            if (ps != P_DONE && ps != P_IDLE) actMask |= 1u << q;
            rare = rare || ps == P_INIT || ps == P_LEVEL;
        }
        if (tid == 0 && iterations > 1) {
            clsCnt[passCls]++;
            clsCyc[passCls] += clock64() - passStart;
        }
        if (shStop || allDone) break;
        if (tid == 0) {
            passStart = clock64();
            bool jac = false, ev = false, qr = false;
            for (int q = 0; q < kG; q++) {
                const int ps = sp[q].pass;
                jac = jac || (ps == P_EVAL && sp[q].ekind == E_JAC);
                ev = ev || ps == P_EVAL;
                qr = qr || (ps >= P_QR1 && ps <= P_QR3);
            }
            passCls = jac ? 0 : ev ? 1 : qr ? 2 : 3;
        }
        // rows per busy slot (once-per-point/level passes keep one row per slot)
        const int nA = __popc(actMask);
        const int rps = (rare || nA > 2) ? 1 : (nA == 1 ? 4 : 2);
        int rowSlot[kG];
        int nSteps = 0;
#pragma unroll
        for (int r = 0; r < kG; r++) {
            const int k = r / rps;  // k-th busy slot
            int sl = -1, seen = 0;
#pragma unroll
            for (int q = 0; q < kG; q++)
                if ((actMask >> q) & 1) {
                    if (seen == k) sl = q;
                    seen++;
                }
            rowSlot[r] = sl;
        }
#pragma unroll
        for (int q = 0; q < kG; q++)
            if ((actMask >> q) & 1) {
                const int ns = (sp[q].len + rps * kC - 1) / (rps * kC);
                nSteps = ns > nSteps ? ns : nSteps;
            }

        // Term waves and the chain wave run separate step loops with the same number of
        // barriers (wave-uniform branches), so neither side's registers are live in the other.
        if (!chainWave) {
            int runBase[kG] = {0, 0, 0, 0};  // INIT: kept pixels before this chunk (same in every term thread)
            Ld L0, L1;
            for (int c = 0; c <= nSteps; c++) {
                if (c < nSteps) {
                    const unsigned long long tc0 = clock64();
                    // ---------------- term waves: chunk c into buffer c & 1 ----------------
                    const int e = c * kC + tid;  // this thread's entry of every slot
                    const int buf = c & 1;
                    // ---- once per point / level: neighbourhood compaction, image-1 samples ----
    #pragma unroll
                    for (int s = 0; s < kG; s++) {
                        const SlotP& P = sp[s];
                        if (!((actMask >> s) & 1) || c * kC >= P.len) continue;
                        const size_t sb = (size_t)s * nOffPad;
                        if (P.pass == P_INIT) {
                            // extractPixelsContour(Vec2d) (:341-374): keep 0 <= p < (boundW, boundH), in
                            // offset order -> entries runBase + (kept pixels before this one in the chunk)
                            int before = 0, total = 0, rank = 0;
                            bool mine = false;
                            double mx = 0, my = 0;
    #pragma unroll
                            for (int b = 0; b < kC / 64; b++) {
                                const long long o2 = offsets[c * kC + 64 * b + lane];
                                const double px = P.ccx + (double)(int)o2, py = P.ccy + (double)(int)(o2 >> 32);
                                const bool v = !(px < 0 || py < 0 || px >= p.boundW || py >= p.boundH);
                                const unsigned long long bm = __ballot(v);
                                const int n = __popcll(bm);
                                if (b < wave) before += n;
                                if (b == wave) {
                                    mine = v;
                                    rank = __popcll(bm & ltMask);
                                    mx = px;
                                    my = py;
                                }
                                total += n;
                            }
                            if (mine) {
                                const int pos = runBase[s] + before + rank;
                                double ux, uy;
                                undistort1(p.cam, mx, my, ux, uy);  // get3dPointsFromImage1Pixels :542
                                RX[sb + pos] = ux;
                                RY[sb + pos] = uy;
                                KI[sb + pos] = e;
                            }
                            runBase[s] += total;
                            if (tid == 0) shCnt[s] = runBase[s];
                        } else if (P.pass == P_LEVEL && e < P.len) {
                            // updateImage1PixelsIntensity (:576-589)
                            const long long o2 = offsets[KI[sb + e]];
                            const double px = P.ccx + (double)(int)o2, py = P.ccy + (double)(int)(o2 >> 32);
                            if (!pixel_good_b(px, py, P.xmax, P.ymax)) {
                                shI1fail[s] = 1;
                            } else {
                                const gu8* img1 = (const gu8*)P.img1;
                                const float fx = (float)(P.scale * px), fy = (float)(P.scale * py);
                                const gu8* g = img1 + (long)(int)floor((double)fy) * P.lw + (int)floor((double)fx);
                                I1[sb + e] = bilinear4(g[0], g[1], g[P.lw], g[P.lw + 1], fx, fy);
                            }
                        }
                    }
                    // residual / Householder passes, software-pipelined by batch: the loads of
                    // the next batch are in flight while the current one is processed
                    Rows R, Rn;
    #pragma unroll
                    for (int r = 0; r < kG; r++) R.slot[r] = Rn.slot[r] = rowSlot[r];
                    R.rps = Rn.rps = rps;
                    R.e0 = c * rps * kC + tid;
                    Rn.e0 = R.e0 + rps * kC;
                    if (c == 0) load_batch(L0, 0, R);
                    load_batch(L1, kB, R);
                    process_batch(L0, 0, R, buf);
                    if (c + 1 < nSteps) load_batch(L0, 0, Rn);
                    process_batch(L1, kB, R, buf);
                    if (tid == 0) cyTerms += clock64() - tc0;
                }
                __syncthreads();
            }
        } else {
            // chain-lane state for this pass
            const int cps = chain ? sp[cslot].pass : P_IDLE;
            const int cSteps = chain ? (sp[cslot].len + rps * kC - 1) / (rps * kC) : 0;
            const int cRow0 = __popc(actMask & ((1u << cslot) - 1)) * rps;  // first row of my slot
            Enorm en;
            en.init(1);
            if (chain) en.agiant = sp[cslot].agiant;
            double csum = 0.;
            const bool cActive = chain && (cwhich == 0 ? (cps >= P_EVAL && cps <= P_QR3)
                                                       : ((cps == P_EVAL && sp[cslot].nev == 2) || cps == P_QR1));
            for (int c = 0; c <= nSteps; c++) {
                if (cActive && c > 0 && c - 1 < cSteps) {
                    const unsigned long long tc0 = clock64();
                    // ---------------- chain lanes: chunk c-1, entry order ----------------
                    const int buf = (c - 1) & 1;
                    if (cps == P_EVAL || cps == P_QR2) {
                        if (!shSlow[buf][cwhich][cslot]) {
                            for (int r = 0; r < rps; r++) en.s2 = chain_sum(en.s2, term[buf][cwhich][cRow0 + r]);
                        } else {
                            ctl.enorm_slow(en, sp[cslot], cslot, cwhich, (c - 1) * rps * kC, rps * kC);
                        }
                        shSlow[buf][cwhich][cslot] = 0;  // buffer reused two steps later, after a barrier
                    } else {
                        for (int r = 0; r < rps; r++) csum = chain_sum(csum, term[buf][cwhich][cRow0 + r]);
                    }
                    if (cl == 0) cyChain += clock64() - tc0;
                }
                __syncthreads();
            }
            // ---------------- per-slot lmdif bookkeeping ----------------
            const unsigned long long tc0 = clock64();
            const double nrm = en.finish();
            const double nrmB = __shfl(nrm, (cl & (kG - 1)) + kG);
            const double sumB = __shfl(csum, (cl & (kG - 1)) + kG);
            if (chain && cwhich == 0 && cps != P_DONE && cps != P_IDLE) {
                PassOut& o = shOut[cslot];
                o.nrm[0] = nrm;
                o.nrm[1] = nrmB;
                o.sum[0] = csum;
                o.sum[1] = sumB;
                o.aqs1 = shAqs1[cslot];
                o.cnt = shCnt[cslot];
                o.fail[0] = shFail[0][cslot];
                o.fail[1] = shFail[1][cslot];
                o.ph3[0] = shPh3[0][cslot];
                o.ph3[1] = shPh3[1][cslot];
                o.i1fail = shI1fail[cslot];
                ctl.after_pass(ss[cslot], sp[cslot], o, cslot);
            }
            if (cl == 0) cyCtl += clock64() - tc0;
        }
    }

    if (chain && cwhich == 0) {
        atomicAdd(p.statEval, (unsigned long long)ctl.cnt_eval);
        atomicAdd(p.statPix, (unsigned long long)ctl.cnt_pix);
    }
    if (tid == 0) {
        atomicAdd(p.statPass + 0, (unsigned long long)iterations);
        atomicAdd(p.statPass + 1, cyTerms);
        atomicAdd(p.statPass + 4, clock64() - cyStart);
        const unsigned long long wt = wall_clock64() - tStart;
        atomicAdd(p.statPass + 5, wt);
        atomicMax(p.statPass + 6, wt);
        for (int k = 0; k < 4; k++) {
            atomicAdd(p.statPass + 7 + k, clsCnt[k]);
            atomicAdd(p.statPass + 11 + k, clsCyc[k]);
        }
        atomicMax(p.statPass + 15, tStart);  // latest workgroup start: late starts = grid > residency
        atomicMax(p.statPass + 16, wall_clock64());
    }
    if (cl == 0) {
        atomicAdd(p.statPass + 2, cyChain);
        atomicAdd(p.statPass + 3, cyCtl);
    }
}

// Between level launches: the points still running, ordered by the evaluations the
// level just finished took, most first (a longest-first schedule for the next level:
// per-point cost is strongly correlated across pyramid levels).  Counting sort, one
// workgroup; the order inside a bin does not matter (points are independent).
__global__ __launch_bounds__(1024) void lm_order_kernel(const int* __restrict__ status, const int* __restrict__ nfev,
                                                      int P, int level, int* __restrict__ order, int* nOrder) {
    constexpr int kBins = 512;
    __shared__ int hist[kBins];
    for (int b = threadIdx.x; b < kBins; b += blockDim.x) hist[b] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < P; i += blockDim.x) {
        if (status[i] != kLMRunning) continue;
        const int n = nfev[8 * i + level];
        atomicAdd(&hist[kBins - 1 - (n < kBins - 1 ? n : kBins - 1)], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int run = 0;
        for (int b = 0; b < kBins; b++) {
            const int c = hist[b];
            hist[b] = run;
            run += c;
        }
        *nOrder = run;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < P; i += blockDim.x) {
        if (status[i] != kLMRunning) continue;
        const int n = nfev[8 * i + level];
        order[atomicAdd(&hist[kBins - 1 - (n < kBins - 1 ? n : kBins - 1)], 1)] = i;
    }
}

template __global__ void lm_kernel<3>(LMParams);
template __global__ void lm_kernel<4>(LMParams);

}  // namespace fm3d
