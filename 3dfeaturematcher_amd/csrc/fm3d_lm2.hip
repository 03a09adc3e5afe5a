// fm3d_lm2.hip -- NormalOptimizer::computeOptimizedNormals on gfx950: one wavefront per point.
//
// Reference: Triangulator/normaloptimizer.cpp:223-452 (optimize_pyramid, optimize,
// computeOptimizedNormals), the residual evaluateNormal (:65-149) and the
// SingleCameraTriangulator geometry it calls (singlecameratriangulator.cpp:341-665),
// minimised by lmfit's lmmin (MINPACK lmdif; fm3d_lmdif.h).
//
// Why the sums are sequential: lmdif decides every step at rounding-noise level
// (ftol = xtol = 30*DBL_EPSILON), so every m_dat-long sum (enorm of fvec, the Jacobian
// column norms, the Householder dot products) is replayed in MINPACK's pixel order,
// bit for bit.  Only the ADDS are sequential; everything feeding
// them is data parallel.
//
// Design:
//   * a workgroup = kW "term" wavefronts + one "chain" wavefront.  Term wave w owns one
//     point ("slot") at a time, pulls the next point from a global queue when its
//     point is done, and runs every pass over the point's neighbourhood itself, 64
//     entries (one per lane) per chunk, with all pass parameters wave-uniform;
//   * the chain wave's lane 2s+k adds slot s's k-th sum of the current pass in entry
//     order, fed through a per-slot LDS ring of kR chunks (producer/consumer counters
//     in LDS, workgroup-scope release/acquire).  Slots never wait for each other: there
//     is no workgroup barrier in the main loop;
//   * between passes, lane 0 of the term wave runs the slot's lmdif bookkeeping;
//   * the first pass of a point compacts its neighbourhood (pixels inside the image
//     bounds, reference order) and precomputes the undistorted rays, so later passes
//     stream exactly m_dat entries;
//   * residuals and Jacobian columns are stored as the float intensity differences
//     dI they are computed from (4 bytes instead of 8): fvec = w*(double)dI and
//     J = (w_j*(double)dI_j - fvec)/h_j are recomputed from them with the same IEEE
//     operations, hence the same bits;
//   * divisions are the hardware sequence without its scaling / fix-up wrappers where the
//     operands need none (fm3d_fastdiv.h: the same bits, checked by
//     tools/micro/div_check.hip); by a pass-uniform denominator (h_j, the Householder
//     norms) they are one multiply by the correctly rounded reciprocal and one Markstein
//     correction;
//   * one workgroup of kW = 15 term waves + the chain wave per CU (4 waves per SIMD).
//
// TREE (fm3d_settings.lmReduction = 1): every m_dat-long sum as a fixed blocked
// tree instead -- each lane adds its entries (e = 64 k + lane) in chunk order, then an xor butterfly
// over the 64 lanes (oracle/fm3d_oracle.c ORC_LM_TREE, bit for bit).  No chain wave and no ring:
// the workgroup's 16th wave is a term wave too, and a pass's sums are the term wave's own.  The
// Jacobian sweep also sums a_0.a_1, a_0.f, a_1.f, so the 2-column Householder QR comes from these
// sums by the reflections' identities (ORC_LM_GRAM) where it is well conditioned; the three
// Householder passes run (tree-summed) only where it is not.  A sum of squares with a component
// outside enorm's intermediate range is replaced by MINPACK's sequential enorm (lane 0, from the
// slabs; rare).  Not the reference's summation order: the normals differ from the sequential
// mode's beyond 1e-4 on a fraction of points (profiles/r05_full_parity.json), so it is opt-in.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include <type_traits>

#include "fm3d_device.h"
#include "fm3d_fastdiv.h"
#include "fm3d_kernels.h"
#include "fm3d_lmdif.h"

namespace fm3d {

namespace {

using namespace lmdif;

constexpr int kW = kLM2Slots;  // term waves (slots) per workgroup
constexpr int kWA = kW + 1;    // per-slot LDS arrays: TREE runs kW + 1 term waves
constexpr int kE = 64;         // entries per chunk: one per lane
constexpr int kR = kLM2Ring;   // chunks in flight per slot (LDS ring depth)
static_assert((kR & (kR - 1)) == 0, "ring depth: a power of two");
constexpr int kRow = kE + 2;   // padded ring row: consecutive rows start 4 banks apart
// doubles per ring position: 2 rows per slot, padded to a multiple of 256 B (64 banks x 4 B)
constexpr int kRS = (2 * kLM2Slots * kRow * 8 + 255) / 256 * 256 / 8;
#ifndef FM3D_EVAL_PIPE
#define FM3D_EVAL_PIPE 1
#endif

// Q_GRAM (TREE only): the Jacobian columns' norms and Gram sums, one sweep after the Jacobian's
enum PassKind2 { Q_IDLE = 0, Q_INIT, Q_LEVEL, Q_EVAL, Q_QR1, Q_QR2, Q_QR3, Q_GRAM, Q_DONE };
enum SumKind { S_NONE = 0, S_ENORM, S_DOT };

typedef __attribute__((address_space(1))) double gdouble;
typedef __attribute__((address_space(1))) float gfloat;
typedef double d2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) d2v gd2v;
typedef __attribute__((address_space(1))) int gint;
typedef __attribute__((address_space(1))) const long long gi64;  // an int2 offset (x low, y high)
typedef __attribute__((address_space(1))) const uint8_t gu8;
typedef __attribute__((address_space(1), aligned(1))) const uint16_t gu16u;  // a byte pair at any address


// ---------------------------------------------------------------- LDS state
// the slot's current pass, written by lane 0 of the slot's term wave
struct SlotP2 {
    int pass, ekind, nev, len, pivot, t0, t1, q0, lw;
    unsigned projOff;  // byte offset of the point's frame pair's ProjConst in the table (p.proj)
    double n0[2], n1[2], n2[2], mm[2], w[2], hj[2];
    // setup_eval's sph2car deferred to the wave (resolve_trig): the angles (phi, theta) of the
    // evaluations whose bit in tpend is set
    double ta[2], tb[2];
    int tpend;
    double scale, xmax, ymax, ccx, ccy, ajn0s, tq, ajn1s, tq0, agiant, wF;
    const uint8_t* img1;
    const uint8_t* img2;
};

// persistent bookkeeping state of a slot (lane 0 of its term wave only)
struct SlotS2 {
    LM s;
    double X0, X1, X2, ccx, ccy, nrm0, nrm1, nrm2;
    double apf, aqf, ff, aps, fs, vfirst, r01, tq0, qtf0, wa4s, usecond, ajn0s, tq, ajn1s;
    double wF, wJ[2];  // weights of the evaluations behind the stored fvec / Jacobian dI values
    long long pev, ppix;  // the point's residual / pixel evaluations (its problem's counters)
    int prob;             // the point's problem (frame pair) in p->prob
    int pidx, m, L, i1ok, ekind, t0, q0, t1, bNaN;
};

// per-pass results handed to the bookkeeping
struct PassOut2 {
    double nrm[2];  // EVAL (per evaluation) / QR2: enorm of the pass's values
    double sum[2];  // QR1 (a_q and fvec products) / QR3 dot products
    double aqs1;    // QR2: transformed a_q at the second kept pixel
    // TREE, Jacobian sweep: sq[j] = sum of a_j^2 (enorm: sqrt), g[0] = a_0.a_1, g[1 + j] = a_j.f;
    // slow: bit j set when column j holds a component outside enorm's intermediate range
    double sq[2], g[3];
    int cnt, fail[2], ph3[2], i1fail, slow;
};

// what the chain lanes need to know about a pass (written before its first chunk)
struct PassDesc {
    int nChunks, id;
    int kind[2];  // SumKind per chain lane (which = 0, 1)
    double agiant;
};

// per-slot views of the slabs: [array][global slot][entry]
struct Slab {
    gdouble* RX;
    gdouble* RY;
    gfloat* I1;
    gfloat* DF;  // fvec as float dI (of the last residual evaluation)
    gfloat* DJ0;
    gfloat* DJ1;
    gint* KI;  // compact entry -> neighbourhood offset index
};
template <int NS>
__device__ inline Slab slab_of(const LMParams& p, long gslot) {
    const size_t n = (size_t)p.nOffPad, G = (size_t)p.nWaves * NS;
    Slab s;
#if FM3D_RAY_AOS
    s.RX = (gdouble*)p.slab + gslot * n * 2;  // (ux, uy) pairs: one 16-byte record per entry
    s.RY = s.RX + 1;
#else
    s.RX = (gdouble*)p.slab + gslot * n;
    s.RY = s.RX + G * n;
#endif
    s.I1 = (gfloat*)p.slabI1 + gslot * n;
    s.DF = s.I1 + G * n;
    s.DJ0 = s.DF + G * n;
    s.DJ1 = s.DJ0 + G * n;
    s.KI = (gint*)(s.DJ1 + G * n);
    return s;
}

// ---------------------------------------------------------------- bookkeeping
// lmdif bookkeeping of one slot, run by lane 0 of its term wave between passes.  Lives
// in LDS: a private object whose address is taken would go to scratch.
struct Ctl2 {
    const LMParams* p;
    Slab sl;
    double eps;
    long long cnt_eval, cnt_pix;
    int tree;  // TREE launch: the Gram form of the QR where it applies (start_qr_tree)

    // the next point of the launch's queue: the problems' points one after the other (each
    // problem one frame pair; its point count on the device or given)
    __device__ void fetch(SlotS2& S, SlotP2& P) {
        int loc = atomicAdd(p->queue, 1), j = 0;
        for (; j < p->nProb; j++) {
            const LMProblem& pr = p->prob[j];
            const int n = pr.Pdev ? *pr.Pdev : pr.P;
            if (loc < n) break;
            loc -= n;
        }
        if (j >= p->nProb) {
            P.pass = Q_DONE;
            return;
        }
        const LMProblem& pr = p->prob[j];
        S.prob = j;
        S.pidx = loc;
        S.pev = 0;
        S.ppix = 0;
        P.projOff = pr.projOff;
        atomicMax(p->statPass + 22, wall_clock64());  // the last point handed out: the queue runs dry
        S.X0 = pr.points[3 * loc + 0];
        S.X1 = pr.points[3 * loc + 1];
        S.X2 = pr.points[3 * loc + 2];
        const double Ident[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        const double Zero[3] = {0, 0, 0};
        double cx, cy;
        project1(p->cam, Ident, Zero, S.X0, S.X1, S.X2, cx, cy);  // extractPixelsContour(Vec3d) :376-397
        S.ccx = cx;
        S.ccy = cy;
        P.pass = Q_INIT;
        P.len = p->nOffPad;
        P.ccx = cx;
        P.ccy = cy;
    }
    __device__ void start_level(SlotS2& S, SlotP2& P) {
        const LevelDesc lv = p->prob[S.prob].lvl[S.L];
        P.pass = Q_LEVEL;
        P.len = S.m;
        P.scale = ldexp(1.0, -S.L);  // 1.0 / float(2^L)  (optimize_pyramid, :225-241)
        P.xmax = (1 / P.scale) * lv.w;
        P.ymax = (1 / P.scale) * lv.h;
        P.img1 = lv.img1;
        P.img2 = lv.img2;
        P.lw = lv.w;
        P.ccx = S.ccx;
        P.ccy = S.ccy;
    }
    __device__ void finish_point(SlotS2& S, SlotP2& P, int code) {
        const LMProblem& pr = p->prob[S.prob];
        pr.status[S.pidx] = code;
        pr.normals[3 * S.pidx + 0] = S.nrm0;
        pr.normals[3 * S.pidx + 1] = S.nrm1;
        pr.normals[3 * S.pidx + 2] = S.nrm2;
        pr.mdat[S.pidx] = S.m;
        atomicAdd(pr.stat + 0, (unsigned long long)S.pev);
        atomicAdd(pr.stat + 1, (unsigned long long)S.ppix);
        fetch(S, P);
    }
    __device__ void level_done(SlotS2& S, SlotP2& P, int info) {
        const LMProblem& pr = p->prob[S.prob];
        pr.info[8 * S.pidx + S.L] = info;
        pr.nfev[8 * S.pidx + S.L] = S.s.nfev;
        sph2car_cr(S.s.x[0], S.s.x[1], S.nrm0, S.nrm1, S.nrm2);
        S.L--;
        if (S.L < 0)
            finish_point(S, P, FM3D_ST_OK);
        else
            start_level(S, P);
    }
    __device__ void abort_level(SlotS2& S, SlotP2& P, int code) {
        const LMProblem& pr = p->prob[S.prob];
        pr.info[8 * S.pidx + S.L] = -code;
        pr.nfev[8 * S.pidx + S.L] = S.s.nfev;
        finish_point(S, P, code);
    }
    // evaluateNormal (normaloptimizer.cpp:65-149), per-call part, for evaluation ev.
    // Returns false if the normal is NaN (the call aborts before touching a pixel).
    // The normal sph2car(phi = a, theta = b) and mm = n . X: inside the reduction range of the
    // correctly rounded sin / cos the four values are finite (no NaN check can fail), and the wave
    // computes them after the bookkeeping, one function per lane (resolve_trig: the same bits);
    // outside it (never on real data) lane 0 computes them here, as before.
    __device__ bool setup_eval(SlotS2& S, SlotP2& P, int ev, double a, double b, double hj) {
        if (fabs(a) < FM3D_CR_RANGE && fabs(b) < FM3D_CR_RANGE) {
            P.ta[ev] = a;
            P.tb[ev] = b;
            P.tpend |= 1 << ev;
        } else {
            double n0, n1, n2;
            sph2car_cr(a, b, n0, n1, n2);  // par = (phi, theta)
            if (n2 != n2 || n1 != n1 || n0 != n0) return false;
            P.n0[ev] = n0;
            P.n1[ev] = n1;
            P.n2[ev] = n2;
            P.mm[ev] = n0 * S.X0 + n1 * S.X1 + n2 * S.X2;
            P.tpend &= ~(1 << ev);
        }
        double w_theta = 1.0, w_phi = 1.0;
        if (fabs(b) - M_PI / 2 > 0 || fabs(a) - M_PI > 0) {
            w_theta = fm3d_exp_cr(fabs(b) - M_PI / 2) + 1;
            w_phi = fm3d_exp_cr(fabs(a) - M_PI + 1) + 1;
        }
        P.w[ev] = w_phi * w_theta;
        P.hj[ev] = hj;
        return true;
    }
    // setup_eval's deferred normals, by the whole wave (all lanes call it): lane 4e + f computes
    // function f of evaluation e -- cos(theta), sin(theta), cos(phi), sin(phi) -- and lane 0 forms
    // sph2car_cr's n0 = cos(theta) cos(phi), n1 = cos(theta) sin(phi), n2 = sin(theta) and mm
    __device__ void resolve_trig(const SlotS2& S, SlotP2& P, int lane) {
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        const int pend = __builtin_amdgcn_readfirstlane(P.tpend);
        if (!pend) return;
        const int e = lane >> 2, f = lane & 3;
        double v = 0.;
        if (e < 2 && ((pend >> e) & 1)) v = fm3d_sincos_sel_cr(f < 2 ? P.tb[e] : P.ta[e], (f & 1) == 0);
        for (int k = 0; k < 2; k++) {
            if (!((pend >> k) & 1)) continue;
            const double ct = __shfl(v, 4 * k), st = __shfl(v, 4 * k + 1), cp = __shfl(v, 4 * k + 2),
                         sp = __shfl(v, 4 * k + 3);
            if (lane == 0) {
                const double n0 = ct * cp, n1 = ct * sp, n2 = st;
                P.n0[k] = n0;
                P.n1[k] = n1;
                P.n2[k] = n2;
                P.mm[k] = n0 * S.X0 + n1 * S.X1 + n2 * S.X2;
            }
        }
        if (lane == 0) P.tpend = 0;
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
    __device__ void count_eval(SlotS2& S) {
        S.s.nfev++;
        cnt_eval++;
        cnt_pix += S.m;
        S.pev++;
        S.ppix += S.m;
    }
    __device__ void eval_pass(SlotS2& S, SlotP2& P, int kind, double a, double b) {
        count_eval(S);
        if (!setup_eval(S, P, 0, a, b, 1.0)) {
            abort_level(S, P, FM3D_ST_NAN_NORMAL);
            return;
        }
        S.ekind = kind;
        S.wF = P.w[0];  // this pass rewrites the stored fvec
        P.pass = Q_EVAL;
        P.len = S.m;
        P.ekind = kind;
        P.nev = 1;
        P.agiant = 1.304e19 / (double)S.m;
    }
    // fdjac2: column j = 0 at (x0 + h0, x1), column j = 1 at (x0, x1 + h1)
    __device__ void jac_pass(SlotS2& S, SlotP2& P) {
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
        S.wJ[0] = P.w[0];
        S.wJ[1] = P.w[1];
        S.ekind = E_JAC;
        P.pass = Q_EVAL;
        P.len = S.m;
        P.ekind = E_JAC;
        P.nev = S.bNaN ? 1 : 2;
        P.agiant = 1.304e19 / (double)S.m;
        P.wF = S.wF;
    }
    // stored fvec / Jacobian column values at entry e (the passes' own operations)
    __device__ double fvec_at(const SlotS2& S, int e) const { return S.wF * (double)sl.DF[e]; }
    __device__ double jcol_at(const SlotS2& S, int j, int e) const {
        const double F = fvec_at(S, e);
        const double r = S.wJ[j] * (double)(j ? sl.DJ1 : sl.DJ0)[e];
        return (r - F) / S.s.h[j];
    }
    __device__ void finalize_qr(SlotS2& S, SlotP2& P, double qtf1) {
        S.s.r[0] = S.t0 ? -S.ajn0s : 0.;
        S.s.r[1] = 0.;
        S.s.r[2] = S.r01;
        S.s.r[3] = S.t1 ? -S.ajn1s : 0.;
        S.s.qtf[0] = S.qtf0;
        S.s.qtf[1] = qtf1;
        after_qr(S, P);
    }
    __device__ void after_qr(SlotS2& S, SlotP2& P) {
        int info = lm_after_qr(S.s);
        if (info) {
            level_done(S, P, info);
        } else {
            lm_inner_step(S.s);
            eval_pass(S, P, E_TRIAL, S.s.wa2[0], S.s.wa2[1]);
        }
    }
    // qrfac with column pivoting for n = 2, on the Jacobian columns of the slab
    __device__ void start_qr(SlotS2& S, SlotP2& P) {
        LM& s = S.s;
        const int pc = (s.acnorm[1] > s.acnorm[0]) ? 1 : 0;  // pivot column = larger norm
        s.ipvt[0] = pc;
        s.ipvt[1] = 1 - pc;
        S.apf = jcol_at(S, pc, 0);
        S.aqf = jcol_at(S, 1 - pc, 0);
        S.ff = fvec_at(S, 0);
        S.aps = jcol_at(S, pc, 1);
        S.fs = fvec_at(S, 1);
        const double ajn0 = s.acnorm[pc];  // == enorm of the pivot column (same elements, same order)
        S.t0 = ajn0 != 0.;
        S.ajn0s = (S.t0 && S.apf < 0.) ? -ajn0 : ajn0;
        if (!S.t0) S.ajn0s = 1.;  // unused
        S.vfirst = S.t0 ? (S.apf / S.ajn0s) + 1. : S.apf;
        P.pivot = pc;
        P.len = S.m;
        P.t0 = S.t0;
        P.ajn0s = S.ajn0s;
        P.wF = S.wF;
        P.w[0] = S.wJ[0];
        P.w[1] = S.wJ[1];
        P.hj[0] = s.h[0];
        P.hj[1] = s.h[1];
        if (S.t0) {
            P.pass = Q_QR1;
        } else {
            S.tq = 0.;
            S.r01 = S.aqf;
            S.q0 = 0;  // vfirst == apf == 0
            S.tq0 = 0.;
            S.qtf0 = S.ff;
            qr2(S, P);
        }
    }
    // TREE: one sweep over the stored Jacobian columns for their norms and Gram sums (Q_GRAM)
    __device__ void gram_pass(SlotS2& S, SlotP2& P) {
        P.pass = Q_GRAM;
        P.len = S.m;
        P.pivot = 0;
        P.wF = S.wF;
        P.w[0] = S.wJ[0];
        P.w[1] = S.wJ[1];
        P.hj[0] = S.s.h[0];
        P.hj[1] = S.s.h[1];
        P.agiant = 1.304e19 / (double)S.m;
    }
    // TREE: the 2-column QR from the Jacobian sweep's tree sums where it is well conditioned
    // (oracle/fm3d_oracle.c orc_qr_tree, ORC_LM_GRAM: the same operations), else the Householder
    // passes with tree sums
    __device__ void start_qr_tree(SlotS2& S, SlotP2& P, const PassOut2& o) {
        LM& s = S.s;
        const int pc = (s.acnorm[1] > s.acnorm[0]) ? 1 : 0;
        if (!o.slow && s.acnorm[pc] != 0.) {
            const double apf = jcol_at(S, pc, 0), aqf = jcol_at(S, 1 - pc, 0);
            const double Spq = o.g[0], Spf = o.g[1 + pc], Sqf = o.g[2 - pc], Sqq = o.sq[1 - pc];
            const double s0 = apf < 0. ? -s.acnorm[pc] : s.acnorm[pc];
            const double r01 = -(Spq / s0), qtf0 = -(Spf / s0), d = Sqq - r01 * r01;
            if (__builtin_isfinite(Spq) && __builtin_isfinite(Spf) && __builtin_isfinite(Sqf) &&
                __builtin_isfinite(Sqq) && d > 1e-6 * Sqq) {  // ORC_GRAM_C
                const double v0 = apf / s0 + 1., v1 = jcol_at(S, pc, 1) / s0, t = (Spq / s0 + aqf) / v0;
                const double a1 = jcol_at(S, 1 - pc, 1) - t * v1;
                double s1 = sqrt(d);
                if (a1 < 0.) s1 = -s1;
                s.ipvt[0] = pc;
                s.ipvt[1] = 1 - pc;
                s.r[0] = -s0;
                s.r[1] = 0.;
                s.r[2] = r01;
                s.r[3] = -s1;
                s.qtf[0] = qtf0;
                s.qtf[1] = -((Sqf - r01 * qtf0) / s1);
                after_qr(S, P);
                return;
            }
        }
        start_qr(S, P);
    }
    __device__ void qr2(SlotS2& S, SlotP2& P) {
        P.pass = Q_QR2;
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

    // TREE: MINPACK's sequential enorm of a pass's values recomputed from the slabs, for a sum of
    // squares with a component outside enorm's intermediate range (rare; orc_enorm_tree's
    // fallback).  kind 0: the residual; 1 / 2: Jacobian column 0 / 1; 3: QR2's transformed a_q
    // (entries 1 ..).  The same IEEE operations as the passes (their fast divisions round alike).
    __device__ __noinline__ double seq_enorm(const SlotP2& P, int kind, int len) const {
        Enorm en;
        en.init(kind == 3 ? len - 1 : len);
        const int pc = P.pivot;
        for (int e = kind == 3 ? 1 : 0; e < len; e++) {
            double v;
            if (kind == 0) {
                v = P.w[0] * (double)sl.DF[e];
            } else if (kind < 3) {
                const int j = kind - 1;
                v = (P.w[j] * (double)(j ? sl.DJ1 : sl.DJ0)[e] - P.wF * (double)sl.DF[e]) / P.hj[j];
            } else {
                const double F = P.wF * (double)sl.DF[e];
                const double ap = (P.w[pc] * (double)(pc ? sl.DJ1 : sl.DJ0)[e] - F) / P.hj[pc];
                v = (P.w[1 - pc] * (double)(pc ? sl.DJ0 : sl.DJ1)[e] - F) / P.hj[1 - pc];
                if (P.t0) v = v - P.tq * (ap / P.ajn0s);
            }
            en.add(v);
        }
        return en.finish();
    }

    __device__ __noinline__ void after_pass(SlotS2& S, SlotP2& P, const PassOut2& o) {
        const int ps = P.pass;
        if (ps == Q_INIT) {
            S.m = o.cnt;
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
        } else if (ps == Q_LEVEL) {
            S.i1ok = o.i1fail ? 0 : 1;
            // car2sph (tools.cpp:767-771) -> lmdif from the current normal
            S.s.x[1] = fm3d_atan2_cr(S.nrm2, sqrt(S.nrm0 * S.nrm0 + S.nrm1 * S.nrm1));
            S.s.x[0] = fm3d_atan2_cr(S.nrm1, S.nrm0);
            S.s.nfev = 0;
            S.s.iter = 1;
            S.s.par = 0.;
            S.s.delta = 0.;
            S.s.xnorm = 0.;
            if (S.m < 2)
                level_done(S, P, 0);  // lmdif: m < n -> improper input, info 0, no evaluation
            else
                eval_pass(S, P, E_INITIAL, S.s.x[0], S.s.x[1]);
        } else if (ps == Q_EVAL) {
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
                if (!tree) s.acnorm[0] = o.nrm[0];
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
                if (tree) {
                    gram_pass(S, P);
                } else {
                    s.acnorm[1] = o.nrm[1];
                    start_qr(S, P);
                }
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
        } else if (ps == Q_QR1) {
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
        } else if (ps == Q_QR2) {
            const double ajn1 = o.nrm[0];
            S.t1 = ajn1 != 0.;
            S.ajn1s = (S.t1 && o.aqs1 < 0.) ? -ajn1 : ajn1;
            if (!S.t1) S.ajn1s = 1.;  // unused
            S.usecond = S.t1 ? (o.aqs1 / S.ajn1s) + 1. : o.aqs1;
            S.wa4s = S.q0 ? S.fs + (S.aps / S.ajn0s) * S.tq0 : S.fs;
            if (S.usecond != 0.) {
                P.pass = Q_QR3;
                P.t1 = S.t1;
                P.ajn1s = S.ajn1s;
                P.q0 = S.q0;
                P.tq0 = S.tq0;
            } else {
                finalize_qr(S, P, S.wa4s);
            }
        } else if (ps == Q_GRAM) {
            S.s.acnorm[0] = o.nrm[0];
            S.s.acnorm[1] = o.nrm[1];
            start_qr_tree(S, P, o);
        } else if (ps == Q_QR3) {
            const double tq1 = -o.sum[0] / S.usecond;
            finalize_qr(S, P, S.wa4s + S.usecond * tq1);
        }
    }
};

struct Shared {
    // chunk terms (rows padded to kRow; the slow flags travel in the tags):
    // ring[pos][(2s + k) * kRow + e]: ring position pos holds, for every slot s and sum k, one
    // row, the chain lane's (2s + k).  Rows of one position lie 528 B apart (16 B mod 256) and a
    // position spans a multiple of 256 B, so in the chain's ds_read_b128 every lane of a 16-lane
    // group reads its own four banks whatever ring positions the slots are at (conflict-free).
    alignas(256) double ring[kR][kRS];
    int rowTag[kWA][kR];            // (chunk index << 2) | slow flags of the terms a ring position holds (published last)
    int consumed[kWA][2];           // chunks consumed, per chain lane (monotonic)
    int resultId[kWA][2];           // id of the last pass whose result is published
    double result[kWA][2];
    Enorm chainEn[64];  // MINPACK enorm state of each chain lane (s2 lives in its register)
    int done[kWA];
    int exited;  // TREE: term waves past their loop (the last one records the group's lifetime)
    // tail help: a wave whose slot has no more points takes every other chunk of a busy slot's
    // summed passes (one helper per slot, attached for good)
    int helper[kWA];                // 1 once a helper is attached
    int annSeq[kWA];                // passes announced to the helper (monotonic)
    int annBase[kWA], annId[kWA];    // the announced pass: first chunk index, pass id
    int helpDone[kWA];              // id of the last announced pass whose helper share is complete
    int hfail[kWA][2], hph3[kWA][2]; // the helper share's failures (as fail0/fail1, ph30/ph31 != 0)
    int hAtt[kWA], hSeen[kWA], hAnn[kWA];  // per wave (lane 0): attached slot, passes taken, passes announced
    // per-wave statistics, kept in LDS (lane 0) so that they hold no scalar registers across
    // the pass loops: class passes / cycles, terms / control cycles, producer waits, passes
    struct WaveStat {
        unsigned long long cnt[4], cyc[4], terms, ctl, wait, nPass, iter, t0;
    } ws[kWA];
    PassDesc pd[kWA];
    SlotP2 sp[kWA];
    SlotS2 ss[kWA];
    PassOut2 out[kWA];
    Ctl2 ctl[kWA];
    LMParams P;
};

// the workgroup's LDS state, at namespace scope so that the wave-role functions below
// address it directly (ds_* instructions) without a generic pointer
__shared__ Shared g_sh;

__device__ __forceinline__ int lds_load_acq(int* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store_rel(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// sum += row[0..64) in index order: 64 dependent adds, fed by ds_read_b128 into four
// register sets of 8 values in rotation, so three sets (24 values) are in flight while one is
// added.  Compiler barriers keep the reads in that order.  (A generic form indexing the sets
// modulo their count compiled to indexed register moves: 4-5x slower rounds.)
__device__ __forceinline__ double chain_sum64(double sum, const double* row) {
#if FM3D_ABL_CHAIN
    // ablation (timing experiments only, wrong sums): one add per chunk
    return sum + row[0];
#endif
    const double2* R = reinterpret_cast<const double2*>(row);
    double2 v0[4], v1[4], v2[4], v3[4];
    auto ld = [&](double2 (&v)[4], int k) {
#pragma unroll
        for (int i = 0; i < 4; i++) v[i] = R[4 * k + i];
        __asm__ __volatile__("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    auto add = [&](const double2 (&v)[4]) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            sum += v[i].x;
            sum += v[i].y;
        }
        __asm__ __volatile__("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    ld(v0, 0);
    ld(v1, 1);
    ld(v2, 2);
    ld(v3, 3);
    add(v0);
    ld(v0, 4);
    add(v1);
    ld(v1, 5);
    add(v2);
    ld(v2, 6);
    add(v3);
    ld(v3, 7);
    add(v0);
    add(v1);
    add(v2);
    add(v3);
    return sum;
}

__device__ __forceinline__ int rfl(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ unsigned long long rfl_u64(unsigned long long v) {
    return ((unsigned long long)(unsigned)rfl((int)(v >> 32)) << 32) | (unsigned)rfl((int)v);
}
__device__ __forceinline__ const uint8_t* rfl_ptr(const uint8_t* q) {
    const unsigned long long v = (unsigned long long)q;
    return (const uint8_t*)(((unsigned long long)(unsigned)rfl((int)(v >> 32)) << 32) | (unsigned)rfl((int)v));
}

// ---------------------------------------------------------------- term wave
// Publishes chunk c (slot w's running chunk index) into ring position c % kR: waits for ring
// space, writes the two term rows and their slow flags, then releases the position's tag.
struct Producer {
    Shared* sh;
    int w, lane, me;  // me: the producing wave (w: the slot it publishes for)
    int cmin;  // chunks both chain lanes had consumed at the last read of their counters
    unsigned long long deadline;  // wall clock: the watchdog ends a wait that a broken chain never releases

    // Waits for ring space for chunk c (both chain lanes have consumed chunk c - kR).  Called
    // before the chunk's terms are computed, so that the term code is one basic block.  The
    // counters are read only when the space seen last time is used up, the clock only when
    // still full.  c and cmin are wave-uniform (SGPRs; readfirstlane on every LDS read).
    __device__ __forceinline__ void reserve(int c) {
        if (c >= cmin + kR) {
            cmin = rfl(min(lds_load_acq(&sh->consumed[w][0]), lds_load_acq(&sh->consumed[w][1])));
            if (c >= cmin + kR) {
                const long long c0 = clock64();
                do {
                    __builtin_amdgcn_s_sleep(1);
                    cmin = rfl(min(lds_load_acq(&sh->consumed[w][0]), lds_load_acq(&sh->consumed[w][1])));
                } while (c >= cmin + kR && wall_clock64() < deadline);
                const unsigned long long dt = clock64() - c0;
                if (lane == 0) sh->ws[me].wait += dt;
            }
        }
    }
    // Publishes chunk c (reserved) into ring position c % kR: the term rows, then the tag.
    // TWO: the pass has a second sum (otherwise the second row is not written: its chain lane
    // sums whatever the row holds and publishes nothing).
    template <bool TWO = true>
    __device__ __forceinline__ void write(int c, double t0, double t1, int slowBits) {
        const int pos = c & (kR - 1);
        double* row0 = &sh->ring[pos][2 * w * kRow];
        row0[lane] = t0;
        if (TWO) row0[kRow + lane] = t1;
        // every lane's ring stores are done before the tag is published (lgkmcnt is per wave).
        // The tag carries the chunk index and the two sums' slow flags (bit k: sum k holds raw
        // values); it is written by every lane (same address, same value): no lane-0 branch
#if FM3D_TAG_NOWAIT
        __hip_atomic_store(&sh->rowTag[w][pos], (c << 2) | slowBits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#else
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
        lds_store_rel(&sh->rowTag[w][pos], (c << 2) | slowBits);
#endif
    }
    template <bool TWO = true>
    __device__ __forceinline__ void put(int c, double t0, double t1, int slowBits) {
        reserve(c);
        write<TWO>(c, t0, t1, slowBits);
    }
#ifndef FM3D_SLOW_BRANCH
#define FM3D_SLOW_BRANCH 1
#endif
    // The same with the enorm terms t_k = x_k^2 and the raw values v_k: sum k carries v_k where
    // slow_k (wave-uniform; rare).  FM3D_SLOW_BRANCH: the rows are written with the terms and, in a
    // branch only a slow chunk takes, overwritten with the raw values, so the common chunk spends
    // no VALU selects on the rows or the tag (the asm keeps the compiler from turning the branch
    // back into selects)
    template <bool TWO = true>
    __device__ __forceinline__ void write_terms(int c, double t0, double v0, bool slow0, double t1, double v1,
                                                bool slow1) {
#if FM3D_SLOW_BRANCH
        const int pos = c & (kR - 1);
        double* row0 = &sh->ring[pos][2 * w * kRow];
        row0[lane] = t0;
        if (TWO) row0[kRow + lane] = t1;
        int slowBits = 0;
        if (slow0 || (TWO && slow1)) {
            asm volatile("" ::: "memory");
            if (slow0) row0[lane] = v0;
            if (TWO && slow1) row0[kRow + lane] = v1;
            slowBits = (slow0 ? 1 : 0) | ((TWO && slow1) ? 2 : 0);
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the rows before the tag (as write)
        lds_store_rel(&sh->rowTag[w][pos], (c << 2) | slowBits);
#else
        write<TWO>(c, slow0 ? v0 : t0, slow1 ? v1 : t1, (slow0 ? 1 : 0) | (slow1 ? 2 : 0));
#endif
    }
};

typedef __attribute__((address_space(4))) const ProjConst cProjConst;

// The projection constants re-read (scalar loads, scalar cache) at every use: 21 uniform
// doubles kept live across the pass loops would not fit the SGPR budget and get spilled
// to VGPR lanes (a v_readlane per use).  The offset (0, or the pass's frame pair's entry of
// the table, SlotP2::projOff) is opaque to the compiler, so the loads are not hoisted out
// of the loop.  Every entry holds the same slab bases.
__device__ __forceinline__ const cProjConst* proj_consts(const ProjConst* p) {
    int z;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
    return (const cProjConst*)((const __attribute__((address_space(4))) char*)p + z);
}
__device__ __forceinline__ const cProjConst* proj_consts(const ProjConst* p, unsigned off) {
    unsigned z;
    asm volatile("s_mov_b32 %0, %1" : "=s"(z) : "s"(off));
    return (const cProjConst*)((const __attribute__((address_space(4))) char*)p + z);
}

// One residual evaluation of a neighbourhood entry: projectPointToPlane (:421-470),
// isInBoundingBox (:646-655), projectPointsToImage2 (:591-644) and the gather address,
// reduced to what the summed passes consume:
//  * inbox: isInBoundingBox of the plane point; false for a NaN coordinate too (the
//    NaN-plane / bounding-box distinction, failure codes 2 / 3, is recomputed for the rare
//    failing lane by plane_code);
//  * good: inbox and isPixelGood of the camera-2 pixel (NaN -> false).  u, v are only
//    used when good, so the r6 NaN propagation of project1 is not needed: an infinite or
//    NaN r6 makes u or v infinite or NaN either way;
//  * off: byte offset of the bilinear window in image 2 (0 when not good).
// Lane masks: every test below is the ballot of one compare (the compare's own SGPR result; the
// term code runs with all 64 lanes active), combined with scalar ANDs.  A ballot of a combined
// bool would cost two extra VALU instructions (v_cndmask + v_cmp) per ballot.
typedef unsigned long long LaneMask;
// v where the lane's bit of m is set, else +0 (v_cndmask with the mask as its selector)
__device__ __forceinline__ double sel_mask(double v, LaneMask m) {
    unsigned lo = __double2loint(v), hi = __double2hiint(v);
    asm("v_cndmask_b32_e64 %0, 0, %0, %1" : "+v"(lo) : "s"(m));
    asm("v_cndmask_b32_e64 %0, 0, %0, %1" : "+v"(hi) : "s"(m));
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ unsigned sel_mask_u32(unsigned v, LaneMask m) {
    asm("v_cndmask_b32_e64 %0, 0, %0, %1" : "+v"(v) : "s"(m));
    return v;
}
// lanes whose entry k*64 + lane lies below len (scalar arithmetic only)
__device__ __forceinline__ LaneMask in_mask(int k, int len) {
    const int rem = len - k * kE;
    return rem >= kE ? ~0ull : (rem <= 0 ? 0ull : ((1ull << rem) - 1));
}

struct Geo2 {
    float fx, fy;
    unsigned off;
    LaneMask inbox, good;  // lane masks
};
// MMOK: div_nn_ok(mm) holds (pass-uniform), so the ray-plane quotient takes the fast sequence.
// xmaxb / ymaxb: the bit patterns of the level bounds xmax, ymax (> 0).  u >= 0 && u <= xmax is
// bits(u) <= bits(xmax) as unsigned integers, because u is never -0 (u = xd*fx + cx with cx > 0,
// host-checked): negative values and NaNs have the sign or exponent bits that put them above.
// a2 = r2 + 2*x*x and a3 = r2 + 2*y*y are single FMAs: 2*RN(x*x) == RN(2x*x) (a power-of-two
// scaling) wherever x*x is normal, so fma(xx, 2, r2) rounds the same exact sum; where x*x is
// subnormal, |x|, |y| < 1e-150 and u, v round to cx, cy either way.  Likewise k*(2xy) is
// (2k)*RN(xy) (pc->k2d, k3d): one add fewer per evaluation; where xy is subnormal the term is far
// below an ulp of x*cdist (or u, v round to cx, cy).
// MULTI: the launch's problems have different poses -- the pass's entry of the table (projOff,
// one more scalar register live across the pass loops: +3-6 % cycles per evaluation pass,
// measured); otherwise entry 0
template <bool MMOK, bool MULTI>
__device__ __forceinline__ Geo2 geometry2(const LMParams& p, unsigned projOff, double ux, double uy, double n0,
                                          double n1, double n2, double mm, double scale,
                                          unsigned long long xmaxb, unsigned long long ymaxb, int lw, double cm) {
    const cProjConst* pc = MULTI ? proj_consts(p.proj, projOff) : proj_consts(p.proj);
    Geo2 r;
    const double nn = n0 * ux + n1 * uy + n2 * 1.;
    const double kk = MMOK ? div_nn(mm, nn, true) : mm / nn;
    const double P0 = kk * ux, P1 = kk * uy, P2 = kk * 1.;
    r.inbox = __ballot(fabs(P0) < cm) & __ballot(fabs(P1) < cm) & __ballot(P2 > 0.) & __ballot(P2 < cm);
    double x = pc->R[0] * P0 + pc->R[1] * P1 + pc->R[2] * P2 + pc->t[0];
    double y = pc->R[3] * P0 + pc->R[4] * P1 + pc->R[5] * P2 + pc->t[1];
    const double z = recip_z_lo(pc->R[6] * P0 + pc->R[7] * P1 + pc->R[8] * P2 + pc->t[2]);
    x *= z;
    y *= z;
    const double xx = x * x, yy = y * y;
    const double r2 = xx + yy;
    const double r4 = r2 * r2;
    const double r6 = r4 * r2;
    const double xy = x * y;
    const double a2 = __builtin_fma(xx, 2., r2);
    const double a3 = __builtin_fma(yy, 2., r2);
    const double cdist = 1 + pc->cam.k[0] * r2 + pc->cam.k[1] * r4 + pc->cam.k[4] * r6;
    const double xd = x * cdist + pc->k2d * xy + pc->cam.k[3] * a2;
    const double yd = y * cdist + pc->cam.k[2] * a3 + pc->k3d * xy;
    const double u = xd * pc->cam.fx + pc->cam.cx;
    const double v = yd * pc->cam.fy + pc->cam.cy;
    r.good = r.inbox & __ballot((unsigned long long)__double_as_longlong(u) <= xmaxb) &
             __ballot((unsigned long long)__double_as_longlong(v) <= ymaxb);
    r.fx = (float)(scale * u);
    r.fy = (float)(scale * v);
    const unsigned o = __umul24((unsigned)(int)floorf(r.fy), (unsigned)lw) + (unsigned)(int)floorf(r.fx);
    r.off = sel_mask_u32(o, r.good);
    return r;
}

// failure code (2 NaN plane point, 3 outside the bounding box) of an entry whose inbox is
// false: the rare path of the summed passes
__device__ __noinline__ int plane_code(double ux, double uy, double n0, double n1, double n2, double mm) {
    const double nn = n0 * ux + n1 * uy + n2 * 1.;
    const double kk = mm / nn;
    const double P0 = kk * ux, P1 = kk * uy, P2 = kk * 1.;
    return (P0 != P0 || P1 != P1 || P2 != P2) ? 2 : 3;
}

// getBilinearInterpPix32f on the gathered window, the floors taken from the sample
// coordinates (exact: |x| < 2^24 wherever the value is used)
__device__ __forceinline__ float bilinear_w(unsigned lo, unsigned hi, float x, float y) {
    const float x0 = floorf(x), y0 = floorf(y);
    const float b00 = (float)(lo & 0xff), b01 = (float)((lo >> 8) & 0xff);
    const float b10 = (float)(hi & 0xff), b11 = (float)((hi >> 8) & 0xff);
    const float xm0 = 1.0f - (x - x0), xm1 = (x - x0);
    const float ym0 = 1.0f - (y - y0), ym1 = (y - y0);
    return xm0 * (b00 * ym0 + b10 * ym1) + xm1 * (b01 * ym0 + b11 * ym1);
}

// the same with the fractions x - floor(x), y - floor(y) given
// (as two-lane float vectors: v_pk_mul_f32 / v_pk_add_f32 do the two columns' independent
// products and sums, each rounded as the scalar operation; 11 instructions instead of 17)
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float bilinear_f(unsigned lo, unsigned hi, float xf, float yf) {
    const f32x2 b0 = {(float)(lo & 0xff), (float)((lo >> 8) & 0xff)};  // b00, b01
    const f32x2 b1 = {(float)(hi & 0xff), (float)((hi >> 8) & 0xff)};  // b10, b11
    const float ym0 = 1.0f - yf, ym1 = yf;
    const f32x2 sc = b0 * ym0 + b1 * ym1;  // (b00 ym0 + b10 ym1, b01 ym0 + b11 ym1)
    const f32x2 xm = {1.0f - xf, xf};
    const f32x2 q = xm * sc;
    return q.x + q.y;  // xm0 * (...) + xm1 * (...)
}

// enorm term with the slow-path flag: x^2 is the term whenever no lane of the chunk needs
// MINPACK's small/large component handling (x = 0 adds +0, as enorm does).  slow: whether
// any lane of the wave does (a wave-uniform ballot of the lane tests).
__device__ __forceinline__ double enorm_term2(double x, double agiant, bool& slow) {
    const double xa = fabs(x);
    slow = (__ballot(!(xa < agiant)) | (__ballot(xa <= 3.834e-20) & __ballot(xa != 0.))) != 0;
    return x * x;
}

// ======================= chain wave =======================
// Lane 2s+k adds sum k of slot s's current pass, chunk by chunk in entry order.  A
// function of its own (not inlined) so that its registers are allocated apart from the
// term waves' code.  MINPACK's enorm state beyond the running s2 lives in LDS
// (g_sh.chainEn): only chunks with raw values (chain_slow) and the pass result touch it.

// a chunk of raw values again from acc0 (the running s2 before it), with MINPACK's full enorm
__device__ __forceinline__ double chain_slow(int lane, double acc0, const double* row) {
    Enorm en = g_sh.chainEn[lane];
    en.s2 = acc0;
    for (int i = 0; i < kE; i++) en.add(row[i]);
    g_sh.chainEn[lane] = en;
    return en.s2;
}
__device__ __forceinline__ double chain_finish(int lane, double acc) {
    Enorm en = g_sh.chainEn[lane];
    en.s2 = acc;
    return en.finish();
}

__device__ __noinline__ void chain_wave(int lane, unsigned long long tStart, long long maxTicks,
                                        unsigned long long* statBusy, unsigned long long* statRounds) {
    // the chain's dependent adds bound a pass's last chunk: let it issue first
    __builtin_amdgcn_s_setprio(3);
    const int s = lane >> 1, which = lane & 1;
    bool alive = s < kW;
    const int ss_ = alive ? s : 0;
    int cur = 0, rem = 0, kind = S_NONE, pid = 0;
    bool inPass = false;
    double acc = 0.;  // running sum: enorm s2 (S_ENORM) or the dot product (S_DOT)
    // busy time: one clock read per busy round (the span to the next round's read)
    unsigned long long busy = 0, tLast = 0, rounds = 0, chunks = 0;
    bool wasBusy = false;
    for (;;) {
        if ((long long)(wall_clock64() - tStart) > maxTicks) break;
        if (!__any(alive)) break;
#ifndef FM3D_CHAIN_ONETRIP
#define FM3D_CHAIN_ONETRIP 1
#endif
#if FM3D_CHAIN_ONETRIP
        // the four ring tags of a round in one LDS round trip: relaxed loads, one acquire fence
        // (the pass descriptor and the rows are read after it); chunks past the pass are cut by rem
        auto tagRel = [&](int b) {
            return alive ? __hip_atomic_load(&g_sh.rowTag[ss_][(cur + b) & (kR - 1)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : -1;
        };
        const int tag0 = tagRel(0), tg1 = tagRel(1), tg2 = tagRel(2), tg3 = tagRel(3);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#else
        const int tag0 = alive ? lds_load_acq(&g_sh.rowTag[ss_][cur & (kR - 1)]) : -1;
#endif
        const bool have = (tag0 >> 2) == cur;
        if (have && !inPass) {
            const PassDesc& d = g_sh.pd[ss_];
            rem = d.nChunks;
            kind = d.kind[which];
            pid = d.id;
            Enorm& en = g_sh.chainEn[lane];
            en.init(1);
            en.agiant = d.agiant;
            acc = 0.;
            inPass = true;
        }
        if (__any(have)) {
            const unsigned long long t = clock64();
            if (wasBusy) busy += t - tLast;
            tLast = t;
            wasBusy = true;
            // up to two chunks per lane per round, never past the pass's last chunk; every
            // lane runs the same add chain (S_NONE lanes sum zeros they never publish)
#ifndef FM3D_CHAIN_NB
#define FM3D_CHAIN_NB 4
#endif
#if FM3D_CHAIN_NB == 4
            // up to four chunks per lane and round: the three further tags read together (relaxed),
            // then one acquire fence before the rows are read
#if FM3D_CHAIN_ONETRIP
            const int tag1 = (have && rem >= 2) ? tg1 : -1, tag2 = (have && rem >= 3) ? tg2 : -1;
            const int tag3 = (have && rem >= 4) ? tg3 : -1;
#else
            const int tag1 = (have && rem >= 2) ? __hip_atomic_load(&g_sh.rowTag[ss_][(cur + 1) & (kR - 1)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : -1;
            const int tag2 = (have && rem >= 3) ? __hip_atomic_load(&g_sh.rowTag[ss_][(cur + 2) & (kR - 1)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : -1;
            const int tag3 = (have && rem >= 4) ? __hip_atomic_load(&g_sh.rowTag[ss_][(cur + 3) & (kR - 1)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : -1;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#endif
            int nb = have ? 1 : 0;
            if (nb == 1 && (tag1 >> 2) == cur + 1) nb = 2;
            if (nb == 2 && (tag2 >> 2) == cur + 2) nb = 3;
            if (nb == 3 && (tag3 >> 2) == cur + 3) nb = 4;
            const int slowm = (tag0 & 3) | ((tag1 & 3) << 2) | ((tag2 & 3) << 4) | ((tag3 & 3) << 6);
#else
            const int tag1 = (have && rem >= 2) ? lds_load_acq(&g_sh.rowTag[ss_][(cur + 1) & (kR - 1)]) : -1;
            const int nb = have ? (((tag1 >> 2) == cur + 1) ? 2 : 1) : 0;
#endif
            rounds++;
            chunks += nb;
#pragma nounroll
            for (int b = 0; b < FM3D_CHAIN_NB; b++) {
                if (b < nb) {
                    const double* row = &g_sh.ring[cur & (kR - 1)][lane * kRow];
#if FM3D_CHAIN_NB == 4
                    const bool slow = ((slowm >> (2 * b + which)) & 1) != 0;
#else
                    const bool slow = (((b ? tag1 : tag0) >> which) & 1) != 0;
#endif
                    const double acc0 = acc;
                    acc = chain_sum64(acc, row);
                    // a chunk of raw values (rare): again, with MINPACK's full enorm
                    if (kind == S_ENORM && slow) acc = chain_slow(lane, acc0, row);
                    cur++;
                    rem--;
                }
            }
            if (nb > 0) lds_store_rel(&g_sh.consumed[ss_][which], cur);
            if (have && rem == 0) {
                g_sh.result[ss_][which] = kind == S_ENORM ? chain_finish(lane, acc) : acc;
                lds_store_rel(&g_sh.resultId[ss_][which], pid);
                inPass = false;
            }
        } else {
            if (wasBusy) {
                busy += clock64() - tLast;
                wasBusy = false;
            }
            // done is set after the slot's last pass completed: every chunk was consumed
            if (alive && !inPass && lds_load_acq(&g_sh.done[ss_])) alive = false;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (lane == 0) {
        atomicAdd(statBusy, busy);
        atomicAdd(statRounds, rounds);
    }
    for (int o = 32; o > 0; o >>= 1) chunks += __shfl_xor(chunks, o);
    if (lane == 0) atomicAdd(statRounds + 1, chunks);
}

}  // namespace

// 4 waves per SIMD: one workgroup of 16 waves per CU (128 VGPRs)
template <bool MULTI, bool TREE>
__global__ __launch_bounds__(kLM2Threads, 4) void lm2_kernel(LMParams p) {
    Shared& sh = g_sh;
    constexpr int NS = TREE ? kWA : kW;  // term waves (slots) of the workgroup
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const unsigned long long tStart = wall_clock64(), cyStart = clock64();
    if (tid == 0) {
        sh.P = p;
        sh.exited = 0;
    }
    if (tid < NS) {
        for (int k = 0; k < kR; k++) sh.rowTag[tid][k] = -1;
        sh.consumed[tid][0] = sh.consumed[tid][1] = 0;
        sh.resultId[tid][0] = sh.resultId[tid][1] = 0;
        sh.done[tid] = 0;
        sh.helper[tid] = sh.annSeq[tid] = sh.helpDone[tid] = 0;
        sh.hAtt[tid] = -2;  // -2: the wave runs its own slot; -1: helper, not attached
        sh.hSeen[tid] = sh.hAnn[tid] = 0;
    }
    __syncthreads();

    if (wave < NS) {
        // ======================= term wave: slot w =======================
        const int w = rfl(wave);
        const long gslot = (long)blockIdx.x * NS + w;
        Ctl2& ctl = sh.ctl[w];

        // the summed passes address the slabs as grid-uniform array bases (ProjConst, scalar
        // loads) + one 32-bit byte offset per entry (global_load ... vOffset, sBase)
        if (lane == 0) {
            ctl.p = &sh.P;
            ctl.sl = slab_of<NS>(p, gslot);
            ctl.tree = TREE;
            ctl.eps = sqrt(p.epsfcn > DBL_EPSILON ? p.epsfcn : DBL_EPSILON);
            ctl.cnt_eval = 0;
            ctl.cnt_pix = 0;
        }
        PassOut2& OUT = sh.out[w];
        Producer prod{&sh, w, lane, w, 0, tStart + (unsigned long long)p.maxTicks};  // publishes into slot prod.w's ring
        int chunkSeq = 0;  // chunks of this slot published so far (all passes)
        // sh.hAtt[w] != -2: no points left for slot w; the wave helps slot prod.w
        const double cm = (double)p.cmax;
        const gi64* __restrict__ offsets = (const gi64*)p.offsets;
        const unsigned long long ltMask = (1ull << lane) - 1;
        int passId = 0;
        Shared::WaveStat& WS = sh.ws[w];
        if (lane == 0) {
            for (int k = 0; k < 4; k++) WS.cnt[k] = WS.cyc[k] = 0;
            WS.terms = WS.ctl = WS.wait = WS.nPass = WS.iter = 0;
            sh.sp[w].tpend = 0;
            ctl.fetch(sh.ss[w], sh.sp[w]);
        }
        ctl.resolve_trig(sh.ss[w], sh.sp[w], lane);
        for (;;) {
            if ((long long)rfl_u64(lane == 0 ? ++WS.iter : 0) > p.maxIter ||
                (long long)(wall_clock64() - tStart) > p.maxTicks) {
                if (lane == 0) atomicExch(p.overflow, 1);  // cannot happen for a correct state machine
                break;
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            bool own = true;
            int hBase = 0;
            if (rfl(sh.hAtt[w]) != -2) {
                // helper: the attached slot's next announced pass; else attach to a busy slot
                // without a helper; else leave.  A slot's owner announces its passes while the
                // slot is not done and waits for each share, so a detach never strands a pass.
                int go = 0, att = 0;
                if (lane == 0) {
                    att = sh.hAtt[w];
                    int seen = sh.hSeen[w];
                    for (;;) {
                        if (att >= 0) {
                            if (lds_load_acq(&sh.annSeq[att]) > seen) {
                                seen++;
                                hBase = sh.annBase[att];
                                go = 1;
                                break;
                            }
                            if (lds_load_acq(&sh.done[att])) {
                                att = -1;
                                continue;
                            }
                            if ((long long)(wall_clock64() - tStart) > p.maxTicks) break;
                            __builtin_amdgcn_s_sleep(2);
                            continue;
                        }
                        for (int s = 0; s < kW && att < 0; s++)
                            if (s != w && !lds_load_acq(&sh.done[s]) && lds_load_acq(&sh.helper[s]) == 0 &&
                                atomicCAS(&sh.helper[s], 0, 1) == 0) {
                                att = s;
                                seen = 0;  // a slot announces to its first and only helper
                            }
                        if (att < 0) break;
                    }
                    sh.hAtt[w] = att;
                    sh.hSeen[w] = seen;
                }
                if (!rfl(go)) break;
                att = rfl(att);
                hBase = rfl(hBase);
                own = false;
                if (prod.w != att) {
                    prod.w = att;
                    prod.cmin = 0;
                }
            }
            const int tw = prod.w;
            SlotP2& SP = sh.sp[tw];
            SlotS2& SS = sh.ss[tw];
            const int pass = rfl(SP.pass);
            if (own && pass == Q_DONE) {
                if (!p.coop) break;
                if (lane == 0) {
                    lds_store_rel(&sh.done[w], 1);
                    sh.hAtt[w] = -1;  // enter the helper branch above
                }
                continue;
            }
            if (lane == 0) WS.t0 = clock64();
            const int len = rfl(SP.len);
            const int nCh = (len + kE - 1) / kE;
            int cls = 3;
            if (pass == Q_INIT) {
                // ---- extractPixelsContour(Vec2d) (:341-374): keep 0 <= p < (boundW, boundH) in
                // offset order -> compact entries; undistorted rays (get3dPointsFromImage1Pixels :542)
                // (the slab views are re-read from LDS here: held across the loop they would take
                // 14 scalar registers)
                const Slab sl2 = ctl.sl;
                const double ccx = SP.ccx, ccy = SP.ccy;
                int base = 0;
                for (int k = 0; k < nCh; k++) {
                    const int e = k * kE + lane;
                    const long long o2 = offsets[e];
                    const double px = ccx + (double)(int)o2, py = ccy + (double)(int)(o2 >> 32);
                    const bool v = !(px < 0 || py < 0 || px >= p.boundW || py >= p.boundH);
                    const unsigned long long bm = __ballot(v);
                    if (v) {
                        const int pos = base + __popcll(bm & ltMask);
                        double ux, uy;
                        undistort1(p.cam, px, py, ux, uy);
#if FM3D_RAY_AOS
                        *(gd2v*)(sl2.RX + 2 * pos) = d2v{ux, uy};
#else
                        sl2.RX[pos] = ux;
                        sl2.RY[pos] = uy;
#endif
                        sl2.KI[pos] = e;
                    }
                    base += __popcll(bm);
                }
                if (lane == 0) OUT.cnt = base;
            } else if (pass == Q_LEVEL) {
                // ---- updateImage1PixelsIntensity (:576-589)
                const Slab sl2 = ctl.sl;
                const double ccx = SP.ccx, ccy = SP.ccy, scale = SP.scale, xmax = SP.xmax, ymax = SP.ymax;
                const gu8* img1 = (const gu8*)SP.img1;
                const int lw = rfl(SP.lw);
                bool bad = false;
                for (int k = 0; k < nCh; k++) {
                    const int e = k * kE + lane;
                    if (e < len) {
                        const long long o2 = offsets[sl2.KI[e]];
                        const double px = ccx + (double)(int)o2, py = ccy + (double)(int)(o2 >> 32);
                        if (!pixel_good_b(px, py, xmax, ymax)) {
                            bad = true;
                        } else {
                            const float fx = (float)(scale * px), fy = (float)(scale * py);
                            const gu8* g = img1 + (long)(int)floorf(fy) * lw + (int)floorf(fx);
                            sl2.I1[e] = bilinear4(g[0], g[1], g[lw], g[lw + 1], fx, fy);
                        }
                    }
                }
                const bool anyBad = __ballot(bad) != 0;
                if (lane == 0) OUT.i1fail = anyBad ? 1 : 0;
            } else {
                // ---- a summed pass: terms here, sums by the chain lanes
                // chunk k of the pass is the slot's chunk cbase + k.  Split with a helper: the
                // owner computes chunks 0, 2, 4, ..., the helper 1, 3, 5, ... (k0, kS)
                int cbase = hBase, k0 = 1, kS = 2;
                if (own) {
                    passId++;
                    if (lane == 0) WS.nPass++;
                    cbase = chunkSeq;
                    chunkSeq = cbase + nCh;
                    k0 = 0;
                    kS = (p.coop && rfl(lds_load_acq(&sh.helper[w])) != 0) ? 2 : 1;  // 2: split
                }
                cbase = rfl(cbase);
                k0 = rfl(k0);
                kS = rfl(kS);
                const unsigned s8 = (unsigned)(((size_t)blockIdx.x * NS + tw) * p.nOffPad * 8);  // slot tw's, < 2^32 (host-checked)
                const int ekind = rfl(SP.ekind);
                const int nev = rfl(SP.nev);
                const bool jac = pass == Q_EVAL && ekind == E_JAC;
                cls = jac ? 0 : (pass == Q_EVAL ? 1 : 2);
                const double agiant = SP.agiant;
                if (!TREE && own && lane == 0) {
                    PassDesc& d = sh.pd[w];
                    d.nChunks = nCh;
                    d.id = passId;
                    d.agiant = agiant;
                    d.kind[0] = (pass == Q_QR1 || pass == Q_QR3) ? S_DOT : S_ENORM;
                    d.kind[1] = pass == Q_QR1 ? S_DOT : ((pass == Q_EVAL && nev == 2) ? S_ENORM : S_NONE);
                    if (kS == 2) {  // SP, SS and the pass descriptor are written: announce
                        sh.annBase[w] = cbase;
                        sh.annId[w] = passId;
                        lds_store_rel(&sh.annSeq[w], ++sh.hAnn[w]);
                    }
                }
                int fail0 = 0x7fffffff, fail1 = 0x7fffffff;
                int ph30 = 0, ph31 = 0;  // image-2 failures seen (wave-uniform flags)
                double aqs1 = 0.;
                // TREE: the lane's partial sums of the pass (entries 64 k + lane in chunk order) and
                // the wave-uniform enorm slow flags of sums 0 / 1
                double ta0 = 0., ta1 = 0., ta2 = 0., ta3 = 0., ta4 = 0.;
                bool tslow0 = false, tslow1 = false;
                if (pass == Q_EVAL) {
                    const double n00 = SP.n0[0], n10 = SP.n1[0], n20 = SP.n2[0], mm0 = SP.mm[0], w0 = SP.w[0];
                    const double n01 = SP.n0[1], n11 = SP.n1[1], n21 = SP.n2[1], mm1 = SP.mm[1], w1 = SP.w[1];
                    const double h0 = SP.hj[0], h1 = SP.hj[1], wF = SP.wF;
                    const double y0 = 1. / h0, y1 = 1. / h1;
                    const bool mok0 = mdiv_ok(h0), mok1 = mdiv_ok(h1);
                    const double scale = SP.scale;
                    const unsigned long long xmaxb = (unsigned long long)__double_as_longlong(SP.xmax);
                    const unsigned long long ymaxb = (unsigned long long)__double_as_longlong(SP.ymax);
                    const uint8_t* img2 = SP.img2;
                    const int lw = rfl(SP.lw);
                    const unsigned projOff = MULTI ? (unsigned)rfl((int)SP.projOff) : 0u;
                    const bool i1ok = rfl(SS.i1ok) != 0;
                    const gu8* img2b = (const gu8*)rfl_ptr(img2);
                    // The fast form (FAST): the ray-plane quotients take div_nn's fast sequence
                    // (div_nn_ok of the pass's numerators) and the JAC divisions by h_j have no
                    // per-lane guard.  The latter holds because the divided numerators of good
                    // pixels, w_j*dI_j - wF*dI_F, combine samples in [0, 255] (|dI| < 256) with the
                    // pass-uniform weights; other lanes are zeroed after the division.
                    const bool fast = !p.safe && div_nn_ok(mm0) && (nev < 2 || div_nn_ok(mm1)) &&
                                      (!jac || (mok0 && 256. * 1.01 * (w0 + wF) < 1e99 &&
                                                (nev < 2 || (mok1 && 256. * 1.01 * (w1 + wF) < 1e99))));
                    // the slab bases, once per pass (scalar registers; used where FM3D_EVAL_HOIST)
#ifndef FM3D_EVAL_HOIST
#define FM3D_EVAL_HOIST 1
#endif
                    struct SlabB {
                        const char *slabRX, *slabRY, *slabI1;
                        char *slabDF, *slabDJ0, *slabDJ1;
                    };
                    const SlabB sbh = [&] {
                        const cProjConst* q = proj_consts(p.proj);
                        return SlabB{q->slabRX, q->slabRY, q->slabI1, q->slabDF, q->slabDJ0, q->slabDJ1};
                    }();
                    // NEV evaluations per entry (2: both forward-difference columns); JAC: the
                    // values are Jacobian columns (r - fvec)/h_j, else the residual fvec itself
                    auto run = [&](auto nevc, auto jacc, auto fastc) {
                        constexpr int NEV = decltype(nevc)::value;
                        constexpr bool JAC = decltype(jacc)::value;
                        constexpr bool FAST = decltype(fastc)::value;
                        // hoisted bases in the single-evaluation passes; the Jacobian passes,
                        // short of scalar registers, re-read them (hoisted there, they spill)
                        auto sb = [&]() {
                            if constexpr (FM3D_EVAL_HOIST && !JAC)
                                return &sbh;
                            else
                                return proj_consts(p.proj);
                        };
                        struct Ld {
                            double ux, uy, dF;
                            float i1;
                        };
                        auto geo = [&](double ux, double uy, double n0, double n1, double n2, double mm) {
                            return FAST ? geometry2<true, MULTI>(p, projOff, ux, uy, n0, n1, n2, mm, scale, xmaxb,
                                                                 ymaxb, lw, cm)
                                        : geometry2<false, MULTI>(p, projOff, ux, uy, n0, n1, n2, mm, scale, xmaxb,
                                                                  ymaxb, lw, cm);
                        };
                        auto jdiv = [&](double a, double h, double y, bool mok) {
                            return FAST ? mdiv_fast(a, h, y) : mdiv(a, h, y, mok);
                        };
                        // o8 / o4: byte offsets of the chunk's entries in the 8- / 4-byte slab arrays.
                        // Entries past len (up to three chunks past the pass) read slab padding.  The
                        // slab streams are read once per pass (nontemporal: they leave L2 to the
                        // image gathers).
                        auto load = [&](unsigned o8, unsigned o4) {
                            const auto* pc = sb();
                            Ld L;
#if FM3D_RAY_AOS
                            // the entry's (ux, uy) record: one 16-byte load (byte offset 2 * o8)
                            const d2v r = __builtin_nontemporal_load((const gd2v*)(pc->slabRX + 2 * o8));
                            L.ux = r.x;
                            L.uy = r.y;
#else
                            L.ux = __builtin_nontemporal_load((const gdouble*)(pc->slabRX + o8));
                            L.uy = __builtin_nontemporal_load((const gdouble*)(pc->slabRY + o8));
#endif
                            L.i1 = __builtin_nontemporal_load((const gfloat*)(pc->slabI1 + o4));
                            L.dF = JAC ? (double)__builtin_nontemporal_load((const gfloat*)(pc->slabDF + o4)) : 0.;
                            return L;
                        };
                        auto gather = [&](unsigned off) {  // two byte pairs: (y0, x0..x0+1), (y0+1, ...)
                            return make_uint2(*(const gu16u*)(img2b + off), *(const gu16u*)(img2b + (off + lw)));
                        };
                        auto chunk = [&](const Ld& L, int k, unsigned o4) {
                            if constexpr (!TREE) prod.reserve(cbase + k);
                            const LaneMask in = in_mask(k, len), ok = i1ok ? in : 0ull;
                            const Geo2 g0 = geo(L.ux, L.uy, n00, n10, n20, mm0);
                            Geo2 g1;
                            if (NEV == 2) g1 = geo(L.ux, L.uy, n01, n11, n21, mm1);
                            // gathers for every lane: a failed entry reads the image's first bytes
                            const uint2 a = gather(g0.off);
                            uint2 c;
                            if (NEV == 2) c = gather(g1.off);
                            // failures: first NaN-plane / bounding-box pixel in index order; image-2 flags
                            {
                                const LaneMask b0 = in & ~g0.inbox;
                                if (b0 && fail0 == 0x7fffffff) {
                                    const int l = __ffsll((long long)b0) - 1;
                                    const int cd = plane_code(L.ux, L.uy, n00, n10, n20, mm0);
                                    fail0 = (k * kE + l) * 4 + __shfl(cd, l);
                                }
                                ph30 |= (in & g0.inbox & ~g0.good) != 0;
                                if (NEV == 2) {
                                    const LaneMask b1 = in & ~g1.inbox;
                                    if (b1 && fail1 == 0x7fffffff) {
                                        const int l = __ffsll((long long)b1) - 1;
                                        const int cd = plane_code(L.ux, L.uy, n01, n11, n21, mm1);
                                        fail1 = (k * kE + l) * 4 + __shfl(cd, l);
                                    }
                                    ph31 |= (in & g1.inbox & ~g1.good) != 0;
                                }
                            }
                            // evaluateNormal :145-148 (fvec), fdjac2 forward differences (JAC)
                            const float dI0 = L.i1 - bilinear_w(a.x, a.y, g0.fx, g0.fy);
                            const double r0 = w0 * (double)dI0;
                            double v0 = JAC ? jdiv(r0 - wF * L.dF, h0, y0, mok0) : r0;
                            v0 = sel_mask(v0, ok & g0.good);
                            {
                                const auto* pc = sb();
                                *(gfloat*)((JAC ? pc->slabDJ0 : pc->slabDF) + o4) = dI0;
                            }
                            bool slow0 = false, slow1 = false;
                            const double t0 = enorm_term2(v0, agiant, slow0);
                            double v1 = 0., t1 = 0.;
                            if (NEV == 2) {
                                const float dI1 = L.i1 - bilinear_w(c.x, c.y, g1.fx, g1.fy);
                                const double r1 = w1 * (double)dI1;
                                v1 = jdiv(r1 - wF * L.dF, h1, y1, mok1);
                                v1 = sel_mask(v1, ok & g1.good);
                                *(gfloat*)(sb()->slabDJ1 + o4) = dI1;
                                t1 = enorm_term2(v1, agiant, slow1);
                            }
                            if constexpr (TREE) {
                                if (!JAC) {  // the Jacobian's sums come from the Q_GRAM sweep
                                    ta0 += t0;
                                    tslow0 |= slow0;
                                }
                            } else {
                                prod.write_terms<NEV == 2>(cbase + k, t0, v0, slow0, t1, v1, slow1);
                            }
                        };
                        // this wave's chunks: k0, k0 + kS, ...; st8 / st4: the offset step between them
                        unsigned o8 = s8 + lane * 8u + (unsigned)k0 * 512u, o4 = o8 >> 1;
                        const unsigned st8 = (unsigned)kS * 512u, st4 = st8 >> 1;
                        if (NEV == 2 && FM3D_EVAL_PIPE) {
                            // both forward-difference columns of a chunk side by side (their
                            // geometries interleave), software-pipelined: chunk k + 1's geometries and
                            // gathers are computed while chunk k's gathers are in flight, then chunk
                            // k's samples and terms; unrolled by two chunks so that the stages
                            // alternate without copies.  Failures are taken in entry order.
                            struct St2 {
                                float xf0, yf0, xf1, yf1, i1, dF;
                                uint2 a, c;
                                LaneMask ok0, ok1;  // in & i1ok & good, per column
                            };
                            auto front2 = [&](const Ld& L, int k) {
                                const LaneMask in = in_mask(k, len), ok = i1ok ? in : 0ull;
                                const Geo2 g0 = geo(L.ux, L.uy, n00, n10, n20, mm0);
                                const Geo2 g1 = geo(L.ux, L.uy, n01, n11, n21, mm1);
                                St2 S;
                                S.a = gather(g0.off);  // every lane: a failed entry reads the image's first bytes
                                S.c = gather(g1.off);
                                const LaneMask b0 = in & ~g0.inbox;
                                if (b0 && fail0 == 0x7fffffff) {
                                    const int l = __ffsll((long long)b0) - 1;
                                    const int cd = plane_code(L.ux, L.uy, n00, n10, n20, mm0);
                                    fail0 = (k * kE + l) * 4 + __shfl(cd, l);
                                }
                                ph30 |= (in & g0.inbox & ~g0.good) != 0;
                                const LaneMask b1 = in & ~g1.inbox;
                                if (b1 && fail1 == 0x7fffffff) {
                                    const int l = __ffsll((long long)b1) - 1;
                                    const int cd = plane_code(L.ux, L.uy, n01, n11, n21, mm1);
                                    fail1 = (k * kE + l) * 4 + __shfl(cd, l);
                                }
                                ph31 |= (in & g1.inbox & ~g1.good) != 0;
                                S.xf0 = g0.fx - floorf(g0.fx);  // the bilinear fractions
                                S.yf0 = g0.fy - floorf(g0.fy);
                                S.xf1 = g1.fx - floorf(g1.fx);
                                S.yf1 = g1.fy - floorf(g1.fy);
                                S.i1 = L.i1;
                                S.dF = (float)L.dF;  // a float value: exact
                                S.ok0 = ok & g0.good;
                                S.ok1 = ok & g1.good;
                                return S;
                            };
                            auto back2 = [&](const St2& S, int k, unsigned oo) {
                                // evaluateNormal :145-148, fdjac2 forward differences
                                const float dI0 = S.i1 - bilinear_f(S.a.x, S.a.y, S.xf0, S.yf0);
                                const float dI1 = S.i1 - bilinear_f(S.c.x, S.c.y, S.xf1, S.yf1);
                                if constexpr (TREE) {
                                    // the columns' values and sums come from the Q_GRAM sweep
                                    const auto* pc = sb();
                                    *(gfloat*)(pc->slabDJ0 + oo) = dI0;
                                    *(gfloat*)(pc->slabDJ1 + oo) = dI1;
                                    return;
                                }
                                const double F = wF * (double)S.dF;
                                double v0 = jdiv(w0 * (double)dI0 - F, h0, y0, mok0);
                                double v1 = jdiv(w1 * (double)dI1 - F, h1, y1, mok1);
                                v0 = sel_mask(v0, S.ok0);
                                v1 = sel_mask(v1, S.ok1);
                                bool slow0, slow1;
                                const double t0 = enorm_term2(v0, agiant, slow0);
                                const double t1 = enorm_term2(v1, agiant, slow1);
                                prod.reserve(cbase + k);
                                {
                                    const auto* pc = sb();
                                    *(gfloat*)(pc->slabDJ0 + oo) = dI0;
                                    *(gfloat*)(pc->slabDJ1 + oo) = dI1;
                                }
                                prod.write_terms<true>(cbase + k, t0, v0, slow0, t1, v1, slow1);
                            };
                            // A stage past the last chunk computes garbage from slab padding (its
                            // entries are not `in`: no failures); no branch between gathers and use
                            Ld A = load(o8, o4), B = load(o8 + st8, o4 + st4);
                            St2 S = front2(A, k0), N;
                            A = load(o8 + 2 * st8, o4 + 2 * st4);
                            for (int k = k0; k < nCh; k += 2 * kS) {
                                N = front2(B, k + kS);
                                B = load(o8 + 3 * st8, o4 + 3 * st4);
                                back2(S, k, o4);
                                if (k + kS >= nCh) break;  // wave-uniform
                                S = front2(A, k + 2 * kS);
                                A = load(o8 + 4 * st8, o4 + 4 * st4);
                                back2(N, k + kS, o4 + st4);
                                o8 += 2 * st8;
                                o4 += 2 * st4;
                            }
                        } else if (NEV == 2) {
                            // (the unpipelined form, FM3D_EVAL_PIPE=0)
                            // two chunks of slab loads in flight ahead of the one being computed
                            Ld A = load(o8, o4), B = load(o8 + st8, o4 + st4);
                            for (int k = k0; k < nCh; k += 2 * kS) {
                                const Ld C = load(o8 + 2 * st8, o4 + 2 * st4);
                                chunk(A, k, o4);
                                A = C;
                                if (k + kS < nCh) {
                                    const Ld D = load(o8 + 3 * st8, o4 + 3 * st4);
                                    chunk(B, k + kS, o4 + st4);
                                    B = D;
                                }
                                o8 += 2 * st8;
                                o4 += 2 * st4;
                            }
                        } else if (FM3D_EVAL_PIPE) {
                            // one evaluation per entry: two chunks side by side (their geometries
                            // interleave), software-pipelined: the geometry and the image-2 gathers
                            // of pair p + 1 are computed while pair p's gathers are in flight, then
                            // pair p's samples, residuals and terms.  Failures are still taken in
                            // entry order (pair p's in the previous iteration).
                            struct St {
                                float fxA, fyA, fxB, fyB, i1A, i1B, dFA, dFB;
                                uint2 a, b;
                                LaneMask okA, okB;  // in & i1ok & good
                            };
                            auto front = [&](const Ld& A, const Ld& B, int k) {
                                const int kB = k + kS;
                                const LaneMask inA = in_mask(k, len), inB = in_mask(kB, len);
                                const Geo2 gA = geo(A.ux, A.uy, n00, n10, n20, mm0);
                                // past the last chunk B holds slab padding: its entries are not
                                // `in`, its gathers read the image's first bytes, nothing is stored
                                const Geo2 gB = geo(B.ux, B.uy, n00, n10, n20, mm0);
                                St S;
                                S.a = gather(gA.off);
                                S.b = gather(gB.off);
                                const LaneMask bA = inA & ~gA.inbox;
                                const LaneMask bB = inB & ~gB.inbox;
                                if ((bA | bB) && fail0 == 0x7fffffff) {
                                    const bool first = bA != 0;
                                    const int l = __ffsll((long long)(first ? bA : bB)) - 1;
                                    const int cd = first ? plane_code(A.ux, A.uy, n00, n10, n20, mm0)
                                                         : plane_code(B.ux, B.uy, n00, n10, n20, mm0);
                                    fail0 = ((first ? k : kB) * kE + l) * 4 + __shfl(cd, l);
                                }
                                ph30 |= ((inA & gA.inbox & ~gA.good) | (inB & gB.inbox & ~gB.good)) != 0;
                                S.fxA = gA.fx - floorf(gA.fx);  // the bilinear fractions (the floors are the geometry's)
                                S.fyA = gA.fy - floorf(gA.fy);
                                S.fxB = gB.fx - floorf(gB.fx);
                                S.fyB = gB.fy - floorf(gB.fy);
                                S.i1A = A.i1;
                                S.i1B = B.i1;
                                S.dFA = (float)A.dF;  // a float value: exact
                                S.dFB = (float)B.dF;
                                S.okA = (i1ok ? inA : 0ull) & gA.good;
                                S.okB = (i1ok ? inB : 0ull) & gB.good;
                                return S;
                            };
                            // the residual / Jacobian value of one chunk of the stage (the samples wait
                            // for the stage's gathers)
                            auto value = [&](float xf, float yf, uint2 w, float i1, float dF, LaneMask ok, float& dI) {
                                dI = i1 - bilinear_f(w.x, w.y, xf, yf);
                                const double r = w0 * (double)dI;
                                const double v = JAC ? jdiv(r - wF * (double)dF, h0, y0, mok0) : r;
                                return sel_mask(v, ok);
                            };
                            auto publish = [&](double v, float dI, unsigned oo, int kk) {
                                {
                                    const auto* pc = sb();
                                    *(gfloat*)((JAC ? pc->slabDJ0 : pc->slabDF) + oo) = dI;
                                }
                                bool slow;
                                const double t = enorm_term2(v, agiant, slow);
                                if constexpr (TREE) {
                                    ta0 += t;
                                    tslow0 |= slow;
                                } else {
                                    prod.write_terms<false>(cbase + kk, t, v, slow, 0., 0., false);
                                }
                            };
                            // both chunks' values first (no branch between the gathers and their
                            // use), then the ring space, then the stores of the chunks that exist
                            auto back = [&](const St& S, int k, unsigned oo) {
                                const int kB = k + kS;
                                const bool two = kB < nCh;  // wave-uniform
                                float dIA, dIB;
                                const double vA = value(S.fxA, S.fyA, S.a, S.i1A, S.dFA, S.okA, dIA);
                                const double vB = value(S.fxB, S.fyB, S.b, S.i1B, S.dFB, S.okB, dIB);
                                if constexpr (!TREE) prod.reserve(cbase + (two ? kB : k));  // space for both chunks
                                publish(vA, dIA, oo, k);
                                if (two) publish(vB, dIB, oo + st4, kB);
                            };
                            // unrolled by two pairs, so that the stages alternate without copies.
                            // A stage past the last chunk computes garbage from slab padding and
                            // the image's first bytes (its entries are not `in`: no failures, no
                            // stores); it keeps the loop free of branches between gathers and use.
                            Ld A = load(o8, o4), B = load(o8 + st8, o4 + st4);
                            St S = front(A, B, k0), N;
                            A = load(o8 + 2 * st8, o4 + 2 * st4);
                            B = load(o8 + 3 * st8, o4 + 3 * st4);
                            for (int k = k0; k < nCh; k += 4 * kS) {
                                N = front(A, B, k + 2 * kS);
                                A = load(o8 + 4 * st8, o4 + 4 * st4);
                                B = load(o8 + 5 * st8, o4 + 5 * st4);
                                back(S, k, o4);
                                if (k + 2 * kS >= nCh) break;  // wave-uniform
                                S = front(A, B, k + 4 * kS);
                                A = load(o8 + 6 * st8, o4 + 6 * st4);
                                B = load(o8 + 7 * st8, o4 + 7 * st4);
                                back(N, k + 2 * kS, o4 + 2 * st4);
                                o8 += 4 * st8;
                                o4 += 4 * st4;
                            }
                        } else {
                            // (the unpipelined form, FM3D_EVAL_PIPE=0)
                            // one evaluation per entry: two chunks side by side, so the two
                            // independent geometries interleave (as the two columns of a Jacobian
                            // pass do); the slab loads of the next pair are issued once the pair's
                            // geometry has consumed its own
                            Ld A = load(o8, o4), B = load(o8 + st8, o4 + st4);
                            for (int k = k0; k < nCh; k += 2 * kS) {
                                const int kB = k + kS;
                                const bool two = kB < nCh;  // wave-uniform
                                if constexpr (!TREE) prod.reserve(cbase + (two ? kB : k));  // space for both chunks
                                const LaneMask inA = in_mask(k, len), inB = in_mask(kB, len);
                                const Geo2 gA = geo(A.ux, A.uy, n00, n10, n20, mm0);
                                // past the last chunk B holds slab padding: its entries are not
                                // `in`, its gathers read the image's first bytes, nothing is stored
                                const Geo2 gB = geo(B.ux, B.uy, n00, n10, n20, mm0);
                                const uint2 a = gather(gA.off), b = gather(gB.off);
                                const float i1A = A.i1, i1B = B.i1;
                                const double dFA = A.dF, dFB = B.dF;
                                // failures in entry order: chunk k before chunk k + 1
                                const LaneMask bA = inA & ~gA.inbox;
                                const LaneMask bB = inB & ~gB.inbox;
                                if ((bA | bB) && fail0 == 0x7fffffff) {
                                    const bool first = bA != 0;
                                    const int l = __ffsll((long long)(first ? bA : bB)) - 1;
                                    const int cd = first ? plane_code(A.ux, A.uy, n00, n10, n20, mm0)
                                                         : plane_code(B.ux, B.uy, n00, n10, n20, mm0);
                                    fail0 = ((first ? k : kB) * kE + l) * 4 + __shfl(cd, l);
                                }
                                ph30 |= ((inA & gA.inbox & ~gA.good) | (inB & gB.inbox & ~gB.good)) != 0;
                                A = load(o8 + 2 * st8, o4 + 2 * st4);
                                B = load(o8 + 3 * st8, o4 + 3 * st4);
                                auto back1 = [&](const Geo2& g, uint2 w, float i1, double dF, LaneMask in, unsigned oo, int kk) {
                                    const float dI = i1 - bilinear_w(w.x, w.y, g.fx, g.fy);
                                    const double r = w0 * (double)dI;
                                    double v = JAC ? jdiv(r - wF * dF, h0, y0, mok0) : r;
                                    v = sel_mask(v, (i1ok ? in : 0ull) & g.good);
                                    {
                                        const auto* pc = sb();
                                        *(gfloat*)((JAC ? pc->slabDJ0 : pc->slabDF) + oo) = dI;
                                    }
                                    bool slow;
                                    const double t = enorm_term2(v, agiant, slow);
                                    if constexpr (TREE) {
                                        ta0 += t;
                                        tslow0 |= slow;
                                    } else {
                                        prod.write_terms<false>(cbase + kk, t, v, slow, 0., 0., false);
                                    }
                                };
                                back1(gA, a, i1A, dFA, inA, o4, k);
                                if (two) back1(gB, b, i1B, dFB, inB, o4 + st4, kB);
                                o8 += 2 * st8;
                                o4 += 2 * st4;
                            }
                        }
                    };
                    using I1 = std::integral_constant<int, 1>;
                    using I2 = std::integral_constant<int, 2>;
                    using T = std::true_type;
                    using F = std::false_type;
                    if (fast) {
                        if (nev == 2)
                            run(I2(), T(), T());
                        else if (jac)
                            run(I1(), T(), T());
                        else
                            run(I1(), F(), T());
                    } else {
                        if (nev == 2)
                            run(I2(), T(), F());
                        else if (jac)
                            run(I1(), T(), F());
                        else
                            run(I1(), F(), F());
                    }
                } else {
                    // ---- Householder passes (qrfac / lmdif qtf for n = 2) on the stored columns
                    const int pc = rfl(SP.pivot), t0f = rfl(SP.t0), t1f = rfl(SP.t1), q0f = rfl(SP.q0);
                    const double wF = SP.wF, wp = SP.w[pc], wq = SP.w[1 - pc], hp = SP.hj[pc], hq = SP.hj[1 - pc];
                    const double yp = 1. / hp, yq = 1. / hq;
                    const bool mokp = mdiv_ok(hp), mokq = mdiv_ok(hq);
                    const double ajn0s = SP.ajn0s, ya0 = 1. / ajn0s, tq = SP.tq;
                    const bool moka0 = mdiv_ok(ajn0s);
                    const double ajn1s = SP.ajn1s, ya1 = 1. / ajn1s, tq0 = SP.tq0;
                    const bool moka1 = mdiv_ok(ajn1s);
                    // The fast form: no per-lane guard in mdiv and no flag selects.  A pass runs only
                    // after evaluations whose every kept pixel was good, so each stored dI (in-range
                    // entries) is a difference of two samples in [0, 255]: |dI| < 256.  The numerators
                    // are then bounded by the pass-uniform weights, and within these bounds every
                    // quotient the pass forms stays below mdiv's 1e100 (the 1.01 covers the roundings).
                    // Entries past len compute garbage the edge chunks zero.
                    const double bnum = 256. * 1.01 * (wp + wq + 2. * wF);
                    const double bap = bnum / fabs(hp), baq = bnum / fabs(hq);
                    // (Q_GRAM: the columns themselves, no Householder quotient)
                    bool fast = !p.safe && t0f && q0f && mokp && mokq && moka0 && bnum < 1e99 && bap < 1e99 &&
                                baq < 1e99 && (pass != Q_QR3 || (t1f && moka1 &&
                                baq + fabs(tq) * (bap / fabs(ajn0s) + 1.) < 1e99));
                    if constexpr (TREE)
                        if (pass == Q_GRAM) fast = !p.safe && mokp && mokq && bnum < 1e99 && bap < 1e99 && baq < 1e99;
                    auto run = [&](auto kindc, auto fastc) {
                        constexpr int KIND = decltype(kindc)::value;
                        constexpr bool FAST = decltype(fastc)::value;
                        struct Ld {
                            float p, q, f;
                        };
                        // o4: byte offset of the chunk's entries in the 4-byte slab arrays
#ifndef FM3D_QR_HOIST
#define FM3D_QR_HOIST 1
#endif
#if FM3D_QR_HOIST
                        // the three slab bases once per pass (scalar registers; the per-chunk
                        // re-read cost a dozen scalar instructions per chunk)
                        const cProjConst* pcs0 = proj_consts(p.proj);
                        const char* const Dp0 = pc ? pcs0->slabDJ1 : pcs0->slabDJ0;
                        const char* const Dq0 = pc ? pcs0->slabDJ0 : pcs0->slabDJ1;
                        const char* const Df0 = pcs0->slabDF;
#endif
                        auto load = [&](unsigned o4) {
#if FM3D_QR_HOIST
                            const char* Dp = Dp0;
                            const char* Dq = Dq0;
                            struct {
                                const char* slabDF;
                            } s0{Df0}, *pcs = &s0;
#else
                            const cProjConst* pcs = proj_consts(p.proj);
                            const char* Dp = pc ? pcs->slabDJ1 : pcs->slabDJ0;
                            const char* Dq = pc ? pcs->slabDJ0 : pcs->slabDJ1;
#endif
                            Ld L;
                            L.p = __builtin_nontemporal_load((const gfloat*)(Dp + o4));
                            L.q = __builtin_nontemporal_load((const gfloat*)(Dq + o4));
                            L.f = __builtin_nontemporal_load((const gfloat*)(pcs->slabDF + o4));  // J = (w_j dI_j - F) / h_j needs F
                            return L;
                        };
                        auto dv = [&](double a, double d, double y, bool mok) {
                            return FAST ? mdiv_fast(a, d, y) : mdiv(a, d, y, mok);
                        };
                        // EDGE: the first or the last chunk (the diagonal entries 0 and 1, entries
                        // past len); every other chunk skips those tests
                        struct Terms {
                            double t0, t1, a;  // a: QR2's raw value, published instead of t0 if slow
                            bool slow;
                            double g0, g1, g2;  // Q_GRAM: a_0.a_1, a_0.f, a_1.f terms (t0, t1: a_0^2, a_1^2)
                            bool slow1;
                        };
                        auto chunk = [&](const Ld& L, int k, auto edgec) {
                            constexpr bool EDGE = decltype(edgec)::value;
                            const int e = k * kE + lane;
                            const bool in = e < len;
                            // the stored columns: F = wF*dI_F, J_j = (w_j*dI_j - F)/h_j (as the JAC pass)
                            const double F = wF * (double)L.f;
                            const double ap = dv(wp * (double)L.p - F, hp, yp, mokp);
                            const double aq = dv(wq * (double)L.q - F, hq, yq, mokq);
                            double t0 = 0., t1 = 0., a = 0., g0 = 0., g1 = 0., g2 = 0.;
                            bool slow = false, slow1 = false;
                            if constexpr (KIND == Q_GRAM) {
                                // the columns (pivot 0: ap = a_0, aq = a_1), their squares (enorm) and
                                // the Gram sums of start_qr_tree; entries past len add +0
                                const double a0 = (EDGE && !in) ? 0. : ap, a1 = (EDGE && !in) ? 0. : aq;
                                const double f = (EDGE && !in) ? 0. : F;
                                t0 = enorm_term2(a0, agiant, slow);
                                t1 = enorm_term2(a1, agiant, slow1);
                                g0 = a0 * a1;
                                g1 = a0 * f;
                                g2 = a1 * f;
                            } else if constexpr (KIND == Q_QR1) {
                                // qrfac column j = 0: v = a_p / ajnorm (+1 on the diagonal); v*a_q, v*f
                                double v = dv(ap, ajn0s, ya0, moka0);
                                if (EDGE && e == 0) v = v + 1.;
                                t0 = v * aq;
                                t1 = v * F;
                                if (EDGE && !in) t0 = t1 = 0.;
                            } else if constexpr (KIND == Q_QR2) {
                                // a_q' = a_q - temp * v below the diagonal -> ajnorm of column 1
                                a = aq;
                                if (FAST || t0f) a = a - tq * dv(ap, ajn0s, ya0, moka0);
                                if (EDGE) {
                                    a = (in && e > 0) ? a : 0.;
                                    if (e == 1) aqs1 = a;
                                }
                                t0 = enorm_term2(a, agiant, slow);
                            } else {
                                // lmdif qtf, j = 1: u_i * wa4_i
                                const double v = (FAST || t0f) ? dv(ap, ajn0s, ya0, moka0) : 0.;
                                double b = aq;
                                if (FAST || t0f) b = b - tq * v;
                                double u = (FAST || t1f) ? dv(b, ajn1s, ya1, moka1) : b;
                                if (EDGE && (FAST || t1f) && e == 1) u = u + 1.;
                                double wa = F;
                                if (FAST || q0f) wa = wa + v * tq0;
                                t0 = u * wa;
                                if (EDGE && !(in && e > 0)) t0 = 0.;
                            }
                            return Terms{t0, t1, a, slow, g0, g1, g2, slow1};
                        };
                        // kQD chunks of loads in flight: this pass computes little per entry.  A
                        // buffer is refilled after its chunk is consumed (no register copies)
#ifndef FM3D_QR_DEPTH
#define FM3D_QR_DEPTH 8
#endif
                        constexpr int kQD = FM3D_QR_DEPTH;
                        unsigned o4 = (s8 >> 1) + lane * 4u + (unsigned)k0 * 256u;
                        const unsigned st4 = (unsigned)kS * 256u;
                        Ld buf[kQD];
#pragma unroll
                        for (int j = 0; j < kQD; j++) {
                            buf[j] = load(o4);
                            o4 += st4;
                        }
                        // o4: the prefetch offset, kQD chunks ahead (one running offset keeps the
                        // per-chunk offsets out of the scalar registers)
                        for (int k = k0; k < nCh; k += kQD * kS) {
#pragma unroll
                            for (int j = 0; j < kQD; j++) {
                                const int kc = k + j * kS;
                                if (kc < nCh) {
                                    const Terms T = (kc == 0 || kc == nCh - 1) ? chunk(buf[j], kc, std::true_type())
                                                                               : chunk(buf[j], kc, std::false_type());
                                    if constexpr (TREE) {
                                        ta0 += T.t0;
                                        if (KIND == Q_QR1 || KIND == Q_GRAM) ta1 += T.t1;
                                        if (KIND == Q_GRAM) {
                                            ta2 += T.g0;
                                            ta3 += T.g1;
                                            ta4 += T.g2;
                                            tslow1 |= T.slow1;
                                        }
                                        tslow0 |= T.slow;
                                    } else {
                                        prod.reserve(cbase + kc);
                                        prod.write_terms<KIND == Q_QR1>(cbase + kc, T.t0, T.a, T.slow, T.t1, 0., false);
                                    }
                                    buf[j] = load(o4);
                                }
                                o4 += st4;
                            }
                        }
                    };
                    if (TREE && pass == Q_GRAM) {
                        if constexpr (TREE) {
                            if (fast)
                                run(std::integral_constant<int, Q_GRAM>(), std::true_type());
                            else
                                run(std::integral_constant<int, Q_GRAM>(), std::false_type());
                        }
                    } else if (fast) {
                        if (pass == Q_QR1)
                            run(std::integral_constant<int, Q_QR1>(), std::true_type());
                        else if (pass == Q_QR2)
                            run(std::integral_constant<int, Q_QR2>(), std::true_type());
                        else
                            run(std::integral_constant<int, Q_QR3>(), std::true_type());
                    } else {
                        if (pass == Q_QR1)
                            run(std::integral_constant<int, Q_QR1>(), std::false_type());
                        else if (pass == Q_QR2)
                            run(std::integral_constant<int, Q_QR2>(), std::false_type());
                        else
                            run(std::integral_constant<int, Q_QR3>(), std::false_type());
                    }
                    aqs1 = __shfl(aqs1, 1);  // QR2: entry 1 lives in lane 1 of chunk 0
                }
                if (!own) {
                    // the helper share is complete: its slab stores, then its failures
                    __builtin_amdgcn_s_waitcnt(0);
                    if (lane == 0) {
                        sh.hfail[tw][0] = fail0;
                        sh.hfail[tw][1] = fail1;
                        sh.hph3[tw][0] = ph30 != 0;
                        sh.hph3[tw][1] = ph31 != 0;
                        lds_store_rel(&sh.helpDone[tw], sh.annId[tw]);
                    }
                } else if constexpr (TREE) {
                    // ---- the pass's sums: the xor butterfly of the lanes' partial sums (every lane
                    // ends with the same value; ORC_LM_TREE's orc_tree_finish)
                    const bool two = pass == Q_QR1 || pass == Q_GRAM;
                    const bool gram = pass == Q_GRAM;
                    for (int o = 32; o > 0; o >>= 1) {
                        ta0 += __shfl_xor(ta0, o);
                        if (two) ta1 += __shfl_xor(ta1, o);
                        if (gram) {
                            ta2 += __shfl_xor(ta2, o);
                            ta3 += __shfl_xor(ta3, o);
                            ta4 += __shfl_xor(ta4, o);
                        }
                    }
                    // sums of squares (enorm): the residual, QR2's a_q', the Gram sweep's columns (the
                    // Jacobian pass itself has no sums in TREE)
                    const bool en = (pass == Q_EVAL && !jac) || pass == Q_QR2 || pass == Q_GRAM;
                    if (lane == 0) {
                        double r0 = ta0, r1 = ta1;
                        if (en) {
                            r0 = tslow0 ? ctl.seq_enorm(SP, pass == Q_QR2 ? 3 : (pass == Q_GRAM ? 1 : 0), len) : sqrt(ta0);
                            if (two) r1 = tslow1 ? ctl.seq_enorm(SP, 2, len) : sqrt(ta1);
                        }
                        OUT.nrm[0] = OUT.sum[0] = r0;
                        OUT.nrm[1] = OUT.sum[1] = r1;
                        OUT.sq[0] = ta0;
                        OUT.sq[1] = ta1;
                        OUT.g[0] = ta2;
                        OUT.g[1] = ta3;
                        OUT.g[2] = ta4;
                        OUT.slow = (tslow0 ? 1 : 0) | (tslow1 ? 2 : 0);
                        OUT.fail[0] = fail0;
                        OUT.fail[1] = fail1;
                        OUT.ph3[0] = ph30 != 0;
                        OUT.ph3[1] = ph31 != 0;
                        OUT.aqs1 = aqs1;
                    }
                } else {
                    // ---- the chain lanes' results of this pass (and the helper share)
                    const long long c0 = clock64();
                    while ((lds_load_acq(&sh.resultId[w][0]) != passId || lds_load_acq(&sh.resultId[w][1]) != passId) &&
                           wall_clock64() < prod.deadline)
                        __builtin_amdgcn_s_sleep(1);
                    bool hp0 = false, hp1 = false;
                    if (kS == 2) {
                        while (lds_load_acq(&sh.helpDone[w]) != passId && wall_clock64() < prod.deadline)
                            __builtin_amdgcn_s_sleep(1);
                        fail0 = min(fail0, sh.hfail[w][0]);
                        fail1 = min(fail1, sh.hfail[w][1]);
                        hp0 = sh.hph3[w][0] != 0;
                        hp1 = sh.hph3[w][1] != 0;
                    }
                    if (lane == 0) {
                        WS.wait += clock64() - c0;
                        OUT.nrm[0] = OUT.sum[0] = sh.result[w][0];
                        OUT.nrm[1] = OUT.sum[1] = sh.result[w][1];
                        OUT.fail[0] = fail0;
                        OUT.fail[1] = fail1;
                        OUT.ph3[0] = ph30 != 0 || hp0;
                        OUT.ph3[1] = ph31 != 0 || hp1;
                        OUT.aqs1 = aqs1;
                    }
                }
            }
            // every lane's slab and LDS stores are done before the bookkeeping reads them
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            if (lane == 0) {
                const unsigned long long tp1 = clock64();
                if (own) ctl.after_pass(SS, SP, OUT);
                const unsigned long long tp2 = clock64();
                WS.terms += tp1 - WS.t0;
                WS.ctl += tp2 - tp1;
                WS.cnt[cls]++;
                WS.cyc[cls] += tp2 - WS.t0;
            }
            if (own) ctl.resolve_trig(SS, SP, lane);
            __builtin_amdgcn_s_waitcnt(0);
        }
        if (lane == 0) {
            lds_store_rel(&sh.done[w], 1);
            atomicAdd(p.statEval, (unsigned long long)ctl.cnt_eval);
            atomicAdd(p.statPix, (unsigned long long)ctl.cnt_pix);
            atomicAdd(p.statPass + 0, WS.nPass);
            atomicAdd(p.statPass + 1, WS.terms);
            atomicAdd(p.statPass + 3, WS.ctl);
            for (int k = 0; k < 4; k++) {
                atomicAdd(p.statPass + 7 + k, WS.cnt[k]);
                atomicAdd(p.statPass + 11 + k, WS.cyc[k]);
            }
            atomicAdd(p.statPass + 21, WS.wait);
        }
    } else {
        chain_wave(lane, tStart, p.maxTicks, p.statPass + 2, p.statPass + 18);
    }
    // the group's lifetime, recorded by the wave that leaves last: the chain wave (it leaves once
    // every slot is done), or in TREE mode, which has none, the last term wave past its loop
    bool lastWave = false;
    if (lane == 0) lastWave = TREE ? atomicAdd(&sh.exited, 1) == NS - 1 : wave == kW;
    if (lastWave) {
        atomicAdd(p.statPass + 4, clock64() - cyStart);
        const unsigned long long wt = wall_clock64() - tStart;
        atomicAdd(p.statPass + 5, wt);
        atomicMax(p.statPass + 6, wt);
        atomicMax(p.statPass + 15, tStart);
        atomicMax(p.statPass + 16, wall_clock64());
        atomicMin(p.statPass + 17, tStart);
    }
}

// one pose for every problem of the launch (one frame pair, or linked pairs of one rig pose), and
// a pose per problem
template __global__ void lm2_kernel<false, false>(LMParams p);
template __global__ void lm2_kernel<true, false>(LMParams p);
template __global__ void lm2_kernel<false, true>(LMParams p);
template __global__ void lm2_kernel<true, true>(LMParams p);

}  // namespace fm3d
