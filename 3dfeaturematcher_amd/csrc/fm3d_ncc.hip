// fm3d_ncc.hip -- NCC scoring of candidate surface normals (BASELINE.json configs[2..3]: "patch NCC
// over 16 / 32 normal hypotheses").
//
// The reference has no NCC search (NormalOptimizer runs lmfit's LM over (phi, theta),
// normaloptimizer.cpp:247-292), so this is an extension on the reference's own residual geometry,
// checked against the oracle's restatement (oracle/fm3d_oracle.c orc_ncc_hypotheses), not against
// the reference.  Per point, on pyramid level 0 of fm3d_set_images:
//   * the extractPixelsContour neighbourhood (singlecameratriangulator.cpp:341-397) and its
//     undistorted rays (:542) and image-1 samples (:576-589);
//   * H = Hphi x Htheta normals sph2car(phi0 + dphi, theta0 + dtheta) on a grid of half width `span`
//     around car2sph(X/|X|), the LM's initial guess (normaloptimizer.cpp:342-343);
//   * per normal the evaluateNormal geometry (:65-149 through :421-470, :591-665): ray-plane
//     intersection, bounding box, camera-2 projection, isPixelGood, image-2 sample; any failing pixel
//     (or a flat patch) gives the score -2, else NCC(I1, I2) over the m_dat pixels.
// One 256-thread workgroup per point: the rays and image-1 samples of 256 entries at a time in LDS
// (each computed once, not once per wave); wave w scores hypotheses w, w+4, ...; lane l sums the
// entries of offset index = l (mod 64) in order, then a fixed xor tree over the wave (the oracle's order).
#include <hip/hip_runtime.h>

#include "fm3d_device.h"
#include "fm3d_fastdiv.h"
#include "fm3d_kernels.h"
#include "fm3d_lmdif.h"

namespace fm3d {

namespace {

constexpr int kNccMaxPerWave = 8;  // hypotheses per wave (H <= 32)
constexpr int kNccChunk = 512;     // neighbourhood entries staged in LDS at a time

__device__ __forceinline__ double ncc_uniform(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane((int)b), hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double xor_sum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// The evaluateNormal geometry of one neighbourhood entry through one hypothesis' plane (ray-plane
// intersection :421-470, isInBoundingBox :646-655, projectPointsToImage2 :591-644, isPixelGood
// :657-665), without the ray-plane division (round 5; the oracle's orc_ncc_hypotheses states the
// same arithmetic, this mode has no reference counterpart to keep the reference's order for):
//  * the plane point is P = (mm / nn) r for the ray r = (ux, uy, 1), nn = n . r.  The bounding box
//    |P0| < cm, |P1| < cm, 0 < P2 < cm reads |mm ux| < cm |nn|, |mm uy| < cm |nn|, |mm| < cm |nn| with
//    mm and nn of one sign (nn = 0 fails every test, as P = inf / NaN did);
//  * camera 2 sees P at (mm q + nn t2) / nn, q = R2 r staged once per entry (q0..q2), so the
//    normalised coordinates are (mm q0 + nn t0) / (mm q2 + nn t2) and (mm q1 + nn t1) / (the same):
//    one reciprocal (recip_z_lo, one guard), no quotient mm / nn;
//  * r2 + 2x^2 as fma(x*x, 2, r2) (2*RN(x*x) == RN(2x*x)) and k 2xy as (2k) RN(xy) (k2d, k3d; the
//    LM kernel's geometry2 states why the bits agree); project1's NaN for an infinite r6
//    dropped (such a u or v is infinite or NaN: not good);
//  * every product-and-sum after the undistortion fused (round 5): nn, the camera-2 coordinates, the
//    distortion polynomial, xd / yd and the pixel coordinates (orc_ncc_project states the same
//    fused operations on the host, C99 fma);
//  * 0 <= u <= xmax as bits(u) <= bits(xmax): u is never -0.0 (the host hands the kernel a
//    principal point of +0.0 for -0.0, fm3d_host.cpp lm_camera), negatives and NaNs lie above.
typedef unsigned long long LaneMask;
// v where the lane's bit of m is set, else 0 (v_cndmask with the SGPR mask as selector)
__device__ __forceinline__ unsigned ncc_sel_u32(unsigned v, LaneMask m) {
    asm("v_cndmask_b32_e64 %0, 0, %0, %1" : "+v"(v) : "s"(m));
    return v;
}
// The tests as lane masks (each the ballot of one compare, combined with scalar ANDs; fm3d_lm2.hip
// geometry2's form): good, the float sample coordinates, and the bilinear window's byte offset (0
// where not good: the gather then reads the image's first bytes)
struct NccGeo {
    float fx, fy;
    unsigned off;
    LaneMask good;
};
// csg = cm sgn, sgn the sign of mm as +1 / -1, 0 for mm = 0 or NaN (hypothesis-uniform).
// The limit csg nn equals cm |nn| where mm and nn share a sign and is <= 0 or NaN (every test fails)
// elsewhere, so the sign test costs one multiply
// the part up to camera 2's homogeneous coordinates (X, Y, Z) = mm q + nn t2 and the box mask
struct NccPre {
    double nn, X, Y, Z;
    LaneMask inbox;
};
__device__ __forceinline__ NccPre ncc_geo_pre(const NccParams& p, double ux, double uy, double q0, double q1, double q2,
                                              double n0, double n1, double n2, double mm, double csg) {
    NccPre r;
    r.nn = __builtin_fma(n1, uy, __builtin_fma(n0, ux, n2));
    const double lim = csg * r.nn;
    r.inbox = __ballot(fabs(mm * ux) < lim) & __ballot(fabs(mm * uy) < lim) & __ballot(fabs(mm) < lim);
    r.X = __builtin_fma(r.nn, p.t2[0], mm * q0);
    r.Y = __builtin_fma(r.nn, p.t2[1], mm * q1);
    r.Z = __builtin_fma(r.nn, p.t2[2], mm * q2);
    return r;
}
// the rest, given z = Z ? 1 / Z : 1
__device__ __forceinline__ NccGeo ncc_geo_post(const NccParams& p, const NccPre& pr, double z, double k2d, double k3d,
                                               unsigned long long xmaxb, unsigned long long ymaxb) {
    NccGeo g;
    const LaneMask inbox = pr.inbox;
    const double x = pr.X * z, y = pr.Y * z;
    const double xx = x * x, yy = y * y;
    const double r2 = xx + yy;
    const double r4 = r2 * r2;
    const double r6 = r4 * r2;
    const double xy = x * y;
    const double a2 = __builtin_fma(xx, 2., r2);
    const double a3 = __builtin_fma(yy, 2., r2);
    const double cdist =
        __builtin_fma(p.cam.k[4], r6, __builtin_fma(p.cam.k[1], r4, __builtin_fma(p.cam.k[0], r2, 1.)));
    const double xd = __builtin_fma(p.cam.k[3], a2, __builtin_fma(k2d, xy, x * cdist));
    const double yd = __builtin_fma(k3d, xy, __builtin_fma(p.cam.k[2], a3, y * cdist));
    const double u = __builtin_fma(xd, p.cam.fx, p.cam.cx);
    const double v = __builtin_fma(yd, p.cam.fy, p.cam.cy);
    g.good = inbox & __ballot((unsigned long long)__double_as_longlong(u) <= xmaxb) &
             __ballot((unsigned long long)__double_as_longlong(v) <= ymaxb);
    g.fx = (float)u;
    g.fy = (float)v;
    // truncation is floor on the good lanes (0 <= u, v); the others' offsets are zeroed
    const unsigned o = __umul24((unsigned)(int)g.fy, (unsigned)p.w) + (unsigned)(int)g.fx;
    g.off = ncc_sel_u32(o, g.good);
    return g;
}
__device__ __forceinline__ NccGeo ncc_geometry_m(const NccParams& p, double ux, double uy, double q0, double q1,
                                                 double q2, double n0, double n1, double n2, double mm,
                                                 double csg, double k2d, double k3d,
                                                 unsigned long long xmaxb, unsigned long long ymaxb) {
    const NccPre pr = ncc_geo_pre(p, ux, uy, q0, q1, q2, n0, n1, n2, mm, csg);
    return ncc_geo_post(p, pr, recip_z_lo(pr.Z), k2d, k3d, xmaxb, ymaxb);
}
// getBilinearInterpPix32f (tools.cpp:129-142) on the gathered window, with the fractions
// x - floor(x), y - floor(y), as two-lane float vectors (v_pk_mul_f32 / v_pk_add_f32: each component
// rounded as the scalar operation; fm3d_lm2.hip bilinear_f).  The fractions as v_fract_f32: for a
// good sample (x, y >= 0) x - floor(x) is exact and below 1, so fract's clamp never applies; the
// other lanes' samples are discarded (not in image 1) or their hypothesis is dead
typedef float ncc_f32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((aligned(1))) const uint16_t ncc_u16u;
// the window's rows lo = (b00, b01), hi = (b10, b11) as loaded
__device__ __forceinline__ float ncc_bilinear_w(unsigned lo, unsigned hi, float x, float y) {
    const float xf = __builtin_amdgcn_fractf(x), yf = __builtin_amdgcn_fractf(y);
    const ncc_f32x2 b0 = {(float)(lo & 0xff), (float)(lo >> 8)};  // b00, b01
    const ncc_f32x2 b1 = {(float)(hi & 0xff), (float)(hi >> 8)};  // b10, b11
    const float ym0 = 1.0f - yf, ym1 = yf;
    const ncc_f32x2 sc = b0 * ym0 + b1 * ym1;
    const ncc_f32x2 xm = {1.0f - xf, xf};
    const ncc_f32x2 q = xm * sc;
    return q.x + q.y;
}
__device__ __forceinline__ float ncc_bilinear_f(const uint8_t* img, unsigned off, int w, float x, float y) {
    // both rows by a 32-bit offset from the image base (the window lies inside the image)
    return ncc_bilinear_w(*(ncc_u16u*)(img + off), *(ncc_u16u*)(img + (off + (unsigned)w)), x, y);
}

// KPW: hypotheses per wave the register arrays hold (H <= 4 * KPW); sized to H so that 16 hypotheses
// keep 4 per wave in registers
// NW: waves per point (hypothesis h runs on wave h % NW).  Round 5 A/B at C3 (H = 16, one pair at a
// time, tools/ncc_ab.sh), before the fused arithmetic: NW = 4, KPW = 4 1.497 ms; the plane constants
// made scalar (readfirstlane) 1.498 ms; NW = 8, KPW = 2 (4 waves per SIMD instead of 3) 1.548 /
// 1.554 ms.  With the fused arithmetic the scalar constants bring the kernel under 128 VGPRs, and
// four waves per SIMD then pay (below)
template <int KPW, bool FULL, int NW = 4>
__global__ __launch_bounds__(64 * NW) void ncc_kernel(NccParams p) {
    const int pt = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (pt >= (p.Pdev ? *p.Pdev : p.P)) return;  // the inlier count on the device (pipeline), or P
    const double X0 = p.points[3 * pt], X1 = p.points[3 * pt + 1], X2 = p.points[3 * pt + 2];
    static const double Ident[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    static const double Zero[3] = {0, 0, 0};
    double ccx, ccy;
    project1(p.cam, Ident, Zero, X0, X1, X2, ccx, ccy);
    // the LM's initial guess X * (1/|X|) and its spherical angles
    const double inv = 1. / sqrt(X0 * X0 + X1 * X1 + X2 * X2);
    const double g0 = X0 * inv, g1 = X1 * inv, g2 = X2 * inv;
    const double theta0 = fm3d_atan2(g2, sqrt(g0 * g0 + g1 * g1)), phi0 = fm3d_atan2(g1, g0);
    const int H = p.Hphi * p.Htheta;
    int nh = 0;
    double n0[KPW], n1[KPW], n2[KPW], mm[KPW];
    for (int k = 0; k < KPW; k++) {
        const int h = wave + NW * k;
        if (h < H) {
            const int ip = h / p.Htheta, it = h - ip * p.Htheta;
            const double dphi = p.span * (double)(2 * ip + 1 - p.Hphi) / p.Hphi;
            const double dtheta = p.span * (double)(2 * it + 1 - p.Htheta) / p.Htheta;
            lmdif::sph2car_det(phi0 + dphi, theta0 + dtheta, n0[k], n1[k], n2[k]);
            mm[k] = n0[k] * X0 + n1[k] * X1 + n2[k] * X2;
            nh = k + 1;
        }
    }
    // the image-1 sums are the same for every hypothesis that scores: one that fails anywhere scores -2
    // whatever its sums, and one that never fails takes every in-bounds pixel, in the same order
    double Sa = 0., Saa = 0.;
    double Sb[KPW], Sbb[KPW], Sab[KPW];
    bool bad[KPW];
    for (int k = 0; k < KPW; k++) {
        Sb[k] = Sbb[k] = Sab[k] = 0.;
        bad[k] = false;
    }
    int m = 0;
    const double cm = (double)p.cmax;
    const double k2d = 2. * p.cam.k[2], k3d = 2. * p.cam.k[3];
    const double xmax = (double)p.w, ymax = (double)p.h;  // isPixelGood at scale 1
    const unsigned long long xmaxb = (unsigned long long)__double_as_longlong(xmax);
    const unsigned long long ymaxb = (unsigned long long)__double_as_longlong(ymax);
    double csg[KPW];
    for (int k = 0; k < KPW; k++) {
        csg[k] = mm[k] > 0. ? cm : mm[k] < 0. ? -cm : 0.;
    }
    // the plane constants are wave-uniform: scalar registers (round 5, with the fused arithmetic:
    // 153 -> 113 VGPRs at H = 16, four waves per SIMD instead of three; same box 1.38 -> 1.33 ms
    // at C3, and at H = 32 217 -> 138 VGPRs, 20.4 -> 18.4 ms over 20k points)
    for (int k = 0; k < KPW; k++) {
        n0[k] = ncc_uniform(n0[k]);
        n1[k] = ncc_uniform(n1[k]);
        n2[k] = ncc_uniform(n2[k]);
        mm[k] = ncc_uniform(mm[k]);
        csg[k] = ncc_uniform(csg[k]);
    }
    // hypotheses of this wave that already failed on some entry (wave-uniform): they score -2
    // whatever their sums, so their geometry is not computed again.  Per hypothesis the lanes that
    // failed it so far (a ballot OR, SGPRs): tests and updates stay scalar
    LaneMask dead[KPW];
    for (int k = 0; k < KPW; k++) dead[k] = 0;
    // the hypothesis-independent part of a pixel (its undistorted ray and image-1 sample) once per
    // workgroup, kNccChunk entries at a time in LDS; lane l of every wave then takes the entries l,
    // l + 64, l + 128, ... of each chunk -- the same entries in the same order as a lane-strided scan
    __shared__ double Rx[kNccChunk], Ry[kNccChunk], Q0[kNccChunk], Q1[kNccChunk], Q2[kNccChunk];
    __shared__ float A1[kNccChunk];
    __shared__ int OK[kNccChunk];
    __shared__ int anyBad1S;
    if (threadIdx.x == 0) anyBad1S = 0;
    __syncthreads();
    const int nk = FULL ? KPW : nh;  // FULL: H == NW * KPW, every wave holds KPW hypotheses
    for (int base = 0; base < p.nOffPad; base += kNccChunk) {
        for (int r = 0; r < kNccChunk / (64 * NW); r++) {
            const int sl = threadIdx.x + 64 * NW * r, e = base + sl;
            int in = 0;
            double ux = 0., uy = 0.;
            float I1 = 0.f;
            if (e < p.nOffPad) {
                const int2 o = p.offsets[e];
                const double px = ccx + (double)o.x, py = ccy + (double)o.y;
                in = e < p.nOff && !(px < 0 || py < 0 || px >= p.boundW || py >= p.boundH);
                if (in) {
                    undistort1(p.cam, px, py, ux, uy);
                    if (!pixel_good_b(px, py, xmax, ymax))
                        anyBad1S = 1;  // the same value from any thread
                    else
                        I1 = bilinear(p.img1, p.w, (float)px, (float)py);
                }
            }
            Rx[sl] = ux;
            Ry[sl] = uy;
            Q0[sl] = p.R2[0] * ux + p.R2[1] * uy + p.R2[2];
            Q1[sl] = p.R2[3] * ux + p.R2[4] * uy + p.R2[5];
            Q2[sl] = p.R2[6] * ux + p.R2[7] * uy + p.R2[8];
            A1[sl] = I1;
            OK[sl] = in;
        }
        __syncthreads();
        if (anyBad1S)  // an image-1 pixel fails: every hypothesis scores -2
            for (int k = 0; k < KPW; k++) dead[k] = ~0ull;
        for (int j = 0; j < kNccChunk / 64; j++) {
            const int t = lane + 64 * j;
            if (base + 64 * j >= p.nOffPad) break;  // wave-uniform
            // branch-free over the lanes: an entry outside image 1 (OK 0) was staged with ray (0, 0)
            // and sample 0, and its image-2 sample is zeroed, so it adds +0 to every sum (the partial
            // sums are >= 0: +0 leaves them unchanged); a pixel that fails a hypothesis marks it dead,
            // and a dead hypothesis scores -2 whatever its sums
            const LaneMask okm = __ballot(OK[t] != 0);
            m += (okm >> lane) & 1;
            const double ux = Rx[t], uy = Ry[t], q0 = Q0[t], q1 = Q1[t], q2 = Q2[t];
            const double a = (double)A1[t];
            Sa += a;
            Saa = __builtin_fma(a, a, Saa);  // a*a and a*b are exact (float samples): fusing keeps the bits
#pragma unroll
            for (int k = 0; k < KPW; k++) {
                if (k >= nk) break;
                if (dead[k]) continue;  // wave-uniform
                const NccGeo g = ncc_geometry_m(p, ux, uy, q0, q1, q2, n0[k], n1[k], n2[k], mm[k], csg[k], k2d, k3d,
                                                  xmaxb, ymaxb);
                dead[k] |= okm & ~g.good;
                const float bf = ncc_bilinear_f(p.img2, g.off, p.w, g.fx, g.fy);
                const double b = (double)__uint_as_float(ncc_sel_u32(__float_as_uint(bf), okm));
                Sb[k] += b;
                Sbb[k] = __builtin_fma(b, b, Sbb[k]);
                Sab[k] = __builtin_fma(a, b, Sab[k]);
            }
        }
        __syncthreads();
    }
    for (int k = 0; k < KPW; k++) bad[k] = dead[k] != 0;
    for (int o = 32; o > 0; o >>= 1) m += __shfl_xor(m, o);
    const bool anyBad1 = anyBad1S != 0;
    __shared__ double score[32];
    const double sa = xor_sum(Sa), saa = xor_sum(Saa);
    for (int k = 0; k < nh; k++) {
        const bool fail = anyBad1 || bad[k];  // wave-uniform
        const double sb = xor_sum(Sb[k]), sbb = xor_sum(Sbb[k]), sab = xor_sum(Sab[k]);
        if (lane == 0) {
            double s = -2.;
            if (!fail && m > 0) {
                const double cov = sab - sa * sb / m, va = saa - sa * sa / m, vb = sbb - sb * sb / m;
                if (va > 0 && vb > 0) s = cov / sqrt(va * vb);
            }
            score[wave + NW * k] = s;
            p.scores[(size_t)pt * H + wave + NW * k] = s;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int best = -1;
        double bs = -2.;
        for (int h = 0; h < H; h++)
            if (score[h] > bs) {
                bs = score[h];
                best = h;
            }
        double r0 = g0, r1 = g1, r2 = g2;
        if (best >= 0) {
            const int ip = best / p.Htheta, it = best - ip * p.Htheta;
            const double dphi = p.span * (double)(2 * ip + 1 - p.Hphi) / p.Hphi;
            const double dtheta = p.span * (double)(2 * it + 1 - p.Htheta) / p.Htheta;
            lmdif::sph2car_det(phi0 + dphi, theta0 + dtheta, r0, r1, r2);
        }
        p.best[pt] = best;
        p.normals[3 * pt] = r0;
        p.normals[3 * pt + 1] = r1;
        p.normals[3 * pt + 2] = r2;
    }
}

}  // namespace

void launch_ncc_hypotheses(const NccParams& p, hipStream_t s) {
    if (p.P <= 0) return;
    const int H = p.Hphi * p.Htheta;
    if (H == 16)
        ncc_kernel<4, true><<<p.P, 256, 0, s>>>(p);
    else if (H == 32)
        ncc_kernel<kNccMaxPerWave, true><<<p.P, 256, 0, s>>>(p);
    else if (H <= 8)
        ncc_kernel<2, false><<<p.P, 256, 0, s>>>(p);
    else if (H <= 16)
        ncc_kernel<4, false><<<p.P, 256, 0, s>>>(p);
    else
        ncc_kernel<kNccMaxPerWave, false><<<p.P, 256, 0, s>>>(p);
}

}  // namespace fm3d
