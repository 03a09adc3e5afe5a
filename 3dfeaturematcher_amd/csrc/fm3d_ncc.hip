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
#include "fm3d_kernels.h"
#include "fm3d_lmdif.h"

namespace fm3d {

namespace {

constexpr int kNccMaxPerWave = 8;  // hypotheses per wave (H <= 32)
constexpr int kNccChunk = 512;     // neighbourhood entries staged in LDS at a time

__device__ __forceinline__ double xor_sum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// KPW: hypotheses per wave the register arrays hold (H <= 4 * KPW); sized to H so that 16 hypotheses
// keep 4 per wave in registers (225 VGPRs at 8, 2 waves per SIMD)
template <int KPW, bool FULL>
__global__ __launch_bounds__(256) void ncc_kernel(NccParams p) {
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
        const int h = wave + 4 * k;
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
    const double xmax = (double)p.w, ymax = (double)p.h;  // isPixelGood at scale 1
    // the hypothesis-independent part of a pixel (its undistorted ray and image-1 sample) once per
    // workgroup, kNccChunk entries at a time in LDS; lane l of every wave then takes the entries l,
    // l + 64, l + 128, ... of each chunk -- the same entries in the same order as a lane-strided scan
    __shared__ double Rx[kNccChunk], Ry[kNccChunk];
    __shared__ float A1[kNccChunk];
    __shared__ int OK[kNccChunk];
    __shared__ int anyBad1S;
    if (threadIdx.x == 0) anyBad1S = 0;
    __syncthreads();
    for (int base = 0; base < p.nOffPad; base += kNccChunk) {
        for (int r = 0; r < kNccChunk / 256; r++) {
            const int sl = threadIdx.x + 256 * r, e = base + sl;
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
            A1[sl] = I1;
            OK[sl] = in;
        }
        __syncthreads();
        for (int j = 0; j < kNccChunk / 64; j++) {
            const int t = lane + 64 * j;
            if (base + t >= p.nOffPad) break;
            if (!OK[t]) continue;
            m++;
            const double ux = Rx[t], uy = Ry[t];
            const double a = (double)A1[t];
            Sa += a;
            Saa += a * a;
            const int nk = FULL ? KPW : nh;  // FULL: H == 4 * KPW, every wave holds KPW hypotheses
#pragma unroll
            for (int k = 0; k < KPW; k++) {
                if (k >= nk) break;
                const double nn = n0[k] * ux + n1[k] * uy + n2[k] * 1.;
                const double kk = mm[k] / nn;
                const double P0 = kk * ux, P1 = kk * uy, P2 = kk * 1.;
                const bool inbox = (P0 > -cm && P0 < cm) && (P1 > -cm && P1 < cm) && (P2 > 0. && P2 < cm);  // NaN fails
                double u, v;
                project1(p.cam, p.R2, p.t2, P0, P1, P2, u, v);
                if (!inbox || !pixel_good_b(u, v, xmax, ymax)) {
                    bad[k] = true;
                    continue;
                }
                const double b = (double)bilinear(p.img2, p.w, (float)u, (float)v);
                Sb[k] += b;
                Sbb[k] += b * b;
                Sab[k] += a * b;
            }
        }
        __syncthreads();
    }
    for (int o = 32; o > 0; o >>= 1) m += __shfl_xor(m, o);
    const bool anyBad1 = anyBad1S != 0;
    __shared__ double score[32];
    const double sa = xor_sum(Sa), saa = xor_sum(Saa);
    for (int k = 0; k < nh; k++) {
        const bool fail = anyBad1 || __any(bad[k]);
        const double sb = xor_sum(Sb[k]), sbb = xor_sum(Sbb[k]), sab = xor_sum(Sab[k]);
        if (lane == 0) {
            double s = -2.;
            if (!fail && m > 0) {
                const double cov = sab - sa * sb / m, va = saa - sa * sa / m, vb = sbb - sb * sb / m;
                if (va > 0 && vb > 0) s = cov / sqrt(va * vb);
            }
            score[wave + 4 * k] = s;
            p.scores[(size_t)pt * H + wave + 4 * k] = s;
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
