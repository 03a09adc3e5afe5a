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
// One 256-thread workgroup per point: wave w scores hypotheses w, w+4, ...; lane l sums the entries
// of offset index = l (mod 64) in order, then a fixed xor tree over the wave (the oracle's order).
#include <hip/hip_runtime.h>

#include "fm3d_device.h"
#include "fm3d_kernels.h"
#include "fm3d_lmdif.h"

namespace fm3d {

namespace {

constexpr int kNccMaxPerWave = 8;  // hypotheses per wave (H <= 32)

__device__ __forceinline__ double xor_sum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__global__ __launch_bounds__(256) void ncc_kernel(NccParams p) {
    const int pt = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (pt >= p.P) return;
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
    double n0[kNccMaxPerWave], n1[kNccMaxPerWave], n2[kNccMaxPerWave], mm[kNccMaxPerWave];
    for (int k = 0; k < kNccMaxPerWave; k++) {
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
    double Sa[kNccMaxPerWave], Sb[kNccMaxPerWave], Saa[kNccMaxPerWave], Sbb[kNccMaxPerWave], Sab[kNccMaxPerWave];
    bool bad[kNccMaxPerWave];
    for (int k = 0; k < kNccMaxPerWave; k++) {
        Sa[k] = Sb[k] = Saa[k] = Sbb[k] = Sab[k] = 0.;
        bad[k] = false;
    }
    bool bad1 = false;
    int m = 0;
    const double cm = (double)p.cmax;
    const double xmax = (double)p.w, ymax = (double)p.h;  // isPixelGood at scale 1
    for (int e = lane; e < p.nOffPad; e += 64) {
        const int2 o = p.offsets[e];
        const double px = ccx + (double)o.x, py = ccy + (double)o.y;
        const bool in = e < p.nOff && !(px < 0 || py < 0 || px >= p.boundW || py >= p.boundH);
        if (!in) continue;
        m++;
        double ux, uy;
        undistort1(p.cam, px, py, ux, uy);
        float I1 = 0.f;
        if (!pixel_good_b(px, py, xmax, ymax))
            bad1 = true;
        else
            I1 = bilinear(p.img1, p.w, (float)px, (float)py);
        const double a = (double)I1;
        for (int k = 0; k < nh; k++) {
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
            Sa[k] += a;
            Sb[k] += b;
            Saa[k] += a * a;
            Sbb[k] += b * b;
            Sab[k] += a * b;
        }
    }
    for (int o = 32; o > 0; o >>= 1) m += __shfl_xor(m, o);
    const bool anyBad1 = __any(bad1);
    __shared__ double score[32];
    for (int k = 0; k < nh; k++) {
        const bool fail = anyBad1 || __any(bad[k]);
        const double sa = xor_sum(Sa[k]), sb = xor_sum(Sb[k]), saa = xor_sum(Saa[k]), sbb = xor_sum(Sbb[k]),
                     sab = xor_sum(Sab[k]);
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
    ncc_kernel<<<p.P, 256, 0, s>>>(p);
}

}  // namespace fm3d
