// san_host.cpp -- the host algebra of libfm3d (csrc/fm3d_host.cpp: setg12, Rodrigues both ways,
// Matx44d::inv, gravity, patch size) compiled with host-side AddressSanitizer +
// UndefinedBehaviorSanitizer (hipcc -Xarch_host -fsanitize=...) and driven through the C ABI's
// context-free entry points (no GPU needed), including near-identity and half-turn rotations and
// a singular IMU rotation.  Run by tests/test_sanitizers.py.
#include <cmath>
#include <cstdio>

#include "fm3d.h"

int main() {
    int fails = 0;
    fm3d_settings s;
    if (fm3d_settings_default(&s) != FM3D_OK) fails++;
    const double T1[3] = {5.301099, 8.031408, 1.977258}, r1[3] = {0.153433, 0.149941, -2.658648};
    const double T2[3] = {4.735536, 7.691893, 1.913166}, r2[3] = {0.252828, 0.048977, -2.676886};
    double g[16], R2[9], t2[3], grav[3];
    if (fm3d_g12_from_poses(&s, T1, T2, r1, r2, g) != FM3D_OK) fails++;
    if (fm3d_camera2_from_g12(g, R2, t2) != FM3D_OK) fails++;
    for (int k = 0; k < 9; k++)
        if (!std::isfinite(R2[k])) fails++;
    // rotations the Rodrigues matrix->vector branches treat specially: identity (s < 1e-5, c > 0),
    // half turns (s < 1e-5, c < 0) about each axis, a tiny angle
    const double rots[][3] = {{0, 0, 0}, {M_PI, 0, 0}, {0, M_PI, 0}, {0, 0, M_PI}, {1e-9, 0, 0}, {1, 2, 3}};
    for (const auto& r : rots) {
        double gg[16];
        if (fm3d_g12_from_poses(&s, T1, T1, r, r, gg) != FM3D_OK) fails++;
        if (fm3d_camera2_from_g12(gg, R2, t2) != FM3D_OK) fails++;
        double a[3] = {0, 0, 0};
        if (fm3d_g12_from_poses(&s, T1, T2, a, r, gg) != FM3D_OK) fails++;
        if (fm3d_camera2_from_g12(gg, R2, t2) != FM3D_OK) fails++;
    }
    if (fm3d_gravity(&s, grav) != FM3D_OK || std::fabs(grav[0] * grav[0] + grav[1] * grav[1] + grav[2] * grav[2] - 1) > 1e-12)
        fails++;
    if (fm3d_patch_size(&s) != 128) fails++;
    s.neighEpsilon = 0;
    if (fm3d_patch_size(&s) != 0) fails++;
    if (fm3d_g12_from_poses(nullptr, T1, T2, r1, r2, g) != FM3D_ERR_INVALID) fails++;
    if (fm3d_gravity(nullptr, grav) != FM3D_ERR_INVALID) fails++;
    std::printf("san_host: %s\n", fails ? "FAILED" : "ok");
    return fails ? 1 : 0;
}
