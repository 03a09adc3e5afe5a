/* san_oracle.c -- the CPU oracle (oracle/fm3d_oracle.c, test infrastructure) under
 * AddressSanitizer + UndefinedBehaviorSanitizer: every public entry point on small seeded inputs,
 * including the edge shapes the tests use (no train rows, one train row, 1-pixel images,
 * neighbourhoods cut by the image corners, points outside every image).  Built and run by
 * tests/test_sanitizers.py (tests/native/Makefile); any report aborts with a nonzero status. */
#include <stdio.h>
#include "../../oracle/fm3d_oracle.c"
#include "../../oracle/orc_surf.c"

static unsigned long long rs = 0x9E3779B97F4A7C15ULL;
static unsigned rnd(void) { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return (unsigned)(rs >> 32); }
static double urand(void) { return rnd() / 4294967296.0; }

int main(void)
{
    enum { NA = 300, NB = 257, D = 128 };
    static uint8_t A8[NA * D], B8[NB * D];
    static float Af[NA * D], Bf[NB * D];
    static int idx[NA * 2], q[NA], t[NA];
    static float dist[NA * 2], dd[NA];
    int i, n, nb;
    for (i = 0; i < NA * D; i++) { A8[i] = (uint8_t)rnd(); Af[i] = A8[i] * 0.01f; }
    for (i = 0; i < NB * D; i++) { B8[i] = (uint8_t)rnd(); Bf[i] = B8[i] * 0.01f; }
    for (nb = 0; nb <= NB; nb += (nb < 3 ? 1 : 127)) {
        orc_knn2(1, A8, NA, B8, nb, D, idx, dist, 1);      /* u8 */
        orc_knn2(0, Af, NA, Bf, nb, D, idx, dist, 1);      /* f32 */
        orc_knn2(2, A8, NA, B8, nb, 32, idx, dist, 1);     /* binary, 256 bits */
        n = orc_nndr(idx, dist, NA, 0.8, q, t, dd);
        (void)n;
    }
    /* pyrDown of odd and degenerate sizes */
    {
        static const int sz[][2] = {{1, 1}, {1, 7}, {5, 1}, {33, 17}, {64, 48}};
        static uint8_t src[64 * 48], dst[32 * 24];
        for (i = 0; i < 64 * 48; i++) src[i] = (uint8_t)rnd();
        for (i = 0; i < 5; i++) orc_pyrdown(src, sz[i][0], sz[i][1], dst);
    }
    /* camera, g12, triangulation of random matches */
    orc_camera cam = {357.80, 357.93, 80.0, 60.0, {-0.299957, 0.124129, -6.6e-05, 0.000567, -0.028357}};
    const double rIC[3] = {-1.2005, 1.1981, -1.2041}, tIC[3] = {0.0, 0.015, -0.051};
    const double T1[3] = {5.301099, 8.031408, 1.977258}, r1[3] = {0.153433, 0.149941, -2.658648};
    const double T2[3] = {4.735536, 7.691893, 1.913166}, r2[3] = {0.252828, 0.048977, -2.676886};
    double g12[16], R2[9], t2[3], rv[3], Rm[9];
    orc_setg12(rIC, tIC, T1, T2, r1, r2, g12);
    orc_camera2_from_g12(g12, R2, t2);
    orc_rodrigues_m2v(R2, rv);
    orc_rodrigues_v2m(rv, Rm);
    {
        static float kp1[200 * 2], kp2[200 * 2];
        static int mq[200], mt[200];
        static uint8_t mask[200];
        static double pts[200 * 3];
        for (i = 0; i < 400; i++) { kp1[i] = (float)(urand() * 160); kp2[i] = (float)(urand() * 160); }
        for (i = 0; i < 200; i++) { mq[i] = (int)(rnd() % 200); mt[i] = (int)(rnd() % 200); }
        orc_triangulate(&cam, g12, 1.5, 2.4, kp1, kp2, mq, mt, 200, mask, pts);
    }
    /* normals on a textured 160 x 120 pair: points inside, at the corners, outside every image */
    {
        enum { W = 160, H = 120, P = 12 };
        static uint8_t im1[W * H], im2[W * H];
        static double pts[P * 3], nrm[P * 3], xy[2 * 13 * 13];
        static int st[P], info[P * 8], nfev[P * 8], mdat[P];
        for (i = 0; i < W * H; i++) {
            int x = i % W, y = i / W;
            im1[i] = (uint8_t)(128 + 60 * sin(x * 0.31) * cos(y * 0.23) + 20 * sin((x + y) * 0.7));
            im2[i] = (uint8_t)(128 + 60 * sin((x + 2) * 0.31) * cos(y * 0.23) + 20 * sin((x + y + 2) * 0.7));
        }
        for (i = 0; i < P; i++) {
            pts[3 * i] = (urand() - 0.5) * 1.6;
            pts[3 * i + 1] = (urand() - 0.5) * 1.2;
            pts[3 * i + 2] = 1.8 + 0.4 * urand();
        }
        pts[0] = -0.45 * 2.0; pts[1] = -0.34 * 2.0; pts[2] = 2.0;   /* top-left corner */
        pts[3] = 5.0; pts[4] = 5.0; pts[5] = 2.0;                   /* outside every image */
        for (i = 0; i < 2; i++) {
            const int mode = i ? ORC_LM_DETMATH : ORC_LM_STRICT;
            orc_optimize_normals(&cam, R2, t2, im1, im2, W, H, 2, pts, P, 6, W, H, 1e-10, 2.4, mode, nrm, st, info,
                                 nfev, mdat, 1);
        }
        orc_neighborhood(&cam, pts, 6, 1024, 768, xy, 13 * 13);
        orc_bilinear_sample(im1, W, H, (float)(W - 1), (float)(H - 2));
        /* frames, square neighbourhoods, patches */
        {
            static double fr[P * 16], g[3], sq[2 * 16 * 16 * 3];
            static uint8_t patch[P * 16 * 16];
            orc_gravity(rIC, g);
            orc_features_frames(pts, pts, P, g, fr);
            orc_square_neighborhoods(fr, 2, 0.02, 0.25, sq);
            orc_export_patches(&cam, im1, W, H, fr, P, 0.02, 0.25, ORC_LM_STRICT, patch, NULL);
            orc_export_patches(&cam, im1, W, H, fr, P, 0.02, 0.25, ORC_LM_DETMATH, patch, NULL);
        }
    }
    /* NCC hypotheses: points inside, behind and far outside the images */
    {
        static double nx[9] = {0.05, -0.02, 1.9, 0.0, 0.0, 0.0, 4.0, 4.0, 2.0}, sc[3 * 32], nn[9];
        static int bb[3];
        static uint8_t i1[64 * 48], i2[64 * 48];
        static const double R2i[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, t2i[3] = {0.01, 0, 0};
        orc_camera c0 = {60, 60, 32, 24, {-0.2, 0.05, 0.001, 0.001, 0.0}};
        for (i = 0; i < 64 * 48; i++) { i1[i] = (uint8_t)rnd(); i2[i] = (uint8_t)rnd(); }
        orc_ncc_hypotheses(&c0, R2i, t2i, i1, i2, 64, 48, nx, 3, 5, 64, 48, 2.4, 8, 4, 0.4, sc, nn, bb);
        orc_ncc_hypotheses(&c0, R2i, t2i, i1, i2, 64, 48, nx, 3, 3, 64, 48, 2.4, 1, 1, 0.4, sc, nn, bb);
    }
    /* circular neighbourhoods (given normals and the X/|X| branch) */
    {
        static double X[6] = {0.1, -0.2, 1.9, 0.3, 0.1, 2.1}, N[6] = {0, 0.1, -0.99, 0.2, 0.2, -0.95}, o[2 * 15 * 5 * 3];
        orc_circular_neighborhoods(X, N, 2, 0.16, 15, 5, o);
        orc_circular_neighborhoods(X, NULL, 2, 0.16, 15, 5, o);
    }
    /* SURF detect + describe on textured images of odd / tiny / wide sizes, patches at the border */
    {
        static const int sizes[][2] = {{96, 80}, {33, 29}, {8, 8}, {200, 24}};
        for (i = 0; i < 4; i++) {
            const int w = sizes[i][0], h = sizes[i][1];
            static uint8_t im[200 * 96];
            static orc_kpt k[4096], k2[4096];
            static int kept[4096];
            static float desc[4096 * 128];
            int x, y, nk, m;
            for (y = 0; y < h; y++)
                for (x = 0; x < w; x++) im[y * w + x] = (uint8_t)(128 + 100 * sin(x * 0.37 + y * 0.21) * cos(y * 0.3) + (rnd() & 15));
            nk = orc_surf_detect(im, w, h, 40.f, 4, 2, k, 4096);
            if (nk > 4096) nk = 4096;
            m = orc_surf_describe(im, w, h, k, nk, 1, k2, kept, desc);
            m = orc_surf_describe(im, w, h, k, nk, 0, k2, kept, desc);
            (void)m;
        }
        {
            static uint8_t patch[128 * 128], tiny[25 * 25];
            static orc_kpt kp = {64, 64, 128, -1, 1, 0, 0}, ko;
            static float d[128];
            for (i = 0; i < 128 * 128; i++) patch[i] = (uint8_t)rnd();
            orc_surf_describe(patch, 128, 128, &kp, 1, 1, &ko, NULL, d);
            for (i = 21; i <= 25 * 25 && i <= 600; i += 21) {
                const int W = 21 + (i % 5);
                orc_resize_area21(patch, W, tiny);
            }
            for (i = 1; i <= 20; i++) orc_resize_area_up(patch, i, 21, tiny); /* windows narrower than the patch */
            {   /* small keypoints: enlarged windows, upright and oriented, inside and across the borders */
                static orc_kpt ks[6] = {{64, 64, 4, -1, 1, 0, 0}, {1, 2, 7, -1, 1, 0, 0}, {127, 120, 0.4f, -1, 1, 0, 0},
                                        {30, 0, 6.9f, -1, 1, 0, 0}, {100, 127, 2.2f, -1, 1, 0, 0}, {64, 64, 0.3f, -1, 1, 0, 0}};
                static orc_kpt ko6[6];
                orc_surf_describe2(patch, 128, 128, ks, 5, 1, 1, ko6, NULL, (float[6 * 128]){0});
                orc_surf_describe2(patch, 128, 128, ks, 5, 1, 0, ko6, NULL, (float[6 * 128]){0});
                if (orc_surf_describe2(patch, 128, 128, ks, 6, 1, 1, ko6, NULL, (float[6 * 128]){0}) != -1) return 1;
            }
        }
    }
    puts("san_oracle: ok");
    return 0;
}
