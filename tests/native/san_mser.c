/* san_mser.c -- the MSER oracle (oracle/orc_mser.c, test infrastructure) under AddressSanitizer +
 * UndefinedBehaviorSanitizer: the two flood passes and fitEllipse on seeded images of edge shapes
 * (1 x 1, one row, one column, constant, noise, ramps, a checkerboard) and parameters (Delta 0..255,
 * MinArea 0.., MaxArea 1.., any variation / diversity), plus fitEllipse on degenerate point sets
 * (collinear, repeated points).  Built and run by tests/test_sanitizers.py (tests/native/Makefile);
 * any report aborts with a nonzero status. */
#include <stdio.h>
#include "../../oracle/orc_mser.c"

static unsigned long long rs = 0x9E3779B97F4A7C15ULL;
static unsigned rnd(void) { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return (unsigned)(rs >> 32); }

int main(void)
{
    static const int shapes[][2] = {{1, 1}, {1, 37}, {41, 1}, {2, 2}, {17, 13}, {64, 48}, {200, 150}};
    static const int deltas[] = {0, 1, 5, 255};
    static uint8_t img[200 * 150];
    static orc_mser_kp kp[20000];
    static int pts[2 * 200 * 150];
    int s, kind, d, i;
    long long npts;
    for (s = 0; s < 7; s++)
        for (kind = 0; kind < 5; kind++) {
            const int w = shapes[s][0], h = shapes[s][1];
            for (i = 0; i < w * h; i++) {
                const int x = i % w, y = i / w;
                img[i] = (uint8_t)(kind == 0 ? 77 : kind == 1 ? rnd() : kind == 2 ? (x * 255) / (w > 1 ? w - 1 : 1)
                                   : kind == 3 ? (((x / 3) + (y / 3)) & 1) * 255 : (x * 7 + y * 13 + (rnd() & 7)) & 255);
            }
            for (d = 0; d < 4; d++) {
                /* regions only (a region under 5 points is allowed here), then detection */
                orc_mser_regions(img, w, h, deltas[d], 0, w * h + 1, 10.0, 0.0, NULL, NULL, 0, NULL, 0, &npts);
                orc_mser_regions(img, w, h, deltas[d], 2, 50, 0.25, 0.2, NULL, NULL, 0, NULL, 0, &npts);
                orc_mser_detect(img, w, h, deltas[d], 4, w * h, 1.0, 0.0, kp, 20000);
                orc_mser_detect(img, w, h, deltas[d], 60, 14400, 0.25, 0.2, kp, 20000);
            }
        }
    /* fitEllipse on degenerate sets: collinear (a zero singular value), repeated, tiny */
    for (i = 0; i < 50; i++) {
        pts[2 * i] = i;
        pts[2 * i + 1] = 2 * i + 1;
    }
    {
        float box[5];
        orc_fit_ellipse(pts, 50, box);
        for (i = 0; i < 50; i++) pts[2 * i] = pts[2 * i + 1] = 7;
        orc_fit_ellipse(pts, 50, box);
        if (orc_fit_ellipse(pts, 4, box) != -1) return 1;
    }
    puts("san_mser: ok");
    return 0;
}
