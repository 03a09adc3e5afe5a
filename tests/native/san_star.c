/* san_star.c -- the STAR oracle (oracle/orc_star.c, test infrastructure) under AddressSanitizer +
 * UndefinedBehaviorSanitizer: the pattern set, integrals, responses and detection on seeded images of
 * the edge shapes (the smallest defined image, a one-pattern border, MaxSize 1..128, bright images whose
 * sums pass 2^24, suppression windows up to the border) and the refused inputs.  Built and run by
 * tests/test_sanitizers.py (tests/native/Makefile); any report aborts with a nonzero status. */
#include <stdio.h>
#include "../../oracle/orc_star.c"

static unsigned long long rs = 0x2545F4914F6CDD1DULL;
static unsigned rnd(void) { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return (unsigned)(rs >> 32); }

int main(void)
{
    static const int shapes[][2] = {{7, 7}, {7, 40}, {40, 7}, {31, 29}, {120, 90}, {400, 390}};
    static const int maxs[] = {1, 2, 8, 16, 23, 45, 90, 128, 129};
    static uint8_t img[400 * 390];
    static orc_kpt k[200000];
    int s, m, i, bright;
    for (bright = 0; bright < 2; bright++)
        for (s = 0; s < 6; s++) {
            const int w = shapes[s][0], h = shapes[s][1];
            for (i = 0; i < w * h; i++) img[i] = (uint8_t)(bright ? 200 + rnd() % 56 : rnd());
            for (m = 0; m < 9; m++) {
                int supp;
                for (supp = 0; supp <= 9; supp += 3) {
                    const int n = orc_star_detect(img, w, h, maxs[m], bright ? 0 : 5, 10, 8, supp, k, 200000);
                    (void)n;
                }
            }
        }
    /* refused: 6-pixel side, MaxSize over 128, a window beyond the border */
    if (orc_star_detect(img, 6, 30, 45, 30, 10, 8, 5, k, 10) != -1) return 1;
    if (orc_star_detect(img, 300, 300, 200, 30, 10, 8, 5, k, 10) != -1) return 1;
    if (orc_star_detect(img, 100, 100, 8, 30, 10, 8, 40, k, 10) != -1) return 1;
    puts("san_star: ok");
    return 0;
}
