/*
 * tools/sincosf_sweep.c -- pins the cosf/sinf of the rBRIEF rotation (ORBextractor.cc:120-130)
 * against the host libm, exhaustively.  Test infrastructure: links the oracle's restatement.
 *
 *   make -C oracle && gcc -O2 -fopenmp -ffp-contract=off -Ioracle tools/sincosf_sweep.c \
 *       oracle/_build/liborbg_oracle.so -lm -o /tmp/sincosf_sweep && /tmp/sincosf_sweep
 *
 * 1. orc_glibc_sinf / orc_glibc_cosf (glibc 2.35 flt-32 restated) vs the linked libm's
 *    sinf / cosf for EVERY float in [0, 7) (1,088,421,888 inputs; the rotation angle is
 *    fastAtan2's [0, 360] degrees times (float)(pi / 180), i.e. at most 6.2832).
 * 2. Round 1's pin (correctly rounded double evaluation) vs glibc for every float angle in
 *    [0, 360] degrees, and for each angle where they differ, how many of the 512 rotated
 *    rBRIEF sample offsets cvRound(x*b + y*a), cvRound(x*a - y*b) change (no FMA, the
 *    default; ORBextractor.cc:128-130).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "orb_oracle.h"

static const signed char pat[256][4] = {
#define ORBG_PAIR(a, b, c, d) {a, b, c, d},
#include "orb_pattern.inc"
#undef ORBG_PAIR
};

static int sample_changes(float a0, float b0, float a1, float b1)
{
    int n = 0;
    for (int t = 0; t < 256; t++)
        for (int s = 0; s < 2; s++) {
            const float x = (float)pat[t][2 * s], y = (float)pat[t][2 * s + 1];
            const float ry0 = x * b0 + y * a0, rx0 = x * a0 - y * b0;
            const float ry1 = x * b1 + y * a1, rx1 = x * a1 - y * b1;
            n += (lrintf(ry0) != lrintf(ry1)) || (lrintf(rx0) != lrintf(rx1));
        }
    return n;
}

int main(void)
{
    long bad = 0, n1 = 0;
#pragma omp parallel for reduction(+ : bad, n1) schedule(static, 1 << 16)
    for (uint32_t u = 0; u < 0x40E00000u; u++) {
        float y;
        memcpy(&y, &u, 4);
        const float a = sinf(y), b = orc_glibc_sinf(y), c = cosf(y), d = orc_glibc_cosf(y);
        bad += memcmp(&a, &b, 4) != 0;
        bad += memcmp(&c, &d, 4) != 0;
        n1++;
    }
    printf("glibc restatement vs host libm: %ld floats in [0, 7), %ld mismatches (sinf+cosf)\n",
           n1, bad);

    const uint32_t hi = 0x43B40000u; /* 360.0f */
    long nang = 0, ndiff = 0, nmoved = 0, nsamples = 0;
#pragma omp parallel for reduction(+ : nang, ndiff, nmoved, nsamples) schedule(static, 1 << 16)
    for (uint32_t u = 0; u <= hi; u++) {
        float deg;
        memcpy(&deg, &u, 4);
        float ap, bp, ag, bg;
        orc_brief_sincos_deg(deg, ORC_SINCOS_PINNED, &ap, &bp);
        orc_brief_sincos_deg(deg, ORC_SINCOS_GLIBC, &ag, &bg);
        nang++;
        if (ap != ag || bp != bg) {
            ndiff++;
            const int m = sample_changes(ap, bp, ag, bg);
            if (m) {
                nmoved++;
                nsamples += m;
            }
        }
    }
    printf("angles in [0, 360] deg: %ld; pinned != glibc on %ld; of those %ld move at least one "
           "rounded rBRIEF sample (%ld samples in all)\n", nang, ndiff, nmoved, nsamples);
    return bad != 0;
}
