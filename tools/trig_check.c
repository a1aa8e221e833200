/* Exhaustive check of orbmi's rBRIEF rotation cos/sin (csrc/trig_f64.h) against the pinned
 * semantics P6, (float)cos((double)a) / (float)sin((double)a) with glibc, over EVERY float a in
 * [0, 2*pi + 1e-3] (the angle of IC_Angle in radians: fastAtan2 degrees * (float)(pi / 180)).
 *   gcc -O2 -fopenmp -ffp-contract=off -I orb_slam2_with_comment_amd/csrc tools/trig_check.c -lm
 * Prints the number of floats checked and of mismatches (expected 0). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#define ORBMI_TRIG_HOST 1
#include "trig_f64.h"

int main(void) {
    const float lo = 0.0f, hi = 6.2841854f;
    uint32_t ulo, uhi;
    memcpy(&ulo, &lo, 4);
    memcpy(&uhi, &hi, 4);
    long long bad = 0, n = 0;
#pragma omp parallel for reduction(+ : bad, n) schedule(static, 1 << 16)
    for (long long u = ulo; u <= (long long)uhi; u++) {
        const uint32_t w = (uint32_t)u;
        float a;
        memcpy(&a, &w, 4);
        double s, c;
        orbmi_sincos_f64((double)a, &s, &c);
        const float fs = (float)s, fc = (float)c;
        const float gs = (float)sin((double)a), gc = (float)cos((double)a);
        n++;
        if (memcmp(&fs, &gs, 4) || memcmp(&fc, &gc, 4)) {
            if (bad < 10) printf("mismatch a=%.9g (0x%08x): sin %.9g vs %.9g  cos %.9g vs %.9g\n", a, w, fs, gs, fc, gc);
            bad++;
        }
    }
    printf("checked %lld floats in [0, %.7g]: %lld mismatches\n", n, hi, bad);
    return bad != 0;
}
