// sin and cos in fp64 of an angle 0 <= x <= 2*pi + 1e-3 (rBRIEF's rotation, pinned P6:
// (float)cos((double)a), (float)sin((double)a)): Cody-Waite reduction by pi/2 (n <= 4: n * pio2_1
// is exact) and the fdlibm k_sin / k_cos minimax kernels (y = 0), one rounding per operation
// (-ffp-contract=off).  Far cheaper than the general libm path, and tools/trig_check.c checks
// that both values, rounded to float, equal glibc's for EVERY float in the domain.  Shared by the
// device code and that host check (ORBMI_TRIG_HOST).
#pragma once

#ifdef ORBMI_TRIG_HOST
#include <math.h>
#include <stdint.h>
#include <string.h>
#define ORBMI_TRIG_FN static inline
static inline uint32_t orbmi_trig_hi(double x) { uint64_t u; memcpy(&u, &x, 8); return (uint32_t)(u >> 32); }
static inline double orbmi_trig_from_hi(uint32_t h) { uint64_t u = (uint64_t)h << 32; double x; memcpy(&x, &u, 8); return x; }
#else
#define ORBMI_TRIG_FN __device__ inline
__device__ inline uint32_t orbmi_trig_hi(double x) { return (uint32_t)__double2hiint(x); }
__device__ inline double orbmi_trig_from_hi(uint32_t h) { return __hiloint2double((int)h, 0); }
#endif

ORBMI_TRIG_FN void orbmi_sincos_f64(double x, double* sp, double* cp) {
    const double invpio2 = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00;   // the first 33 bits of pi/2
    const double pio2_1t = 6.07710050650619224932e-11;  // pi/2 - pio2_1
    const double n = rint(x * invpio2);
    const double r = (x - n * pio2_1) - n * pio2_1t;
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double z = r * r;
    // k_sin: r + r^3 (S1 + z (S2 + ... + z S6))
    const double ps = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    const double s = r + (z * r) * (S1 + z * ps);
    // k_cos: 1 - (z/2 - z q) below |r| = 0.3, else with fdlibm's split 1 - qx, qx ~ |r| / 4
    const double q = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    const uint32_t ix = orbmi_trig_hi(r) & 0x7fffffffu;
    double c;
    if (ix < 0x3FD33333u) {
        c = 1.0 - (0.5 * z - z * q);
    } else {
        const double qx = ix > 0x3fe90000u ? 0.28125 : orbmi_trig_from_hi(ix - 0x00200000u);
        const double hz = 0.5 * z - qx;
        const double a = 1.0 - qx;
        c = a - (hz - z * q);
    }
    switch ((int)n & 3) {
        case 0: *sp = s; *cp = c; break;
        case 1: *sp = c; *cp = -s; break;
        case 2: *sp = -s; *cp = -c; break;
        default: *sp = -c; *cp = s; break;
    }
}
