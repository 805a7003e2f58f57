/*
 * bre_fmath.h — portable single-precision transcendental functions (host and device).
 *
 * The photon and camera passes consume random numbers through log / exp / sin / cos
 * (medium free-flight sampling, Beer-Lambert transmittance, Henyey-Greenstein and cosine
 * hemisphere sampling, homogeneous.cpp:50-77, medium.cpp:194-213, sampling.h:159-163).  A
 * Russian-roulette decision that flips on a one-ulp difference between glibc and the GPU's libm
 * would send a photon down a different path, so both sides use these functions, built only from
 * IEEE-exact operations (+ - * /, comparisons, bit manipulation) and compiled without FMA
 * contraction: the results are bit-identical on x86-64 (g++) and gfx950 (hipcc).
 * Accuracy is about 1-2 ulp over the ranges used (Cephes single-precision algorithms).
 */
#ifndef BRE_FMATH_H
#define BRE_FMATH_H

#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define BRE_HD __host__ __device__ __forceinline__
#else
#define BRE_HD static inline
#endif

BRE_HD uint32_t bre_f2u(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}
BRE_HD float bre_u2f(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}

/* round to nearest integer value (ties away from zero), exact for |x| < 2^22 */
BRE_HD float bre_roundf(float x) {
    const float big = 8388608.0f; /* 2^23 */
    float a = x < 0 ? -x : x;
    if (!(a < big)) return x;
    float r = (a + 0.5f);
    /* truncate r toward zero via the 2^23 trick */
    float t = (r + big) - big;
    if (t > r) t = t - 1.0f;
    return x < 0 ? -t : t;
}

/* 2^n for integer n in [-126, 127] */
BRE_HD float bre_pow2i(int n) { return bre_u2f((uint32_t)(n + 127) << 23); }

/* natural logarithm, x > 0 (Cephes logf) */
BRE_HD float bre_logf(float x) {
    if (!(x > 0.0f)) return x == 0.0f ? -bre_u2f(0x7f800000u) : bre_u2f(0x7fc00000u);
    if (x == bre_u2f(0x7f800000u)) return x;
    uint32_t u = bre_f2u(x);
    int e = (int)((u >> 23) & 0xff);
    if (e == 0) { /* subnormal: scale up */
        x = x * 16777216.0f;
        u = bre_f2u(x);
        e = (int)((u >> 23) & 0xff) - 24;
    }
    e -= 126;
    float m = bre_u2f((u & 0x807fffffu) | 0x3f000000u); /* m in [0.5, 1) */
    if (m < 0.70710678118654752440f) {
        e -= 1;
        m = m + m - 1.0f;
    } else {
        m = m - 1.0f;
    }
    const float z = m * m;
    float y = 7.0376836292e-2f;
    y = y * m + -1.1514610310e-1f;
    y = y * m + 1.1676998740e-1f;
    y = y * m + -1.2420140846e-1f;
    y = y * m + 1.4249322787e-1f;
    y = y * m + -1.6668057665e-1f;
    y = y * m + 2.0000714765e-1f;
    y = y * m + -2.4999993993e-1f;
    y = y * m + 3.3333331174e-1f;
    y = y * m * z;
    const float fe = (float)e;
    y = y + -2.12194440e-4f * fe;
    y = y + -0.5f * z;
    float r = m + y;
    r = r + 0.693359375f * fe;
    return r;
}

/* e^x (Cephes expf); returns 0 below -103.97, +inf above 88.72 */
BRE_HD float bre_expf(float x) {
    if (x != x) return x;
    if (x > 88.72283935546875f) return bre_u2f(0x7f800000u);
    if (x < -103.972084045410f) return 0.0f;
    float n = bre_roundf(x * 1.44269504088896341f);
    float r = x - n * 0.693359375f;
    r = r - n * -2.12194440e-4f;
    const float z = r * r;
    float p = 1.9875691500e-4f;
    p = p * r + 1.3981999507e-3f;
    p = p * r + 8.3334519073e-3f;
    p = p * r + 4.1665795894e-2f;
    p = p * r + 1.6666665459e-1f;
    p = p * r + 5.0000001201e-1f;
    p = p * z + r + 1.0f;
    int ni = (int)n;
    if (ni < -126) { /* gradual underflow in two steps */
        p = p * bre_pow2i(-126);
        ni += 126;
        if (ni < -126) return 0.0f;
    }
    if (ni > 127) {
        p = p * bre_pow2i(127);
        ni -= 127;
    }
    return p * bre_pow2i(ni);
}

/* sin and cos of x, |x| <= 2^13 (Cephes sinf/cosf with the 3-part pi/4 reduction) */
BRE_HD void bre_sincosf(float x, float *s, float *c) {
    float sign_s = 1.0f;
    if (x < 0) {
        x = -x;
        sign_s = -1.0f;
    }
    float jf = x * 1.27323954473516f; /* 4/pi */
    int j = (int)jf;
    if (j & 1) {
        j += 1;
    }
    const float y = (float)j;
    j &= 7;
    float z = ((x - y * 0.78515625f) - y * 2.4187564849853515625e-4f) - y * 3.77489497744594108e-8f;
    float sign_c = 1.0f;
    if (j > 3) {
        j -= 4;
        sign_s = -sign_s;
        sign_c = -sign_c;
    }
    if (j > 1) sign_c = -sign_c;
    const float zz = z * z;
    float ps = -1.9515295891e-4f;
    ps = ps * zz + 8.3321608736e-3f;
    ps = ps * zz + -1.6666654611e-1f;
    ps = ps * zz * z + z;
    float pc = 2.443315711809948e-5f;
    pc = pc * zz + -1.388731625493765e-3f;
    pc = pc * zz + 4.166664568298827e-2f;
    pc = pc * zz * zz;
    pc = pc - 0.5f * zz + 1.0f;
    if (j == 1 || j == 2) {
        *s = sign_s * pc;
        *c = sign_c * ps;
    } else {
        *s = sign_s * ps;
        *c = sign_c * pc;
    }
}

#endif /* BRE_FMATH_H */
