/*
 * bre_fmath.h — single-precision log / exp / sin / cos (host and device) that return the x86-64
 * glibc libm's results bit for bit: the functions the reference calls as std::exp, std::log,
 * std::sin and std::cos on a Float (spectrum.h:222-224, homogeneous.cpp:47,74, grid.cpp:76,104,
 * sampling.cpp:127 ConcentricSampleDisk, medium.cpp:194-213 via SphericalDirection).
 *
 * The photon and camera passes consume random numbers through these.  A Russian-roulette decision
 * or a free-flight distance that moves by one ulp sends a photon down a different path, so the GPU,
 * the oracle and the reference must agree to the bit.  Until round 6 both sides used Cephes-form
 * float routines (within 2 ulp of libm): GPU == oracle, but not == libm.  These are instead the
 * algorithms of glibc >= 2.28's expf / logf / sinf / cosf (the ARM optimized-routines designs,
 * glibc sysdeps/ieee754/flt-32/e_expf.c, e_logf.c, s_sinf.c, s_cosf.c, s_sincosf.h): double
 * arithmetic on small tables, with fused multiply-adds exactly where glibc's x86-64 FMA variants
 * (the ones its ifunc picks on any CPU with FMA and AVX2) have them.  Every operation is an IEEE
 * double operation or an explicit fma, so g++ (-ffp-contract=off) and hipcc (gfx950) compute the same
 * bits.  tests/fmath_libm_check.c compares them with the host libm over all 2^32 inputs
 * (profiles/r6/fmath_libm_exhaustive.txt): identical, NaN payloads aside.
 *
 * Table values: 2^(i/32) (expf), the logf subinterval centres and logs (chosen by the designers; read
 * from the image's libm.so data and checked by the exhaustive comparison), the bits of 2/pi.
 */
#ifndef BRE_FMATH_H
#define BRE_FMATH_H

#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define BRE_HD __host__ __device__ __forceinline__
#define BRE_CONST static constexpr
#else
#define BRE_HD static inline
#define BRE_CONST static const
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
BRE_HD uint64_t bre_d2u(double f) {
    uint64_t u;
    memcpy(&u, &f, 8);
    return u;
}
BRE_HD double bre_u2d(uint64_t u) {
    double f;
    memcpy(&f, &u, 8);
    return f;
}
BRE_HD double bre_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }

/* ---- expf (e_expf.c): exp(x) = 2^(k/32) * 2^(r/32), k = round(x * 32 / ln 2) ---- */
/* tab[i] = bits(2^(i/32)) - (i << 47): 2^(k/32) = double(tab[k % 32] + (k << 47)) */
BRE_CONST uint64_t kBreExp2fTab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull,
};

BRE_HD float bre_expf(float x) {
    const uint32_t abstop = (bre_f2u(x) >> 20) & 0x7ff;
    if (abstop >= 0x42b) { /* |x| >= 88 or nan */
        if (bre_f2u(x) == 0xff800000u) return 0.0f;
        if (abstop >= 0x7f8) return x + x;
        if (x > 0x1.62e42ep6f) return bre_u2f(0x7f800000u);
        if (x < -0x1.9fe368p6f) return 0.0f;
    }
    /* z = InvLn2N * x, fused into both of its uses: kd = z + shift (rounds z to an integer in the
       low bits) and r = z - k */
    const double xd = (double)x, inv_ln2n = 0x1.71547652b82fep+0 * 32;
    double kd = bre_fma(inv_ln2n, xd, 0x1.8p+52);
    const uint64_t ki = bre_d2u(kd);
    kd -= 0x1.8p+52;
    const double r = bre_fma(inv_ln2n, xd, -kd);
    const uint64_t t = kBreExp2fTab[ki % 32] + (ki << 47);
    const double s = bre_u2d(t);
    const double zc = bre_fma(0x1.c6af84b912394p-5 / 32 / 32 / 32, r, 0x1.ebfce50fac4f3p-3 / 32 / 32);
    const double r2 = r * r;
    double y = bre_fma(0x1.62e42ff0c52d6p-1 / 32, r, 1.0);
    y = bre_fma(zc, r2, y);
    y = y * s;
    return (float)y;
}

/* ---- logf (e_logf.c): log(x) = log1p(z/c - 1) + log(c) + k ln 2, z in [0x3f330000, 2x) ---- */
BRE_CONST double kBreLogfTab[16][2] = { /* {invc, logc} */
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2},  {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1p+0, 0x0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aap-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2},  {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2},
};

BRE_HD float bre_logf(float x) {
    uint32_t ix = bre_f2u(x);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) { /* x < 2^-126, inf or nan */
        if (ix * 2 == 0) return -bre_u2f(0x7f800000u);
        if (ix == 0x7f800000u) return x;
        if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return bre_u2f(0x7fc00000u);
        ix = bre_f2u(x * 0x1p23f); /* subnormal: normalise */
        ix -= 23u << 23;
    }
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> (23 - 4)) % 16);
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & 0xff800000u);
    const double invc = kBreLogfTab[i][0], logc = kBreLogfTab[i][1];
    const double z = (double)bre_u2f(iz);
    const double r = bre_fma(z, invc, -1.0);
    const double y0 = bre_fma((double)k, 0x1.62e42fefa39efp-1, logc);
    const double r2 = r * r;
    double y = bre_fma(0x1.5575b0be00b6ap-2, r, -0x1.ffffef20a4123p-2);
    y = bre_fma(-0x1.00ea348b88334p-2, r2, y);
    y = bre_fma(y, r2, y0 + r);
    return (float)y;
}

/* ---- sinf / cosf (s_sinf.c, s_cosf.c, s_sincosf.h) ---- */
/* cos / sin polynomial on [-pi/4, pi/4] for quadrants 0-1 ([0]) and 2-3 ([1], signs flipped) */
BRE_CONST double kBreSincosC[2][5] = {
    {0x1p0, -0x1.ffffffd0c621cp-2, 0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16},
    {-0x1p0, 0x1.ffffffd0c621cp-2, -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16},
};
BRE_CONST double kBreSincosS[3] = {-0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13};
/* windows of the bits of 2/pi (0.a2f9836e 4e441529 fc2757d1 f534ddc0 db629599 3c439041...):
   entry j holds bits [8 (j - 3), 8 (j - 3) + 32) of the fraction, zero-extended on the left */
BRE_CONST uint32_t kBreInvPio4[24] = {
    0xa2,       0xa2f9,     0xa2f983,   0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529,
    0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0,
    0x34ddc0db, 0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041,
};

/* the polynomial for quadrant n on the reduced x (x2 = x * x): sine for even n, cosine for odd
   (sinf_poly); t selects the sign-flipped cosine coefficients of quadrants 2-3 */
BRE_HD float bre_sinf_poly(double x, double x2, int t, int n) {
    if ((n & 1) == 0) {
        const double x3 = x * x2;
        const double s1 = bre_fma(x2, kBreSincosS[2], kBreSincosS[1]);
        const double x7 = x3 * x2;
        const double s = bre_fma(x3, kBreSincosS[0], x);
        return (float)bre_fma(x7, s1, s);
    }
    const double x4 = x2 * x2;
    const double c2 = bre_fma(x2, kBreSincosC[t][4], kBreSincosC[t][3]);
    const double c1 = bre_fma(x2, kBreSincosC[t][1], kBreSincosC[t][0]);
    const double x6 = x4 * x2;
    const double c = bre_fma(x4, kBreSincosC[t][2], c1);
    return (float)bre_fma(x6, c2, c);
}

/* |y| < 120: n = round(y * 2/pi) by the 2^24-scaled truncation, x = y - n pi/2 */
BRE_HD double bre_reduce_fast(double x, int *np) {
    const double r = x * 0x1.45f306dc9c883p+23;
    const int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return bre_fma(-(double)n, 0x1.921fb54442d18p+0, x);
}

/* |y| >= 120: the quadrant and the reduced value from 96 bits of y * 2/pi in integers */
BRE_HD double bre_reduce_large(uint32_t xi, int *np) {
    const uint32_t *arr = &kBreInvPio4[(xi >> 26) & 15];
    const int shift = (xi >> 23) & 7;
    xi = (xi & 0xffffffu) | 0x800000u;
    xi <<= shift;
    uint64_t res0 = (uint64_t)(uint32_t)(xi * arr[0]);
    const uint64_t res1 = (uint64_t)xi * arr[4];
    const uint64_t res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    const uint64_t n = (res0 + (1ull << 61)) >> 62;
    res0 -= n << 62;
    const double x = (double)(int64_t)res0;
    *np = (int)n;
    return x * 0x1.921fb54442d18p-62;
}

BRE_HD float bre_sinf(float y) {
    double x = y;
    const uint32_t at = (bre_f2u(y) >> 20) & 0x7ff;
    int n;
    if (at < 0x3f4) { /* |y| < pi/4 */
        if (at < 0x398) return y; /* |y| < 2^-12 */
        return bre_sinf_poly(x, x * x, 0, 0);
    }
    int q;
    if (at < 0x42f) { /* |y| < 120 */
        x = bre_reduce_fast(x, &n);
        q = n;
    } else if (at < 0x7f8) {
        const uint32_t xi = bre_f2u(y);
        x = bre_reduce_large(xi, &n);
        q = n + (int)(xi >> 31);
    } else {
        return bre_u2f(0x7fc00000u);
    }
    const double s = ((q & 3) == 1 || (q & 3) == 2) ? -1.0 : 1.0;
    return bre_sinf_poly(x * s, x * x, (q & 2) ? 1 : 0, n);
}

BRE_HD float bre_cosf(float y) {
    double x = y;
    const uint32_t at = (bre_f2u(y) >> 20) & 0x7ff;
    int n;
    if (at < 0x3f4) {
        if (at < 0x398) return 1.0f;
        return bre_sinf_poly(x, x * x, 0, 1);
    }
    int q;
    if (at < 0x42f) {
        x = bre_reduce_fast(x, &n);
        q = n;
    } else if (at < 0x7f8) {
        const uint32_t xi = bre_f2u(y);
        x = bre_reduce_large(xi, &n);
        q = n + (int)(xi >> 31);
    } else {
        return bre_u2f(0x7fc00000u);
    }
    const double s = ((q & 3) == 1 || (q & 3) == 2) ? -1.0 : 1.0;
    return bre_sinf_poly(x * s, x * x, (q & 2) ? 1 : 0, n ^ 1);
}

/* std::sin and std::cos of one argument with one reduction (glibc's sincosf: the same values as
   sinf and cosf, which take the same reduction, sign and coefficient set; g++ itself fuses the
   reference's sin / cos pairs into sincosf) */
BRE_HD void bre_sincosf(float y, float *sinp, float *cosp) {
    double x = y;
    const uint32_t at = (bre_f2u(y) >> 20) & 0x7ff;
    int n;
    if (at < 0x3f4) {
        if (at < 0x398) {
            *sinp = y;
            *cosp = 1.0f;
            return;
        }
        const double x2 = x * x;
        *sinp = bre_sinf_poly(x, x2, 0, 0);
        *cosp = bre_sinf_poly(x, x2, 0, 1);
        return;
    }
    int q;
    if (at < 0x42f) {
        x = bre_reduce_fast(x, &n);
        q = n;
    } else if (at < 0x7f8) {
        const uint32_t xi = bre_f2u(y);
        x = bre_reduce_large(xi, &n);
        q = n + (int)(xi >> 31);
    } else {
        *sinp = *cosp = bre_u2f(0x7fc00000u);
        return;
    }
    const double s = ((q & 3) == 1 || (q & 3) == 2) ? -1.0 : 1.0;
    const int t = (q & 2) ? 1 : 0;
    *sinp = bre_sinf_poly(x * s, x * x, t, n);
    *cosp = bre_sinf_poly(x * s, x * x, t, n ^ 1);
}

#endif /* BRE_FMATH_H */
