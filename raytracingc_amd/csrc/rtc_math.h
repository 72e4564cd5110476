/*
 * rtc_math.h -- compact double-precision log / cos / exp2 for the device path (host-compilable for checks).
 *
 * Why: the reference evaluates Box-Muller in double (moremath.c:99-101: log, sqrt, cos) and the sky in
 * powf (raytracing.c:153,155).  The generic ocml double routines handle every range (Payne-Hanek reduction
 * etc.) and cost ~60 VGPRs inside the render kernel, halving its occupancy.  The arguments here are narrow:
 * log of a RandomValue() in (0, 1], cos of theta = 2*pi*u in [0, 2*pi), exp2 of y*log2(x) <= 0 mostly, so
 * short, classic algorithms suffice:
 *   - log: the fdlibm e_log.c scheme (Sun Microsystems, freely distributable): x = 2^k (1+f),
 *     s = f/(2+f), Remez polynomial Lg1..Lg7 in s^2, < 1 ulp;
 *   - cos: fdlibm's medium-range reduction by pi/2 (33+33+33-bit split of pi/2) and __kernel_cos /
 *     __kernel_sin polynomials (C1..C6, S1..S6), < 1 ulp;
 *   - exp2: t = k + r, |r| <= 1/2, exp(r*ln2) by a degree-14 Taylor polynomial (truncation < 2^-57), ldexp.
 * They are checked against glibc on the exact input sets the renderer can produce
 * (tools/check_devmath.cpp, tests/test_devmath.py): what matters is that the FLOAT values the reference
 * derives from them ((float)sqrt(-2 log u), (float)(rho*cos(theta)), powf) come out identical.
 *
 * Compile with -ffp-contract=off: every fma below is explicit, every other product/sum is rounded.
 */
#pragma once

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define RTC_HD __host__ __device__ __forceinline__
#else
#include <cmath>
#include <cstdint>
#include <cstring>
#define RTC_HD inline
#endif

namespace rtcmath {

RTC_HD unsigned hi_word(double x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return (unsigned)(__double_as_longlong(x) >> 32);
#else
    unsigned long long b;
    memcpy(&b, &x, sizeof b);
    return (unsigned)(b >> 32);
#endif
}

RTC_HD double with_hi_word(unsigned hi)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __longlong_as_double((long long)((unsigned long long)hi << 32));
#else
    unsigned long long b = (unsigned long long)hi << 32;
    double x;
    memcpy(&x, &b, sizeof x);
    return x;
#endif
}

/* natural log for finite x > 0 (0 -> -inf, inf -> inf, x < 0 or NaN -> NaN).  Branch-free in the common
 * domain (selects, not branches: lanes of a wave take different paths otherwise). */
RTC_HD double log(double x)
{
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                 Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    int k;
    double m = frexp(x, &k); /* x = m 2^k, m in [0.5, 1) */
    m *= 2.0;                 /* m in [1, 2) */
    k -= 1;
    /* hx: the 20 high mantissa bits, as fdlibm keeps them; fold m into [sqrt(1/2), sqrt(2)) */
    const unsigned hx = hi_word(m) & 0x000fffffu;
    const bool fold = hx >= 0x6a09eu;
    m = fold ? m * 0.5 : m;
    k = fold ? k + 1 : k;
    const double f = m - 1.0; /* exact (Sterbenz) */
    const double dk = (double)k;
    /* -2^-20 <= f < 2^-20: short series (fdlibm); the general forms below give dk*(ln2_hi+ln2_lo) at f = 0 */
    const double Rs = f * f * (0.5 - 0.33333333333333333 * f);
    const double small = dk * ln2_hi - ((Rs - dk * ln2_lo) - f);
    const double s = f / (2.0 + f);
    const double z = s * s;
    const double w = z * z;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    const double R = t2 + t1;
    const double hfsq = 0.5 * f * f;
    const double nearSqrt2 = dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    const double other = dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
    const int i = (int)hx - 0x6147a, j = 0x6b851 - (int)hx;
    double r = (i | j) > 0 ? nearSqrt2 : other;
    r = ((0x000fffffu & (2u + hx)) < 3u) ? small : r;
    r = x == 0.0 ? -__builtin_inf() : r;
    r = x == __builtin_inf() ? x : r;
    return (x >= 0.0) ? r : __builtin_nan(""); /* x < 0 or NaN */
}

/* fdlibm __kernel_cos(x, y), |x| <= pi/4, y the tail of x (selects instead of branches) */
RTC_HD double kcos(double x, double y)
{
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03, C3 = 2.48015872894767294178e-05,
                 C4 = -2.75573143513906633035e-07, C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const unsigned ix = hi_word(x) & 0x7fffffffu;
    const double z = x * x;
    const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    const double small = 1.0 - (0.5 * z - (z * r - x * y)); /* |x| < 0.3 */
    const double qx = ix > 0x3fe90000u ? 0.28125 : with_hi_word(ix - 0x00200000u); /* x/4 (high word only) */
    const double hz = 0.5 * z - qx;
    const double a = 1.0 - qx;
    const double big = a - (hz - (z * r - x * y));
    return ix < 0x3e400000u ? 1.0 : (ix < 0x3FD33333u ? small : big);
}

/* fdlibm __kernel_sin(x, y, iy=1), |x| <= pi/4 */
RTC_HD double ksin(double x, double y)
{
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03, S3 = -1.98412698298579493134e-04,
                 S4 = 2.75573137070700676789e-06, S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const unsigned ix = hi_word(x) & 0x7fffffffu;
    const double z = x * x;
    const double v = z * x;
    const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    const double res = x - ((z * (0.5 * y - v * r) - y) - v * S1);
    return ix < 0x3e400000u ? x : res;
}

/* cos for |x| < 2^19 * pi/2 (fdlibm __ieee754_rem_pio2 medium case); larger |x| is not produced here */
RTC_HD double cos(double x)
{
    const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
                 pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
                 pio2_2t = 2.02226624879595063154e-21, pio2_3 = 2.02226624871116645580e-21,
                 pio2_3t = 8.47842766036889956997e-32;
    const unsigned ix = hi_word(x) & 0x7fffffffu;
    const bool tiny = ix <= 0x3fe921fbu; /* |x| <= pi/4: no reduction */
    const double fn = tiny ? 0.0 : rint(x * invpio2);
    const int n = (int)fn;
    double r = x - fn * pio2_1;
    double w = fn * pio2_1t;
    double y0 = r - w;
    const int j = (int)(ix >> 20);
    int i = j - (int)((hi_word(y0) >> 20) & 0x7ffu);
    if (!tiny && i > 16) { /* cancellation near a multiple of pi/2: 2nd iteration, 118 bits of pi/2 */
        double t = r;
        w = fn * pio2_2;
        r = t - w;
        w = fn * pio2_2t - ((t - r) - w);
        y0 = r - w;
        i = j - (int)((hi_word(y0) >> 20) & 0x7ffu);
        if (i > 49) { /* 3rd iteration: 151 bits */
            t = r;
            w = fn * pio2_3;
            r = t - w;
            w = fn * pio2_3t - ((t - r) - w);
            y0 = r - w;
        }
    }
    const double y1 = tiny ? 0.0 : (r - y0) - w;
    const double c = kcos(y0, y1), sn = ksin(y0, y1);
    const int q = n & 3;
    const double res = q == 0 ? c : (q == 1 ? -sn : (q == 2 ? -c : sn));
    return ix >= 0x7ff00000u ? x - x : res; /* inf or NaN -> NaN */
}

/* 2^t */
RTC_HD double exp2(double t)
{
    if (t != t)
        return t;
    if (t >= 1024.0)
        return __builtin_inf();
    if (t < -1080.0)
        return 0.0;
    const double k = rint(t);
    const double z = (t - k) * 6.93147180559945286227e-01; /* |z| <= ln2/2 */
    double p = 1.1470745597729725e-11;                      /* 1/14! */
    p = fma(p, z, 1.6059043836821613e-10);                  /* 1/13! */
    p = fma(p, z, 2.08767569878680989792e-09);              /* 1/12! */
    p = fma(p, z, 2.50521083854417187751e-08);              /* 1/11! */
    p = fma(p, z, 2.75573192239858906526e-07);              /* 1/10! */
    p = fma(p, z, 2.75573192239858906526e-06);              /* 1/9!  */
    p = fma(p, z, 2.48015873015873015873e-05);              /* 1/8!  */
    p = fma(p, z, 1.98412698412698412698e-04);              /* 1/7!  */
    p = fma(p, z, 1.38888888888888888889e-03);              /* 1/6!  */
    p = fma(p, z, 8.33333333333333333333e-03);              /* 1/5!  */
    p = fma(p, z, 4.16666666666666666667e-02);              /* 1/4!  */
    p = fma(p, z, 1.66666666666666666667e-01);              /* 1/3!  */
    p = fma(p, z, 0.5);
    p = fma(p, z, 1.0);
    p = fma(p, z, 1.0);
    return ldexp(p, (int)k);
}

/* powf(x, y) of raytracing.c:153,155 for x >= 0 (or NaN): exp2(y * log2(x)) in double, rounded once */
RTC_HD float pow_ref(float x, float y)
{
    if (y == 0.f || x == 1.f)
        return 1.f;
    if (x == 0.f)
        return y > 0.f ? 0.f : __builtin_inff();
    const double l2 = rtcmath::log((double)x) * 1.44269504088896338700e+00; /* log2(x) */
    return (float)rtcmath::exp2((double)y * l2);
}

} // namespace rtcmath
