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

/* ---- glibc's powf, restated -----------------------------------------------------------------------------
 * The reference calls powf (raytracing.c:153,155) from glibc 2.35 libm.  That powf is ARM's optimized-routines
 * algorithm (sysdeps/ieee754/flt-32/e_powf.c, published under MIT / Apache-2.0): log2(x) from a 16-entry
 * {1/c, log2 c} table and a degree-5 polynomial in r = z/c - 1, then y*log2(x), then 2^t from a 32-entry table
 * of 2^(i/32) and a degree-3 polynomial, all in double, with ONE final rounding to float.  It is not correctly
 * rounded (<= 0.82 ulp), so matching it bit for bit needs the same tables, coefficients and operation order.
 * On x86-64 glibc picks its FMA build (__powf_fma) on every CPU with FMA + AVX2; that build contracts each
 * a*b+c below into a fused multiply-add (FMA = true).  The table and coefficient values are glibc's
 * __powf_log2_data / __exp2f_data (tools/extract_glibc_powf.py reads them out of libm.so.6);
 * tools/check_devmath.cpp checks this restatement against libm's powf on every float x in [0, 1]. */
namespace powf_data {
constexpr double kLog2Tab[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.efec65b963019p-2}, {0x1.571ed4aaf883dp+0, -0x1.b0b6832d4fca4p-2},
    {0x1.49539f0f010b0p+0, -0x1.7418b0a1fb77bp-2}, {0x1.3c995b0b80385p+0, -0x1.39de91a6dcf7bp-2},
    {0x1.30d190c8864a5p+0, -0x1.01d9bf3f2b631p-2}, {0x1.25e227b0b8ea0p+0, -0x1.97c1d1b3b7af0p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.2f9e393af3c9fp-3}, {0x1.12358f08ae5bap+0, -0x1.960cbbf788d5cp-4},
    {0x1.0953f419900a7p+0, -0x1.a6f9db6475fcep-5}, {0x1.0000000000000p+0, 0x0.0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.338ca9f24f53dp-4},  {0x1.ca4b31f026aa0p-1, 0x1.476a9543891bap-3},
    {0x1.b2036576afce6p-1, 0x1.e840b4ac4e4d2p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.40645f0c6651cp-2},
    {0x1.886e6037841edp-1, 0x1.88e9c2c1b9ff8p-2},  {0x1.767dcf5534862p-1, 0x1.ce0a44eb17bccp-2},
};
constexpr double kLog2Poly[5] = {0x1.27616c9496e0bp-2, -0x1.71969a075c67ap-2, 0x1.ec70a6ca7baddp-2,
                                 -0x1.7154748bef6c8p-1, 0x1.71547652ab82bp+0};
/* asuint64(2^(i/32)) - (i << 47) */
constexpr unsigned long long kExp2Tab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull,
};
constexpr double kExp2Poly[3] = {0x1.c6af84b912394p-5, 0x1.ebfce50fac4f3p-3, 0x1.62e42ff0c52d6p-1};
constexpr double kExp2Shift = 0x1.8p+52 / 32; /* __exp2f_data.shift_scaled */
constexpr unsigned kSignBias = 1u << (5 + 11);
} // namespace powf_data

RTC_HD unsigned f2u(float f)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __float_as_uint(f);
#else
    unsigned u;
    memcpy(&u, &f, 4);
    return u;
#endif
}
RTC_HD float u2f(unsigned u)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __uint_as_float(u);
#else
    float f;
    memcpy(&f, &u, 4);
    return f;
#endif
}
RTC_HD unsigned long long d2u(double d)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return (unsigned long long)__double_as_longlong(d);
#else
    unsigned long long u;
    memcpy(&u, &d, 8);
    return u;
#endif
}
RTC_HD double u2d(unsigned long long u)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __longlong_as_double((long long)u);
#else
    double d;
    memcpy(&d, &u, 8);
    return d;
#endif
}

/* a*b + c as the chosen glibc build evaluates it: fused (FMA build) or two roundings */
template <bool FMA> RTC_HD double mad(double a, double b, double c) { return FMA ? fma(a, b, c) : a * b + c; }

/* 0: not an integer, 1: odd integer, 2: even integer (e_powf.c checkint) */
RTC_HD int powf_checkint(unsigned iy)
{
    const int e = (int)(iy >> 23 & 0xff);
    if (e < 0x7f)
        return 0;
    if (e > 0x7f + 23)
        return 2;
    if (iy & ((1u << (0x7f + 23 - e)) - 1))
        return 0;
    if (iy & (1u << (0x7f + 23 - e)))
        return 1;
    return 2;
}
RTC_HD bool powf_zeroinfnan(unsigned ix) { return 2 * ix - 1 >= 2u * 0x7f800000u - 1; }

/* tables: glibc's by default; the device passes copies staged in LDS (same values) */
template <bool FMA> RTC_HD double powf_log2(unsigned ix, const double (*tab)[2] = powf_data::kLog2Tab) /* e_powf.c log2_inline */
{
    const unsigned tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> (23 - 4)) % 16);
    const unsigned top = tmp & 0xff800000u;
    const unsigned iz = ix - top;
    const int k = (int)top >> 23; /* arithmetic shift */
    const double invc = tab[i][0], logc = tab[i][1];
    const double z = (double)u2f(iz);
    const double r = mad<FMA>(z, invc, -1.0);
    const double y0 = logc + (double)k;
    const double *A = powf_data::kLog2Poly;
    const double r2 = r * r;
    double y = mad<FMA>(A[0], r, A[1]);
    const double p = mad<FMA>(A[2], r, A[3]);
    const double r4 = r2 * r2;
    double q = mad<FMA>(A[4], r, y0);
    q = mad<FMA>(p, r2, q);
    y = mad<FMA>(y, r4, q);
    return y;
}

template <bool FMA>
RTC_HD float powf_exp2(double xd, unsigned signBias,
                       const unsigned long long *tab = powf_data::kExp2Tab) /* e_powf.c exp2_inline */
{
    double kd = xd + powf_data::kExp2Shift;
    const unsigned long long ki = d2u(kd);
    kd -= powf_data::kExp2Shift;
    const double r = xd - kd;
    unsigned long long t = tab[ki % 32];
    const unsigned long long ski = ki + signBias;
    t += ski << (52 - 5);
    const double s = u2d(t);
    const double *C = powf_data::kExp2Poly;
    const double z = mad<FMA>(C[0], r, C[1]);
    const double r2 = r * r;
    double y = mad<FMA>(C[2], r, 1.0);
    y = mad<FMA>(z, r2, y);
    y = y * s;
    return (float)y;
}

/* powf(x, y) for a special y (+-0, +-inf, NaN: powf_zeroinfnan(iy)), any x -- e_powf.c's first special case */
RTC_HD float powf_special_y(float x, float y)
{
    const unsigned ix = f2u(x), iy = f2u(y);
    /* signalling NaN: quiet bit clear */
    auto sig = [](unsigned u) { return (u & 0x7fc00000u) == 0x7f800000u && (u & 0x003fffffu) != 0; };
    if (2 * iy == 0)
        return sig(ix) ? x + y : 1.0f;
    if (ix == 0x3f800000u)
        return sig(iy) ? x + y : 1.0f;
    if (2 * ix > 2u * 0x7f800000u || 2 * iy > 2u * 0x7f800000u)
        return x + y;
    if (2 * ix == 2u * 0x3f800000u)
        return 1.0f;
    if ((2 * ix < 2u * 0x3f800000u) == !(iy & 0x80000000u))
        return 0.0f;
    return y * y;
}

template <bool FMA>
RTC_HD float powf_glibc(float x, float y, const double (*log2tab)[2] = powf_data::kLog2Tab,
                        const unsigned long long *exp2tab = powf_data::kExp2Tab) /* e_powf.c __powf, round-to-nearest */
{
    unsigned signBias = 0;
    unsigned ix = f2u(x), iy = f2u(y);
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u || powf_zeroinfnan(iy)) {
        if (powf_zeroinfnan(iy))
            return powf_special_y(x, y);
        if (powf_zeroinfnan(ix)) {
            float x2 = x * x;
            if ((ix & 0x80000000u) && powf_checkint(iy) == 1)
                x2 = -x2;
            return (iy & 0x80000000u) ? 1.0f / x2 : x2;
        }
        if (ix & 0x80000000u) { /* finite x < 0 */
            const int yint = powf_checkint(iy);
            if (yint == 0)
                return __builtin_nanf("");
            if (yint == 1)
                signBias = powf_data::kSignBias;
            ix &= 0x7fffffffu;
        }
        if (ix < 0x00800000u) { /* subnormal x: normalise */
            ix = f2u(x * 0x1p23f);
            ix &= 0x7fffffffu;
            ix -= 23u << 23;
        }
    }
    const double logx = powf_log2<FMA>(ix, log2tab);
    const double ylogx = (double)y * logx;
    if ((d2u(ylogx) >> 47 & 0xffff) >= d2u(126.0) >> 47) {
        if (ylogx > 0x1.fffffffd1d571p+6)
            return signBias ? -__builtin_inff() : __builtin_inff();
        if (ylogx <= -150.0)
            return signBias ? -0.0f : 0.0f;
    }
    return powf_exp2<FMA>(ylogx, signBias, exp2tab);
}

/* powf_glibc for the environment's arguments, branch-free: x with the sign bit clear (+0, subnormal, normal,
 * +inf or NaN) and y finite and nonzero.  The main path runs for every x (bounded table indices whatever
 * the bits) and glibc's special results are selected over it: x = +0 -> 0 (1/0 = inf for y < 0), NaN ->
 * x*x (1/(x*x) for y < 0), +inf -> inf (0 for y < 0), subnormal x normalised first, the over/underflow
 * limits of the exp2 step.  Bit-identical to powf_glibc on every such x (tools/exact_probe.hip). */
template <bool FMA>
RTC_HD float powf_glibc_pos(float x, float y, const double (*log2tab)[2] = powf_data::kLog2Tab,
                            const unsigned long long *exp2tab = powf_data::kExp2Tab)
{
    const unsigned ix = f2u(x), iy = f2u(y);
    const bool sub = ix < 0x00800000u;
    const unsigned ixs = (f2u(x * 0x1p23f) & 0x7fffffffu) - (23u << 23);
    const double logx = powf_log2<FMA>(sub ? ixs : ix, log2tab);
    const double ylogx = (double)y * logx;
    float r = powf_exp2<FMA>(ylogx, 0u, exp2tab);
    r = ylogx > 0x1.fffffffd1d571p+6 ? __builtin_inff() : r;
    r = ylogx <= -150.0 ? 0.0f : r;
    const bool yneg = (iy & 0x80000000u) != 0;
    const float x2 = x * x;
    r = ix == 0u ? (yneg ? __builtin_inff() : 0.0f) : r;
    r = ix == 0x7f800000u ? (yneg ? 0.0f : __builtin_inff()) : r;
    r = ix > 0x7f800000u ? (yneg ? 1.0f / x2 : x2) : r;
    return r;
}

/* getEnvironmentLight's sky term powf(x, 0.35f) (raytracing.c:153) for a normal x in [2^-126, 1] (smoothstep's value
 * above the horizon): glibc's main path alone.  There 0.35 log2(x) lies in [-44.1, 0], so none of powf_glibc_pos's
 * special results (x = 0, inf, NaN, subnormal x, the exp2 step's overflow and underflow limits) applies and its selects
 * are no-ops.  Bit-identical to powf_glibc(x, 0.35f) on every such x (tools/exact_probe.hip). */
RTC_HD float powf_sky_unit(float x, const double (*log2tab)[2] = powf_data::kLog2Tab,
                           const unsigned long long *exp2tab = powf_data::kExp2Tab)
{
    const double logx = powf_log2<true>(f2u(x), log2tab);
    return powf_exp2<true>((double)0.35f * logx, 0u, exp2tab);
}

/* ---- certified fast Box-Muller (RandomValueNormalDistrubtion, moremath.c:97-102) -----------------------
 * The reference's rho = (float)sqrt(-2 log(u)) and n = (float)((double)rho * cos((double)theta)) need glibc's
 * log and cos only up to the final float rounding.  The fast path evaluates them with short table-driven
 * schemes (no divide, no branches) and CERTIFIES each float: it is returned only when the double value lies
 * farther from the float rounding midpoint than the combined error bound of the fast evaluation and of the
 * reference's own double evaluation (glibc log / cos, double sqrt / product roundings) -- then both round to
 * the same float.  Otherwise the caller falls back to the exact restatement (log / cos above).  The bounds are
 * measured exhaustively (tools/check_devmath.cpp: every float u in (0, 1], every float theta in [0, 2 pi]), and
 * the rho path's final floats are compared with glibc's on every input.
 *   log: u = 2^k z (glibc's reduction on the float bits), r = z invc - 1 exact (invc a float), log u =
 *        k ln2 + logc + log1p(r), log1p by a degree-7 polynomial, |r| <= 2^-7;
 *   cos: theta = j 2pi/64 + t (j * kBmStepHi exact), |t| <= pi/64, cos theta = cos_j cos t - sin_j sin t. */
#include "rtc_bm_tables.h"

constexpr double kBmLn2Hi = 6.93147180369123816490e-01, kBmLn2Lo = 1.90821492927058770002e-10; /* 43-bit hi */
constexpr double kBmRhoTol = 0x1p-44; /* relative to rho */
constexpr double kBmNrmTol = 0x1p-46; /* absolute, per unit rho */

/* f32 sqrt for the Newton seed of bm_rho_d: v_sqrt_f32 on the device (<= 1 ulp for the normal arguments it gets
 * here), the correctly rounded sqrtf on the host -- the seed's error enters only through the Newton step's bound */
RTC_HD float bm_sqrtf(float x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_sqrtf(x);
#else
    return sqrtf(x);
#endif
}
/* 1 / x for x in [2^-125, 2^125] (rtc_device.h rcp_cr: v_rcp_f32 and two FMA Newton steps, the IEEE quotient for every
 * such x), inf for x = 0 */
RTC_HD float bm_rcpf(float x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    float r = __builtin_amdgcn_rcpf(x);
    r = __builtin_fmaf(__builtin_fmaf(-x, r, 1.0f), r, r);
    return __builtin_fmaf(__builtin_fmaf(-x, r, 1.0f), r, r);
#else
    return 1.0f / x;
#endif
}

/* half an ulp of a normal float f (exponent field E >= 1), as a double */
RTC_HD double bm_half_ulp(float f) { return u2d((unsigned long long)(((f2u(f) >> 23) & 0xffu) + 1023u - 151u) << 52); }

/* sqrt(-2 log((double)u)) in double, for u in (0, 1] (the fast scheme, before certification) */
RTC_HD double bm_rho_d(float u, const BmLogEntry *logTab = kBmLogTab)
{
    const unsigned iu = f2u(u);
    const unsigned tmp = iu - 0x3f330000u;
    const BmLogEntry e = logTab[(tmp >> 16) & 127u];
    const double dk = (double)((int)tmp >> 23);
    const double r = fma((double)u2f(iu - (tmp & 0xff800000u)), (double)e.invc, -1.0); /* exact */
    /* log1p(r) = r + r^2 (-1/2 + r/3 - r^2/4 + r^3/5 - r^4/6): the dropped r^7/7 is below 2^-51.8 absolute (|r| <=
     * 2^-7 in the entry of c = 1), the largest relative error of rho it leaves is 1.7e-14 = 2^-45.8 (at u = 1 - 2^-7,
     * exhaustive over every float u, tools/check_devmath.cpp), inside kBmRhoTol = 2^-44 */
    double q = -1.0 / 6.0;
    q = fma(q, r, 0.2);
    q = fma(q, r, -0.25);
    q = fma(q, r, 1.0 / 3.0);
    q = fma(q, r, -0.5);
    const double p = fma(r * r, q, r);
    const double hi = fma(dk, kBmLn2Hi, e.logcHi);
    const double lo = fma(dk, kBmLn2Lo, (double)e.logcLo) + p;
    const double L = -2.0 * (hi + lo);
    /* sqrt(L) without the correctly rounded double square root: the f32 root of (float)L, rf = sqrt(L) (1 + d) with
     * |d| <= 2^-23 + 2^-25 (the rounding of L, v_sqrt_f32's ulp), and one Newton step in double, rho = rf + (L - rf^2)
     * / (2 rf), its quotient from the correctly rounded f32 1 / (2 rf): the step leaves d^2 / 2 < 2^-46.6 and the
     * quotient's error |d| 2^-24 < 2^-46.7 of rho, together inside kBmRhoTol = 2^-44 (every float u is checked on the
     * GPU, tools/exact_probe.hip).  L >= 2^-23 for u < 1 (the RNG's u are >= 2^-32, so L < 45); u = 1 gives L = 0: rf
     * = 0, its 1 / rf inf and rho NaN -- not certified (bm_rho_fast) */
    const float rf = bm_sqrtf((float)L);
    const double e2 = fma(-(double)rf, (double)rf, L);
    const float hq = 0.5f * bm_rcpf(rf);
    return fma(e2, (double)hq, (double)rf);
}
/* rho = (float)sqrt(-2 log((double)u)) for u in (0, 1]; false: not certified (use the exact path) */
RTC_HD bool bm_rho_fast(float u, float &rho, const BmLogEntry *logTab = kBmLogTab)
{
    const double rd = bm_rho_d(u, logTab);
    const float f = (float)rd;
    rho = f;
    const double d = fabs(rd - (double)f);
    return (f2u(f) & 0x7f800000u) != 0u && f2u(u) >= 0x00800000u && d < fma(-rd, kBmRhoTol, bm_half_ulp(f));
}
/* cos((double)theta) in double for theta in [0, 2 pi] (the fast scheme) */
RTC_HD double bm_cos_d(float theta, const double (*cosTab)[2] = kBmCosTab)
{
    const double th = (double)theta;
    const double jd = rint(th * kBmInvStep);
    double t = fma(-jd, kBmStepHi, th); /* exact */
    t = fma(-jd, kBmStepLo, t);
    const double z = t * t;
    /* z = t^2 <= 2^-8.7: cos t = 1 - z/2 + z^2/24 - z^3/720 (the dropped z^4/8! < 2^-50), sin t = t (1 - z/6 + z^2/120 -
     * z^3/5040) (the dropped t z^4/9! < 2^-57) */
    double c = -1.0 / 720.0;
    c = fma(c, z, 1.0 / 24.0);
    c = fma(c, z, -0.5);
    c = fma(c, z, 1.0);
    double sn = -1.0 / 5040.0;
    sn = fma(sn, z, 1.0 / 120.0);
    sn = fma(sn, z, -1.0 / 6.0);
    sn = fma(sn * z, t, t);
    const int j = (int)jd & 63;
    return fma(cosTab[j][0], c, -cosTab[j][1] * sn);
}
/* n = (float)((double)rho * cos((double)theta)) for theta = (float)(2 pi u) in [0, 2 pi]; false: not certified */
RTC_HD bool bm_normal_fast(float rho, float theta, float &n, const double (*cosTab)[2] = kBmCosTab)
{
    const double rd = (double)rho * bm_cos_d(theta, cosTab);
    const float f = (float)rd;
    n = f;
    const double d = fabs(rd - (double)f);
    return (f2u(f) & 0x7f800000u) != 0u && d < fma(-(double)rho, kBmNrmTol, bm_half_ulp(f));
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
