// Exhaustive check of raytracingc_amd/csrc/rtc_math.h against glibc on the input sets the renderer produces.
//   g++ -O2 -ffp-contract=off -fopenmp -std=c++17 tools/check_devmath.cpp -o /tmp/check_devmath
//   /tmp/check_devmath [stride]      (stride 1 = every float; larger = sampled)
// Reports, per function, how many inputs give a different double / a different float result than glibc.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../raytracingc_amd/csrc/rtc_math.h"

static float f_of(uint32_t b)
{
    float f;
    memcpy(&f, &b, 4);
    return f;
}

int main(int argc, char **argv)
{
    const uint32_t stride = argc > 1 ? (uint32_t)atoi(argv[1]) : 1;
    // 1. log of u in (0, 1] -> rho = (float)sqrt(-2 log u)   (moremath.c:100)
    long long n1 = 0, dlog = 0, drho = 0;
#pragma omp parallel for reduction(+ : n1, dlog, drho) schedule(static, 65536)
    for (long long b = 1; b <= 0x3f800000LL; b += stride) {
        const double u = (double)f_of((uint32_t)b);
        const double a = rtcmath::log(u), g = ::log(u);
        n1++;
        dlog += (a != g);
        drho += ((float)sqrt(-2 * a) != (float)sqrt(-2 * g));
    }
    printf("log: %lld inputs, %lld double != glibc, %lld float rho != glibc\n", n1, dlog, drho);
    // 2. cos of theta in [0, 2*pi) as a float (moremath.c:99-101)
    long long n2 = 0, dcos = 0, dprod = 0;
#pragma omp parallel for reduction(+ : n2, dcos, dprod) schedule(static, 65536)
    for (long long b = 0; b <= 0x40c90fdbLL; b += stride) {
        const double t = (double)f_of((uint32_t)b);
        const double a = rtcmath::cos(t), g = ::cos(t);
        n2++;
        dcos += (a != g);
        // a product with a few typical rho values
        const float rhos[4] = {0.37f, 1.0f, 1.7724539f, 3.3f};
        for (float r : rhos)
            dprod += ((float)((double)r * a) != (float)((double)r * g));
    }
    printf("cos: %lld inputs, %lld double != glibc, %lld float rho*cos != glibc (4 rho each)\n", n2, dcos, dprod);
    // 2b. the certified fast Box-Muller path (rtc_math.h bm_*): the fast schemes' largest errors against glibc
    //     (they must stay within the certification tolerances), the rho path's certified floats against glibc's
    //     on every u, and certified normals on random (u1, u2) draws
    {
        long long nr = 0, certR = 0, wrongR = 0;
        double maxRelRho = 0.0;
#pragma omp parallel for reduction(+ : nr, certR, wrongR) reduction(max : maxRelRho) schedule(static, 65536)
        for (long long b = 1; b <= 0x3f800000LL; b += stride) {
            const float u = f_of((uint32_t)b);
            const double g = sqrt(-2 * ::log((double)u));
            const double a = rtcmath::bm_rho_d(u);
            if (g > 0 && b >= 0x00800000LL) /* normal u (the RNG's are 0 or >= 2^-32) */
                maxRelRho = fmax(maxRelRho, fabs(a - g) / g);
            float rho;
            const bool ok = rtcmath::bm_rho_fast(u, rho);
            nr++;
            certR += ok;
            wrongR += ok && rtcmath::f2u(rho) != rtcmath::f2u((float)g);
        }
        printf("bm_rho: %lld inputs, %lld certified, %lld certified != glibc, max rel err %.3g (tol %.3g)\n", nr, certR,
               wrongR, maxRelRho, rtcmath::kBmRhoTol);
        long long nc = 0;
        double maxAbsCos = 0.0;
#pragma omp parallel for reduction(+ : nc) reduction(max : maxAbsCos) schedule(static, 65536)
        for (long long b = 0; b <= 0x40c90fdbLL; b += stride) {
            const float t = f_of((uint32_t)b);
            nc++;
            maxAbsCos = fmax(maxAbsCos, fabs(rtcmath::bm_cos_d(t) - ::cos((double)t)));
        }
        printf("bm_cos: %lld inputs, max abs err %.3g (tol %.3g)\n", nc, maxAbsCos, rtcmath::kBmNrmTol);
        long long nn = 0, certN = 0, wrongN = 0;
#pragma omp parallel for reduction(+ : nn, certN, wrongN) schedule(static, 1 << 16)
        for (long long k = 0; k < 400000000LL / (long long)stride + 1; ++k) {
            uint64_t x = (uint64_t)k * 0x9e3779b97f4a7c15ull;
            x ^= x >> 29, x *= 0xbf58476d1ce4e5b9ull, x ^= x >> 32;
            const float u1 = (float)fma((double)(uint32_t)x, 0x1p-64, (double)(uint32_t)x * 0x1p-32);
            const float u2 = (float)fma((double)(uint32_t)(x >> 32), 0x1p-64, (double)(uint32_t)(x >> 32) * 0x1p-32);
            const float theta = (float)(2 * 3.14159265 * (double)u1);
            const float rho = (float)sqrt(-2 * ::log((double)u2));
            const float g = (float)((double)rho * ::cos((double)theta));
            float n;
            const bool ok = rtcmath::bm_normal_fast(rho, theta, n);
            nn++;
            certN += ok;
            wrongN += ok && rtcmath::f2u(n) != rtcmath::f2u(g);
        }
        printf("bm_normal: %lld draws, %lld certified, %lld certified != glibc\n", nn, certN, wrongN);
    }
    // 3. powf(x, y) for x in [0, 1] (raytracing.c:153,155)
    const float ys[3] = {0.35f, 22.f, 7.5f};
    for (float y : ys) {
        long long n3 = 0, dglibc = 0, dcr = 0;
#pragma omp parallel for reduction(+ : n3, dglibc, dcr) schedule(static, 65536)
        for (long long b = 0; b <= 0x3f800000LL; b += stride) {
            const float x = f_of((uint32_t)b);
            const float a = rtcmath::pow_ref(x, y);
            const float g = powf(x, y);
            const float c = (y == 0.f || x == 1.f) ? 1.f : (float)::exp2((double)y * ::log2((double)x));
            n3++;
            dglibc += (a != g);
            dcr += (a != c);
        }
        printf("pow y=%g: %lld inputs, %lld != glibc powf, %lld != double-glibc exp2(y*log2 x)\n", y, n3, dglibc, dcr);
    }
    // 4. the restated glibc powf (FMA build and plain build) against libm's own powf, every float x in [0, 1]
    const float ys2[5] = {0.35f, 22.f, 7.5f, 1.3f, 0.5f};
    for (float y : ys2) {
        long long n4 = 0, dfma = 0, dplain = 0;
#pragma omp parallel for reduction(+ : n4, dfma, dplain) schedule(static, 65536)
        for (long long b = 0; b <= 0x3f800000LL; b += stride) {
            const float x = f_of((uint32_t)b);
            const uint32_t g = rtcmath::f2u(powf(x, y));
            n4++;
            dfma += rtcmath::f2u(rtcmath::powf_glibc<true>(x, y)) != g;
            dplain += rtcmath::f2u(rtcmath::powf_glibc<false>(x, y)) != g;
        }
        printf("glibc-powf y=%g: %lld inputs, fma-build %lld != libm, plain-build %lld != libm\n", y, n4, dfma, dplain);
    }
    // 4b. RandomValue's divide-free form (rtc_device.h random_value) on every u32
    {
        long long dr = 0;
#pragma omp parallel for reduction(+ : dr) schedule(static, 1 << 20)
        for (long long r = 0; r <= 0xffffffffLL; r += stride) {
            const float a = (float)((double)r / 4294967295.0);
            const float b = (float)fma((double)r, 0x1p-64, (double)r * 0x1p-32);
            dr += (a != b);
        }
        printf("random_value: %lld != divide\n", dr);
    }
    // 5. random (x, y) over the whole float range (both signs, subnormals, inf, NaN): bits compared, NaN == NaN
    {
        long long n5 = 0, d5 = 0;
        uint64_t s = 0x9e3779b97f4a7c15ull;
        for (long long k = 0; k < 20000000 / (long long)stride + 1000; ++k) {
            s ^= s << 13, s ^= s >> 7, s ^= s << 17;
            const float x = f_of((uint32_t)s), y = (k & 1) ? f_of((uint32_t)(s >> 32)) : (float)(int)((s >> 40) % 64) - 31.f;
            const float g = powf(x, y), a = rtcmath::powf_glibc<true>(x, y);
            n5++;
            d5 += !((g != g && a != a) || rtcmath::f2u(g) == rtcmath::f2u(a));
        }
        printf("glibc-powf random: %lld inputs, fma-build %lld != libm\n", n5, d5);
    }
    return 0;
}
