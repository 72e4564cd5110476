// Exhaustive GPU check of the exact f32 shortcuts in rtc_device.h against the operations they replace, over
// all 2^32 float bit patterns (test infrastructure; tests/test_gpu_exact.py runs it, `make probe` builds it):
//   sqrt_cr(x)  == (float)sqrt((double)x)        (length(), moremath.c:9)
//   rcp_cr(x)   == 1.f / x  (IEEE f32 divide)     (normalized(), moremath.c:14; (float)(1./x) == 1.f/x)
//   powf_glibc_pos(x, y) == powf_glibc(x, y) bit for bit, every x with the sign bit clear, y in kPowY;
//   powf_sky_unit(x) == powf_glibc(x, 0.35f), every normal x in [2^-126, 1]
//                                                 (getEnvironmentLight's powf, raytracing.c:153,155)
//   bm_rho_fast(u) == (float)sqrt(-2 log u) (exact restatement) whenever certified, every float u in (0, 1];
//   bm_normal_fast(rho, theta) == (float)(rho cos theta) likewise, every float theta in [0, 2 pi] x 4 rho
//                                                 (the certified fast Box-Muller path, moremath.c:97-102)
//   smoothstep_k<S>(x) == smoothstep(inf, sup, x) bit for bit, all 2^32 x, both of getEnvironmentLight's
//                                                 smoothsteps (raytracing.c:153,156; moremath.c:49-53)
// Prints one line per check: "<name> mismatches <n> checked <m>".  Exit status 0 iff every count is 0.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../raytracingc_amd/csrc/rtc_device.h"

using namespace rtcdev;

__device__ __forceinline__ bool same(float a, float b)
{
    return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
}

__global__ void check(unsigned long long base, unsigned long long *bad)
{
    const unsigned long long i = base + blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    const float x = __uint_as_float((unsigned)i);
    unsigned b0 = 0, b1 = 0;
    double xd = (double)x;
    asm volatile("" : "+v"(xd)); /* keep the double sqrt (no fptrunc(sqrt(fpext)) -> sqrtf folding) */
    if (!same(sqrt_cr(x), (float)__builtin_sqrt(xd)))
        b0 = 1;
    if (!same(rcp_cr(x), 1.f / x))
        b1 = 1;
    const unsigned long long m0 = __ballot(b0), m1 = __ballot(b1);
    if ((threadIdx.x & 63) == 0) {
        if (m0)
            atomicAdd(&bad[0], (unsigned long long)__popcll(m0));
        if (m1)
            atomicAdd(&bad[1], (unsigned long long)__popcll(m1));
    }
}

__constant__ float kPowY[8] = {0.35f, 22.f, 7.5f, 1.3f, 0.5f, -3.f, 150.f, 1e-5f};

__global__ void check_pow(unsigned long long base, unsigned long long *bad)
{
    const unsigned long long i = base + blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    const float x = __uint_as_float((unsigned)i); /* i < 2^31: sign bit clear */
    unsigned b = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const float y = kPowY[k];
        if (__float_as_uint(rtcmath::powf_glibc_pos<true>(x, y)) != __float_as_uint(rtcmath::powf_glibc<true>(x, y)))
            b++;
    }
    const unsigned long long m = __ballot(b != 0);
    if ((threadIdx.x & 63) == 0 && m)
        atomicAdd(&bad[2], (unsigned long long)__popcll(m));
    const bool unit = i >= 0x00800000ull && i <= 0x3f800000ull &&
                      __float_as_uint(rtcmath::powf_sky_unit(x)) != __float_as_uint(rtcmath::powf_glibc<true>(x, 0.35f));
    const unsigned long long mu = __ballot(unit);
    if ((threadIdx.x & 63) == 0 && mu)
        atomicAdd(&bad[6], (unsigned long long)__popcll(mu));
}

__device__ __forceinline__ float smoothstep_div(float inf, float sup, float x)
{
    float d = sup - inf;
    asm volatile("" : "+v"(d)); /* an IEEE f32 divide, as moremath.c:51 */
    x = clamp01((x - inf) / d);
    return (float)((double)(x * x) * (3.0 - 2.0 * (double)x));
}

__global__ void check_smooth(unsigned long long base, unsigned long long *bad)
{
    const unsigned long long i = base + blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    const float x = __uint_as_float((unsigned)i);
    const bool b0 = !same(smoothstep_k<kSkyStep>(x), smoothstep_div(0.f, 0.74f, x));
    const bool b1 = !same(smoothstep_k<kGroundStep>(x), smoothstep_div(-0.01f, 0.f, x));
    const unsigned long long m0 = __ballot(b0), m1 = __ballot(b1);
    if ((threadIdx.x & 63) == 0) {
        if (m0)
            atomicAdd(&bad[3], (unsigned long long)__popcll(m0));
        if (m1)
            atomicAdd(&bad[4], (unsigned long long)__popcll(m1));
    }
}

__global__ void check_bm(unsigned long long base, unsigned long long *bad)
{
    const unsigned long long i = base + blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    unsigned b = 0, c = 0;
    if (i >= 1 && i <= 0x3f800000ull) { /* u in (0, 1] */
        const float u = __uint_as_float((unsigned)i);
        float rho;
        if (rtcmath::bm_rho_fast(u, rho)) {
            c++;
            b += __float_as_uint(rho) != __float_as_uint((float)__builtin_sqrt(-2 * rtcmath::log((double)u)));
        }
    }
    if (i <= 0x40c90fdbull) { /* theta in [0, 2 pi] */
        const float t = __uint_as_float((unsigned)i);
        const float rhos[4] = {0.37f, 1.0f, 1.7724539f, 3.3f};
        for (float r : rhos) {
            float n;
            if (rtcmath::bm_normal_fast(r, t, n)) {
                c++;
                b += __float_as_uint(n) != __float_as_uint((float)((double)r * rtcmath::cos((double)t)));
            }
        }
    }
    const unsigned long long m = __ballot(b != 0);
    if ((threadIdx.x & 63) == 0 && m)
        atomicAdd(&bad[5], (unsigned long long)__popcll(m));
    (void)c;
}

int main()
{
    unsigned long long *bad;
    if (hipMalloc(&bad, 7 * sizeof(unsigned long long)) != hipSuccess) {
        printf("no device\n");
        return 2;
    }
    (void)hipMemset(bad, 0, 7 * sizeof(unsigned long long));
    const unsigned long long chunk = 1ull << 30;
    for (unsigned long long base = 0; base < (1ull << 32); base += chunk)
        hipLaunchKernelGGL(check, dim3((unsigned)(chunk / 256)), dim3(256), 0, nullptr, base, bad);
    for (unsigned long long base = 0; base < (1ull << 31); base += chunk)
        hipLaunchKernelGGL(check_pow, dim3((unsigned)(chunk / 256)), dim3(256), 0, nullptr, base, bad);
    for (unsigned long long base = 0; base < (1ull << 31); base += chunk)
        hipLaunchKernelGGL(check_bm, dim3((unsigned)(chunk / 256)), dim3(256), 0, nullptr, base, bad);
    for (unsigned long long base = 0; base < (1ull << 32); base += chunk)
        hipLaunchKernelGGL(check_smooth, dim3((unsigned)(chunk / 256)), dim3(256), 0, nullptr, base, bad);
    unsigned long long h[7] = {0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpy(h, bad, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) {
        printf("copy failed\n");
        return 2;
    }
    printf("sqrt_cr mismatches %llu checked %llu\n", h[0], 1ull << 32);
    printf("rcp_cr mismatches %llu checked %llu\n", h[1], 1ull << 32);
    printf("powf_glibc_pos mismatches %llu checked %llu\n", h[2], 8ull << 31);
    printf("smoothstep_sky mismatches %llu checked %llu\n", h[3], 1ull << 32);
    printf("smoothstep_ground mismatches %llu checked %llu\n", h[4], 1ull << 32);
    printf("bm_fast mismatches %llu checked %llu\n", h[5], 0x3f800000ull + 4 * 0x40c90fdcull);
    printf("powf_sky_unit mismatches %llu checked %llu\n", h[6], 0x3f800000ull - 0x00800000ull + 1);
    return (h[0] | h[1] | h[2] | h[3] | h[4] | h[5] | h[6]) ? 1 : 0;
}
