// Exhaustive GPU check of the exact f32 shortcuts in rtc_device.h against the operations they replace, over
// all 2^32 float bit patterns (test infrastructure; tests/test_gpu_exact.py runs it, `make probe` builds it):
//   sqrt_cr(x)  == (float)sqrt((double)x)        (length(), moremath.c:9)
//   rcp_cr(x)   == 1.f / x  (IEEE f32 divide)     (normalized(), moremath.c:14; (float)(1./x) == 1.f/x)
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

int main()
{
    unsigned long long *bad;
    if (hipMalloc(&bad, 2 * sizeof(unsigned long long)) != hipSuccess) {
        printf("no device\n");
        return 2;
    }
    (void)hipMemset(bad, 0, 2 * sizeof(unsigned long long));
    const unsigned long long chunk = 1ull << 30;
    for (unsigned long long base = 0; base < (1ull << 32); base += chunk)
        hipLaunchKernelGGL(check, dim3((unsigned)(chunk / 256)), dim3(256), 0, nullptr, base, bad);
    unsigned long long h[2] = {0, 0};
    if (hipMemcpy(h, bad, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) {
        printf("copy failed\n");
        return 2;
    }
    printf("sqrt_cr mismatches %llu checked %llu\n", h[0], 1ull << 32);
    printf("rcp_cr mismatches %llu checked %llu\n", h[1], 1ull << 32);
    return (h[0] | h[1]) ? 1 : 0;
}
