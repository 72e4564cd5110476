// Micro-benchmark of the sky path's pieces on the GPU (not part of the product):
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 tools/sky_bench.hip -o /tmp/sky_bench
// One thread per pixel of a 1920x1080 frame, 64 "samples" each:
//   0: write-only (launch + store cost)            1: 64 accumulations of a constant
//   2: environment once + 64 accumulations           3: environment every sample (opaque direction)
//   4: like 3 with the powf tables in LDS            5: like 3, 2 pixels per thread (ILP)
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../raytracingc_amd/csrc/rtc_device.h"

using namespace rtcdev;

template <int MODE> __device__ __forceinline__ V3 dir_of(int x, int y)
{
    if (MODE >= 6) { /* the default camera of main.c:114-116 (basis main.c:252-255) */
        const V3 ex{0.7132819890975952f, 0.0f, -0.7008771300315857f};
        const V3 ey{-0.026064898818731308f, 0.9993083477020264f, -0.026526223868131638f};
        const V3 ez{0.7003923058509827f, 0.03718896582722664f, 0.7127885818481445f};
        const float dx = (float)(x - 960) / 540.f, dy = (float)(y - 540) / 540.f;
        return normalized(add(add(mul(ex, dx), mul(ey, dy)), ez));
    }
    const float dx = (float)(x - 960) / 540.f, dy = (float)(y - 540) / 540.f;
    return normalized(V3{dx * 0.7f + 0.1f, dy - 0.2f, 1.f});
}

template <int MODE>
__global__ __launch_bounds__(256) void sky(EnvParams env, unsigned char *out, int W, int H, int spp)
{
    __shared__ PowTablesLds sPow;
    if (MODE == 4 || MODE == 6) {
        sPow.fill(threadIdx.x);
        __syncthreads();
        sPow.attach(env);
    }
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= W || y >= H)
        return;
    V3 d = dir_of<MODE>(x, y);
    V3 acc{0.f, 0.f, 0.f};
    const float inv = 1.f / (float)spp;
    if (MODE == 1) {
        for (int s = 0; s < spp; ++s)
            acc = add(acc, mul(V3{0.5f, 0.6f, 0.7f}, inv));
    } else if (MODE == 2) {
        const V3 l = environment(d, env);
        for (int s = 0; s < spp; ++s)
            acc = add(acc, mul(l, inv));
    } else if (MODE == 3 || MODE == 4 || MODE == 6) {
        for (int s = 0; s < spp; ++s) {
            asm volatile("" : "+v"(d.x), "+v"(d.y), "+v"(d.z));
            acc = add(acc, mul(environment(d, env), inv));
        }
    } else if (MODE == 5) {
        V3 d2 = dir_of<MODE>(x + 1, y);
        V3 acc2{0.f, 0.f, 0.f};
        for (int s = 0; s < spp; s += 2) {
            asm volatile("" : "+v"(d.x), "+v"(d.y), "+v"(d.z), "+v"(d2.x), "+v"(d2.y), "+v"(d2.z));
            acc = add(acc, mul(environment(d, env), inv));
            acc2 = add(acc2, mul(environment(d2, env), inv));
        }
        acc = add(acc, acc2);
    }
    const size_t o = (size_t)y * W + x;
    out[3 * o] = float_to_u8(acc.x);
    out[3 * o + 1] = float_to_u8(acc.y);
    out[3 * o + 2] = float_to_u8(acc.z);
}

template <int MODE> float run(EnvParams env, unsigned char *out)
{
    dim3 grid(120, 68);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(sky<MODE>, grid, dim3(256), 0, nullptr, env, out, 1920, 1080, 64);
    hipEventRecord(a);
    for (int i = 0; i < 5; ++i)
        hipLaunchKernelGGL(sky<MODE>, grid, dim3(256), 0, nullptr, env, out, 1920, 1080, 64);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main()
{
    EnvParams env{};
    env.sun = V3{-0.2f, -0.6f, 0.77f};
    env.horizon = V3{1.f, 1.f, 1.f};
    env.zenith = V3{0.263f, 0.969f, 0.871f};
    env.ground = V3{0.66f, 0.66f, 0.66f};
    env.focus = 22.f;
    env.intensity = 0.75f;
    unsigned char *out;
    hipMalloc(&out, 1920 * 1080 * 3);
    printf("mode0 write-only      %.3f ms\n", run<0>(env, out));
    printf("mode1 64 const acc    %.3f ms\n", run<1>(env, out));
    printf("mode2 env once        %.3f ms\n", run<2>(env, out));
    printf("mode3 env per sample  %.3f ms\n", run<3>(env, out));
    printf("mode4 env/sample LDS  %.3f ms\n", run<4>(env, out));
    printf("mode5 2 px per thread %.3f ms\n", run<5>(env, out));
    env.sun = V3{-0.22283440828323364f, -0.6313641667366028f, 0.7427813410758972f};
    printf("mode6 real camera+sun %.3f ms\n", run<6>(env, out));
    hipFree(out);
    return 0;
}
