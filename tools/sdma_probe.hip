// Does a D2H copy slow a concurrently running kernel, by copy engine?  (test infrastructure; not the product)
//   busy kernel alone | + hipMemcpyAsync D2H (runtime blit kernel) | + hsa_amd_memory_async_copy (SDMA)
// Build: hipcc --offload-arch=gfx950 -O2 tools/sdma_probe.hip -o /tmp/sdma_probe -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
#define HK(x) do { hsa_status_t s_ = (x); if (s_ != HSA_STATUS_SUCCESS) { printf("HSA %d at %d\n", (int)s_, __LINE__); return 1; } } while (0)

__global__ void busy(float *out, int iters)
{
    float a = threadIdx.x * 1e-3f, b = 1.0001f;
    for (int i = 0; i < iters; ++i)
        a = a * b + 1e-7f;
    if (a == 12345.f)
        out[threadIdx.x] = a;
}

static std::vector<hsa_agent_t> g_gpu, g_cpu;
static hsa_status_t collect(hsa_agent_t a, void *)
{
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU)
        g_gpu.push_back(a);
    else if (t == HSA_DEVICE_TYPE_CPU)
        g_cpu.push_back(a);
    return HSA_STATUS_SUCCESS;
}

int main()
{
    const size_t n = 1920 * 1080 * 3;
    unsigned char *dsrc, *hdst;
    float *dout;
    CK(hipMalloc(&dsrc, n));
    CK(hipMalloc(&dout, 4096));
    CK(hipHostMalloc(&hdst, n, 0));
    CK(hipMemset(dsrc, 7, n));
    hipStream_t ks, cs;
    CK(hipStreamCreateWithFlags(&ks, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    HK(hsa_init());
    HK(hsa_iterate_agents(collect, nullptr));
    printf("agents: %zu gpu, %zu cpu\n", g_gpu.size(), g_cpu.size());
    hsa_signal_t sig;
    HK(hsa_signal_create(1, 0, nullptr, &sig));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int iters = 200000, grid = 256 * 8;
    auto run_busy = [&](int mode) -> float {
        hipEventRecord(e0, ks);
        hipLaunchKernelGGL(busy, dim3(grid), dim3(256), 0, ks, dout, iters);
        hipEventRecord(e1, ks);
        for (int c = 0; c < 4; ++c) {
            if (mode == 1) {
                hipMemcpyAsync(hdst, dsrc, n, hipMemcpyDeviceToHost, cs);
            } else if (mode == 2) {
                hsa_signal_store_screlease(sig, 1);
                hsa_amd_memory_async_copy(hdst, g_cpu[0], dsrc, g_gpu[0], n, 0, nullptr, sig);
                hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
            }
        }
        hipStreamSynchronize(cs);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        return ms;
    };
    for (int rep = 0; rep < 3; ++rep)
        for (int mode = 0; mode < 3; ++mode)
            printf("mode %s busy kernel %.4f ms\n", mode == 0 ? "alone" : (mode == 1 ? "+blit D2H x4" : "+SDMA D2H x4"), run_busy(mode));
    /* the SDMA copy alone, and its data */
    memset(hdst, 0, n);
    auto t0 = std::chrono::steady_clock::now();
    for (int c = 0; c < 10; ++c) {
        hsa_signal_store_screlease(sig, 1);
        HK(hsa_amd_memory_async_copy(hdst, g_cpu[0], dsrc, g_gpu[0], n, 0, nullptr, sig));
        hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
    }
    auto t1 = std::chrono::steady_clock::now();
    printf("SDMA D2H alone %.4f ms per copy, data ok %d\n",
           std::chrono::duration<double, std::milli>(t1 - t0).count() / 10, hdst[0] == 7 && hdst[n - 1] == 7);
    return 0;
}
