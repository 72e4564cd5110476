// Blocking SDMA copies through the HSA runtime (test infrastructure for tools/sdma_overlap_probe.py; not the
// product).  Build: g++ -O2 -shared -fPIC tools/sdma_copy.cpp -o raytracingc_amd/_lib/libsdma_copy.so
//   -I/opt/rocm/include -L/opt/rocm/lib -lhsa-runtime64
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cstdint>
#include <vector>

static std::vector<hsa_agent_t> g_gpu, g_cpu;
static hsa_signal_t g_sig;
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

extern "C" int sdma_init()
{
    if (hsa_init() != HSA_STATUS_SUCCESS)
        return 1;
    if (hsa_iterate_agents(collect, nullptr) != HSA_STATUS_SUCCESS || g_gpu.empty() || g_cpu.empty())
        return 2;
    return hsa_signal_create(1, 0, nullptr, &g_sig) == HSA_STATUS_SUCCESS ? 0 : 3;
}

extern "C" int sdma_copy_d2h(void *dst, const void *src, size_t n)
{
    hsa_signal_store_screlease(g_sig, 1);
    if (hsa_amd_memory_async_copy(dst, g_cpu[0], src, g_gpu[0], n, 0, nullptr, g_sig) != HSA_STATUS_SUCCESS)
        return 1;
    hsa_signal_wait_scacquire(g_sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
    return 0;
}
